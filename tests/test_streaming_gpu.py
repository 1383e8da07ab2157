"""GPU parity of the host-resident streamed path (streaming.reproject_host):
band-wise H2D -> K1 -> D2H on three streams == the reference goldens and the
resident K1 launch, bit for bit, for every band height (1 row, partial tile
rows, whole tile rows) and several dim-0 slices."""

from __future__ import annotations

import numpy as np
import pytest

from helpers import assert_bitwise_equal, load_golden, reproject_golden_inputs

pytestmark = pytest.mark.gpu


def _plan(g):
    import xcube_resampling_amd as xrs

    ds, tgm = reproject_golden_inputs(g)
    sgm = xrs.GridMapping.from_dataset(ds)
    return xrs.plan_reproject(sgm, tgm, xrs.Transformer.from_crs(tgm.crs, sgm.crs,
                                                                  always_xy=True))


@pytest.mark.parametrize("band_rows", [None, 1, 5, 13])
@pytest.mark.parametrize("interp", ["nearest", "bilinear", "triangular"])
def test_streamed_matches_reference_goldens(interp, band_rows):
    from xcube_resampling_amd import streaming

    for case in ("f32", "i16"):
        g = load_golden(f"reproject_{case}.npz")
        out = streaming.reproject_host(g["data"], _plan(g), interp, g["fill"].item(),
                                       band_rows=band_rows)
        assert_bitwise_equal(out, g[f"out_{interp}"], f"{case}/{interp} band_rows={band_rows}")


def test_streamed_multi_slice_matches_resident():
    """1536x2048 source, 3 slices, 1900x1700 target in 256^2 tiles."""
    import torch

    import xcube_resampling_amd as xrs
    from xcube_resampling_amd import kernels, streaming

    rng = np.random.default_rng(11)
    h, w = 1536, 2048
    lon = -5.0 + (np.arange(w) + 0.5) * 0.0045
    lat = 60.0 - (np.arange(h) + 0.5) * 0.003
    sgm = xrs.GridMapping.from_coords(xrs.DataArray(lon, "lon", name="lon"),
                                      xrs.DataArray(lat, "lat", name="lat"), "EPSG:4326")
    tgm = xrs.GridMapping.regular((1700, 1900), (-520000.0, 7450000.0), (480.0, 470.0),
                                  "EPSG:3857", tile_size=256)
    plan = xrs.plan_reproject(sgm, tgm, xrs.Transformer.from_crs(tgm.crs, sgm.crs,
                                                                  always_xy=True))
    data = rng.random((3, h, w), dtype=np.float32)
    data.ravel()[rng.choice(data.size, data.size // 500, replace=False)] = np.nan
    dev = torch.from_numpy(data).cuda()
    ref = kernels.reproject(dev, plan, "bilinear", np.nan).cpu().numpy()
    for band in (None, 100, 700):
        got = streaming.reproject_host(data, plan, "bilinear", np.nan, band_rows=band)
        assert_bitwise_equal(got, ref, f"band_rows={band}")
    ref32 = kernels.reproject(dev, plan, "bilinear", np.nan, out_dtype=np.float32).cpu().numpy()
    out = np.empty_like(ref32)
    got32 = streaming.reproject_host(data, plan, "bilinear", np.nan, out_dtype=np.float32,
                                     out=out)
    assert got32 is out
    assert_bitwise_equal(got32, ref32, "f32 out")


def test_dataset_api_streams_host_arrays():
    import xcube_resampling_amd as xrs

    g = load_golden("reproject_f32.npz")
    ds, tgm = reproject_golden_inputs(g)
    with xrs.set_options(host_streaming_min_bytes=0):
        out = xrs.reproject_dataset(ds, tgm, interp_methods="bilinear",
                                    fill_values=g["fill"].item())
        ds2 = xrs.Dataset(data_vars={"v": (("lat", "lon"), g["data"][1])},
                          coords={"lon": ("lon", g["src_lon"]), "lat": ("lat", g["src_lat"])})
        out2 = xrs.reproject_dataset(ds2, tgm)
    assert isinstance(out["v"].data, np.ndarray)
    assert_bitwise_equal(out["v"].values, g["out_bilinear"])
    assert out2["v"].dims == ("y", "x")
    assert_bitwise_equal(out2["v"].values, g["out_bilinear"][1])


def test_streamed_errors():
    from xcube_resampling_amd import streaming

    g = load_golden("reproject_f32.npz")
    plan = _plan(g)
    with pytest.raises(NotImplementedError, match="interp_methods must be one of"):
        streaming.reproject_host(g["data"], plan, "cubic", np.nan)
    with pytest.raises(ValueError, match="does not match the plan"):
        streaming.reproject_host(g["data"][:, :-1], plan, "nearest", np.nan)


def test_pinned_transfers_in_affine_and_rectify_paths():
    """The dataset APIs move numpy arrays of at least host_streaming_min_bytes
    through the page-locked staging buffers (streaming.host_to_device /
    device_to_host, several staging chunks at the sizes below): same bits as
    the small-array path."""
    import xcube_resampling_amd as xrs

    rng = np.random.default_rng(5)
    # affine (coarsen 4x4 mean, 3-D) on a regular EPSG:4326 grid
    n = 256
    res = 2.0 ** -8
    lon = (np.arange(n) + 0.5) * res
    lat = n * res - (np.arange(n) + 0.5) * res
    data = rng.random((2, n, n), dtype=np.float32)
    data.ravel()[rng.choice(data.size, 100, replace=False)] = np.nan
    ds = xrs.Dataset(data_vars={"v": (("t", "lat", "lon"), data)},
                     coords={"lon": ("lon", lon), "lat": ("lat", lat)})
    tgm = xrs.GridMapping.regular((n // 4, n // 4), (0, 0), res * 4, "EPSG:4326")
    # irregular swath for rectify
    h, w = 120, 100
    ii, jj = np.meshgrid(np.arange(w), np.arange(h))
    slat = 60 - 0.0027 * jj - 0.0004 * ii
    slon = 5 + 0.0045 * ii + 0.0009 * jj
    sds = xrs.Dataset(data_vars={"v": (("y", "x"), rng.random((h, w), dtype=np.float32))},
                      coords={"lon": (("y", "x"), slon), "lat": (("y", "x"), slat)})
    results = []
    for min_bytes in (1 << 40, 0):
        with xrs.set_options(host_streaming_min_bytes=min_bytes):
            a = xrs.affine_transform_dataset(ds, tgm, agg_methods="mean")["v"].values
            r = xrs.rectify_dataset(sds, interp_methods="bilinear")["v"].values
        assert isinstance(a, np.ndarray) and isinstance(r, np.ndarray)
        results.append((a, r))
    assert_bitwise_equal(results[1][0], results[0][0], "affine")
    assert_bitwise_equal(results[1][1], results[0][1], "rectify")
    assert np.isfinite(results[0][1]).sum() > h * w // 2


def test_streamed_from_read_only_memmap(tmp_path):
    """A file-backed, read-only source (np.load(mmap_mode='r')) streams
    through the staging buffers like any array — same bits."""
    from xcube_resampling_amd import streaming

    g = load_golden("reproject_f32.npz")
    np.save(tmp_path / "src.npy", g["data"])
    src = np.load(tmp_path / "src.npy", mmap_mode="r")
    out = streaming.reproject_host(src, _plan(g), "bilinear", g["fill"].item(), band_rows=7)
    assert_bitwise_equal(out, g["out_bilinear"], "memmap source")


# ---- affine / rectify band pipelines (streaming.affine_host / rectify_host) ------
AFFINE_CASES = [
    # (matrix, out (h, w), out chunks (h, w), order, agg)
    (((0.9216, 0.0, 102.4), (0.0, 0.9216, 51.2)), (700, 650), (128, 160), 0, "first"),
    (((0.5, 0.0, 3.25), (0.0, 0.5, 7.5)), (900, 800), (256, 200), 1, "first"),
    (((4.0, 0.0, 0.0), (0.0, 4.0, 0.0)), (200, 220), (64, 100), 1, "mean"),
    (((3.0, 0.0, 1.0), (0.0, 3.0, 2.0)), (180, 200), (60, 75), 1, "max"),
]


@pytest.mark.parametrize("band_chunks", [1, 2, None])
@pytest.mark.parametrize("case", range(len(AFFINE_CASES)))
def test_affine_streamed_matches_resident(case, band_chunks):
    """Bands of whole output chunk rows, each reading only its chunks' input
    slices (the device source is poisoned with NaN bytes beforehand, so a read
    outside a band's rows would show) == the resident launch, bit for bit."""
    import torch

    import xcube_resampling_amd.affine as A
    from xcube_resampling_amd import kernels, streaming

    m, out_shape, chunks, order, agg = AFFINE_CASES[case]
    rng = np.random.default_rng(case)
    src = rng.random((2, 800, 900), dtype=np.float32)
    src.ravel()[rng.choice(src.size, 300, replace=False)] = np.nan
    plan = A.plan_affine(src.shape, src.dtype, m, (2,) + out_shape, (1,) + chunks, order, agg,
                         False, np.nan)
    ref = kernels.affine(torch.from_numpy(src).cuda(), plan).cpu().numpy()
    out = streaming.affine_host(src, plan, band_chunks=band_chunks, poison=True)
    assert out is not None
    assert_bitwise_equal(out, ref, f"affine case {case} band_chunks={band_chunks}")


def _swath_ij(h, w, reverse):
    import torch

    import xcube_resampling_amd as xrs
    from xcube_resampling_amd import rectify as R

    ii, jj = np.meshgrid(np.arange(w), np.arange(h))
    rng = np.random.default_rng(11)
    sign = 1 if reverse else -1
    lat = 60 + sign * 0.0027 * jj - 0.0004 * ii + rng.normal(0, 1e-4, (h, w))
    lon = 5 + 0.0045 * ii + 0.0009 * jj + rng.normal(0, 1e-4, (h, w))
    sgm = xrs.GridMapping.from_coords(xrs.DataArray(lon, ("y", "x"), name="lon"),
                                      xrs.DataArray(lat, ("y", "x"), name="lat"), "EPSG:4326")
    tgm = sgm.to_regular(tile_size=128)
    return R._compute_target_source_ij(sgm, tgm, 1e-3)


@pytest.mark.parametrize("reverse", [False, True])
@pytest.mark.parametrize("band_rows", [1, 37, None])
def test_rectify_streamed_matches_resident(band_rows, reverse):
    """K6 in target row bands, each reading only the source rows its
    positions reach (bounded per row from ij; a swath whose rows run against
    the target's exercises out-of-order row needs) == the resident K6."""
    import torch

    from xcube_resampling_amd import kernels, streaming

    h, w = 600, 500
    ij = _swath_ij(h, w, reverse)
    rng = np.random.default_rng(3)
    src = rng.random((2, h, w), dtype=np.float32)
    for interp in ("nearest", "bilinear", "triangular"):
        ref = kernels.rectify_var(ij, torch.from_numpy(src).cuda(), interp, np.nan).cpu().numpy()
        out = streaming.rectify_host(src, ij, interp, np.nan, band_rows=band_rows, poison=True)
        assert_bitwise_equal(out, ref, f"rectify {interp} band_rows={band_rows}")
    assert np.isfinite(ref).mean() > 0.4


def test_staging_round_trip_multi_chunk():
    """host_to_device / device_to_host through the staging buffers: arrays of
    several 16 MiB chunks plus a ragged tail, odd dtypes and a read-only view,
    land bit for bit; the pinned buffers are reused across calls."""
    from xcube_resampling_amd import streaming
    from xcube_resampling_amd.options import set_options

    rng = np.random.default_rng(9)
    n = 3 * (streaming._STAGE_BYTES // 4) + 12345
    cases = [rng.random(n, dtype=np.float32).reshape(-1, 5) if n % 5 == 0 else
             rng.random(n, dtype=np.float32),
             rng.integers(-2**15, 2**15, 2 * streaming._STAGE_BYTES // 2 + 7, dtype=np.int16),
             rng.random((1000, 2049))]
    ro = rng.random((3000, 3001))
    ro.flags.writeable = False
    cases.append(ro)
    with set_options(host_streaming_min_bytes=0):
        for a in cases:
            d = streaming.host_to_device(a, "cuda:0")
            assert tuple(d.shape) == a.shape
            back = streaming.device_to_host(d)
            assert back.dtype == a.dtype
            assert np.array_equal(back.view(np.uint8), np.ascontiguousarray(a).view(np.uint8))
    with streaming._staging() as a:
        assert len(a.bufs) == 2
    with streaming._staging() as b:      # a drained pair is handed out again
        assert b is a


def test_staging_concurrent_threads():
    """Streamed copies from several host threads at once (a threaded chunk
    scheduler calling the dataset APIs): a thread borrows a page-locked pair
    from the pool for each transfer, so no thread's bytes land in another's
    array, and the pool never holds more than _POOL_MAX pairs (ADVICE r04:
    no pinned pair per thread for the life of the thread)."""
    from concurrent.futures import ThreadPoolExecutor

    import torch

    from xcube_resampling_amd import streaming
    from xcube_resampling_amd.options import set_options

    import threading

    n = 2 * (streaming._STAGE_BYTES // 4) + 999
    start = threading.Barrier(4, timeout=60)   # four distinct threads, copying together

    def work(k):
        torch.cuda.set_device(0)
        start.wait()
        a = np.random.default_rng(100 + k).random(n, dtype=np.float32)
        ok = True
        for _ in range(3):
            d = streaming.host_to_device(a, "cuda:0")
            ok &= np.array_equal(streaming.device_to_host(d), a)
        return ok

    with set_options(host_streaming_min_bytes=0), ThreadPoolExecutor(4) as ex:
        res = list(ex.map(work, range(4)))
    assert all(res)
    assert 1 <= streaming._POOL_MADE <= streaming._POOL_MAX
    assert len(streaming._POOL_FREE) == streaming._POOL_MADE   # every pair returned


def test_host_register_copy_unregister_then_fresh_pageable_copy():
    """The sequence behind round 3's illegal-address faults:
    register a page-aligned host buffer -> async copy to the device ->
    unregister -> free the pages -> a fresh allocation of the same size (the
    kernel usually hands back the same addresses) -> a pageable copy from it.
    Every copy lands the bytes it was given; a malloc'd numpy array is
    refused."""
    import ctypes
    import mmap

    import torch

    from xcube_resampling_amd import _native

    lib = _native.lib()
    page = mmap.PAGESIZE
    nbytes = 64 * (1 << 20)
    assert nbytes % page == 0
    dev = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream()
    rng = np.random.default_rng(4)
    addrs = []
    for k in range(3):
        buf = mmap.mmap(-1, nbytes)
        host = np.frombuffer(buf, dtype=np.float32)
        host[:] = rng.random(host.size, dtype=np.float32)
        ptr = host.ctypes.data
        addrs.append(ptr)
        assert ptr % page == 0
        assert lib.xrs_host_register(ctypes.c_void_p(ptr), nbytes) == _native.XRS_OK
        _native.check(lib.xrs_copy_async(ctypes.c_void_p(dev.data_ptr()), ctypes.c_void_p(ptr),
                                         nbytes, ctypes.c_void_p(stream.cuda_stream)),
                      "xrs_copy_async")
        streams = (ctypes.c_void_p * 1)(stream.cuda_stream)   # the stream that copied
        _native.check(lib.xrs_host_unregister(ctypes.c_void_p(ptr), streams, 1),
                      "xrs_host_unregister")
        expect = host.copy()
        assert_bitwise_equal(dev.cpu().numpy(), expect, f"registered copy {k}")
        del host
        buf.close()                                  # the pages go back to the kernel
        fresh = np.frombuffer(mmap.mmap(-1, nbytes), dtype=np.float32)
        fresh[:] = rng.random(fresh.size, dtype=np.float32)
        got = torch.from_numpy(fresh).cuda()         # pageable copy from the fresh range
        assert_bitwise_equal(got.cpu().numpy(), fresh, f"pageable copy after unregister {k}")
        del got, fresh
    heap = np.empty(nbytes // 4 + 3, np.float32)     # malloc'd: starts inside a page
    if heap.ctypes.data % page:
        assert lib.xrs_host_register(ctypes.c_void_p(heap.ctypes.data),
                                     heap.nbytes) == _native.XRS_ERR_ARG

"""Multi-GPU behind the dataset API (xcube_resampling_amd.multidevice), on the
one-GPU test box: ``devices=[0, 0]`` (and three parts) runs each variable's
partitions from several host threads on their own HIP streams of the same
GPU — the code an 8-GPU node runs with ``devices=list(range(8))``.  Every
result is bit-identical to the single-device call and to the oracle or the
reference's goldens (reproject.py:230-252, rectify.py:347-370,
affine.py:336-362: partitions are independent)."""

from __future__ import annotations

import numpy as np
import pytest

import configs
from fixtures import dataset_2x2_irregular, reference_goldens
from helpers import assert_bitwise_equal, load_golden, reproject_golden_inputs

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
@pytest.mark.parametrize("case", ["f32", "i16", "u8", "pad"])
def test_reproject_dataset_devices_match_goldens(case, devices):
    """Host (numpy) dataset in, numpy out; the golden fixtures were made by
    the reference's own _reproject_block.  "pad" (y scale < 0.95) is
    downscaled through the affine path first by the dataset API, so it is
    compared with the single-device call (both partitioned paths in one
    call); the others with the goldens."""
    import xcube_resampling_amd as xrs

    g = load_golden(f"reproject_{case}.npz")
    ds, tgm = reproject_golden_inputs(g)
    for interp in ("nearest", "bilinear", "triangular"):
        out = xrs.reproject_dataset(ds, tgm, interp_methods=interp,
                                    fill_values=g["fill"].item(), devices=devices)
        assert isinstance(out["v"].values, np.ndarray)
        if case == "pad":
            exp = xrs.reproject_dataset(ds, tgm, interp_methods=interp,
                                        fill_values=g["fill"].item())["v"].values
        else:
            exp = g[f"out_{interp}"]
        assert_bitwise_equal(out["v"].values, exp, f"{case}/{interp}")


def test_config2_devices_match_single_device_and_oracle():
    """Config 2 (8192^2 f32 -> EPSG:3857, bilinear f64, device-resident):
    two parts on the GPU == the single-device call (oracle-pinned on all 16
    tiles in test_configs_gpu) == the oracle on a tile of each part."""
    import torch

    import xcube_resampling_amd as xrs

    size = 8192
    o = configs.reproject_oracle(size)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(2)
    src = torch.rand((1, size, size), generator=gen, device="cuda", dtype=torch.float32)
    ds = xrs.Dataset(data_vars={"v": (("time", "lat", "lon"), src)},
                     coords={"lon": ("lon", o["lon"]), "lat": ("lat", o["lat"])})
    tgm = xrs.GridMapping.regular((size, size), configs.REPROJECT_TGT_MIN, (830, 950),
                                  "EPSG:3857", tile_size=2048)
    one = xrs.reproject_dataset(ds, tgm, interp_methods="bilinear")["v"].data
    with xrs.set_options(devices=[0, 0]):    # the option form
        two = xrs.reproject_dataset(ds, tgm, interp_methods="bilinear")["v"].data
    assert two.device == src.device and two.dtype == torch.float64
    assert torch.equal(one.view(torch.int64), two.view(torch.int64))
    host = lambda j0, j1, i0, i1: src[:, j0:j1, i0:i1].cpu().numpy()  # noqa: E731
    for j, i in ((0, 0), (o["nty"] - 1, o["ntx"] - 1)):
        ref, (r0, r1, c0, c1) = configs.oracle_tile(o, host, j, i, "bilinear")
        assert_bitwise_equal(two[:, r0:r1, c0:c1].cpu().numpy(), ref, f"tile ({j}, {i})")


def test_reproject_devices_multi_variable_and_2d():
    """Several variables (2-D and 3-D, float and int) in one call: each is
    split over the devices and equals the single-device result."""
    import xcube_resampling_amd as xrs

    g = load_golden("reproject_f32.npz")
    ds, tgm = reproject_golden_inputs(g)
    ds["w"] = xrs.DataArray((g["data"][0] * 1000).astype(np.int16), ("lat", "lon"))
    one = xrs.reproject_dataset(ds, tgm, interp_methods="nearest")
    two = xrs.reproject_dataset(ds, tgm, interp_methods="nearest", devices=["cuda:0", 0])
    for k in ("v", "w"):
        assert two[k].dims == one[k].dims
        assert_bitwise_equal(two[k].values, one[k].values, k)


@pytest.mark.parametrize("agg", ["mean", "max", "count", "first"])
@pytest.mark.parametrize("on_device", [False, True])
def test_affine_coarsen_devices_match_oracle(agg, on_device):
    """Config-3 shape in miniature (1024^2 f32 with NaN -> 256^2, scale 4):
    output chunk rows over three parts, each holding its footprints' source
    rows == the oracle."""
    import torch

    import xcube_resampling_amd.affine as A
    from oracle import affine_ref
    from xcube_resampling_amd import multidevice

    rng = np.random.default_rng(5)
    a = rng.random((1024, 1024), dtype=np.float32)
    a.ravel()[rng.choice(a.size, a.size // 1000, replace=False)] = np.nan
    m = ((4.0, 0.0, 0.0), (0.0, 4.0, 0.0))
    ref = affine_ref.resample_array(a, m, (256, 256), (64, 128), 1, agg, False, np.nan)
    src = torch.from_numpy(a).cuda() if on_device else a
    with multidevice.use_devices([0, 0, 0]):
        got = A._resample_array(src, None, None, m, (256, 256), (64, 128), 1, agg, False,
                                np.nan)
    assert isinstance(got, np.ndarray) != on_device
    got = got.cpu().numpy() if on_device else got
    assert_bitwise_equal(got, np.asarray(ref), agg)


@pytest.mark.parametrize("nan_row", [None, 300, 5, 1020])
def test_affine_recover_nans_devices(nan_row):
    """recover_nans: da.any(mask) is the whole array's (affine.py:347-349);
    with the NaN in a row only one part reads — or in rows no part's
    footprint reads (5, 1020) — the decision, and every value, equal the
    oracle's."""
    import xcube_resampling_amd.affine as A
    from oracle import affine_ref
    from xcube_resampling_amd import multidevice

    rng = np.random.default_rng(8)
    a = rng.random((2, 1024, 512)).astype(np.float32)
    if nan_row is not None:
        a[1, nan_row, 100] = np.nan
    m = ((1.5, 0.0, 3.0), (0.0, 0.75, 200.0))   # reads rows [200, ~584) only
    oshape, ochunks = (2, 512, 300), (1, 128, 128)
    ref = affine_ref.resample_array(a, m, oshape, ochunks, 1, "first", True, np.nan)
    with multidevice.use_devices([0, 0]):
        got = A._resample_array(a, None, None, m, oshape, ochunks, 1, "first", True, np.nan)
    assert_bitwise_equal(got, np.asarray(ref), f"nan_row={nan_row}")


def test_affine_transform_dataset_devices():
    import xcube_resampling_amd as xrs
    from oracle import affine_ref

    rng = np.random.default_rng(9)
    n = 512
    a = rng.random((n, n), dtype=np.float32)
    res = 2.0 ** -10
    ds = xrs.Dataset(data_vars={"v": (("lat", "lon"), a)},
                     coords={"lon": ("lon", (np.arange(n) + 0.5) * res),
                             "lat": ("lat", 0.5 - (np.arange(n) + 0.5) * res)})
    tgm = xrs.GridMapping.regular((n // 4, n // 4), (0, 0), 2.0 ** -8, "EPSG:4326", tile_size=32)
    out = xrs.affine_transform_dataset(ds, tgm, devices=[0, 0])
    m = tgm.ij_transform_to(xrs.GridMapping.from_dataset(ds))
    ref = affine_ref.resample_array(a, m, (n // 4, n // 4), (32, 32), 1, "mean", False, np.nan)
    assert_bitwise_equal(out["v"].values, ref)


def _swath(rng, h, w):
    i = np.arange(w)[None, :]
    j = np.arange(h)[:, None]
    lon = 5.0 + 0.0045 * i + 0.0009 * j + rng.normal(0, 0.0002, (h, w))
    lat = 60.0 - 0.0027 * j - 0.0004 * i + 1e-8 * (i - w / 2) ** 2 \
        + rng.normal(0, 0.0001, (h, w))
    return lon, lat


@pytest.mark.parametrize("interp", ["nearest", "bilinear", "triangular"])
@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_rectify_dataset_devices_match_oracle(interp, devices):
    """A 700x900 jittered swath rectified to 1000x760 in 128x96 tiles: the
    tile runs of 2-3 parts (K5 + K6 each) == the single-device call == the C
    oracle of the reference's numba kernels; two variables (3-D float, 2-D
    int) in one call."""
    import xcube_resampling_amd as xrs
    from oracle import gridmapping_ref as gref
    from oracle import rectify_ref

    rng = np.random.default_rng(7)
    h, w = 700, 900
    lon, lat = _swath(rng, h, w)
    var = rng.random((2, h, w)).astype(np.float32)
    ivar = rng.integers(0, 60000, (h, w)).astype(np.uint16)
    size, xy_min, res, tile = (1000, 760), (5.3, 58.3), 0.0025, (128, 96)
    ds = xrs.Dataset(data_vars={"v": (("t", "y", "x"), var), "q": (("y", "x"), ivar)},
                     coords={"lon": (("y", "x"), lon), "lat": (("y", "x"), lat)})
    tgm = xrs.GridMapping.regular(size, xy_min, res, "EPSG:4326", tile_size=tile)
    one = xrs.rectify_dataset(ds, target_gm=tgm, interp_methods=interp)
    many = xrs.rectify_dataset(ds, target_gm=tgm, interp_methods=interp, devices=devices)
    geo = gref.regular_geometry(size, xy_min, res, tile_size=tile)
    exp_ij, _ = rectify_ref.compute_target_source_ij(lon, lat, size, tile, geo["xy_bbox"],
                                                     geo["xy_res"], False, threads=8)
    for k, arr, fill in (("v", var, np.nan), ("q", ivar[None], 65535)):
        exp = rectify_ref.compute_var_image(exp_ij, arr, fill, interp, tile, threads=8)
        exp = exp if arr.shape[0] > 1 or k == "v" else exp[0]
        assert_bitwise_equal(many[k].values, one[k].values, f"{k} vs single device")
        assert_bitwise_equal(many[k].values, exp, f"{k} vs oracle")


def test_rectify_devices_reference_goldens_and_device_data():
    """The reference's 13x13 rectify golden with tiles of 5 over 2 parts,
    and a device-resident variable (the result stays on its device)."""
    import torch

    import xcube_resampling_amd as xrs

    gold = reference_goldens("tests/test_rectify.py")["__helpers__"]["expected_rad_13x13"]
    tgm = xrs.GridMapping.regular((13, 13), (-0.25, 49.75), 0.5, "EPSG:4326", tile_size=5)
    out = xrs.rectify_dataset(dataset_2x2_irregular(), target_gm=tgm, interp_methods=0,
                              devices=[0, 0])
    np.testing.assert_almost_equal(out["rad"].values, gold)
    ds = dataset_2x2_irregular()
    ds["rad"] = xrs.DataArray(torch.from_numpy(np.asarray(ds["rad"].values)).cuda(), ("y", "x"))
    out = xrs.resample_in_space(ds, target_gm=tgm, interp_methods=0, devices=[0, 0])
    assert out["rad"].data.is_cuda
    np.testing.assert_almost_equal(out["rad"].data.cpu().numpy(), gold)


def test_devices_non_separable_reprojection():
    """A non-separable pair (LAEA source -> geographic, the reference's
    test_reproject_complex_dask_array case: 2-D coordinate tables made on
    each device, row bands balanced by rows) over two and three parts ==
    the single-device call; and one variable, whose plan fuses the
    transformation into the gather."""
    import xcube_resampling_amd as xrs
    from fixtures import dataset_large_for_reproject

    tgm = xrs.GridMapping.regular((10, 10), (6.0, 48.0), 0.2, "EPSG:4326", tile_size=(5, 5))
    src = dataset_large_for_reproject()
    # two yx variables: the plan keeps 2-D coordinate tables (one per device)
    src["t2"] = xrs.DataArray(src["temperature"].values[:3] * 2.0, ("time2", "y", "x"))
    for interp in ("nearest", "triangular", "bilinear"):
        one = xrs.reproject_dataset(src, tgm, interp_methods=interp)
        for devices in ([0, 0], [0, 0, 0]):
            many = xrs.reproject_dataset(src, tgm, interp_methods=interp, devices=devices)
            for k in ("temperature", "t2"):
                assert_bitwise_equal(many[k].values, one[k].values,
                                     f"{interp}/{k}/{len(devices)}")
    # one yx variable: the transformation fused into the gather
    one = xrs.reproject_dataset(dataset_large_for_reproject(), tgm, interp_methods=1)
    two = xrs.reproject_dataset(dataset_large_for_reproject(), tgm, interp_methods=1,
                                devices=[0, 0])
    assert_bitwise_equal(two["temperature"].values, one["temperature"].values, "fused")


def test_devices_affine_order1_time_neighbours():
    """Order-1 3-D affine with dask-image's zero-weight time neighbour (the
    per-slice kernel path) split into output row bands over two parts, NaN
    in the data == the oracle."""
    import xcube_resampling_amd.affine as A
    from oracle import affine_ref
    from xcube_resampling_amd import multidevice

    rng = np.random.default_rng(12)
    a = rng.random((3, 300, 260)).astype(np.float32)
    a.ravel()[rng.random(a.size) < 0.002] = np.nan
    m = ((0.7, 0.0, 3.3), (0.0, 0.8, 1.5))
    oshape, ochunks = (3, 240, 200), (2, 64, 64)
    ref = affine_ref.resample_array(a, m, oshape, ochunks, 1, "first", False, np.nan)
    with multidevice.use_devices([0, 0]):
        got = A._resample_array(a, None, None, m, oshape, ochunks, 1, "first", False, np.nan)
    assert_bitwise_equal(got, np.asarray(ref), "order 1, time neighbours")


def test_devices_more_parts_than_rows():
    """More devices than target rows / tiles: the extra parts get empty
    shards and the result is unchanged (reproject, rectify)."""
    import xcube_resampling_amd as xrs

    g = load_golden("reproject_f32.npz")
    ds, tgm = reproject_golden_inputs(g)
    many = xrs.reproject_dataset(ds, tgm, interp_methods="nearest",
                                 devices=[0] * (tgm.height + 3))
    assert_bitwise_equal(many["v"].values, g["out_nearest"], "reproject")
    gold = reference_goldens("tests/test_rectify.py")["__helpers__"]["expected_rad_13x13"]
    rtgm = xrs.GridMapping.regular((13, 13), (-0.25, 49.75), 0.5, "EPSG:4326", tile_size=5)
    out = xrs.rectify_dataset(dataset_2x2_irregular(), target_gm=rtgm, interp_methods=0,
                              devices=[0] * 12)
    np.testing.assert_almost_equal(out["rad"].values, gold)


def test_affine_workspaces_bounded_per_stream():
    """K2/K3 workspaces are keyed by (device, stream) and the cache keeps at
    most _WORKSPACES_MAX of them (one per pool stream, forever):
    twelve streams leave eight entries, the most recent ones, and a stream's
    entry is reused while it stays cached."""
    import torch

    from xcube_resampling_amd import kernels

    dev = torch.device("cuda", 0)
    streams = [torch.cuda.Stream(device=dev) for _ in range(12)]
    for s in streams:
        kernels._workspace(dev, 1 << 16, s)
    keys = [(str(dev), int(s.cuda_stream)) for s in streams]
    assert len(kernels._WORKSPACES) <= kernels._WORKSPACES_MAX
    assert all(k in kernels._WORKSPACES for k in keys[-kernels._WORKSPACES_MAX:])
    assert not any(k in kernels._WORKSPACES for k in keys[:12 - kernels._WORKSPACES_MAX])
    ws = kernels._workspace(dev, 1 << 10, streams[-1])
    assert ws is kernels._workspace(dev, 1 << 12, streams[-1])   # cached, large enough
    torch.cuda.synchronize()

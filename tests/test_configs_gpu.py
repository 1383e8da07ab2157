"""GPU parity at the BASELINE.json config geometries.

Every expected value comes from the oracle with the ORACLE's own geometry —
its windows (_get_scr_bboxes_indices, reproject.py:385-469), its float32
window origins and its affine matrix — never from the product's plan, so the
host-side window math is checked at full size together with the kernels.
Bar: bit-exact (float64 bilinear as the reference returns it; the float32
output mode is that value rounded once)."""

from __future__ import annotations

import numpy as np
import pytest

import configs
from helpers import assert_bitwise_equal

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nan_frac", [0.0, 0.001])
def test_config1_affine_nearest_1024_full_geometry(nan_frac):
    """Config 1: affine nearest 1024^2 f32 EPSG:4326 (scale 0.9216, offset
    102.4 px; fill at the far edges) through affine_transform_dataset ==
    the oracle (dask-image chunk restatement + scipy order 0), bit for bit."""
    import xcube_resampling_amd as xrs
    from oracle import affine_ref

    lon, lat, geo, m = configs.config1_oracle()
    n = configs.C1_SIZE
    rng = np.random.default_rng(20250905)
    a = rng.random((1, n, n), dtype=np.float32)
    if nan_frac:
        a.ravel()[rng.choice(a.size, int(a.size * nan_frac), replace=False)] = np.nan
    ds = xrs.Dataset(data_vars={"v": (("time", "lat", "lon"), a)},
                     coords={"lon": ("lon", lon), "lat": ("lat", lat)})
    tgm = xrs.GridMapping.regular((n, n), configs.C1_TGT_MIN, configs.C1_TGT_RES, "EPSG:4326")
    out = xrs.affine_transform_dataset(ds, tgm, interp_methods=0)["v"].values
    tw, th = geo["tile_size"]
    ref = affine_ref.resample_array(a, m, (1, n, n), (1, th, tw), 0, "first", False, np.nan)
    assert_bitwise_equal(out, np.asarray(ref), "config 1")
    assert np.isnan(ref[0, :, -1]).all() and np.isfinite(ref[0, :, 0]).mean() > 0.99


def test_config2_reproject_bilinear_8192_f64():
    """Config 2: reproject bilinear 8192^2 f32 EPSG:4326 -> EPSG:3857 in
    2048^2 tiles, float64 output (the reference's bilinear dtype), through
    reproject_dataset on a device-resident source; ALL 16 tiles against the
    oracle's block on the oracle's window."""
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
    out = xrs.reproject_dataset(ds, tgm, interp_methods="bilinear")["v"].data
    assert out.dtype == torch.float64
    host = lambda j0, j1, i0, i1: src[:, j0:j1, i0:i1].cpu().numpy()  # noqa: E731
    tiles = [(j, i) for j in range(o["nty"]) for i in range(o["ntx"])]
    assert len(tiles) == 16
    for j, i in tiles:
        ref, (r0, r1, c0, c1) = configs.oracle_tile(o, host, j, i, "bilinear")
        assert ref.dtype == np.float64
        assert_bitwise_equal(out[:, r0:r1, c0:c1].cpu().numpy(), ref, f"tile ({j}, {i})")


@pytest.mark.parametrize("interp", ["nearest", "triangular"])
def test_config2_other_methods_all_tiles(interp):
    """Config 2 nearest / triangular through the K1 launch: ALL 16 tiles
    against the oracle's block on the oracle's window."""
    import torch

    from xcube_resampling_amd import kernels
    import bench

    size = 8192
    o = configs.reproject_oracle(size)
    _, _, plan, _, _ = bench.workload(size, 2048)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(3)
    src = torch.rand((1, size, size), generator=gen, device="cuda", dtype=torch.float32)
    out = kernels.reproject(src, plan, interp, float("nan"))
    host = lambda j0, j1, i0, i1: src[:, j0:j1, i0:i1].cpu().numpy()  # noqa: E731
    tiles = [(j, i) for j in range(o["nty"]) for i in range(o["ntx"])]
    assert len(tiles) == 16
    for j, i in tiles:
        ref, (r0, r1, c0, c1) = configs.oracle_tile(o, host, j, i, interp)
        assert_bitwise_equal(out[:, r0:r1, c0:c1].cpu().numpy(), ref, f"{interp} ({j}, {i})")


def _same_bits(actual, expected) -> bool:
    """Bit-equal (NaN == NaN) without assert_bitwise_equal's per-byte view:
    equal words, or every differing word a NaN on both sides."""
    u = {8: np.uint64, 4: np.uint32}[actual.dtype.itemsize]
    a, e = actual.view(u), expected.view(u)
    ne = a != e
    if not ne.any():
        return True
    return bool((np.isnan(actual[ne]) & np.isnan(expected[ne])).all())


def test_config5_full_size_all_tiles():
    """Config 5 at full size — 40960^2 f32 bilinear EPSG:4326 -> EPSG:3857,
    400 tiles of 2048^2 in ONE launch, float64 output (the reference's dtype)
    and the float32 output mode of the bench: EVERY tile == the oracle's
    _reproject_block (reproject.py:268-335) on the oracle's window
    (reproject.py:385-469), bit for bit.  The source goes to the host once;
    the results come back one tile row at a time and the oracle runs the
    row's tiles on a thread pool sized to the box's CPU share, so host memory
    stays bounded (~7 GB source + one tile row of results)."""
    import os
    from concurrent.futures import ThreadPoolExecutor

    import torch

    import bench
    from xcube_resampling_amd import kernels

    size = 40960
    o = configs.reproject_oracle(size)
    _, _, plan, _, _ = bench.workload(size, 2048)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(5)
    src = torch.rand((1, size, size), generator=gen, device="cuda", dtype=torch.float32)
    out64 = kernels.reproject(src, plan, "bilinear", float("nan"))
    out32 = kernels.reproject(src, plan, "bilinear", float("nan"), out_dtype=np.float32)
    src_host = src.cpu().numpy()
    del src
    host = lambda j0, j1, i0, i1: src_host[:, j0:j1, i0:i1]  # noqa: E731
    workers = max(1, min(16, len(os.sched_getaffinity(0))))
    tile = o["tile"]
    checked = 0
    with ThreadPoolExecutor(max_workers=workers) as pool:
        for j in range(o["nty"]):
            r0, r1 = j * tile, min(size, (j + 1) * tile)
            row64 = out64[:, r0:r1].cpu().numpy()
            row32 = out32[:, r0:r1].cpu().numpy()

            def check(i, j=j, row64=row64, row32=row32):
                ref, (t0, t1, c0, c1) = configs.oracle_tile(o, host, j, i, "bilinear")
                assert ref.dtype == np.float64 and (t0, t1) == (r0, r1)
                a64 = np.ascontiguousarray(row64[:, :, c0:c1])
                a32 = np.ascontiguousarray(row32[:, :, c0:c1])
                if not _same_bits(a64, ref):
                    assert_bitwise_equal(a64, ref, f"f64 tile ({j}, {i})")
                r32 = ref.astype(np.float32)
                if not _same_bits(a32, r32):
                    assert_bitwise_equal(a32, r32, f"f32 tile ({j}, {i})")
                return 1

            checked += sum(pool.map(check, range(o["ntx"])))
    assert checked == o["ntx"] * o["nty"] == 400

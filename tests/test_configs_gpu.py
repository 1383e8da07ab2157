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


def test_config5_full_size_sampled_tiles():
    """Config 5 at full size — 40960^2 f32 bilinear EPSG:4326 -> EPSG:3857,
    400 tiles of 2048^2 in ONE launch, float64 output (the reference's dtype)
    and the float32 output mode of the bench: one tile in every tile row plus
    the corners (24 tiles) == the oracle's _reproject_block on the oracle's
    windows, bit for bit."""
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
    host = lambda j0, j1, i0, i1: src[:, j0:j1, i0:i1].cpu().numpy()  # noqa: E731
    tiles = configs.sample_tiles(o["ntx"], o["nty"])
    assert len({j for j, _ in tiles}) == o["nty"]
    for j, i in tiles:
        ref, (r0, r1, c0, c1) = configs.oracle_tile(o, host, j, i, "bilinear")
        assert ref.dtype == np.float64
        assert_bitwise_equal(out64[:, r0:r1, c0:c1].cpu().numpy(), ref, f"f64 tile ({j}, {i})")
        assert_bitwise_equal(out32[:, r0:r1, c0:c1].cpu().numpy(), ref.astype(np.float32),
                             f"f32 tile ({j}, {i})")

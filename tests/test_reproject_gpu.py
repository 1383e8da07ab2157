"""GPU parity tests of K1 (xrs_reproject) — the reference's reproject path.

Bar: bit-exact against the reference's own outputs (golden fixtures produced
by executing reproject.py:268-335/385-469/499-530) for nearest, bilinear
(float64, as the reference returns) and triangular, float and integer
dtypes; bit-exact against the oracle on larger seeded inputs; float32 output
mode within 1e-6 relative of the float64 reference (it is the same float64
value rounded once)."""

from __future__ import annotations

import numpy as np
import pytest

from helpers import assert_bitwise_equal, load_golden, reproject_golden_inputs

pytestmark = pytest.mark.gpu

CASES = ["f32", "u8", "i16", "pad"]
NO_DOWNSCALE = ["f32", "u8", "i16"]  # "pad" has y_scale < 0.95: the dataset API downscales first


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("interp", ["nearest", "bilinear", "triangular"])
def test_kernel_matches_reference_bitwise(case, interp):
    """K1 on the product's plan == the reference's per-tile blocks."""
    import torch

    import xcube_resampling_amd as xrs
    from xcube_resampling_amd import kernels

    g = load_golden(f"reproject_{case}.npz")
    ds, tgm = reproject_golden_inputs(g)
    sgm = xrs.GridMapping.from_dataset(ds)
    plan = xrs.plan_reproject(sgm, tgm, xrs.Transformer.from_crs(tgm.crs, sgm.crs, always_xy=True))
    src = torch.from_numpy(g["data"]).cuda()
    out = kernels.reproject(src, plan, interp, g["fill"].item())
    assert_bitwise_equal(out.cpu().numpy(), g[f"out_{interp}"], f"{case}/{interp}")


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 20, 23, 24, 25, 28])
def test_every_gather_variant_is_bit_identical(variant, monkeypatch):
    """The A/B schedules of K1 (XRS_REPROJECT_VARIANT) differ only in load
    order / work shape: all reproduce the reference bit for bit, incl. a small
    band height (items that split tiles) and a single block per CU (grid loop)."""
    import torch

    import xcube_resampling_amd as xrs
    from xcube_resampling_amd import kernels

    monkeypatch.setenv("XRS_REPROJECT_VARIANT", str(variant))
    for case in ("f32", "i16"):
        g = load_golden(f"reproject_{case}.npz")
        ds, tgm = reproject_golden_inputs(g)
        sgm = xrs.GridMapping.from_dataset(ds)
        plan = xrs.plan_reproject(sgm, tgm, xrs.Transformer.from_crs(tgm.crs, sgm.crs,
                                                                      always_xy=True))
        src = torch.from_numpy(g["data"]).cuda()
        for interp in ("nearest", "bilinear", "triangular"):
            for band, bpc in (("", ""), ("5", "1")):
                monkeypatch.setenv("XRS_REPROJECT_BAND", band or "0")
                monkeypatch.setenv("XRS_REPROJECT_BLOCKS_PER_CU", bpc or "0")
                out = kernels.reproject(src, plan, interp, g["fill"].item())
                assert_bitwise_equal(out.cpu().numpy(), g[f"out_{interp}"],
                                     f"v{variant} {case}/{interp} band={band} bpc={bpc}")


@pytest.mark.parametrize("case", NO_DOWNSCALE)
@pytest.mark.parametrize("interp", ["nearest", "bilinear", "triangular"])
def test_reproject_dataset_matches_reference_bitwise(case, interp):
    import xcube_resampling_amd as xrs

    g = load_golden(f"reproject_{case}.npz")
    ds, tgm = reproject_golden_inputs(g)
    out = xrs.reproject_dataset(ds, tgm, interp_methods=interp, fill_values=g["fill"].item())
    assert_bitwise_equal(out["v"].values, g[f"out_{interp}"], f"{case}/{interp}")
    assert out["v"].dims == ("time", "y", "x")


def test_reproject_2d_variable_and_coords():
    import xcube_resampling_amd as xrs

    g = load_golden("reproject_f32.npz")
    ds = xrs.Dataset(data_vars={"v": (("lat", "lon"), g["data"][1])},
                     coords={"lon": ("lon", g["src_lon"]), "lat": ("lat", g["src_lat"])})
    _, tgm = reproject_golden_inputs(g)
    out = xrs.reproject_dataset(ds, tgm)  # default interp for floats: bilinear
    assert_bitwise_equal(out["v"].values, g["out_bilinear"][1])
    assert out["v"].dims == ("y", "x")
    assert_bitwise_equal(out["x"].values, tgm.x_coords.values)
    assert_bitwise_equal(out["y"].values, tgm.y_coords.values)
    assert "spatial_ref" in out.coords


def test_float32_output_mode_within_tolerance():
    import xcube_resampling_amd as xrs

    g = load_golden("reproject_f32.npz")
    ds, tgm = reproject_golden_inputs(g)
    with xrs.set_options(reproject_bilinear_dtype="source"):
        out = xrs.reproject_dataset(ds, tgm, interp_methods="bilinear")
    v = out["v"].values
    assert v.dtype == np.float32
    ref = g["out_bilinear"]
    assert_bitwise_equal(v, ref.astype(np.float32))  # single rounding of the f64 value
    np.testing.assert_allclose(v, ref, rtol=1e-6, equal_nan=True)


@pytest.mark.parametrize("interp", ["nearest", "bilinear", "triangular"])
def test_kernel_matches_oracle_on_larger_tiled_raster(interp):
    """1024x768 source, 900x700 target in 128x96 tiles (partial edge tiles),
    0.1 % NaN: kernel == oracle bit for bit."""
    import xcube_resampling_amd as xrs
    from oracle import gridmapping_ref as gref
    from oracle import reproject_ref

    rng = np.random.default_rng(20250905)
    h, w = 768, 1024
    xr, yr = 0.0075, 0.005
    lon = -5.0 + (np.arange(w) + 0.5) * xr
    lat = 55.0 - (np.arange(h) + 0.5) * yr
    data = rng.random((1, h, w), dtype=np.float32)
    data.ravel()[rng.choice(data.size, data.size // 1000, replace=False)] = np.nan
    ds = xrs.Dataset(data_vars={"v": (("t", "lat", "lon"), data)},
                     coords={"lon": ("lon", lon), "lat": ("lat", lat)})
    tsize, tmin, tres, ttile = (900, 700), (-540000.0, 6500000.0), (800.0, 840.0), (128, 96)
    tgm = xrs.GridMapping.regular(tsize, tmin, tres, "EPSG:3857", tile_size=ttile)
    out = xrs.reproject_dataset(ds, tgm, interp_methods=interp)
    geo = gref.regular_geometry(tsize, tmin, tres, tile_size=ttile)
    ref = reproject_ref.reproject_array(
        data, gref.webmerc_inverse, lambda *b: gref.transform_bounds(gref.webmerc_inverse, *b),
        lon, lat, xr, yr, geo["x_coords"], geo["y_coords"], geo["xy_bboxes"], ttile[0], ttile[1],
        interp, np.nan)
    assert_bitwise_equal(out["v"].values, ref, interp)


def test_device_resident_input_stays_on_device():
    import torch

    import xcube_resampling_amd as xrs

    g = load_golden("reproject_f32.npz")
    ds, tgm = reproject_golden_inputs(g)
    dev = torch.from_numpy(g["data"]).cuda()
    ds_dev = xrs.Dataset(data_vars={"v": (("time", "lat", "lon"), dev)}, coords=ds.coords)
    out = xrs.reproject_dataset(ds_dev, tgm, interp_methods="nearest")
    assert out["v"].data.is_cuda
    assert_bitwise_equal(out["v"].values, g["out_nearest"])


@pytest.mark.parametrize("interp", ["nearest", "bilinear", "triangular"])
def test_2d_coordinate_mode_matches_reference(interp):
    """K1c (per-pixel index math from 2-D coordinate tables, the path for
    non-separable CRS pairs) == the reference outputs."""
    import dataclasses

    import torch

    import xcube_resampling_amd as xrs
    from xcube_resampling_amd import kernels

    g = load_golden("reproject_f32.npz")
    ds, tgm = reproject_golden_inputs(g)
    sgm = xrs.GridMapping.from_dataset(ds)
    tr = xrs.Transformer.from_crs(tgm.crs, sgm.crs, always_xy=True)
    plan = xrs.plan_reproject(sgm, tgm, tr)
    xx, yy = np.meshgrid(tgm.x_coords.values, tgm.y_coords.values)
    sx, sy = tr.transform(xx, yy)
    plan2 = dataclasses.replace(plan, coord_mode=1, src_x=sx, src_y=sy, _device_cache={})
    out = kernels.reproject(torch.from_numpy(g["data"]).cuda(), plan2, interp, np.nan)
    assert_bitwise_equal(out.cpu().numpy(), g[f"out_{interp}"], interp)


def test_row_band_sharding_matches_whole_raster():
    """Target row bands computed separately from per-band source bands (the
    multi-GPU partition) == the whole raster."""
    import torch

    import xcube_resampling_amd as xrs
    from xcube_resampling_amd import kernels

    g = load_golden("reproject_f32.npz")
    ds, tgm = reproject_golden_inputs(g)
    sgm = xrs.GridMapping.from_dataset(ds)
    plan = xrs.plan_reproject(sgm, tgm, xrs.Transformer.from_crs(tgm.crs, sgm.crs,
                                                                  always_xy=True))
    src = torch.from_numpy(g["data"]).cuda()
    parts = []
    for r0, r1 in [(0, 7), (7, 20), (20, 36)]:
        j0, j1 = plan.source_rows_for(r0, r1)
        band = src[:, j0:j1].contiguous()
        parts.append(kernels.reproject(band, plan, "bilinear", np.nan, rows=(r0, r1),
                                       src_row0=j0).cpu().numpy())
    assert_bitwise_equal(np.concatenate(parts, axis=1), g["out_bilinear"])


def test_config5_full_size_sampled_tiles():
    """BASELINE config 5 at full size — 40960^2 f32 bilinear EPSG:4326 ->
    EPSG:3857, 400 tiles of 2048^2 in one launch: corner, centre and edge tiles
    of the device result == the oracle's _reproject_block (reproject.py:268-335)
    on each tile's window, bit for bit (the float32 output is the reference's
    float64 value rounded once)."""
    import torch

    import bench
    from oracle import gridmapping_ref as gref
    from oracle import reproject_ref
    from xcube_resampling_amd import kernels

    size = 40960
    _, tgm, plan, _, _ = bench.workload(size, 2048)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(5)
    src = torch.rand((1, size, size), generator=gen, device="cuda", dtype=torch.float32)
    out = kernels.reproject(src, plan, "bilinear", float("nan"), out_dtype=np.float32)
    ntx, nty = plan.num_tiles
    th, tw = plan.tile_height, plan.tile_width
    xc, yc = tgm.x_coords.values, tgm.y_coords.values
    wy, wx = plan.win_height, plan.win_width
    for j, i in [(0, 0), (0, ntx - 1), (nty // 2, ntx // 2), (nty - 1, 0), (nty - 1, ntx - 1)]:
        t = j * ntx + i
        r0, r1 = j * th, min(plan.dst_height, (j + 1) * th)
        c0, c1 = i * tw, min(plan.dst_width, (i + 1) * tw)
        sxx, syy = gref.webmerc_inverse(*np.meshgrid(xc[c0:c1], yc[r0:r1]))
        wi0, wj0 = (int(v) for v in plan.tile_win[t])
        win = np.full((1, wy, wx), np.nan, np.float32)
        sj0, sj1 = max(wj0, 0), min(wj0 + wy, size)
        si0, si1 = max(wi0, 0), min(wi0 + wx, size)
        win[:, sj0 - wj0:sj1 - wj0, si0 - wi0:si1 - wi0] = src[:, sj0:sj1, si0:si1].cpu().numpy()
        x_coord = np.full((wx, 1, 1), plan.tile_x0[t], np.float32)
        y_coord = np.full((wy, 1, 1), plan.tile_y0[t], np.float32)
        ref = reproject_ref.reproject_block(sxx, syy, win, x_coord, y_coord, plan.x_res,
                                            plan.y_res, "bilinear")
        assert ref.dtype == np.float64
        assert_bitwise_equal(out[:, r0:r1, c0:c1].cpu().numpy(), ref.astype(np.float32),
                             f"tile ({j}, {i})")

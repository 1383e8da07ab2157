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


@pytest.mark.parametrize("band,bpc", [(5, 0), (1, 0), (32, 1), (7, 1), (8, 0), (3, 1), (4, 0),
                                      (2, 0), (1, 1), (64, 0), (65, 0), (100, 1), (200, 0)])
def test_work_shapes_are_bit_identical(band, bpc):
    """K1's work decomposition (target rows per work item, grid cap) changes
    only which block computes a pixel: items that split tiles (5 / 1 rows), a
    single block per CU (grid-stride loop), items taller than the 64 rows one
    resolve of the row entries covers (65-200 rows: the entries are resolved
    again every 64 rows) — all reproduce the reference bit for bit.  The
    shapes are forced through the test-only knobs (xrs_testing_set); the
    product never reads them from the environment.  Each shape runs with the
    column coordinates generated in the kernel (coord_mode 2) and read from
    the src_x table (coord_mode 0)."""
    import dataclasses

    import torch

    import xcube_resampling_amd as xrs
    from xcube_resampling_amd import kernels
    from xcube_resampling_amd._native import testing_knob

    for case in ("f32", "i16"):
        g = load_golden(f"reproject_{case}.npz")
        ds, tgm = reproject_golden_inputs(g)
        sgm = xrs.GridMapping.from_dataset(ds)
        plan = xrs.plan_reproject(sgm, tgm, xrs.Transformer.from_crs(tgm.crs, sgm.crs,
                                                                      always_xy=True))
        assert plan.x_gen is not None
        # coord_mode 2 (column generators) and 0 (the src_x table)
        table = dataclasses.replace(plan, x_gen=None, _device_cache={})
        src = torch.from_numpy(g["data"]).cuda()
        for interp in ("nearest", "bilinear", "triangular"):
            for p, mode in ((plan, "gen"), (table, "table")):
                with testing_knob("reproject_band", band), \
                        testing_knob("reproject_blocks_per_cu", bpc):
                    out = kernels.reproject(src, p, interp, g["fill"].item())
                assert_bitwise_equal(out.cpu().numpy(), g[f"out_{interp}"],
                                     f"{case}/{interp} band={band} bpc={bpc} {mode}")


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

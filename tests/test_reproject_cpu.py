"""CPU tests of the reproject path: the oracle and the product's host-side
plan against fixtures produced by the reference's own functions
(tests/golden/make_goldens.py)."""

from __future__ import annotations

import math

import numpy as np
import pytest

from helpers import assert_bitwise_equal, load_golden, reproject_golden_inputs
from oracle import gridmapping_ref as gref
from oracle import reproject_ref

CASES = ["f32", "u8", "i16", "pad"]


def _oracle_run(g, interp):
    tsize = tuple(int(v) for v in g["tsize"])
    ttile = tuple(int(v) for v in g["ttile"])
    geo = gref.regular_geometry(tsize, tuple(g["txy_min"]), tuple(g["tres"]), tile_size=ttile)
    return reproject_ref.reproject_array(
        g["data"], gref.webmerc_inverse,
        lambda *b: gref.transform_bounds(gref.webmerc_inverse, *b),
        g["src_lon"], g["src_lat"], float(g["x_res"]), float(g["y_res"]),
        geo["x_coords"], geo["y_coords"], geo["xy_bboxes"], ttile[0], ttile[1], interp,
        g["fill"].item())


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("interp", ["nearest", "bilinear", "triangular"])
def test_oracle_matches_reference_outputs(case, interp):
    g = load_golden(f"reproject_{case}.npz")
    assert_bitwise_equal(_oracle_run(g, interp), g[f"out_{interp}"], f"{case}/{interp}")


def test_reference_bilinear_returns_float64():
    # hard part 1: float32 values x float64 weights -> float64
    g = load_golden("reproject_f32.npz")
    assert g["out_bilinear"].dtype == np.float64
    assert g["out_nearest"].dtype == np.float32
    assert g["out_triangular"].dtype == np.float32


@pytest.mark.parametrize("case", CASES)
def test_product_plan_matches_reference_windows(case):
    """plan_reproject (host side of the product) == _get_scr_bboxes_indices."""
    import xcube_resampling_amd as xrs

    g = load_golden(f"reproject_{case}.npz")
    ds, tgm = reproject_golden_inputs(g)
    sgm = xrs.GridMapping.from_dataset(ds)
    assert sgm.x_res == float(g["x_res"]) and sgm.y_res == float(g["y_res"])
    tr = xrs.Transformer.from_crs(tgm.crs, sgm.crs, always_xy=True)
    plan = xrs.plan_reproject(sgm, tgm, tr)
    np.testing.assert_array_equal(plan.scr_ij_bboxes, g["scr_ij_bboxes"])
    assert plan.pad_width == tuple(tuple(int(v) for v in p) for p in g["pad_width"])
    assert plan.win_width == g["x_coords"].shape[0]
    assert plan.win_height == g["y_coords"].shape[0]
    ntx, nty = plan.num_tiles
    assert_bitwise_equal(plan.tile_x0, g["x_coords"][0].reshape(-1), "tile_x0")
    assert_bitwise_equal(plan.tile_y0, g["y_coords"][0].reshape(-1), "tile_y0")
    # unpadded window origins
    pad_top, pad_left = plan.pad_width[1][0], plan.pad_width[2][0]
    np.testing.assert_array_equal(plan.tile_win[:, 0], g["scr_ij_bboxes"][0].ravel() - pad_left)
    np.testing.assert_array_equal(plan.tile_win[:, 1], g["scr_ij_bboxes"][1].ravel() - pad_top)
    # separable coordinate tables == the per-pixel transform of the meshgrid
    geo = gref.regular_geometry(tuple(int(v) for v in g["tsize"]), tuple(g["txy_min"]),
                                tuple(g["tres"]), tile_size=tuple(int(v) for v in g["ttile"]))
    xx, yy = np.meshgrid(geo["x_coords"], geo["y_coords"])
    sxx, syy = gref.webmerc_inverse(xx, yy)
    assert_bitwise_equal(np.broadcast_to(plan.src_x[None, :], sxx.shape), sxx, "src_x")
    assert_bitwise_equal(np.broadcast_to(plan.src_y[:, None], syy.shape), syy, "src_y")


def test_target_coords_are_blockwise_linspace():
    import xcube_resampling_amd as xrs

    gm = xrs.GridMapping.regular((1000, 700), (-2226000, 3504000), (830, 950), "EPSG:3857",
                                 tile_size=256)
    geo = gref.regular_geometry((1000, 700), (-2226000, 3504000), (830, 950), tile_size=(256, 256))
    assert_bitwise_equal(gm.x_coords.values, geo["x_coords"])
    assert_bitwise_equal(gm.y_coords.values, geo["y_coords"])
    np.testing.assert_array_equal(gm.xy_bboxes, geo["xy_bboxes"])


def test_webmerc_roundtrip():
    import xcube_resampling_amd as xrs

    lon = np.linspace(-179.9, 179.9, 101)
    lat = np.linspace(-85, 85, 101)
    x, y = xrs.crs.webmerc_forward(lon, lat)
    lon2, lat2 = xrs.crs.webmerc_inverse(x, y)
    np.testing.assert_allclose(lon2, lon, rtol=0, atol=1e-12)
    np.testing.assert_allclose(lat2, lat, rtol=0, atol=1e-12)
    # the oracle's independent restatement agrees bit for bit
    ox, oy = gref.webmerc_inverse(x, y)
    assert_bitwise_equal(lon2, ox)
    assert_bitwise_equal(lat2, oy)


def test_unknown_interp_method_raises():
    g = load_golden("reproject_f32.npz")
    with pytest.raises(NotImplementedError, match="interp_methods must be one of"):
        _oracle_run(g, "cubic")


def test_non_separable_plan_fuses_only_above_table_budget():
    """A 2-D (non-separable) plan keeps device coordinate tables unless they
    would exceed the reproject_table_max_bytes option (or fuse_transform is
    set); separable plans never fuse (host logic, no device needed)."""
    import dataclasses

    import xcube_resampling_amd as xrs

    sgm = xrs.GridMapping.regular((300, 200), (400000.0, 5500000.0), 100.0, "EPSG:32632",
                                  tile_size=128)
    tgm = xrs.GridMapping.regular((250, 150), (4150000.0, 2950000.0), 100.0, "EPSG:3035",
                                  tile_size=128)
    plan = xrs.plan_reproject(sgm, tgm, xrs.Transformer.from_crs(tgm.crs, sgm.crs,
                                                                 always_xy=True))
    assert plan.coord_mode == 1 and plan.src_x is None
    assert not plan.fused_transform("cuda:0")
    with xrs.set_options(reproject_table_max_bytes=16 * 250 * 150 - 1):
        assert plan.fused_transform("cuda:0")
    with xrs.set_options(reproject_table_max_bytes=16 * 250 * 150):
        assert not plan.fused_transform("cuda:0")
    assert dataclasses.replace(plan, fuse_transform=True).fused_transform("cuda:0")
    with pytest.raises(ValueError):
        with xrs.set_options(reproject_table_max_bytes=-1):
            pass
    geo = xrs.GridMapping.regular((300, 200), (10.0, 50.0), 0.001, "EPSG:4326", tile_size=128)
    merc = xrs.GridMapping.regular((250, 150), (1113195.0, 6446276.0), 100.0, "EPSG:3857",
                                   tile_size=128)
    sep = xrs.plan_reproject(geo, merc, xrs.Transformer.from_crs(merc.crs, geo.crs,
                                                                 always_xy=True))
    assert sep.coord_mode == 0
    with xrs.set_options(reproject_table_max_bytes=0):
        assert not sep.fused_transform("cuda:0")

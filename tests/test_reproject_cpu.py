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


@pytest.mark.parametrize("size,tile,crs_pair", [
    ((900, 700), (128, 96), ("EPSG:3857", "EPSG:4326")),     # partial last tile column
    ((4096, 512), (2048, 512), ("EPSG:3857", "EPSG:4326")),
    ((1000, 300), (1000, 300), ("EPSG:4326", "EPSG:3857")),  # one tile column, forward webmerc
    ((777, 65), (64, 65), ("EPSG:4326", "EPSG:4326")),        # identity
    ((513, 40), (64, 40), ("EPSG:3857", "EPSG:4326")),       # a last block of one column
])
def test_column_generators_reproduce_src_x(size, tile, crs_pair):
    """coord_mode 2 (K1 computes its column coordinates): the records
    reproduce the plan's src_x bit for bit on regular target grids — dask's
    blockwise linspace per tile column, then the separable transformation's
    scalings — and are refused (None) the moment one column differs."""
    import xcube_resampling_amd as xrs
    from xcube_resampling_amd.reproject import column_generators

    tcrs, scrs = crs_pair
    xmin = -500000.0 if tcrs == "EPSG:3857" else -4.25
    res = 800.0 if tcrs == "EPSG:3857" else 0.0071
    tgm = xrs.GridMapping.regular(size, (xmin, 6500000.0 if tcrs == "EPSG:3857" else 50.0),
                                  res, tcrs, tile_size=tile)
    tr = xrs.Transformer.from_crs(tgm.crs, scrs, always_xy=True)
    tx = tgm.x_coords.values
    src_x = tr.transform_x(tx)
    recs = column_generators(tx, tile[0], src_x, tr.separable_x_scales())
    assert recs is not None and recs.shape == (4 * -(-size[0] // tile[0]) + 2,)
    # the kernel's evaluation, restated
    m1, m2 = recs[-2:]
    got = np.empty_like(src_x)
    for c in range(size[0]):
        tx_i, k = divmod(c, tile[0])
        start, stop, step, n = recs[4 * tx_i:4 * tx_i + 4]
        v = stop if k == int(n) - 1 else k * step + start
        got[c] = (v * m1) * m2
    assert_bitwise_equal(got, src_x)
    bad = src_x.copy()
    bad[size[0] // 2] = np.nextafter(bad[size[0] // 2], np.inf)
    assert column_generators(tx, tile[0], bad, tr.separable_x_scales()) is None
    assert column_generators(tx, tile[0], src_x, None) is None


def test_reproject_plans_use_column_generators():
    """The bench workload (config 5) and the golden plans qualify for
    coord_mode 2; a non-separable plan has no generators."""
    import xcube_resampling_amd as xrs

    g = load_golden("reproject_f32.npz")
    ds, tgm = reproject_golden_inputs(g)
    sgm = xrs.GridMapping.from_dataset(ds)
    plan = xrs.plan_reproject(sgm, tgm, xrs.Transformer.from_crs(tgm.crs, sgm.crs,
                                                                  always_xy=True))
    assert plan.coord_mode == 0 and plan.x_gen is not None
    utm = xrs.GridMapping.regular((64, 48), (500000.0, 5500000.0), 100.0, "EPSG:32632",
                                  tile_size=32)
    plan2 = xrs.plan_reproject(sgm, utm, xrs.Transformer.from_crs(utm.crs, sgm.crs,
                                                                   always_xy=True))
    assert plan2.coord_mode == 1 and plan2.x_gen is None


@pytest.mark.parametrize("crs_pair", [("EPSG:3857", "EPSG:4326"), ("EPSG:4326", "EPSG:3857"),
                                      ("EPSG:3035", "EPSG:32632"), ("EPSG:32632", "EPSG:3035"),
                                      ("EPSG:4326", "EPSG:4326")])
def test_transform_bounds_many_equals_tile_by_tile(crs_pair):
    """plan_reproject's vectorised source bounds (one transform of every
    tile's densified edges) equal transform_bounds tile by tile, bit for bit,
    including tiles whose points are all outside the projection (inf)."""
    import xcube_resampling_amd as xrs

    tr = xrs.Transformer.from_crs(crs_pair[0], crs_pair[1], always_xy=True)
    rng = np.random.default_rng(7)
    if crs_pair[0] == "EPSG:3857":
        lo, hi, span = -2.0e7, 2.0e7, 4.0e5
    elif crs_pair[0] == "EPSG:4326":
        lo, hi, span = -80.0, 80.0, 3.0
    else:
        lo, hi, span = 2.0e5, 6.0e6, 2.0e5
    x0 = rng.uniform(lo, hi, 64)
    y0 = rng.uniform(lo, hi, 64) if crs_pair[0] != "EPSG:4326" else rng.uniform(-80, 80, 64)
    w = rng.uniform(0.1, 1.0, 64) * span
    bb = np.stack([x0, y0, x0 + w, y0 + w], axis=1)
    if crs_pair[0] == "EPSG:3857":
        bb[0] = [1e30, 1e30, 2e30, 2e30]   # nothing finite
    with np.errstate(over="ignore", invalid="ignore"):
        many = tr.transform_bounds_many(bb)
        one = np.array([tr.transform_bounds(*b) for b in bb])
    assert many.shape == one.shape
    np.testing.assert_array_equal(many.view(np.int64), one.view(np.int64))


def test_plan_bboxes_vectorised_equal_per_tile_loop():
    """The config-5 plan's tile windows through the vectorised bounds equal
    the per-tile computation (reproject.py:385-403)."""
    import bench

    sgm, tgm, plan, _, _ = bench.workload(8192, 2048)
    import xcube_resampling_amd as xrs

    tr = xrs.Transformer.from_crs(tgm.crs, sgm.crs, always_xy=True)
    origin = sgm.x_coords.values[0], sgm.y_coords.values[0]
    exp = []
    for xy_bbox in tgm.xy_bboxes:
        sb = tr.transform_bounds(*xy_bbox)
        exp.append([math.floor((sb[0] - origin[0]) / sgm.x_res),
                    math.floor((origin[1] - sb[3]) / sgm.y_res),
                    math.ceil((sb[2] - origin[0]) / sgm.x_res),
                    math.ceil((origin[1] - sb[1]) / sgm.y_res)])
    exp = np.array(exp)
    i_diff, j_diff = exp[:, 2] - exp[:, 0], exp[:, 3] - exp[:, 1]
    i_start = exp[:, 0] - (i_diff.max() + 1 - i_diff) // 2
    j_start = exp[:, 1] - (j_diff.max() + 1 - j_diff) // 2
    np.testing.assert_array_equal(plan.tile_win, np.stack([i_start, j_start], axis=1))
    assert plan.win_width == i_diff.max() + 1 and plan.win_height == j_diff.max() + 1

"""CPU tests of the rectify path: the C restatement of the numba kernels
(oracle/rectify_ref.c) against fixtures produced by executing the reference's
own kernels (tests/golden/make_goldens.py) and the reference's bbox test
goldens (tests/gridmapping/test_bboxes.py)."""

from __future__ import annotations

import numpy as np
import pytest

from fixtures import reference_goldens
from helpers import assert_bitwise_equal, load_golden
from oracle import rectify_ref

CASES = ["f32", "fine", "u8_jup", "nan"]
BORDER_BOX = np.array([[12.4, 51.6, 12.6, 51.7]])


def _geometry(g):
    from oracle import gridmapping_ref as gref

    size = tuple(int(v) for v in g["size"])
    tile = tuple(int(v) for v in g["tile"])
    geo = gref.regular_geometry(size, tuple(g["xy_min"]), float(g["res"]), tile_size=tile,
                                is_j_axis_up=bool(g["j_up"]))
    return size, tile, geo


@pytest.mark.parametrize("case", CASES)
def test_oracle_rectify_matches_reference_kernels(case):
    g = load_golden(f"rectify_{case}.npz")
    size, tile, geo = _geometry(g)
    ij, bb = rectify_ref.compute_target_source_ij(g["lon"], g["lat"], size, tile, geo["xy_bbox"],
                                                  geo["xy_res"], bool(g["j_up"]))
    np.testing.assert_array_equal(bb, g["ij_bboxes"])
    assert_bitwise_equal(ij, g["ij"], "ij")
    for interp in ("nearest", "bilinear", "triangular"):
        out = rectify_ref.compute_var_image(ij, g["var"], g["fill"].item(), interp, tile)
        assert_bitwise_equal(out, g[f"out_{interp}"], interp)


def test_oracle_bboxes_match_reference_test_goldens():
    gold = reference_goldens("tests/gridmapping/test_bboxes.py")
    lon, lat = np.meshgrid(np.linspace(10.0, 20.0, 11), np.linspace(50.0, 60.0, 11))
    a0, a1, a2 = 0.0, 5.0, 10.0
    tiles = np.array([[10.0 + a0, 50.0 + a0, 10.0 + a1, 50.0 + a1],
                      [10.0 + a1, 50.0 + a0, 10.0 + a2, 50.0 + a1],
                      [10.0 + a0, 50.0 + a1, 10.0 + a1, 50.0 + a2],
                      [10.0 + a1, 50.0 + a1, 10.0 + a2, 50.0 + a2]])
    cases = [("test_all_included", [(np.array([[10.0, 50.0, 20.0, 60.0]]), 0.0, 0)]),
             ("test_tiles", [(tiles, 0.0, 0)]),
             ("test_none_found", [(tiles + 11.0, 0.0, 0)]),
             ("test_with_border", [(BORDER_BOX, 0.0, 0), (BORDER_BOX, 0.5, 0),
                                   (BORDER_BOX, 1.0, 0), (BORDER_BOX, 2.0, 0),
                                   (BORDER_BOX, 2.0, 2)])]
    for name, calls in cases:
        for (boxes, xb, ib), (exp, _) in zip(calls, gold[name]):
            got = rectify_ref.compute_ij_bboxes(lon, lat, boxes, xb, ib)
            np.testing.assert_array_equal(got, exp.astype(np.int64), err_msg=name)


def test_product_tile_records():
    """rectify_tiles (product host code) derives the reference's per-tile
    windows and offsets (rectify.py:391-418) from K4's bboxes — checked here
    with the oracle's bboxes substituted (no GPU)."""
    import xcube_resampling_amd as xrs
    from xcube_resampling_amd import rectify as R

    g = load_golden("rectify_f32.npz")
    size, tile, geo = _geometry(g)
    tgm = xrs.GridMapping.regular(size, tuple(g["xy_min"]), float(g["res"]), "EPSG:4326",
                                  tile_size=tile)
    sgm = xrs.GridMapping.from_coords(xrs.DataArray(g["lon"], ("y", "x"), name="lon"),
                                      xrs.DataArray(g["lat"], ("y", "x"), name="lat"),
                                      "EPSG:4326")
    orig = type(sgm).ij_bboxes_from_xy_bboxes
    try:
        type(sgm).ij_bboxes_from_xy_bboxes = (
            lambda self, b, xy_border=0.0, ij_border=0, ij_bboxes=None, grid=None:
            rectify_ref.compute_ij_bboxes(g["lon"], g["lat"], b, xy_border, ij_border))
        tiles, ntx, bb, border = R.rectify_tiles(sgm, tgm)
    finally:
        type(sgm).ij_bboxes_from_xy_bboxes = orig
    np.testing.assert_array_equal(bb, g["ij_bboxes"])
    assert border == float(g["xy_border"])
    assert ntx == -(-size[0] // tile[0])
    t = tiles[1]
    assert (t["c0"], t["r0"], t["tw"], t["th"]) == (tile[0], 0, tile[0], tile[1])
    i_min, j_min, i_max, j_max = bb[1]
    assert (t["si0"], t["sj0"]) == (i_min, j_min)
    assert t["swin"] == min(i_max + 1, g["lon"].shape[1]) - i_min


def test_box_grid_decided_on_the_host():
    """K4's grid mode (and rectify_tiles_device's key scratch) is decided
    from the boxes alone, before any launch: the tiles of a regular grid
    qualify; a box list that is not one (or a wrong grid shape) does not."""
    from xcube_resampling_amd import kernels

    xs = np.array([0.0, 1.0, 2.5, 3.0])
    ys = np.array([10.0, 9.0, 7.5])
    boxes = [(xs[i], ys[j + 1], xs[i + 1], ys[j]) for j in range(2) for i in range(3)]
    b, ntx, nty = kernels._box_grid(boxes, 0.25, (3, 2))
    assert (ntx, nty) == (3, 2) and b.shape == (6, 4)
    assert np.array_equal(b[0], [-0.25, 8.75, 1.25, 10.25])
    assert kernels._box_grid(boxes, 0.25, (2, 3))[1:] == (0, 0)
    assert kernels._box_grid(boxes, 0.25, (4, 2))[1:] == (0, 0)      # 8 != 6 boxes
    assert kernels._box_grid(boxes, 0.25, None)[1:] == (0, 0)
    skew = [list(bx) for bx in boxes]
    skew[4][0] += 0.1
    assert kernels._box_grid(skew, 0.0, (3, 2))[1:] == (0, 0)

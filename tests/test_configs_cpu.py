"""CPU checks of the product's host-side geometry at the BASELINE config
sizes against the oracle: the reference's per-tile windows
(_get_scr_bboxes_indices, reproject.py:385-469) incl. the float32 window
origins, at configs 2 and 5; the config-1 affine matrix (base.py:461-478)."""

from __future__ import annotations

import numpy as np
import pytest

import configs
from helpers import assert_bitwise_equal


@pytest.mark.parametrize("size", [8192, 40960])
def test_plan_matches_oracle_windows_at_config_size(size):
    import bench

    o = configs.reproject_oracle(size)
    _, tgm, plan, lon, lat = bench.workload(size, 2048)
    assert_bitwise_equal(lon, o["lon"], "source lon")
    assert_bitwise_equal(lat, o["lat"], "source lat")
    assert_bitwise_equal(tgm.x_coords.values, o["geo"]["x_coords"], "target x")
    assert_bitwise_equal(tgm.y_coords.values, o["geo"]["y_coords"], "target y")
    np.testing.assert_array_equal(np.asarray(tgm.xy_bboxes), o["geo"]["xy_bboxes"])
    assert plan.num_tiles == (o["ntx"], o["nty"])
    np.testing.assert_array_equal(plan.scr_ij_bboxes, o["bboxes"])
    assert plan.pad_width == tuple(tuple(int(v) for v in p) for p in o["pad"])
    assert plan.win_width == o["x_coords"].shape[0]
    assert plan.win_height == o["y_coords"].shape[0]
    # the per-tile window origins the reference rounds to float32 (427-453)
    assert_bitwise_equal(plan.tile_x0, o["x_coords"][0].reshape(-1), "tile_x0")
    assert_bitwise_equal(plan.tile_y0, o["y_coords"][0].reshape(-1), "tile_y0")
    pt, pl = plan.pad_width[1][0], plan.pad_width[2][0]
    np.testing.assert_array_equal(plan.tile_win[:, 0], o["bboxes"][0].ravel() - pl)
    np.testing.assert_array_equal(plan.tile_win[:, 1], o["bboxes"][1].ravel() - pt)
    # the separable coordinate tables: one transform per column / row ==
    # the per-pixel transform of the meshgrid (reproject.py:472-496)
    from oracle import gridmapping_ref as gref

    for j in (0, o["nty"] // 2, o["nty"] - 1):
        r = slice(j * 2048, j * 2048 + 3)
        sxx, syy = gref.webmerc_inverse(*np.meshgrid(o["geo"]["x_coords"], o["geo"]["y_coords"][r]))
        assert_bitwise_equal(np.broadcast_to(plan.src_x[None, :], sxx.shape), sxx, "src_x")
        assert_bitwise_equal(np.broadcast_to(plan.src_y[r, None], syy.shape), syy, "src_y")


def test_config1_affine_matrix_matches_oracle():
    import xcube_resampling_amd as xrs

    lon, lat, geo, m = configs.config1_oracle()
    sgm = xrs.GridMapping.from_coords(xrs.DataArray(lon, "lon", name="lon"),
                                      xrs.DataArray(lat, "lat", name="lat"), "EPSG:4326")
    tgm = xrs.GridMapping.regular((configs.C1_SIZE,) * 2, configs.C1_TGT_MIN, configs.C1_TGT_RES,
                                  "EPSG:4326")
    assert tgm.ij_transform_to(sgm) == m
    assert abs(m[0][0] - 0.9216) < 1e-12 and abs(m[0][2] - 102.4) < 1e-9

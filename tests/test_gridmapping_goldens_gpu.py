"""GridMapping goldens that need the device: ij_bbox(es)_from_xy_bbox(es)
run the K4 kernel (xrs_ij_bboxes) — the reference's compute_ij_bboxes seam
(gridmapping/bboxes.py:28-106 via base.py:565-629).  Expected values from
the reference's tests/gridmapping/test_base.py:456-512 (see
test_gridmapping_goldens_cpu.py for the golden mechanism)."""

from __future__ import annotations

import numpy as np
import pytest

from test_gridmapping_goldens_cpu import BASE, Rec, _base_gm

pytestmark = pytest.mark.gpu


def test_base_ij_bbox_from_xy_bbox():
    gm = _base_gm()
    r = Rec(BASE, "GridMappingTest.test_ij_bbox_from_xy_bbox")
    for bbox, border in [((-180, -90, 180, 90), 0), ((-180, -90, 0, 0), 0),
                         ((0, 0, 180, 90), 0), ((-180, -90, 0, 0), 1), ((0, 0, 180, 90), 1),
                         ((-190, -100, -170, -80), 1), ((-190, -100, -180, -90), 1)]:
        r("ij_bbox", gm.ij_bbox_from_xy_bbox(bbox, ij_border=border))
    r.done()
    r = Rec(BASE, "GridMappingTest.test_ij_bboxes_from_xy_bboxes")
    boxes = np.array([[-180, -90, 180, 90], [-180, -90, 0, 0], [0, 0, 180, 90],
                      [-180, -90, 0, 0], [0, 0, 180, 90], [-190, -100, -170, -80],
                      [-190, -100, -180, -90]], dtype=np.float32)
    r("ij_bboxes", gm.ij_bboxes_from_xy_bboxes(xy_bboxes=boxes))
    r.done()



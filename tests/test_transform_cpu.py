"""Host side of the device coordinate transformation (xrs_transform): the
ctypes record matches include/xrs.h byte for byte, and every non-separable
transformer describes its pipeline with the constants of the numpy
restatement (crs.py / projections.py)."""

from __future__ import annotations

import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_proj_step_layout_matches_header(tmp_path):
    import ctypes

    from xcube_resampling_amd._native import ProjStep

    src = tmp_path / "sz.c"
    src.write_text('#include <stddef.h>\n#include <stdio.h>\n#include "xrs.h"\n'
                   "int main(void) { printf(\"%zu %zu %zu %zu\\n\", sizeof(XrsProjStep), "
                   "offsetof(XrsProjStep, c), offsetof(XrsProjStep, qp), "
                   "offsetof(XrsProjStep, cosb1)); return 0; }\n")
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)],
                   check=True)
    size, off_c, off_qp, off_cosb1 = map(int, subprocess.run(
        [str(exe)], check=True, capture_output=True, text=True).stdout.split())
    assert ctypes.sizeof(ProjStep) == size
    assert ProjStep.c.offset == off_c and ProjStep.qp.offset == off_qp
    assert ProjStep.cosb1.offset == off_cosb1


@pytest.mark.parametrize("src,dst,kinds", [
    ("EPSG:32632", "EPSG:3035", ["tmerc_inv", "laea_fwd"]),
    ("EPSG:4326", "EPSG:32633", ["tmerc_fwd"]),
    ("EPSG:3035", "EPSG:4326", ["laea_inv"]),
    ("EPSG:3857", "EPSG:32610", ["webmerc_inv", "tmerc_fwd"]),
    ("EPSG:4326", "EPSG:3857", ["webmerc_fwd"]),
])
def test_transformer_device_steps(src, dst, kinds):
    import xcube_resampling_amd as xrs
    from xcube_resampling_amd._native import PROJ_KINDS
    from xcube_resampling_amd.projections import TransverseMercator, WGS84

    tr = xrs.Transformer.from_crs(src, dst, always_xy=True)
    steps, n = tr.device_steps()
    assert [steps[k].kind for k in range(n)] == [PROJ_KINDS[k] for k in kinds]
    for k in range(n):
        st = steps[k]
        if kinds[k].startswith("tmerc"):
            ref = TransverseMercator(WGS84, 0.9996, 0.0)
            assert st.Qn == ref.Qn and st.Zb == ref.Zb
            assert list(st.c) == list(ref.cgb) + list(ref.cbg) + list(ref.utg) + list(ref.gtu)
            assert st.a == 6378137.0 and st.x0 == 500000.0
        if kinds[k].startswith("laea"):
            assert st.mode == 3 and st.x0 == 4321000.0 and st.y0 == 3210000.0
            assert st.lam0 == np.float64(10.0) * 0.017453292519943296


def test_identity_has_no_steps():
    import xcube_resampling_amd as xrs

    _, n = xrs.Transformer.from_crs("EPSG:32632", "EPSG:32632", always_xy=True).device_steps()
    assert n == 0

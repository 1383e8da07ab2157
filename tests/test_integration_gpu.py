"""The ctypes stub shown in INTEGRATION.md (what a maintainer adds to the
reference) runs as written against libxrs.so and reproduces the reference's
reprojection bit for bit."""

from __future__ import annotations

import os
import re

import numpy as np
import pytest

from helpers import assert_bitwise_equal, load_golden, reproject_golden_inputs

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _stub_namespace():
    import xcube_resampling_amd._native as N

    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    code = re.findall(r"```python\n(.*?)```", text, re.S)[0]
    code = code.replace('"/path/to/libxrs.so"', repr(N.LIB_PATH))
    ns: dict = {}
    exec(compile(code, "INTEGRATION.md", "exec"), ns)
    return ns


@pytest.mark.parametrize("interp", ["nearest", "bilinear"])
def test_integration_stub_matches_reference(interp):
    import xcube_resampling_amd as xrs

    ns = _stub_namespace()
    g = load_golden("reproject_f32.npz")
    ds, tgm = reproject_golden_inputs(g)
    sgm = xrs.GridMapping.from_dataset(ds)
    plan = xrs.plan_reproject(sgm, tgm, xrs.Transformer.from_crs(tgm.crs, sgm.crs,
                                                                  always_xy=True))
    out = ns["reproject_tiles"](
        g["data"], plan.src_x, plan.src_y, plan.tile_x0, plan.tile_y0,
        plan.tile_win.reshape(-1), (plan.win_height, plan.win_width),
        (plan.tile_height, plan.tile_width), (plan.dst_height, plan.dst_width),
        plan.x_res, plan.y_res, interp, np.nan)
    assert_bitwise_equal(out, g[f"out_{interp}"], interp)
    with pytest.raises(NotImplementedError):
        ns["reproject_tiles"](g["data"], plan.src_x, plan.src_y, plan.tile_x0, plan.tile_y0,
                              plan.tile_win.reshape(-1), (plan.win_height, plan.win_width),
                              (plan.tile_height, plan.tile_width),
                              (plan.dst_height, plan.dst_width), plan.x_res, plan.y_res,
                              "cubic", np.nan)

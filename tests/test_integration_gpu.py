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
    code = re.findall(r"```python\n(.*?)```", text, re.S)[0]   # the first block: the stub
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


@pytest.mark.parametrize("case", ["f32", "u8", "i16", "pad"])
@pytest.mark.parametrize("interp", ["nearest", "bilinear", "triangular"])
def test_integration_stub_on_reference_window_outputs(case, interp):
    """INTEGRATION.md's mapping driven by the REFERENCE's own window outputs:
    the golden fixtures hold what _get_scr_bboxes_indices returned
    (scr_ij_bboxes, x_coords, y_coords, pad_width, reproject.py:385-469);
    tables_from_windows maps them onto the ABI tables, the target centres are
    transformed per column / row by the oracle, and the stub reproduces the
    reference's blocks bit for bit."""
    from oracle import gridmapping_ref as gref

    ns = _stub_namespace()
    g = load_golden(f"reproject_{case}.npz")
    tx0, ty0, twin, win_hw = ns["tables_from_windows"](g["scr_ij_bboxes"], g["x_coords"],
                                                        g["y_coords"], g["pad_width"])
    tsize = tuple(int(v) for v in g["tsize"])
    ttile = tuple(int(v) for v in g["ttile"])
    geo = gref.regular_geometry(tsize, tuple(g["txy_min"]), tuple(g["tres"]), tile_size=ttile)
    sx, _ = gref.webmerc_inverse(geo["x_coords"], np.zeros(tsize[0]))
    _, sy = gref.webmerc_inverse(np.zeros(tsize[1]), geo["y_coords"])
    out = ns["reproject_tiles"](g["data"], sx, sy, tx0, ty0, twin, win_hw,
                                (ttile[1], ttile[0]), (tsize[1], tsize[0]), float(g["x_res"]),
                                float(g["y_res"]), interp, g["fill"].item())
    assert_bitwise_equal(out, g[f"out_{interp}"], f"{case}/{interp}")


def test_integration_stub_device_per_block_from_threads():
    """The stub's device argument as a dask threaded scheduler would use it:
    blocks (the dim-0 slices of two golden rasters, twice) run from
    four threads, each on device_of_block(k) — every visible GPU in turn (on
    the one-GPU box, all on cuda:0) — and each equals the reference's block."""
    from concurrent.futures import ThreadPoolExecutor

    import torch

    import xcube_resampling_amd as xrs

    ns = _stub_namespace()
    jobs = []
    for case in ("f32", "i16"):
        g = load_golden(f"reproject_{case}.npz")
        ds, tgm = reproject_golden_inputs(g)
        sgm = xrs.GridMapping.from_dataset(ds)
        plan = xrs.plan_reproject(sgm, tgm, xrs.Transformer.from_crs(tgm.crs, sgm.crs,
                                                                      always_xy=True))
        for s in range(g["data"].shape[0]):
            jobs.append((g, plan, s))
    jobs = jobs + jobs
    ngpu = torch.cuda.device_count()

    def block(k):
        g, plan, s = jobs[k]
        dev = ns["device_of_block"](k)
        assert dev.index == k % ngpu
        out = ns["reproject_tiles"](
            g["data"][s:s + 1], plan.src_x, plan.src_y, plan.tile_x0, plan.tile_y0,
            plan.tile_win.reshape(-1), (plan.win_height, plan.win_width),
            (plan.tile_height, plan.tile_width), (plan.dst_height, plan.dst_width),
            plan.x_res, plan.y_res, "bilinear", g["fill"].item(), device=dev)
        exp = g["out_bilinear"][s:s + 1]
        same = (out == exp) | (np.isnan(out) & np.isnan(exp))
        return k, out.dtype, exp.dtype, int((~same).sum())

    serial = [block(k) for k in range(len(jobs))]
    assert all(r[3] == 0 for r in serial), serial
    with ThreadPoolExecutor(4) as ex:
        threaded = list(ex.map(block, range(len(jobs))))
    assert all(r[3] == 0 for r in threaded), threaded

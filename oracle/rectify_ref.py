"""ORACLE (test infrastructure only) — the reference's rectify path on the CPU.

Python driver restating the tiling of xcube_resampling/rectify.py
(_compute_target_source_ij 312-370, _compute_target_source_ij_block 373-419,
_compute_var_image_block 605-635) around plain-C restatements of the numba
kernels (rectify_ref.c: compute_ij_bboxes bboxes.py:28-106,
_compute_target_source_ij_sequential/_line rectify.py:424-576,
_compute_var_image_sequential/_for_dest_line rectify.py:640-734).
Built by ``make -C oracle`` (__graft_entry__.build()).
"""

from __future__ import annotations

import ctypes
import math
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from . import gridmapping_ref as gref

_LIB = None
_HERE = os.path.dirname(os.path.abspath(__file__))


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "_build", "librectify_ref.so")
        if not os.path.exists(path):
            raise RuntimeError("oracle C library not built: run `make -C oracle`")
        L = ctypes.CDLL(path)
        P, I, D = ctypes.c_void_p, ctypes.c_int64, ctypes.c_double
        L.compute_ij_bboxes.argtypes = [P, P, I, I, P, I, D, I, P]
        L.compute_target_source_ij_sequential.argtypes = [P, P, I, I, I, I, P, I, I, D, D, D, D, D]
        L.compute_var_image_sequential.argtypes = [P, I, I, I, P, I, I, I, I, ctypes.c_int, P, P]
        _LIB = L
    return _LIB


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def compute_ij_bboxes(x_image, y_image, xy_boxes, xy_border, ij_border):
    x = np.ascontiguousarray(x_image, np.float64)
    y = np.ascontiguousarray(y_image, np.float64)
    boxes = np.ascontiguousarray(xy_boxes, np.float64).reshape(-1, 4)
    out = np.full(boxes.shape, -1, np.int64)
    lib().compute_ij_bboxes(_p(x), _p(y), x.shape[0], x.shape[1], _p(boxes), boxes.shape[0],
                            float(xy_border), int(ij_border), _p(out))
    return out


def target_tiles(size, tile_size):
    w, h = size
    tw, th = tile_size
    return [(r0, min(h, r0 + th), c0, min(w, c0 + tw)) for r0 in range(0, h, th)
            for c0 in range(0, w, tw)]


def compute_target_source_ij(src_x, src_y, size, tile_size, xy_bbox, xy_res, j_up=False,
                             uv_delta=1e-3, threads=1, tile_ids=None):
    """rectify.py:312-419 for a target grid (size, tile_size, xy_bbox, xy_res);
    ``tile_ids``: only those target tiles (raster order), the others NaN — a
    dask worker's share of the tiles (rectify.py:347-370)."""
    w, h = size
    tw, th = tile_size
    x_min, y_min, x_max, y_max = xy_bbox
    x_res, y_res = xy_res
    xy_border = min(min(2 * (w / tw) * x_res, 2 * (h / th) * y_res),
                    min(0.5 * (x_max - x_min), 0.5 * (y_max - y_min)))
    boxes = gref.xy_bboxes(size, tile_size, xy_bbox, xy_res, j_up)
    src_x = np.ascontiguousarray(src_x, np.float64)
    src_y = np.ascontiguousarray(src_y, np.float64)
    ij_bboxes = compute_ij_bboxes(src_x, src_y, boxes, xy_border, 1)
    out = np.full((2, h, w), np.nan)

    def block(k_tile):
        k, (r0, r1, c0, c1) = k_tile
        i_min, j_min, i_max, j_max = (int(v) for v in ij_bboxes[k])
        blk = np.full((2, r1 - r0, c1 - c0), np.nan)
        if i_min == -1:
            return k, blk
        wx = np.ascontiguousarray(src_x[j_min:j_max + 1, i_min:i_max + 1])
        wy = np.ascontiguousarray(src_y[j_min:j_max + 1, i_min:i_max + 1])
        x_off = x_min + c0 * x_res
        y_off = (y_min + r0 * y_res) if j_up else (y_max - r0 * y_res)
        lib().compute_target_source_ij_sequential(
            _p(wx), _p(wy), wx.shape[0], wx.shape[1], i_min, j_min, _p(blk), r1 - r0, c1 - c0,
            x_off, y_off, x_res, y_res if j_up else -y_res, uv_delta)
        return k, blk

    tiles = list(enumerate(target_tiles(size, tile_size)))
    if tile_ids is not None:
        keep = set(int(t) for t in tile_ids)
        tiles = [kt for kt in tiles if kt[0] in keep]
    with ThreadPoolExecutor(max_workers=threads) as ex:
        for k, blk in ex.map(block, tiles):
            r0, r1, c0, c1 = dict(tiles)[k]
            out[:, r0:r1, c0:c1] = blk
    return out, ij_bboxes


def compute_var_image(ij, var, fill_value, interp, tile_size, threads=1, tile_ids=None):
    """rectify.py:579-635: per target tile, source sub-window + sequential loop
    (``tile_ids``: only those tiles, the others fill)."""
    codes = {"nearest": 0, "bilinear": 1, "triangular": 2}
    if interp not in codes:
        raise NotImplementedError(
            f"interp_methods must be one of 0, 1, 'nearest', 'bilinear', "
            f"'triangular', was '{interp}'.")
    var = np.asarray(var)
    squeeze = var.ndim == 2
    if squeeze:
        var = var[None]
    n, sh, sw = var.shape
    _, h, w = ij.shape
    out = np.full((n, h, w), fill_value, dtype=var.dtype)

    def block(t):
        r0, r1, c0, c1 = t
        tij = np.ascontiguousarray(ij[:, r0:r1, c0:c1])
        if np.all(np.isnan(tij[0])):
            return t, None
        b0 = int(np.nanmin(tij[0]))
        b1 = int(np.nanmin(tij[1]))
        b2 = min(int(np.nanmax(tij[0])) + 2, sw)
        b3 = min(int(np.nanmax(tij[1])) + 2, sh)
        win = np.ascontiguousarray(var[:, b1:b3, b0:b2].astype(np.float64))
        vals = np.zeros((n, r1 - r0, c1 - c0))
        written = np.zeros((r1 - r0, c1 - c0), np.uint8)
        lib().compute_var_image_sequential(_p(win), n, win.shape[1], win.shape[2], _p(tij),
                                           r1 - r0, c1 - c0, b0, b1, codes[interp], _p(vals),
                                           _p(written))
        return t, (vals, written.astype(bool))

    tl = target_tiles((w, h), tile_size)
    if tile_ids is not None:
        tl = [tl[int(t)] for t in tile_ids]
    with ThreadPoolExecutor(max_workers=threads) as ex:
        for (r0, r1, c0, c1), res in ex.map(block, tl):
            if res is None:
                continue
            vals, written = res
            blk = out[:, r0:r1, c0:c1]
            blk[:, written] = vals[:, written].astype(var.dtype)
    return out[0] if squeeze else out

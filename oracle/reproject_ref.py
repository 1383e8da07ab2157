"""ORACLE (test infrastructure only) — numpy restatement of the reference's
reproject path, tile by tile, exactly as the dask graph evaluates it.

Follows xcube_resampling/reproject.py:
  _reproject_block             268-335   reproject_block()
  _get_scr_bboxes_indices      385-469   get_scr_bboxes_indices()
  _reorganize_data_array_slice 499-530   reorganize_data_array_slice()
  _transform_gridpoints        472-496   (meshgrid + transform per tile)
  _reproject_data_array        189-265   reproject_array()
"""

from __future__ import annotations

import math

import numpy as np


def reproject_block(source_xx, source_yy, scr_data, x_coord, y_coord, scr_x_res, scr_y_res,
                    interp_method):
    """reproject.py:268-335 (numpy, literal)."""
    ix = (source_xx - x_coord[0]) / scr_x_res
    iy = (source_yy - y_coord[0]) / -scr_y_res
    if interp_method == "nearest":
        ix = np.rint(ix).astype(np.int16)
        iy = np.rint(iy).astype(np.int16)
        return scr_data[:, iy, ix]
    if interp_method not in ("triangular", "bilinear"):
        raise NotImplementedError(
            f"interp_methods must be one of 0, 1, 'nearest', 'bilinear', 'triangular', "
            f"was '{interp_method}'.")
    ix_ceil = np.ceil(ix).astype(np.int16)
    ix_floor = np.floor(ix).astype(np.int16)
    iy_ceil = np.ceil(iy).astype(np.int16)
    iy_floor = np.floor(iy).astype(np.int16)
    diff_ix = ix - ix_floor
    diff_iy = iy - iy_floor
    v00 = scr_data[:, iy_floor, ix_floor]
    v01 = scr_data[:, iy_floor, ix_ceil]
    v10 = scr_data[:, iy_ceil, ix_floor]
    v11 = scr_data[:, iy_ceil, ix_ceil]
    if interp_method == "bilinear":
        u0 = v00 + diff_ix * (v01 - v00)
        u1 = v10 + diff_ix * (v11 - v10)
        return u0 + diff_iy * (u1 - u0)
    mask = diff_ix + diff_iy < 1.0
    n = scr_data.shape[0]
    m3 = np.repeat(mask[np.newaxis], n, axis=0)
    dx3 = np.repeat(diff_ix[np.newaxis], n, axis=0)
    dy3 = np.repeat(diff_iy[np.newaxis], n, axis=0)
    out = np.zeros((n, iy.shape[0], iy.shape[1]), dtype=scr_data.dtype)
    out[m3] = v00[m3] + dx3[m3] * (v01[m3] - v00[m3]) + dy3[m3] * (v10[m3] - v00[m3])
    nm = ~m3
    out[nm] = (v11[nm] + (1.0 - dx3[nm]) * (v10[nm] - v11[nm])
               + (1.0 - dy3[nm]) * (v01[nm] - v11[nm]))
    return out


def get_scr_bboxes_indices(transform_bounds, src_x_coords, src_y_coords, src_x_res, src_y_res,
                           src_width, src_height, target_xy_bboxes, num_tiles_x, num_tiles_y):
    """reproject.py:385-469 (loops as written; dask arrays -> numpy)."""
    origin = src_x_coords[0], src_y_coords[0]
    b = np.full((4, num_tiles_y, num_tiles_x), -1, dtype=np.int32)
    for idx, xy_bbox in enumerate(target_xy_bboxes):
        j, i = np.unravel_index(idx, (num_tiles_y, num_tiles_x))
        s = transform_bounds(*xy_bbox)
        b[:, j, i] = [math.floor((s[0] - origin[0]) / src_x_res),
                      math.floor((origin[1] - s[3]) / src_y_res),
                      math.ceil((s[2] - origin[0]) / src_x_res),
                      math.ceil((origin[1] - s[1]) / src_y_res)]
    i_diff = b[2] - b[0]
    j_diff = b[3] - b[1]
    i_diff_max = np.max(i_diff) + 1
    j_diff_max = np.max(j_diff) + 1
    for i in range(num_tiles_x):
        for j in range(num_tiles_y):
            bb = b[:, j, i]
            i_start = bb[0] - (i_diff_max - i_diff[j, i]) // 2
            j_start = bb[1] - (j_diff_max - j_diff[j, i]) // 2
            b[:, j, i] = [i_start, j_start, i_start + i_diff_max, j_start + j_diff_max]
    x_coords = np.zeros((i_diff_max, num_tiles_y, num_tiles_x), dtype=np.float32)
    y_coords = np.zeros((j_diff_max, num_tiles_y, num_tiles_x), dtype=np.float32)
    i_min = np.min(b[0])
    i_max = np.max(b[2])
    j_min = np.min(b[[1, 3]])
    j_max = np.max(b[[1, 3]])
    x_coord = np.arange(src_x_coords[0] + i_min * src_x_res, src_x_coords[0] + i_max * src_x_res,
                        src_x_res)
    y_res = src_y_coords[1] - src_y_coords[0]
    y_coord = np.arange(src_y_coords[0] + j_min * y_res, src_y_coords[0] + j_max * y_res, y_res)
    for i in range(num_tiles_x):
        for j in range(num_tiles_y):
            s0 = b[0, j, i] - i_min
            x_coords[:, j, i] = x_coord[s0:s0 + i_diff_max]
            t0 = b[1, j, i] - j_min
            y_coords[:, j, i] = y_coord[t0:t0 + j_diff_max]
    pad_width = ((0, 0),
                 (-min(0, int(j_min)), max(0, int(j_max - src_height))),
                 (-min(0, int(i_min)), max(0, int(i_max - src_width))))
    b[[1, 3]] += pad_width[1][0]
    b[[0, 2]] += pad_width[2][0]
    return b, x_coords, y_coords, pad_width


def reorganize_data_array_slice(array, x_coords, y_coords, scr_ij_bboxes, pad_width, fill_value):
    """reproject.py:499-530 (da.pad + per-tile window copy)."""
    wy, wx = y_coords.shape[0], x_coords.shape[0]
    nty, ntx = scr_ij_bboxes.shape[1], scr_ij_bboxes.shape[2]
    out = np.zeros((array.shape[0], wy * nty, wx * ntx), dtype=array.dtype)
    data_in = np.pad(array, pad_width, mode="constant", constant_values=fill_value)
    for i in range(ntx):
        for j in range(nty):
            bb = scr_ij_bboxes[:, j, i]
            out[:, j * wy:(j + 1) * wy, i * wx:(i + 1) * wx] = data_in[:, bb[1]:bb[3], bb[0]:bb[2]]
    return out


def reproject_array(array, transform, transform_bounds, src_x_coords, src_y_coords, src_x_res,
                    src_y_res, dst_x_coords, dst_y_coords, dst_xy_bboxes, tile_w, tile_h,
                    interp_method, fill_value, tiles=None):
    """reproject.py:189-265 + 472-496 for one (n, H, W) array.

    `transform(xx, yy)` maps target-CRS points to the source CRS (always_xy).
    `tiles`: optional list of (tj, ti) to evaluate (others left as zeros) —
    used to time a bounded sample for the CPU baseline.
    Returns an (n, H', W') array in the dtype the reference produces.
    """
    n, src_h, src_w = array.shape
    dst_w, dst_h = len(dst_x_coords), len(dst_y_coords)
    ntx, nty = math.ceil(dst_w / tile_w), math.ceil(dst_h / tile_h)
    b, xc, yc, pad = get_scr_bboxes_indices(transform_bounds, src_x_coords, src_y_coords,
                                            src_x_res, src_y_res, src_w, src_h, dst_xy_bboxes,
                                            ntx, nty)
    wy, wx = yc.shape[0], xc.shape[0]
    out = None
    todo = tiles if tiles is not None else [(j, i) for j in range(nty) for i in range(ntx)]
    for j, i in todo:
        r0, r1 = j * tile_h, min(dst_h, (j + 1) * tile_h)
        c0, c1 = i * tile_w, min(dst_w, (i + 1) * tile_w)
        xx, yy = np.meshgrid(dst_x_coords[c0:c1], dst_y_coords[r0:r1])
        sxx, syy = transform(xx, yy)
        bb = b[:, j, i]
        win = _padded_window(array, pad, bb, fill_value)
        res = reproject_block(sxx, syy, win, xc[:, j, i].reshape(-1, 1, 1),
                              yc[:, j, i].reshape(-1, 1, 1), src_x_res, src_y_res, interp_method)
        if out is None:
            out = np.zeros((n, dst_h, dst_w), dtype=res.dtype)
        out[:, r0:r1, c0:c1] = res
    return out


def _padded_window(array, pad, bb, fill_value):
    """data_in[:, bb[1]:bb[3], bb[0]:bb[2]] of the padded array, without
    materialising the whole pad (same values as reorganize_data_array_slice)."""
    n, h, w = array.shape
    pt, pl = pad[1][0], pad[2][0]
    j0, j1, i0, i1 = bb[1] - pt, bb[3] - pt, bb[0] - pl, bb[2] - pl
    win = np.empty((n, j1 - j0, i1 - i0), dtype=array.dtype)
    win[...] = np.array(fill_value).astype(array.dtype)
    sj0, sj1, si0, si1 = max(0, j0), min(h, j1), max(0, i0), min(w, i1)
    if sj1 > sj0 and si1 > si0:
        win[:, sj0 - j0:sj1 - j0, si0 - i0:si1 - i0] = array[:, sj0:sj1, si0:si1]
    return win

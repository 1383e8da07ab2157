"""ORACLE (test infrastructure only) — grid geometry numerics of the
reference, restated independently of the product's GridMapping.

  dask_linspace        dask.array.linspace (creation.py) as used by
                       gridmapping/regular.py:44-63
  regular_geometry     gridmapping/regular.py:87-129 (+ helpers.py:39-48)
  xy_bboxes            gridmapping/base.py:503-533
  webmerc_inverse /    PROJ webmerc (merc_s_inverse / merc_s_forward) with
  webmerc_forward      inv_prepare's x*ra de-scaling and unitconvert — PROJ is
                       not in the reference tree: restated from PROJ's
                       published algorithm; PARITY UNPINNED for this step.
  transform_bounds     PROJ proj_trans_bounds (21 densified points per edge)
"""

from __future__ import annotations

import math

import numpy as np

A_WGS84 = 6378137.0
DEG_TO_RAD = 0.017453292519943296


def to_int_or_float(x):
    """helpers.py:39-48."""
    if isinstance(x, int):
        return x
    xf = float(x)
    xi = round(xf)
    return xi if math.isclose(xi, xf, rel_tol=1e-5) else xf


def dask_linspace(start, stop, num, chunk):
    step = float(stop - start) / (num - 1)
    out, blockstart, pos = [], start, 0
    while pos < num:
        bs = min(chunk, num - pos)
        out.append(np.linspace(blockstart, blockstart + ((bs - 1) * step), bs))
        blockstart = blockstart + (step * bs)
        pos += bs
    return np.concatenate(out)


def regular_geometry(size, xy_min, xy_res, tile_size=None, is_j_axis_up=False):
    """Pixel-centre coordinates, bbox and tile boxes of GridMapping.regular."""
    w, h = size
    xr, yr = (xy_res, xy_res) if np.isscalar(xy_res) else xy_res
    xr, yr = to_int_or_float(xr), to_int_or_float(yr)
    x_min = to_int_or_float(to_int_or_float(xy_min[0]))
    y_min = to_int_or_float(to_int_or_float(xy_min[1]))
    x_max = to_int_or_float(x_min + xr * w)
    y_max = to_int_or_float(y_min + yr * h)
    tw, th = tile_size if tile_size else (w, h)
    xs = dask_linspace(x_min + xr / 2, x_max - xr / 2, w, tw)
    y1, y2 = y_min + yr / 2, y_max - yr / 2
    if not is_j_axis_up:
        y1, y2 = y2, y1
    ys = dask_linspace(y1, y2, h, th)
    return dict(x_coords=xs, y_coords=ys, xy_bbox=(x_min, y_min, x_max, y_max),
                xy_res=(xr, yr), tile_size=(tw, th),
                xy_bboxes=xy_bboxes((w, h), (tw, th), (x_min, y_min, x_max, y_max), (xr, yr),
                                    is_j_axis_up))


def xy_bboxes(size, tile_size, xy_bbox, xy_res, is_j_axis_up=False):
    w, h = size
    tw, th = tile_size
    boxes = []
    for y0 in range(0, h, th):
        for x0 in range(0, w, tw):
            boxes.append((x0, y0, min(w, x0 + tw), min(h, y0 + th)))
    ij = np.array(boxes, dtype=np.int64)
    x_min, y_min, x_max, y_max = xy_bbox
    xr, yr = xy_res
    if is_j_axis_up:
        return np.array([x_min, y_min, x_min, y_min]) + np.array([xr, yr, xr, yr]) * ij
    out = np.array([x_min, y_max, x_min, y_max]) + np.array([xr, -yr, xr, -yr]) * ij
    out[:, [1, 3]] = out[:, [3, 1]]
    return out


def webmerc_inverse(x, y):
    ra = 1.0 / A_WGS84
    f = 1.0 / DEG_TO_RAD
    x = np.asarray(x, np.float64)
    y = np.asarray(y, np.float64)
    return (x * ra) * f, np.arctan(np.sinh(y * ra)) * f


def webmerc_forward(lon, lat):
    lam = np.asarray(lon, np.float64) * DEG_TO_RAD
    phi = np.asarray(lat, np.float64) * DEG_TO_RAD
    return A_WGS84 * lam, A_WGS84 * np.arcsinh(np.tan(phi))


def transform_bounds(transform, left, bottom, right, top, densify_pts=21):
    side = densify_pts + 1
    dx = (right - left) / side
    dy = (top - bottom) / side
    k = np.arange(side, dtype=np.float64)
    xs = np.concatenate([np.full(side, left), left + k * dx, np.full(side, right), right - k * dx])
    ys = np.concatenate([top - k * dy, np.full(side, bottom), bottom + k * dy, np.full(side, top)])
    tx, ty = transform(xs, ys)
    ok = np.isfinite(tx) & np.isfinite(ty)
    return float(tx[ok].min()), float(ty[ok].min()), float(tx[ok].max()), float(ty[ok].max())


# --------------------------------------------------------------------------
# affine-package matrix arithmetic (affine >= 2.2, not installed here; its
# published __invert__ / __mul__ restated) as used by
# gridmapping/base.py:437-478 (ij_to_xy_transform, xy_to_ij_transform,
# ij_transform_to) through helpers.py:51-56 (_from_affine / _to_affine)
# --------------------------------------------------------------------------

def affine_invert(m):
    """affine.Affine.__invert__: idet = 1 / (a*e - b*d), then the closed form."""
    (a, b, c), (d, e, f) = m
    idet = 1.0 / (a * e - b * d)
    ra = e * idet
    rb = -b * idet
    rd = -d * idet
    re = a * idet
    return (ra, rb, -c * ra - f * rb), (rd, re, -c * rd - f * re)


def affine_mul(s, o):
    """affine.Affine.__mul__ (s * o, both 2x3)."""
    (sa, sb, sc), (sd, se, sf) = s
    (oa, ob, oc), (od, oe, of) = o
    return ((sa * oa + sb * od, sa * ob + sb * oe, sa * oc + sb * of + sc),
            (sd * oa + se * od, sd * ob + se * oe, sd * oc + se * of + sf))


def ij_to_xy_transform(xy_bbox, xy_res, is_j_axis_up=False):
    """base.py:437-451."""
    x_min, y_min, _, y_max = xy_bbox
    x_res, y_res = xy_res
    if is_j_axis_up:
        return (x_res, 0.0, x_min), (0.0, y_res, y_min)
    return (x_res, 0.0, x_min), (0.0, -y_res, y_max)


def ij_transform_to(src_ij_to_xy, tgt_ij_to_xy):
    """base.py:461-478 with self = target, other = source: image coordinates
    of the target -> image coordinates of the source (affine.py:121)."""
    return affine_mul(affine_invert(src_ij_to_xy), tgt_ij_to_xy)

"""BASELINE.json configs as test geometry, stated twice:
through the product's API and through the oracle, so parity tests compare
the two at the benchmark sizes.

  config 1  affine nearest 1024^2 f32, EPSG:4326 (scale 0.9216, 102.4 px offset)
  config 2  reproject bilinear 8192^2 f32 EPSG:4326 -> EPSG:3857, 2048^2 tiles
  config 5  reproject bilinear 40960^2 (as config 2, finer), 2048^2 tiles
"""

from __future__ import annotations

import math

import numpy as np

from oracle import gridmapping_ref as gref
from oracle import reproject_ref

# config 1
C1_SIZE = 1024
C1_SRC_RES = 2.0 ** -10
C1_SRC_X0, C1_SRC_Y1 = 10.0, 51.0
C1_TGT_MIN, C1_TGT_RES = (10.1, 50.05), 0.0009

# configs 2 / 5 (bench.workload)
REPROJECT_SRC_X0, REPROJECT_SRC_Y0 = -20.0, 70.96
REPROJECT_TGT_MIN = (-2226000.0, 3504000.0)


def config1_oracle():
    """Source pixel centres, target geometry and the affine matrix, all from
    the oracle (affine-package arithmetic restated in oracle/gridmapping_ref)."""
    n = C1_SIZE
    lon = C1_SRC_X0 + (np.arange(n) + 0.5) * C1_SRC_RES
    lat = C1_SRC_Y1 - (np.arange(n) + 0.5) * C1_SRC_RES
    src_bbox = (C1_SRC_X0, C1_SRC_Y1 - n * C1_SRC_RES, C1_SRC_X0 + n * C1_SRC_RES, C1_SRC_Y1)
    geo = gref.regular_geometry((n, n), C1_TGT_MIN, C1_TGT_RES)
    m = gref.ij_transform_to(gref.ij_to_xy_transform(src_bbox, (C1_SRC_RES, C1_SRC_RES)),
                             gref.ij_to_xy_transform(geo["xy_bbox"], geo["xy_res"]))
    return lon, lat, geo, m


def reproject_oracle(size: int, tile: int = 2048):
    """Oracle geometry of configs 2 (8192) / 5 (40960): source pixel centres,
    target geometry and the reference's windows (_get_scr_bboxes_indices,
    reproject.py:385-469) computed by the oracle."""
    scale = 40960 / size
    xres, yres = 0.0015 * scale, 0.001 * scale
    lon = REPROJECT_SRC_X0 + (np.arange(size) + 0.5) * xres
    lat = REPROJECT_SRC_Y0 - (np.arange(size) + 0.5) * yres
    geo = gref.regular_geometry((size, size), REPROJECT_TGT_MIN, (166 * scale, 190 * scale),
                                tile_size=(tile, tile))
    ntx = nty = math.ceil(size / tile)
    win = reproject_ref.get_scr_bboxes_indices(
        lambda *b: gref.transform_bounds(gref.webmerc_inverse, *b), lon, lat, xres, yres,
        size, size, geo["xy_bboxes"], ntx, nty)
    return dict(lon=lon, lat=lat, x_res=xres, y_res=yres, geo=geo, tile=tile, ntx=ntx, nty=nty,
                bboxes=win[0], x_coords=win[1], y_coords=win[2], pad=win[3])


def oracle_tile(o: dict, src_host_window, j: int, i: int, interp: str):
    """The reference's block for target tile (j, i): _transform_gridpoints
    (reproject.py:472-496) + _reproject_block (268-335) on the tile's padded
    window.  `src_host_window(j0, j1, i0, i1)` returns source rows / columns
    [j0, j1) x [i0, i1) (clipped to the source) as an (n, rows, cols) array."""
    tile, geo = o["tile"], o["geo"]
    size = len(o["lon"])
    r0, r1 = j * tile, min(size, (j + 1) * tile)
    c0, c1 = i * tile, min(size, (i + 1) * tile)
    sxx, syy = gref.webmerc_inverse(*np.meshgrid(geo["x_coords"][c0:c1], geo["y_coords"][r0:r1]))
    bb = o["bboxes"][:, j, i]
    pt, pl = o["pad"][1][0], o["pad"][2][0]
    wj0, wj1, wi0, wi1 = int(bb[1]) - pt, int(bb[3]) - pt, int(bb[0]) - pl, int(bb[2]) - pl
    sj0, sj1, si0, si1 = max(0, wj0), min(size, wj1), max(0, wi0), min(size, wi1)
    part = src_host_window(sj0, sj1, si0, si1)
    win = np.full((part.shape[0], wj1 - wj0, wi1 - wi0), np.nan, part.dtype)
    win[:, sj0 - wj0:sj1 - wj0, si0 - wi0:si1 - wi0] = part
    out = reproject_ref.reproject_block(sxx, syy, win, o["x_coords"][:, j, i].reshape(-1, 1, 1),
                                        o["y_coords"][:, j, i].reshape(-1, 1, 1), o["x_res"],
                                        o["y_res"], interp)
    return out, (r0, r1, c0, c1)


def sample_tiles(ntx: int, nty: int):
    """At least one tile per tile row (a column walking across the raster),
    plus the four corners."""
    tiles = {(j, (7 * j + 3) % ntx) for j in range(nty)}
    tiles |= {(0, 0), (0, ntx - 1), (nty - 1, 0), (nty - 1, ntx - 1)}
    return sorted(tiles)

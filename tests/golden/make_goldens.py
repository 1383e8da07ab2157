"""Generate golden fixtures by EXECUTING the reference's own functions.

Run in the development container (needs /root/reference; never on the GPU box):

    python tests/golden/make_goldens.py

Writes small .npz fixtures next to this script.  Each fixture holds the inputs
and the reference's outputs; tests compare the oracle (oracle/) and the HIP
kernels against them.  See refload.py for how reference functions are run
without xarray/dask/numba.
"""

from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, HERE)

from refload import chunked, load_functions  # noqa: E402

from oracle import gridmapping_ref as gref  # noqa: E402  (geometry + PROJ restatement)

SEED = 20250905


class _Values:
    def __init__(self, v):
        self.values = np.asarray(v)


class _SourceGM:
    def __init__(self, x, y, x_res, y_res):
        self.x_coords, self.y_coords = _Values(x), _Values(y)
        self.x_res, self.y_res = x_res, y_res
        self.width, self.height = len(x), len(y)


class _TargetGM:
    def __init__(self, geo, size):
        self.width, self.height = size
        self.tile_width, self.tile_height = geo["tile_size"]
        self.xy_bboxes = geo["xy_bboxes"]
        self.x_coords, self.y_coords = _Values(geo["x_coords"]), _Values(geo["y_coords"])


class _Transformer:
    """target (EPSG:3857) -> source (EPSG:4326), always_xy."""

    transform = staticmethod(gref.webmerc_inverse)

    def transform_bounds(self, *b):
        return gref.transform_bounds(gref.webmerc_inverse, *b)


def reproject_case(name, data, src_lon, src_lat, x_res, y_res, tsize, txy_min, tres, ttile,
                   interps, fill):
    ref = load_functions("xcube_resampling/reproject.py",
                         ["_reproject_block", "_get_scr_bboxes_indices",
                          "_reorganize_data_array_slice"])
    sgm = _SourceGM(src_lon, src_lat, x_res, y_res)
    geo = gref.regular_geometry(tsize, txy_min, tres, tile_size=ttile)
    tgm = _TargetGM(geo, tsize)
    tr = _Transformer()
    b, xc, yc, pad = ref["_get_scr_bboxes_indices"](tr, sgm, tgm)
    arr = chunked(data, ((data.shape[0],), (data.shape[1],), (data.shape[2],)))
    scr = ref["_reorganize_data_array_slice"](arr, xc, yc, b, pad, fill)
    wy, wx = yc.shape[0], xc.shape[0]
    tw, th = ttile
    W, H = tsize
    sxx, syy = np.meshgrid(geo["x_coords"], geo["y_coords"])
    sxx, syy = tr.transform(sxx, syy)
    out = {}
    for interp in interps:
        res = None
        for j in range(b.shape[1]):
            for i in range(b.shape[2]):
                r0, r1, c0, c1 = j * th, min(H, (j + 1) * th), i * tw, min(W, (i + 1) * tw)
                blk = ref["_reproject_block"](
                    sxx[r0:r1, c0:c1], syy[r0:r1, c0:c1],
                    scr[:, j * wy:(j + 1) * wy, i * wx:(i + 1) * wx],
                    xc[:, j:j + 1, i:i + 1], yc[:, j:j + 1, i:i + 1], x_res, y_res, interp)
                if res is None:
                    res = np.zeros((data.shape[0], H, W), dtype=blk.dtype)
                res[:, r0:r1, c0:c1] = blk
        out[f"out_{interp}"] = res
    np.savez_compressed(
        os.path.join(HERE, f"reproject_{name}.npz"),
        data=data, src_lon=src_lon, src_lat=src_lat, x_res=x_res, y_res=y_res,
        tsize=np.array(tsize), txy_min=np.array(txy_min, dtype=np.float64),
        tres=np.array(tres, dtype=np.float64), ttile=np.array(ttile), fill=fill,
        scr_ij_bboxes=b, x_coords=xc, y_coords=yc, pad_width=np.array(pad),
        interps=np.array(interps), **out)
    print(f"reproject_{name}: data {data.shape} {data.dtype} -> {tsize} tiles {ttile}, "
          f"windows {wx}x{wy}, pad {pad}")


class _ValuesView:
    """Stand-in for an xarray.DataArray inside the reference block functions
    (only slicing + .values are used)."""

    def __init__(self, a):
        self._a = np.asarray(a)

    def __getitem__(self, k):
        return _ValuesView(self._a[k])

    @property
    def values(self):
        return self._a

    @property
    def shape(self):
        return self._a.shape

    @property
    def dtype(self):
        return self._a.dtype


def _swath(rng, h, w, lon0, lat0, dlon_i, dlon_j, dlat_i, dlat_j, curv, jitter):
    i = np.arange(w)[None, :]
    j = np.arange(h)[:, None]
    lon = lon0 + dlon_i * i + dlon_j * j
    lat = lat0 - dlat_j * j - dlat_i * i + curv * (i - w / 2) ** 2
    lon = lon + rng.normal(0, jitter * dlon_i, (h, w))
    lat = lat + rng.normal(0, jitter * dlat_j, (h, w))
    return lon, lat


def rectify_case(name, rng, h, w, size, xy_min, res, tile, nvar, dtype, j_up=False, nan_px=0):
    ref = load_functions("xcube_resampling/rectify.py", [
        "_compute_target_source_ij_block", "_compute_target_source_ij_sequential",
        "_compute_target_source_ij_line", "_compute_var_image_block",
        "_compute_var_image_sequential", "_compute_var_image_for_dest_line",
        "_fdet", "_fu", "_fv", "_fclamp", "_iclamp"])
    bb = load_functions("xcube_resampling/gridmapping/bboxes.py", ["compute_ij_bboxes"])
    lon, lat = _swath(rng, h, w, 5.0, 60.0, 0.045, 0.009, 0.004, 0.027, 1e-6, 0.05)
    if nan_px:
        lon.ravel()[rng.choice(lon.size, nan_px, replace=False)] = np.nan
    if np.issubdtype(dtype, np.floating):
        var = rng.random((nvar, h, w)).astype(dtype)
    else:
        var = rng.integers(0, 250, (nvar, h, w)).astype(dtype)
    W, H = size
    tw, th = tile
    geo = gref.regular_geometry(size, xy_min, res, tile_size=tile, is_j_axis_up=j_up)
    x_min, y_min, x_max, y_max = geo["xy_bbox"]
    x_res, y_res = geo["xy_res"]
    xy_border = min(min(2 * (W / tw) * x_res, 2 * (H / th) * y_res),
                    min(0.5 * (x_max - x_min), 0.5 * (y_max - y_min)))
    boxes = geo["xy_bboxes"]
    ij_bboxes = np.full_like(boxes, -1, dtype=np.int64)
    bb["compute_ij_bboxes"](lon, lat, boxes, xy_border, 1, ij_bboxes)
    xy = _ValuesView(np.stack([lon, lat]))
    ij = np.full((2, H, W), np.nan)
    k = 0
    tiles = [(r0, min(H, r0 + th), c0, min(W, c0 + tw)) for r0 in range(0, H, th)
             for c0 in range(0, W, tw)]
    for (r0, r1, c0, c1) in tiles:
        blk = ref["_compute_target_source_ij_block"](
            np.float64, k, (2, r1 - r0, c1 - c0), ((0, 2), (r0, r1), (c0, c1)), xy, ij_bboxes,
            x_min, y_min, y_max, x_res, y_res, j_up, 1e-3)
        ij[:, r0:r1, c0:c1] = blk
        k += 1
    outs = {}
    fill = np.nan if np.issubdtype(dtype, np.floating) else 255
    for interp in ("nearest", "bilinear", "triangular"):
        res_ = np.empty((nvar, H, W), dtype=dtype)
        for (r0, r1, c0, c1) in tiles:
            blk = ref["_compute_var_image_block"](ij[:, r0:r1, c0:c1], _ValuesView(var), fill,
                                                  interp, (nvar, r1 - r0, c1 - c0))
            res_[:, r0:r1, c0:c1] = blk
        outs[f"out_{interp}"] = res_
    np.savez_compressed(os.path.join(HERE, f"rectify_{name}.npz"), lon=lon, lat=lat, var=var,
                        size=np.array(size), xy_min=np.array(xy_min, float),
                        res=np.array(res, float), tile=np.array(tile), j_up=j_up, fill=fill,
                        xy_border=xy_border, ij_bboxes=ij_bboxes, ij=ij, **outs)
    print(f"rectify_{name}: src {h}x{w} -> {size} tiles {tile}, "
          f"{int(np.sum(~np.isnan(ij[0])))} px with a source")


def main():
    rng = np.random.default_rng(SEED)
    # 1) float32 (n=2), lon/lat 4326 source, 3857 target with partial edge tiles
    h, w = 48, 64
    x_res, y_res = 0.25, 0.2
    lon = -8.0 + (np.arange(w) + 0.5) * x_res
    lat = 60.0 - (np.arange(h) + 0.5) * y_res
    data = rng.random((2, h, w), dtype=np.float32)
    data[0, 5, 7] = np.nan
    data[1, 20, 33] = np.nan
    reproject_case("f32", data, lon, lat, x_res, y_res, (40, 36), (-1000000.0, 6200000.0),
                   (24000, 31000), (16, 16), ["nearest", "bilinear", "triangular"], np.nan)
    # 2) uint8 nearest + int16 bilinear/triangular: integer semantics (wrapping diffs)
    d8 = rng.integers(0, 256, (1, h, w), dtype=np.uint8)
    reproject_case("u8", d8, lon, lat, x_res, y_res, (33, 29), (-900000.0, 6300000.0),
                   (26000, 30000), (12, 10), ["nearest", "bilinear", "triangular"], 255)
    d16 = rng.integers(-3000, 3000, (1, h, w), dtype=np.int16)
    reproject_case("i16", d16, lon, lat, x_res, y_res, (33, 29), (-900000.0, 6300000.0),
                   (26000, 30000), (12, 10), ["nearest", "bilinear", "triangular"], -1)
    # 3) target extends beyond the source (constant padding, fill everywhere outside)
    d = rng.random((1, h, w), dtype=np.float32)
    reproject_case("pad", d, lon, lat, x_res, y_res, (50, 40), (-1400000.0, 5600000.0),
                   (25000, 40000), (25, 20), ["nearest", "bilinear", "triangular"], np.nan)
    # rectify: OLCI-like jittered swath, tiled target, finer/coarser targets
    rectify_case("f32", rng, 24, 30, (40, 30), (5.0, 59.1), 0.03, (16, 12), 2, np.float32)
    rectify_case("fine", rng, 12, 14, (50, 44), (5.05, 59.5), 0.012, (20, 20), 1, np.float64)
    rectify_case("u8_jup", rng, 20, 22, (30, 26), (5.0, 59.3), 0.03, (11, 9), 1, np.uint8,
                 j_up=True)
    rectify_case("nan", rng, 22, 26, (36, 28), (5.0, 59.2), 0.03, (13, 15), 1, np.float32,
                 nan_px=6)


if __name__ == "__main__":
    main()

"""Irregular (2-D coordinates) -> regular grid (reference: rectify.py).

Host side restates ``rectify_dataset`` (rectify.py:54-179),
``_transform_coords`` (182-231), ``_downscale_source_dataset`` (234-260),
``_rectify_data_array`` (263-309) and the tiling math of
``_compute_target_source_ij`` (312-370, incl. the empirical ``xy_border``)
and ``_compute_target_source_ij_block`` (373-419: per-tile source window and
target offsets).  The pixel work runs on the device:

* K4 ``xrs_ij_bboxes``   per target tile, the source pixel bbox (numba
                         compute_ij_bboxes, gridmapping/bboxes.py:28-106);
* K5 ``xrs_rectify_ij``  per target pixel, the fractional source (i, j) of the
                         first source quad that covers it (numba kernels,
                         rectify.py:424-576) — computed once, shared by all
                         variables, and kept in HBM;
* K6 ``xrs_rectify_var`` per variable, sampling at those positions
                         (rectify.py:605-734).
"""

from __future__ import annotations

from collections.abc import Iterable

import numpy as np

from . import kernels, multidevice
from .affine import resample_dataset
from .constants import SCALE_LIMIT, UV_DELTA
from .crs import Transformer
from .dataset import DataArray, Dataset
from .device import is_device_array, require_device, to_device
from . import streaming
from .options import get_options
from .streaming import device_to_host, host_to_device
from .gridmapping import GridMapping
from .gridmapping.helpers import chunk_sizes
from .utils import (
    _get_fill_value,
    _get_interp_method_str,
    _is_equal_crs,
    _prep_interp_methods_downscale,
    _select_variables,
    as_dataset,
    normalize_grid_mapping,
)


def rectify_dataset(source_ds, target_gm: GridMapping | None = None,
                    source_gm: GridMapping | None = None,
                    variables: str | Iterable[str] | None = None, interp_methods=None,
                    agg_methods=None, recover_nans=False, fill_values=None,
                    tile_size=None, devices=None) -> Dataset:
    """Rectify a dataset with 2-D coordinates onto a regular grid
    (rectify.py:54-179; same arguments, defaults and errors).
    ``devices`` (engine extension): split the target tiles over these GPUs
    (``multidevice``; default: the ``devices`` option, else the current
    device)."""
    with multidevice.use_devices(devices):
        return _rectify_dataset(source_ds, target_gm, source_gm, variables, interp_methods,
                                agg_methods, recover_nans, fill_values, tile_size)


def _rectify_dataset(source_ds, target_gm, source_gm, variables, interp_methods, agg_methods,
                     recover_nans, fill_values, tile_size) -> Dataset:
    source_ds = as_dataset(source_ds)
    if source_gm is None:
        source_gm = GridMapping.from_dataset(source_ds)
    source_ds = normalize_grid_mapping(source_ds, source_gm)
    if target_gm is None:
        target_gm = source_gm.to_regular(tile_size=tile_size)
    if not _is_equal_crs(source_gm, target_gm):
        source_ds = _transform_coords(source_ds, source_gm, target_gm)
        source_gm = GridMapping.from_dataset(source_ds)
    source_ds = _select_variables(source_ds, variables)
    source_ds, source_gm = _downscale_source_dataset(
        source_ds, source_gm, target_gm, interp_methods, agg_methods, recover_nans)

    yx_dims = (source_gm.xy_dim_names[1], source_gm.xy_dim_names[0])
    rect_vars = [k for k, v in source_ds.data_vars.items() if v.dims[-2:] == yx_dims]
    # K6 of the first device-resident variable runs inside K5's resolve pass
    # (xrs_rectify_ij_var); the ij image is kept only for the others.  With
    # 3 target rows per resolve item the fused pass is quicker for every
    # interpolation (config 4: nearest 1.30 vs 1.41 ms, bilinear 1.42 vs
    # 1.45 ms; with 4 rows the bilinear taps cost a wave per SIMD and fusing
    # it was slower, 1.50 vs 1.47 ms)
    devices = multidevice.active_devices()
    parted, fused = {}, None
    if devices is not None:   # every variable over the device list (multidevice)
        parted = _rectify_partitioned(source_ds, source_gm, target_gm, rect_vars,
                                      interp_methods, fill_values, devices)
    else:
        fused = next((k for k in rect_vars if len(source_ds[k].dims) in (2, 3)
                      and not _streams(source_ds[k].data)), None)
        if fused is not None:
            da = source_ds[fused]
            src = _var_device(da.data)
            target_source_ij, out = _compute_target_source_ij(
                source_gm, target_gm, UV_DELTA, var=(
                    src, _get_interp_method_str(interp_methods, fused, da),
                    _get_fill_value(fill_values, fused, da), len(rect_vars) > 1))
            fused_da = _rectified_array(da, target_gm, out)
        else:
            target_source_ij = _compute_target_source_ij(source_gm, target_gm, UV_DELTA)

    x_name, y_name = source_gm.xy_var_names
    coords = {k: v for k, v in source_ds.coords.items() if k not in (x_name, y_name)}
    tx_name, ty_name = target_gm.xy_var_names
    target_coords = target_gm.to_coords()
    coords[tx_name] = target_coords[tx_name]
    coords[ty_name] = target_coords[ty_name]
    coords["spatial_ref"] = DataArray(np.array(0), (), target_gm.crs.to_cf())
    target_ds = Dataset(coords=coords, attrs=source_ds.attrs)

    for var_name, data_array in source_ds.data_vars.items():
        if data_array.dims[-2:] == yx_dims:
            assert len(data_array.dims) in (2, 3), \
                f"Data variable {var_name} has {len(data_array.dims)} dimensions."
            if var_name == fused:
                target_ds[var_name] = fused_da
                continue
            if var_name in parted:
                target_ds[var_name] = parted[var_name]
                continue
            target_ds[var_name] = _rectify_data_array(
                data_array, var_name, target_gm, target_source_ij, interp_methods, fill_values)
        elif yx_dims[0] not in data_array.dims and yx_dims[1] not in data_array.dims:
            target_ds[var_name] = data_array
    return target_ds


def _transform_coords(source_ds: Dataset, source_gm: GridMapping,
                      target_gm: GridMapping) -> Dataset:
    """rectify.py:182-231 — 2-D source coordinates into the target CRS, per
    point on the device (xrs_transform); the host keeps a copy for the
    GridMapping analysis of the transformed coordinates."""
    tr = Transformer.from_crs(source_gm.crs, target_gm.crs, always_xy=True)
    sx, sy = source_gm.x_coords.values, source_gm.y_coords.values
    if tr.is_identity:
        xx, yy = tr.transform(sx, sy)
    else:
        shape = np.shape(sx)
        xd, yd = kernels.transform(tr, np.reshape(sx, (1, -1)), np.reshape(sy, (1, -1)), False,
                                   require_device())
        xx, yy = device_to_host(xd).reshape(shape), device_to_host(yd).reshape(shape)
    source_ds = source_ds.drop_vars(source_gm.xy_var_names)
    yx_dims = (source_gm.xy_dim_names[1], source_gm.xy_dim_names[0])
    names = ("lon", "lat") if target_gm.crs.is_geographic else ("transformed_x", "transformed_y")
    return source_ds.assign_coords({
        "spatial_ref": DataArray(np.array(0), (), target_gm.crs.to_cf()),
        names[0]: DataArray(xx, yx_dims),
        names[1]: DataArray(yy, yx_dims),
    })


def _downscale_source_dataset(source_ds, source_gm: GridMapping, target_gm: GridMapping,
                              interp_methods, agg_methods, recover_nans):
    """rectify.py:234-260."""
    x_scale = source_gm.x_res / target_gm.x_res
    y_scale = source_gm.y_res / target_gm.y_res
    if x_scale < SCALE_LIMIT or y_scale < SCALE_LIMIT:
        w, h = round(x_scale * source_gm.width), round(y_scale * source_gm.height)
        downscaled_size = (w if w >= 2 else 2, h if h >= 2 else 2)
        source_ds = resample_dataset(
            source_ds, ((1 / x_scale, 0, 0), (0, 1 / y_scale, 0)),
            (source_gm.xy_dim_names[1], source_gm.xy_dim_names[0]), downscaled_size,
            source_gm.tile_size, _prep_interp_methods_downscale(interp_methods), agg_methods,
            recover_nans)
        source_gm = GridMapping.from_dataset(source_ds)
    return source_ds, source_gm


def rectify_tiles(source_gm: GridMapping, target_gm: GridMapping, uv_delta: float = UV_DELTA,
                  xy=None):
    """Host tiling of rectify.py:312-419: xy_border, per-tile source bboxes
    (K4), per-tile source windows and target offsets (TILE_INFO records).
    ``xy``: the source coordinates already on the device (x, y), else they are
    taken from ``source_gm``."""
    dst_w, dst_h = target_gm.width, target_gm.height
    tw, th = target_gm.tile_width, target_gm.tile_height
    dst_x_min, dst_y_min, dst_x_max, dst_y_max = target_gm.xy_bbox
    dst_x_res, dst_y_res = target_gm.xy_res
    j_up = target_gm.is_j_axis_up
    num_tiles_x = dst_w / tw
    num_tiles_y = dst_h / th
    xy_border = min(min(2 * num_tiles_x * target_gm.x_res, 2 * num_tiles_y * target_gm.y_res),
                    min(0.5 * (dst_x_max - dst_x_min), 0.5 * (dst_y_max - dst_y_min)))
    ys = chunk_sizes(dst_h, th)
    xs = chunk_sizes(dst_w, tw)
    if xy is None:
        src_ij_bboxes = source_gm.ij_bboxes_from_xy_bboxes(
            target_gm.xy_bboxes, xy_border=xy_border, ij_border=1, grid=(len(xs), len(ys)))
    else:  # base.py:565-629 on coordinates already resident in HBM
        src_ij_bboxes = kernels.ij_bboxes(xy[0], xy[1], target_gm.xy_bboxes, xy_border, 1,
                                          grid=(len(xs), len(ys)))
    tiles = tile_records(target_gm, src_ij_bboxes, source_gm.width, source_gm.height)
    return tiles, len(xs), src_ij_bboxes, xy_border


def tile_records(target_gm: GridMapping, src_ij_bboxes, src_w: int, src_h: int) -> np.ndarray:
    """TILE_INFO records (kernels.py) of the target tiles from their source ij
    bboxes (rectify.py:391-418; host arithmetic only)."""
    dst_w, dst_h = target_gm.width, target_gm.height
    tw, th = target_gm.tile_width, target_gm.tile_height
    dst_x_min, dst_y_min, dst_x_max, dst_y_max = target_gm.xy_bbox
    dst_x_res, dst_y_res = target_gm.xy_res
    j_up = target_gm.is_j_axis_up
    ys = chunk_sizes(dst_h, th)
    xs = chunk_sizes(dst_w, tw)
    src_ij_bboxes = np.asarray(src_ij_bboxes)
    tiles = np.zeros(len(ys) * len(xs), dtype=kernels.TILE_INFO_DTYPE)
    r0s = np.repeat(np.concatenate([[0], np.cumsum(ys)[:-1]]), len(xs))
    c0s = np.tile(np.concatenate([[0], np.cumsum(xs)[:-1]]), len(ys))
    tiles["r0"], tiles["c0"] = r0s, c0s
    tiles["th"], tiles["tw"] = np.repeat(ys, len(xs)), np.tile(xs, len(ys))
    i_min, j_min, i_max, j_max = (src_ij_bboxes[:, k] for k in range(4))
    none = i_min == -1
    tiles["si0"] = np.where(none, -1, i_min)
    tiles["sj0"] = np.where(none, -1, j_min)
    tiles["swin"] = np.where(none, 0, np.minimum(i_max + 1, src_w) - i_min)
    tiles["shin"] = np.where(none, 0, np.minimum(j_max + 1, src_h) - j_min)
    # rectify.py:402-406 (python float arithmetic, element by element)
    tiles["x_off"] = [dst_x_min + int(c0) * dst_x_res for c0 in c0s]
    tiles["y_off"] = [(dst_y_min + int(r0) * dst_y_res) if j_up else (dst_y_max - int(r0) * dst_y_res)
                      for r0 in r0s]
    return tiles


def rectify_tile_run(source_gm: GridMapping, target_gm: GridMapping, src, shard, interp: str,
                     fill, tiles=None, uv_delta: float = UV_DELTA):
    """One rank's share of a rectification split by ``sharding.rectify_shard``
    (coordinates and the variable `src` (n, H, W) replicated on every rank):
    K5 on the rank's run of target tiles, K6 on the target rows they cover.
    Returns the (n, row1 - row0, W') device band; pixels of tiles the rank
    does not own are `fill` (``sharding.merge_tile_runs`` assembles the
    ranks' bands)."""
    device = require_device(getattr(src, "device", None))
    xy = source_gm.xy_coords.data
    xy = (host_to_device(xy[0], device, np.float64), host_to_device(xy[1], device, np.float64))
    if tiles is None:
        tiles, _, _, _ = rectify_tiles(source_gm, target_gm, uv_delta, xy=xy)
    ntx = len(chunk_sizes(target_gm.width, target_gm.tile_width))
    dst_y_scale = target_gm.y_res if target_gm.is_j_axis_up else -target_gm.y_res
    run = tiles[shard.tile0:shard.tile1]
    ij = kernels.rectify_ij(xy[0], xy[1], run, ntx, target_gm.height, target_gm.width,
                            target_gm.x_res, dst_y_scale, uv_delta, init_nan=True)
    return kernels.rectify_var(ij, src, interp, fill, rows=shard.rows)


def _rectify_partitioned(source_ds, source_gm: GridMapping, target_gm: GridMapping, rect_vars,
                         interp_methods, fill_values, devices) -> dict:
    """K5 + K6 over several devices (``multidevice``): the target tiles are
    dealt as contiguous cost-balanced runs (``sharding.rectify_shard``); each
    device gets the source coordinates and the variables (a tile's source
    window can lie anywhere), runs K5 on its tiles and K6 on the target rows
    they cover, and its tiles' pixels are copied into the variable's output.
    Tiles are independent (rectify.py:347-370), so the result is the
    single-device one bit for bit.  Returns {name: DataArray}."""
    from .sharding import rectify_shard

    dev0 = require_device()
    xy = source_gm.xy_coords.data
    xy0 = (host_to_device(xy[0], dev0, np.float64), host_to_device(xy[1], dev0, np.float64))
    tiles, ntx, _, _ = rectify_tiles(source_gm, target_gm, UV_DELTA, xy=xy0)
    world = len(devices)
    shards = [rectify_shard(tiles, world, i) for i in range(world)]
    dst_y_scale = target_gm.y_res if target_gm.is_j_axis_up else -target_gm.y_res

    def part_ij(i, dev):
        sh = shards[i]
        if sh.tile1 <= sh.tile0:
            return None
        x, y = (c if c.device == dev else c.to(dev) for c in xy0)
        return kernels.rectify_ij(x, y, tiles[sh.tile0:sh.tile1], ntx, target_gm.height,
                                  target_gm.width, target_gm.x_res, dst_y_scale, UV_DELTA,
                                  init_nan=True)

    ijs = multidevice.run_parts(devices, part_ij, sources=list(xy0))
    out = {}
    for name in rect_vars:
        da = source_ds[name]
        if len(da.dims) not in (2, 3):
            continue
        interp = _get_interp_method_str(interp_methods, name, da)
        fill = _get_fill_value(fill_values, name, da)
        data = da.data
        on_device = is_device_array(data)
        arr = data if on_device else np.asarray(data)
        if arr.ndim == 2:
            arr = arr.unsqueeze(0) if on_device else arr.reshape((1,) + arr.shape)
        res = multidevice.output_like(arr, (arr.shape[0], target_gm.height, target_gm.width),
                                      da.dtype)

        def part_var(i, dev, arr=arr, res=res, interp=interp, fill=fill):
            sh = shards[i]
            if ijs[i] is None:
                return
            src = multidevice.rows_to_device(arr, 0, arr.shape[1], dev)
            band = kernels.rectify_var(ijs[i], src, interp, fill, rows=sh.rows)
            multidevice.put_tiles(res, band, tiles[sh.tile0:sh.tile1], sh.row0)

        multidevice.run_parts(devices, part_var, sources=[arr])
        out[name] = _rectified_array(da, target_gm, res)
    return out


def _compute_target_source_ij(source_gm: GridMapping, target_gm: GridMapping,
                              uv_delta: float, var=None):
    """rectify.py:312-370 -> device tensor (2, H', W') float64 (K5).  The
    source coordinates are uploaded once and shared by K4 and K5.  With
    ``var=(src, interp, fill, keep_ij)`` the variable is sampled by K5's
    resolve pass: returns (ij or None, the (n, H', W') rectified variable)."""
    device = require_device()
    xy = source_gm.xy_coords.data
    xy = (host_to_device(xy[0], device, np.float64), host_to_device(xy[1], device, np.float64))
    dst_y_scale = target_gm.y_res if target_gm.is_j_axis_up else -target_gm.y_res
    tiles = _device_tiles(source_gm, target_gm, xy)
    if tiles is None:   # boxes not a regular tile grid: host tiling
        tiles, ntx, _, _ = rectify_tiles(source_gm, target_gm, uv_delta, xy=xy)
    else:
        ntx = len(chunk_sizes(target_gm.width, target_gm.tile_width))
    if var is not None:
        src, interp, fill, keep_ij = var
        return kernels.rectify_ij_var(xy[0], xy[1], tiles, target_gm.height, target_gm.width,
                                      target_gm.x_res, dst_y_scale, uv_delta, src, interp, fill,
                                      keep_ij=keep_ij)
    return kernels.rectify_ij(xy[0], xy[1], tiles, ntx, target_gm.height, target_gm.width,
                              target_gm.x_res, dst_y_scale, uv_delta)


def _device_tiles(source_gm: GridMapping, target_gm: GridMapping, xy):
    """rectify_tiles with K4's accumulators turned into tile records and chunk
    offsets on the device (xrs_rectify_tiles): no host synchronisation
    between K4 and K5."""
    dst_w, dst_h = target_gm.width, target_gm.height
    tw, th = target_gm.tile_width, target_gm.tile_height
    dst_x_min, dst_y_min, dst_x_max, dst_y_max = target_gm.xy_bbox
    xy_border = min(min(2 * (dst_w / tw) * target_gm.x_res, 2 * (dst_h / th) * target_gm.y_res),
                    min(0.5 * (dst_x_max - dst_x_min), 0.5 * (dst_y_max - dst_y_min)))
    grid = (len(chunk_sizes(dst_w, tw)), len(chunk_sizes(dst_h, th)))
    return kernels.rectify_tiles_device(
        xy[0], xy[1], target_gm.xy_bboxes, xy_border, 1, grid, (tw, th), (dst_w, dst_h),
        (dst_x_min, dst_y_min, dst_y_max), target_gm.xy_res, target_gm.is_j_axis_up)


def _streams(data) -> bool:
    """A numpy variable large enough for the host band pipeline."""
    return isinstance(data, np.ndarray) and data.ndim in (2, 3) and \
        data.nbytes >= get_options()["host_streaming_min_bytes"]


def _var_device(data):
    """The variable as a (n, H, W) device tensor."""
    src = host_to_device(data, require_device())
    return src.unsqueeze(0) if src.dim() == 2 else src


def _rectify_data_array(data_array: DataArray, var_name, target_gm: GridMapping,
                        target_source_ij, interp_methods, fill_values) -> DataArray:
    """rectify.py:263-309 (K6, one launch for all dim-0 slices)."""
    fill_value = _get_fill_value(fill_values, var_name, data_array)
    interp_method = _get_interp_method_str(interp_methods, var_name, data_array)
    data = data_array.data
    if _streams(data):
        # numpy in, numpy out (rectify.py:297-298): band pipeline
        arr = data.reshape((1,) + data.shape) if data.ndim == 2 else data
        out = streaming.rectify_host(arr, target_source_ij, interp_method, fill_value,
                                     require_device())
    else:
        out = kernels.rectify_var(target_source_ij, _var_device(data), interp_method,
                                  fill_value)
    return _rectified_array(data_array, target_gm, out)


def _rectified_array(data_array: DataArray, target_gm: GridMapping, out) -> DataArray:
    """The (n, H', W') K6 result as the target variable (rectify.py:297-309):
    numpy in, numpy out; device arrays stay on the device."""
    data = data_array.data
    result = device_to_host(out) if is_device_array(out) and not is_device_array(data) else out
    if data.ndim == 2:
        result = result[0]
        dims = (target_gm.xy_dim_names[1], target_gm.xy_dim_names[0])
    else:
        dims = (data_array.dims[0], target_gm.xy_dim_names[1], target_gm.xy_dim_names[0])
    return DataArray(result, dims, data_array.attrs)

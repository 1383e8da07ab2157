"""Regular -> regular reprojection across CRSs (reference: reproject.py).

Host side (this module) restates the reference's orchestration and tiling math
— ``reproject_dataset`` (reproject.py:51-186), ``_reproject_data_array``
(189-265), ``_downscale_source_dataset`` (338-382),
``_get_scr_bboxes_indices`` (385-469) and ``_transform_gridpoints``
(472-496) — and hands ALL target tiles of a variable to one launch of the K1
HIP kernel (``xrs_reproject``), which replaces ``_reproject_block``
(268-335) and the pad/copy of ``_reorganize_data_array_slice`` (499-530).

Device data layout: the source variable lives in HBM as one contiguous
(n, H, W) array (never reorganised into per-tile windows); the target is one
(n, H', W') array.  The per-tile window geometry is a few small tables; the
target pixel coordinates in the source CRS are two 1-D float64 tables
(separable CRS pairs, e.g. EPSG:3857 -> EPSG:4326) instead of the reference's
two materialised (H', W') float64 grids.
"""

from __future__ import annotations

import math
from collections.abc import Iterable
from dataclasses import dataclass, field

import numpy as np

from . import kernels, multidevice, streaming
from .constants import SCALE_LIMIT
from .crs import Transformer
from .dataset import DataArray, Dataset
from .device import is_device_array, require_device, to_device, torch
from .gridmapping import GridMapping
from .options import get_options
from .utils import (
    _get_fill_value,
    _get_interp_method_str,
    _prep_interp_methods_downscale,
    _select_variables,
    as_dataset,
    clip_dataset_by_bbox,
    normalize_grid_mapping,
)


@dataclass
class ReprojectPlan:
    """Host-computed tiling geometry of one (source_gm, target_gm) pair."""

    src_width: int
    src_height: int
    dst_width: int
    dst_height: int
    tile_width: int
    tile_height: int
    x_res: float
    y_res: float
    coord_mode: int              # 0: separable tables, 1: 2-D tables
    src_x: np.ndarray | None     # (W',) or (H', W') float64, target pixel x in source CRS
    src_y: np.ndarray | None     # (H',) or (H', W') float64 (None: 2-D tables made on device)
    tile_x0: np.ndarray          # (ntiles,) float32, window x origin (reproject.py:427-453)
    tile_y0: np.ndarray          # (ntiles,) float32
    tile_win: np.ndarray         # (ntiles, 2) int64, window (i0, j0) in unpadded source indices
    win_width: int
    win_height: int
    scr_ij_bboxes: np.ndarray    # (4, nty, ntx) int32, as returned by the reference (padded)
    pad_width: tuple
    # 2-D plans without host tables: the target grid's pixel-centre axes and the
    # target -> source transformer, evaluated per pixel on the device
    grid_x: np.ndarray | None = None
    grid_y: np.ndarray | None = None
    transformer: Transformer | None = None
    # 2-D plans: evaluate the transformation inside the gather
    # (xrs_reproject_proj) instead of through coordinate tables; also chosen
    # when the tables would exceed the ``reproject_table_max_bytes`` option
    fuse_transform: bool = False
    # separable plans whose src_x the target grid's column generators
    # reproduce bit for bit (``column_generators``): K1 computes the column
    # coordinates instead of reading them (xrs_reproject coord_mode 2)
    x_gen: np.ndarray | None = None
    _device_cache: dict = field(default_factory=dict, repr=False)

    @property
    def num_tiles(self) -> tuple[int, int]:
        return self.scr_ij_bboxes.shape[2], self.scr_ij_bboxes.shape[1]

    def _tile_tables(self, device) -> dict:
        key = ("tiles", str(device))
        tabs = self._device_cache.get(key)
        if tabs is None:
            tabs = dict(
                tile_x0=to_device(self.tile_x0.astype(np.float32), device),
                tile_y0=to_device(self.tile_y0.astype(np.float32), device),
                tile_win=to_device(np.ascontiguousarray(self.tile_win, np.int64), device),
            )
            self._device_cache[key] = tabs
        return tabs

    def device_tables(self, device) -> dict:
        key = str(device)
        tabs = self._device_cache.get(key)
        if tabs is None:
            if self.src_x is None:   # target pixel centres -> source CRS on the device
                from . import kernels
                sx, sy = kernels.transform(self.transformer, self.grid_x, self.grid_y, True,
                                           device)
            else:
                sx = to_device(np.ascontiguousarray(self.src_x, np.float64), device)
                sy = to_device(np.ascontiguousarray(self.src_y, np.float64), device)
            tabs = dict(src_x=sx, src_y=sy, **self._tile_tables(device))
            if self.x_gen is not None and self.coord_mode == 0:
                tabs["x_gen"] = to_device(np.ascontiguousarray(self.x_gen, np.float64), device)
            self._device_cache[key] = tabs
        return tabs

    def fused_transform(self, device) -> bool:
        """True when the next K1 call evaluates the transformation per pixel:
        a 2-D plan without coordinate tables on `device` whose tables would
        exceed ``reproject_table_max_bytes`` (or ``fuse_transform`` set)."""
        if self.coord_mode != 1 or self.src_x is not None or str(device) in self._device_cache:
            return False
        table_bytes = 16 * self.dst_width * self.dst_height
        return self.fuse_transform or table_bytes > get_options()["reproject_table_max_bytes"]

    def device_grid(self, device) -> dict:
        """The target grid's pixel-centre axes + tile tables on `device`
        (xrs_reproject_proj's inputs)."""
        key = ("grid", str(device))
        tabs = self._device_cache.get(key)
        if tabs is None:
            tabs = dict(grid_x=to_device(np.ascontiguousarray(self.grid_x, np.float64), device),
                        grid_y=to_device(np.ascontiguousarray(self.grid_y, np.float64), device),
                        **self._tile_tables(device))
            self._device_cache[key] = tabs
        return tabs

    def host_coords(self) -> tuple[np.ndarray, np.ndarray]:
        """The coordinate tables on the host (2-D plans: the numpy
        restatement of the transformation, reproject.py:472-496)."""
        if self.src_x is not None:
            return self.src_x, self.src_y
        xx, yy = np.meshgrid(self.grid_x, self.grid_y)
        return self.transformer.transform(xx, yy)

    def workspace(self, device, nbytes: int):
        """Device scratch for the axis tables (reused across calls; stream-ordered)."""
        if nbytes <= 0:
            return None
        key = ("ws", str(device))
        ws = self._device_cache.get(key)
        if ws is None or ws.numel() < nbytes:
            ws = torch().empty(nbytes, dtype=torch().uint8, device=device)
            self._device_cache[key] = ws
        return ws

    def _row_read_grid(self):
        """(H', ntiles_x) int64 arrays (lo, hi) of the global source rows the
        floor / ceil taps of each target row read in each tile column
        (reproject.py:279, 286-291, 316-321: int16 window index with
        python-style wrap, window origin, rows outside the source read the
        pad and are not counted); lo > hi where nothing is read."""
        cache = self._device_cache.get("row_read_grid")
        if cache is not None:
            return cache
        ntx, _ = self.num_tiles
        rows = np.arange(self.dst_height)
        ty = rows // self.tile_height
        lo = np.full((self.dst_height, ntx), np.iinfo(np.int64).max, np.int64)
        hi = np.full((self.dst_height, ntx), -1, np.int64)
        for tx in range(ntx):
            t = ty * ntx + tx
            iy = (self.src_y[rows] - self.tile_y0[t].astype(np.float64)) / -self.y_res
            for f in (np.floor, np.ceil):
                with np.errstate(invalid="ignore"):
                    w = f(iy).astype(np.int16).astype(np.int64)
                w = np.where(w < 0, w + self.win_height, w)
                g = self.tile_win[t, 1] + w
                ok = (w >= 0) & (w < self.win_height) & (g >= 0) & (g < self.src_height)
                lo[:, tx] = np.where(ok, np.minimum(lo[:, tx], g), lo[:, tx])
                hi[:, tx] = np.where(ok, np.maximum(hi[:, tx], g), hi[:, tx])
        self._device_cache["row_read_grid"] = (lo, hi)
        return lo, hi

    def row_source_extent(self) -> tuple[np.ndarray, np.ndarray]:
        """Per target row: the lowest and highest global source row read
        (lo > hi: none).  Separable plans only."""
        if self.coord_mode != 0:
            raise NotImplementedError("row extents need separable coordinate tables")
        lo, hi = self._row_read_grid()
        return lo.min(axis=1), hi.max(axis=1)

    def source_cols_read(self) -> int:
        """Number of distinct source columns any target pixel reads (separable
        plans; bilinear floor + ceil taps)."""
        ntx, nty = self.num_tiles
        cols = np.zeros(self.src_width, bool)
        for t in range(ntx * nty):
            tx = t % ntx
            c = np.arange(tx * self.tile_width, min(self.dst_width, (tx + 1) * self.tile_width))
            ix = (self.src_x[c] - self.tile_x0[t].astype(np.float64)) / self.x_res
            for f in (np.floor, np.ceil):
                with np.errstate(invalid="ignore"):
                    w = f(ix).astype(np.int16).astype(np.int64)
                w = np.where(w < 0, w + self.win_width, w)
                g = self.tile_win[t, 0] + w
                ok = (w >= 0) & (w < self.win_width) & (g >= 0) & (g < self.src_width)
                cols[g[ok]] = True
        return int(cols.sum())

    def source_rows_read(self, r0: int, r1: int) -> tuple[int, int]:
        """Global source rows [j0, j1) that K1 reads for target rows [r0, r1)
        — exactly (separable plans) or the union of the tile windows
        (2-D coordinate plans)."""
        if self.coord_mode != 0:
            return self.source_rows_for(r0, r1)
        lo, hi = self.row_source_extent()
        lo, hi = lo[r0:r1], hi[r0:r1]
        ok = hi >= lo
        if not ok.any():
            return 0, 0
        return int(lo[ok].min()), int(hi[ok].max()) + 1

    def source_rows_for(self, r0: int, r1: int) -> tuple[int, int]:
        """Global source rows [j0, j1) read by target rows [r0, r1) (clipped)."""
        tys = range(r0 // self.tile_height, (max(r1, r0 + 1) - 1) // self.tile_height + 1)
        ntx = self.num_tiles[0]
        t = np.array([ty * ntx + tx for ty in tys for tx in range(ntx)], dtype=np.int64)
        j0 = int(self.tile_win[t, 1].min())
        j1 = int(self.tile_win[t, 1].max()) + self.win_height
        return max(0, j0), min(self.src_height, max(0, j1))


def plan_reproject(source_gm: GridMapping, target_gm: GridMapping,
                   transformer: Transformer) -> ReprojectPlan:
    """Restates reproject.py:385-469 and 472-496."""
    num_tiles_x = math.ceil(target_gm.width / target_gm.tile_width)
    num_tiles_y = math.ceil(target_gm.height / target_gm.tile_height)

    origin = source_gm.x_coords.values[0], source_gm.y_coords.values[0]
    bboxes = np.full((4, num_tiles_y, num_tiles_x), -1, dtype=np.int32)
    # all tiles' source bounds in one vectorised transform_bounds (the same
    # values as tile by tile); a tile whose bounds are not finite takes the
    # per-tile loop, which raises as the reference's math.floor does
    sbs = transformer.transform_bounds_many(np.asarray(target_gm.xy_bboxes, dtype=np.float64))
    edges = None
    if np.isfinite(sbs).all():
        sb0, sb1, sb2, sb3 = sbs.T
        edges = np.stack([
            np.floor((sb0 - origin[0]) / source_gm.x_res),
            np.floor((origin[1] - sb3) / source_gm.y_res),
            np.ceil((sb2 - origin[0]) / source_gm.x_res),
            np.ceil((origin[1] - sb1) / source_gm.y_res),
        ]).reshape(4, num_tiles_y, num_tiles_x)
        if (np.abs(edges) > np.iinfo(np.int32).max).any():
            edges = None   # the per-tile assignment raises OverflowError
    if edges is not None:
        bboxes[:] = edges
    else:
        for idx, xy_bbox in enumerate(target_gm.xy_bboxes):
            j, i = np.unravel_index(idx, (num_tiles_y, num_tiles_x))
            sb = transformer.transform_bounds(*xy_bbox)
            bboxes[:, j, i] = [
                math.floor((sb[0] - origin[0]) / source_gm.x_res),
                math.floor((origin[1] - sb[3]) / source_gm.y_res),
                math.ceil((sb[2] - origin[0]) / source_gm.x_res),
                math.ceil((origin[1] - sb[1]) / source_gm.y_res),
            ]

    # uniform window size (reproject.py:405-423)
    i_diff = bboxes[2] - bboxes[0]
    j_diff = bboxes[3] - bboxes[1]
    i_diff_max = np.max(i_diff) + 1
    j_diff_max = np.max(j_diff) + 1
    i_start = bboxes[0] - (i_diff_max - i_diff) // 2
    j_start = bboxes[1] - (j_diff_max - j_diff) // 2
    bboxes = np.stack([i_start, j_start, i_start + i_diff_max, j_start + j_diff_max]).astype(np.int32)

    # window origins (reproject.py:427-450), float32 like the reference's x_coords
    i_min = np.min(bboxes[0])
    i_max = np.max(bboxes[2])
    j_min = np.min(bboxes[[1, 3]])
    j_max = np.max(bboxes[[1, 3]])
    x0 = source_gm.x_coords.values[0]
    x_coord = np.arange(x0 + i_min * source_gm.x_res, x0 + i_max * source_gm.x_res,
                        source_gm.x_res)
    yv = source_gm.y_coords.values
    y_res = yv[1] - yv[0]
    y_coord = np.arange(yv[0] + j_min * y_res, yv[0] + j_max * y_res, y_res)
    tile_x0 = x_coord[(bboxes[0] - i_min).ravel()].astype(np.float32)
    tile_y0 = y_coord[(bboxes[1] - j_min).ravel()].astype(np.float32)
    tile_win = np.stack([bboxes[0].ravel(), bboxes[1].ravel()], axis=1).astype(np.int64)

    pad_width = ((0, 0),
                 (-min(0, int(j_min)), max(0, int(j_max - source_gm.height))),
                 (-min(0, int(i_min)), max(0, int(i_max - source_gm.width))))
    scr_ij_bboxes = bboxes.copy()
    scr_ij_bboxes[[1, 3]] += pad_width[1][0]
    scr_ij_bboxes[[0, 2]] += pad_width[2][0]

    # target pixel centres in the source CRS (reproject.py:472-496)
    tx = target_gm.x_coords.values
    ty = target_gm.y_coords.values
    x_gen = None
    if transformer.is_separable:
        coord_mode = 0
        src_x = transformer.transform_x(tx)
        src_y = transformer.transform_y(ty)
        x_gen = column_generators(tx, target_gm.tile_width, src_x,
                                  transformer.separable_x_scales())
    else:   # evaluated per target pixel on the device (xrs_transform)
        coord_mode = 1
        src_x = src_y = None

    return ReprojectPlan(
        src_width=source_gm.width, src_height=source_gm.height,
        dst_width=target_gm.width, dst_height=target_gm.height,
        tile_width=target_gm.tile_width, tile_height=target_gm.tile_height,
        x_res=source_gm.x_res, y_res=source_gm.y_res, coord_mode=coord_mode,
        src_x=None if src_x is None else np.asarray(src_x, np.float64),
        src_y=None if src_y is None else np.asarray(src_y, np.float64),
        tile_x0=tile_x0, tile_y0=tile_y0, tile_win=tile_win,
        win_width=int(i_diff_max), win_height=int(j_diff_max),
        scr_ij_bboxes=scr_ij_bboxes, pad_width=pad_width,
        grid_x=None if coord_mode == 0 else np.asarray(tx, np.float64),
        grid_y=None if coord_mode == 0 else np.asarray(ty, np.float64),
        transformer=None if coord_mode == 0 else transformer,
        x_gen=x_gen,
    )


def column_generators(tx, tile_w: int, src_x, scales) -> np.ndarray | None:
    """xrs_reproject's coord_mode-2 records (include/xrs.h) for a separable
    plan, or None when they would not reproduce ``src_x`` bit for bit.

    A regular target grid's x coordinates are dask's blockwise linspace of
    the pixel centres, one block per tile column (regular.py:44-52 ->
    ``helpers.dask_linspace``): element k of a block of n is k * step + start,
    the last one stop.  The separable transformation then scales them
    (``Transformer.separable_x_scales``).  K1 can evaluate that itself from
    32 bytes per tile column instead of reading 8 bytes per column — but only
    the comparison below, on every column, licenses it."""
    if scales is None or tile_w < 1:
        return None
    tx = np.asarray(tx, np.float64)
    w = tx.size
    m1, m2 = (float(v) for v in scales)
    gen = np.empty(w, np.float64)
    recs = []
    for b0 in range(0, w, tile_w):
        n = min(tile_w, w - b0)
        start, stop = float(tx[b0]), float(tx[b0 + n - 1])
        step = (stop - start) / (n - 1) if n > 1 else 0.0
        v = np.arange(n, dtype=np.float64) * step + start
        v[-1] = stop
        gen[b0:b0 + n] = v
        recs.append((start, stop, step, float(n)))
    with np.errstate(all="ignore"):
        x = (gen * m1) * m2
    if not np.array_equal(x.view(np.uint64), np.ascontiguousarray(src_x, np.float64).view(np.uint64)):
        return None
    return np.concatenate([np.asarray(recs, np.float64).reshape(-1), [m1, m2]])


def reproject_dataset(source_ds, target_gm: GridMapping, source_gm: GridMapping | None = None,
                      variables: str | Iterable[str] | None = None, interp_methods=None,
                      agg_methods=None, recover_nans=False, fill_values=None,
                      devices=None) -> Dataset:
    """Reproject a dataset to the CRS and grid of ``target_gm``
    (reproject.py:51-186; same arguments, defaults and errors).
    ``devices`` (engine extension): split every variable's target row bands
    over these GPUs (``multidevice``; default: the ``devices`` option, else
    the current device)."""
    with multidevice.use_devices(devices):
        return _reproject_dataset(source_ds, target_gm, source_gm, variables, interp_methods,
                                  agg_methods, recover_nans, fill_values)


def _reproject_dataset(source_ds, target_gm, source_gm, variables, interp_methods, agg_methods,
                       recover_nans, fill_values) -> Dataset:
    source_ds = as_dataset(source_ds)
    if source_gm is None:
        source_gm = GridMapping.from_dataset(source_ds)
    if source_gm.is_j_axis_up:
        v_var = source_gm.xy_var_names[1]
        source_ds = source_ds.isel({v_var: slice(None, None, -1)})
        source_gm = GridMapping.from_dataset(source_ds)

    source_ds = normalize_grid_mapping(source_ds, source_gm)
    source_ds = _select_variables(source_ds, variables)
    transformer = Transformer.from_crs(target_gm.crs, source_gm.crs, always_xy=True)

    source_ds, source_gm = _downscale_source_dataset(
        source_ds, source_gm, target_gm, transformer, interp_methods, agg_methods, recover_nans)

    plan = plan_reproject(source_gm, target_gm, transformer)
    yx_dims = (source_gm.xy_dim_names[1], source_gm.xy_dim_names[0])
    n_vars = sum(1 for v in source_ds.data_vars.values() if v.dims[-2:] == yx_dims)
    if n_vars == 1 and plan.coord_mode == 1 and plan.src_x is None:
        # one variable over a non-separable pair: the transformation fused into
        # the gather (xrs_reproject_proj) beats tables made for one reader
        # (config 2u: 1.58 vs 1.63 ms of kernels; bit-identical results)
        import dataclasses

        plan = dataclasses.replace(plan, fuse_transform=True)

    x_name, y_name = source_gm.xy_var_names
    coords = {k: v for k, v in source_ds.coords.items() if k not in (x_name, y_name)}
    tx_name, ty_name = target_gm.xy_var_names
    coords[tx_name] = DataArray(target_gm.x_coords.values, target_gm.x_coords.dims)
    coords[ty_name] = DataArray(target_gm.y_coords.values, target_gm.y_coords.dims)
    coords["spatial_ref"] = DataArray(np.array(0), (), target_gm.crs.to_cf())
    target_ds = Dataset(coords=coords, attrs=source_ds.attrs)

    for var_name, data_array in source_ds.items():
        if data_array.dims[-2:] == yx_dims:
            assert len(data_array.dims) in (2, 3), \
                f"Data variable {var_name} has {len(data_array.dims)} dimensions."
            target_ds[var_name] = _reproject_data_array(
                data_array, var_name, target_gm, plan, interp_methods, fill_values)
        elif yx_dims[0] not in data_array.dims and yx_dims[1] not in data_array.dims:
            target_ds[var_name] = data_array
    return target_ds


def _reproject_data_array(data_array: DataArray, var_name, target_gm: GridMapping,
                          plan: ReprojectPlan, interp_methods, fill_values) -> DataArray:
    """reproject.py:189-265 — one kernel launch over all tiles and dim-0 slices."""
    fill_value = _get_fill_value(fill_values, var_name, data_array)
    interp_method = _get_interp_method_str(interp_methods, var_name, data_array)
    device = require_device()
    data = data_array.data
    on_device = is_device_array(data)
    out_dtype = None
    if interp_method == "bilinear" and get_options()["reproject_bilinear_dtype"] == "source":
        out_dtype = data_array.dtype if np.issubdtype(data_array.dtype, np.floating) else np.float64
    expanded = len(data_array.dims) == 2
    devices = multidevice.active_devices()
    if devices is not None:
        # the variable's target row bands over several devices (multidevice)
        src = data if on_device else np.asarray(data)
        src = src.unsqueeze(0) if (expanded and on_device) else \
            (src.reshape((1,) + src.shape) if expanded else src)
        result = _reproject_partitioned(src, plan, interp_method, fill_value, out_dtype, devices)
    elif not on_device and isinstance(data, np.ndarray) and \
            data.nbytes >= get_options()["host_streaming_min_bytes"]:
        # host array in, host array out (reproject.py:254-255): band pipeline
        src = data.reshape((1,) + data.shape) if expanded else data
        result = streaming.reproject_host(src, plan, interp_method, fill_value,
                                          out_dtype=out_dtype, device=device)
    else:
        src = to_device(data, device)
        if expanded:
            src = src.unsqueeze(0)
        out = kernels.reproject(src, plan, interp_method, fill_value, out_dtype=out_dtype)
        result = out if on_device else out.cpu().numpy()
    if expanded:
        result = result[0]
        dims = (target_gm.xy_dim_names[1], target_gm.xy_dim_names[0])
    else:
        dims = (data_array.dims[0], target_gm.xy_dim_names[1], target_gm.xy_dim_names[0])
    return DataArray(result, dims, data_array.attrs)


def _reproject_partitioned(src, plan: ReprojectPlan, interp: str, fill, out_dtype, devices):
    """K1 over several devices (``multidevice``): target row bands balanced by
    predicted K1 time (``sharding.band_shard``; by rows for 2-D plans), each
    device holding only the source rows its band reads, from one host thread
    and stream per device.  The band results land in one (n, H', W') output —
    numpy for a numpy source, a tensor on the source's device otherwise — bit
    for bit the single-launch result (the kernel takes any row band:
    reproject.py:230-252's per-tile blocks are independent)."""
    from .sharding import band_shard

    od = np.dtype(out_dtype if out_dtype is not None else
                  (np.float64 if interp == "bilinear" else _src_dtype(src)))
    world = len(devices)
    balance = "cost" if plan.coord_mode == 0 else "rows"
    shards = [band_shard(plan, world, i, balance, od.itemsize) for i in range(world)]
    n = src.shape[0]
    out = multidevice.output_like(src, (n, plan.dst_height, plan.dst_width), od)

    def part(i, dev):
        sh = shards[i]
        if sh.row1 <= sh.row0:
            return
        j0, j1 = sh.src_rows
        band = multidevice.rows_to_device(src, j0, j1, dev)
        res = kernels.reproject(band, plan, interp, fill, out_dtype=od, rows=sh.rows, src_row0=j0)
        multidevice.put_rows(out, sh.row0, sh.row1, res)

    multidevice.run_parts(devices, part, sources=[src])
    return out


def _src_dtype(src) -> np.dtype:
    if is_device_array(src):
        from .device import numpy_dtype
        return numpy_dtype(src.dtype)
    return np.dtype(src.dtype)


def _downscale_source_dataset(source_ds, source_gm: GridMapping, target_gm: GridMapping,
                              transformer: Transformer, interp_methods, agg_methods,
                              recover_nans):
    """reproject.py:338-382 — pre-downscale a finer source with the affine path."""
    bbox_trans = transformer.transform_bounds(*target_gm.xy_bbox)
    xres_trans = (bbox_trans[2] - bbox_trans[0]) / target_gm.width
    yres_trans = (bbox_trans[3] - bbox_trans[1]) / target_gm.height
    x_scale = source_gm.x_res / xres_trans
    y_scale = source_gm.y_res / yres_trans
    if x_scale < SCALE_LIMIT or y_scale < SCALE_LIMIT:
        from .affine import affine_transform_dataset

        bbox_trans = (bbox_trans[0] - 2 * source_gm.x_res, bbox_trans[1] - 2 * source_gm.y_res,
                      bbox_trans[2] + 2 * source_gm.x_res, bbox_trans[3] + 2 * source_gm.y_res)
        source_ds = clip_dataset_by_bbox(source_ds, bbox_trans, source_gm.xy_dim_names)
        source_gm = GridMapping.from_dataset(source_ds)
        w, h = round(x_scale * source_gm.width), round(y_scale * source_gm.height)
        downscaled_size = (w if w >= 2 else 2, h if h >= 2 else 2)
        downscale_target_gm = GridMapping.regular(
            size=downscaled_size, xy_min=(source_gm.xy_bbox[0], source_gm.xy_bbox[1]),
            xy_res=(xres_trans, yres_trans), crs=source_gm.crs, tile_size=source_gm.tile_size)
        source_ds = affine_transform_dataset(
            source_ds, downscale_target_gm, source_gm=source_gm,
            interp_methods=_prep_interp_methods_downscale(interp_methods),
            agg_methods=agg_methods, recover_nans=recover_nans)
        source_gm = GridMapping.from_dataset(source_ds)
    return source_ds, source_gm

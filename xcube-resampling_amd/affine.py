"""Same-CRS regular -> regular resampling (reference: affine.py).

Host side restates ``affine_transform_dataset`` (affine.py:52-137),
``resample_dataset`` (140-240) and ``_resample_array``/``_downscale``/
``_upscale`` (243-362), including the parts delegated to third-party code
absent from the reference tree: dask-image's per-output-chunk input footprint
(the chunk offsets/slices that decide scipy's mirror and bounds behaviour) and
dask's auto-chunking of numpy inputs.  All pixel work is one launch of the
K2/K3 HIP kernel (``xrs_affine``): scipy order-0/1 sampling, recover_nans and
the coarsen reducer fused, the div-x intermediate never materialised.
"""

from __future__ import annotations

import math
from collections.abc import Iterable
from dataclasses import dataclass, field

import numpy as np

from . import _native, kernels, multidevice
from .dataset import DataArray, Dataset
from .device import is_device_array, require_device, to_device
from . import streaming
from .options import get_options
from .streaming import device_to_host, host_to_device
from .gridmapping import GridMapping
from .utils import (
    _can_apply_affine_transform,
    _get_agg_method,
    _get_fill_value,
    _get_interp_method_int,
    _get_recover_nan,
    _select_variables,
    as_dataset,
    normalize_grid_mapping,
)

_DASK_CHUNK_LIMIT = 128 * 2**20  # dask "array.chunk-size" default


def dask_auto_chunks(shape, itemsize: int, limit: int = _DASK_CHUNK_LIMIT) -> tuple[int, ...]:
    """dask.array.core.auto_chunks for ``da.asarray(numpy_array)`` (all dims
    "auto", no previous chunks): the chunking the reference's ``da.asarray``
    gives numpy inputs (affine.py:207, reproject.py:210)."""
    chunks: list = [None] * len(shape)
    autos = [i for i in range(len(shape))]
    largest_block = 1
    while autos:
        size = (limit / itemsize / largest_block) ** (1 / len(autos))
        small = [i for i in autos if shape[i] < size]
        if small:
            for i in small:
                chunks[i] = shape[i]
                largest_block *= max(shape[i], 1)
            autos = [i for i in autos if i not in small]
            continue
        for i in autos:
            chunks[i] = _round_to(size, shape[i])
        break
    return tuple(int(c) for c in chunks)


def _round_to(c: float, s: int) -> int:
    """dask.array.core.round_to: the largest factor of s in [c/2, c], else c."""
    if c <= s:
        fs = [f for f in _factors(s) if c / 2 <= f <= c]
        return max(fs) if fs else max(1, int(c))
    return int(c // s * s)


def _factors(n: int) -> set[int]:
    out = set()
    for i in range(1, int(math.isqrt(n)) + 1):
        if n % i == 0:
            out.update((i, n // i))
    return out


def axis_chunk_params(scale: float, offset: float, out_len: int, chunk: int, in_len: int,
                      order: int):
    """dask-image ndinterp.affine_transform footprint along one axis of a
    diagonal transform: per output chunk the input slice start, its length and
    the re-based offset ``offset + scale*chunk_offset - start``."""
    rel, lens, offs = [], [], []
    co = 0
    while co < out_len:
        cs = min(chunk, out_len - co)
        e0 = scale * co + offset
        e1 = scale * (co + cs) + offset
        lo, hi = min(e0, e1), max(e0, e1)
        if order % 2 == 0:
            lo += 0.5
            hi += 0.5
        rel_i = float(np.floor(lo) - order // 2)
        rel_f = float(np.floor(hi) - order // 2 + order)
        if order == 0:
            rel_i -= 1
        rel_i = float(np.clip(rel_i, 0, in_len - 1))
        rel_f = float(np.clip(rel_f, 0, in_len - 1))
        start, stop = int(rel_i), min(int(rel_f) + 2, in_len)
        rel.append(start)
        lens.append(stop - start)
        offs.append((offset + scale * co) - rel_i)
        co += cs
    return (np.array(rel, np.int64), np.array(lens, np.int64), np.array(offs, np.float64))


def _mirror(idx: int, n: int) -> int:
    if n <= 1:
        return 0
    s2 = 2 * n - 2
    if idx >= n:
        idx -= s2 * (idx // s2)
        if idx >= n:
            idx = s2 - idx
    return idx


def time_neighbours(nt: int, chunk: int, order: int) -> np.ndarray | None:
    """Index of the slice scipy weights by 0 (order 1) for every time step:
    t+1, mirrored inside the dask-image input slice of the time chunk."""
    if order != 1:
        return None
    rel, lens, _ = axis_chunk_params(1.0, 0.0, nt, chunk, nt, 1)
    out = np.empty(nt, np.int64)
    for k, (start, n) in enumerate(zip(rel, lens)):
        for tl in range(min(chunk, nt - k * chunk)):
            t = k * chunk + tl
            out[t] = start + _mirror(t - start + 1, int(n))
    return out


def aligned_coarsen_chunks(chunks, multiple: int) -> tuple[int, ...]:
    """dask.array.routines.aligned_coarsen_chunks (dask 2021.10: the rechunk
    da.coarsen applies before chunk.coarsen): chunk sizes made multiples of
    `multiple`, the excess redistributed to the smallest chunks, any remainder
    appended."""
    chunks = np.array(chunks, dtype=np.int64)
    overflow = chunks % multiple
    excess = int(overflow.sum())
    new = chunks - overflow
    valid = new == chunks
    vi, ii = np.where(valid)[0], np.where(~valid)[0]
    order = [*ii[np.argsort(new[ii])], *vi[np.argsort(new[vi])]]
    parts = (multiple,) * (excess // multiple)
    rem = (excess % multiple,) if excess % multiple else ()
    for k, extra in enumerate(parts):
        new[order[k]] += extra
    new = np.array([*new, *rem], dtype=np.int64)
    return tuple(int(c) for c in new[new > 0])


def _has_whole_chunk_windows(chunk_x: np.ndarray, div_x: int) -> bool:
    """True if some dask chunk along x is exactly one coarsen window wide."""
    sizes = np.bincount(chunk_x)
    return bool(np.any(sizes == div_x))


def coarsen_chunk_ids(shape, chunks, factors):
    """Per axis, the id of the dask chunk that holds each index after
    da.coarsen's alignment rechunk (routines.py coarsen: aligned_coarsen_chunks
    on every coarsened axis whose chunks are not multiples of the factor)."""
    ids = []
    for n, c, f in zip(shape, chunks, factors):
        c = min(int(c), n)
        sizes = (c,) * (n // c) + ((n % c,) if n % c else ())
        if f > 1:
            aligned = aligned_coarsen_chunks(sizes, f)
            if aligned != sizes:
                sizes = aligned
        ids.append(np.repeat(np.arange(len(sizes), dtype=np.int32), sizes))
    return tuple(ids)


@dataclass
class AffinePlan:
    out_h: int
    out_w: int
    div_y: int
    div_x: int
    agg_code: int
    order: int
    scale_y: float
    scale_x: float
    chunk_y: int
    rel_y: np.ndarray
    len_y: np.ndarray
    off_y: np.ndarray
    chunk_x: int
    rel_x: np.ndarray
    len_x: np.ndarray
    off_x: np.ndarray
    t_next: np.ndarray | None
    cval: float
    recover_nan: bool
    out_dtype: np.dtype
    # reducers outside the fused K3 (median, mode, std, var): K2 evaluates the
    # div-x intermediate (out_h, out_w above are then its size), K7 coarsens it
    post_agg: str | None = None
    post_div: tuple[int, int] = (1, 1)
    post_dtype: np.dtype | None = None
    post_chunks: tuple | None = None   # dask chunk ids (t, y, x) for float mode
    _cache: dict = field(default_factory=dict, repr=False)

    @property
    def run_weights(self) -> bool:
        """xrs_affine's K3w hint: an order-1 coarsen whose div-x grid has scale 1
        on both axes with some chunk offset off the integral layout (a target
        grid not aligned to the source: contiguous taps, fractional weights).
        Only the kernel choice depends on it, never the result."""
        if self.order != 1 or (self.div_y == 1 and self.div_x == 1):
            return False
        if self.scale_y != 1.0 or self.scale_x != 1.0:
            return False
        offs = np.concatenate([np.asarray(self.off_y, np.float64).ravel(),
                               np.asarray(self.off_x, np.float64).ravel()])
        return bool(np.any(offs != np.floor(offs)))

    def device_tables(self, device) -> dict:
        key = str(device)
        tabs = self._cache.get(key)
        if tabs is None:
            tabs = {k: to_device(getattr(self, k), device)
                    for k in ("rel_y", "len_y", "off_y", "rel_x", "len_x", "off_x")}
            tabs["t_next"] = (to_device(self.t_next, device) if self.t_next is not None
                              else None)
            self._cache[key] = tabs
        return tabs


def _agg_dtype(agg: str, dtype: np.dtype) -> np.dtype:
    """numpy result dtype of the coarsen reducer on a block of `dtype`."""
    dtype = np.dtype(dtype)
    if agg in ("count", "mode"):   # np.count_nonzero; _mode_from_normalized's int64
        return np.dtype(np.int64)
    if np.issubdtype(dtype, np.floating):
        return dtype
    if agg in ("sum", "prod"):
        return np.dtype(np.uint64 if np.issubdtype(dtype, np.unsignedinteger) else np.int64)
    return dtype


def plan_affine(src_shape, dtype, affine_matrix, output_shape, output_chunks, interp: int,
                agg: str, recover_nan: bool, fill_value) -> AffinePlan:
    """affine.py:243-362 decisions for one (nt, H, W) array (``recover_nan``
    must already include the reference's ``da.any(mask)`` test)."""
    ((i_scale, _, i_off), (_, j_scale, j_off)) = affine_matrix
    if interp > 1:
        raise ValueError(
            "interp_methods must be one of 0, 1, 'nearest', 'bilinear'. "
            "Higher order is not supported for 3D arrays in affine transforms, "
            "as it causes unintended blending across the non-spatial (e.g., time) "
            "dimension.")
    nt, h, w = src_shape
    out_h, out_w = output_shape[-2], output_shape[-1]
    tile_h, tile_w = output_chunks[-2], output_chunks[-1]
    # affine.py:253 — note the reference tests affine_matrix[1][0] (not [1][1])
    if (affine_matrix[0][0] > 1 or affine_matrix[1][0] > 1) and interp != 0:
        div_y, div_x = math.ceil(abs(j_scale)), math.ceil(abs(i_scale))
        scale_y, scale_x = j_scale / div_y, i_scale / div_x
        agg_name = agg
    else:
        div_y = div_x = 1
        scale_y, scale_x = j_scale, i_scale
        agg_name = None
    recover = bool(recover_nan and interp > 0 and np.issubdtype(dtype, np.floating))
    inter_dtype = np.dtype(np.float64) if recover else np.dtype(dtype)
    post = {}
    if agg_name is None:
        agg_code, out_dtype = 0, inter_dtype
    else:
        if agg_name not in _native.AGG_CODES:
            raise NotImplementedError(f"aggregation method {agg_name!r} is not supported")
        agg_code, out_dtype = _native.AGG_CODES[agg_name], _agg_dtype(agg_name, inter_dtype)
        t_chunk = output_chunks[0] if len(output_shape) == 3 else nt
        chunks = coarsen_chunk_ids((nt, out_h * div_y, out_w * div_x),
                                   (t_chunk, tile_h, tile_w), (1, div_y, div_x))
        # K3 sums every window row by row; a chunk one window wide is summed
        # as one pairwise loop by numpy (see xrs_coarsen) -> K7 handles it
        whole = _has_whole_chunk_windows(chunks[2], div_x)
        if agg_name not in _native.FUSED_AGGS or whole:
            post = dict(post_agg=agg_name, post_div=(div_y, div_x),
                        post_dtype=np.dtype(out_dtype), post_chunks=chunks)
            agg_code, out_dtype = 0, inter_dtype
    rel_y, len_y, off_y = axis_chunk_params(scale_y, j_off, out_h * div_y, tile_h, h, interp)
    rel_x, len_x, off_x = axis_chunk_params(scale_x, i_off, out_w * div_x, tile_w, w, interp)
    t_next = None
    if len(output_shape) == 3:
        t_next = time_neighbours(nt, output_chunks[0], interp)
    if post:  # K2 writes the intermediate (out*div, div 1), K7 reduces it
        out_h, out_w, div_y, div_x = out_h * div_y, out_w * div_x, 1, 1
    return AffinePlan(out_h=out_h, out_w=out_w, div_y=div_y, div_x=div_x, agg_code=agg_code,
                      order=interp, scale_y=scale_y, scale_x=scale_x, chunk_y=tile_h,
                      rel_y=rel_y, len_y=len_y, off_y=off_y, chunk_x=tile_w, rel_x=rel_x,
                      len_x=len_x, off_x=off_x, t_next=t_next, cval=float(fill_value),
                      recover_nan=recover, out_dtype=np.dtype(out_dtype), **post)


def _resample_array(data, dims, chunks, affine_matrix, output_shape, output_chunks, interp,
                    agg, recover_nan, fill_value):
    """Device execution of affine.py:243-362 for one variable."""
    if len(data.shape) > 3:
        raise NotImplementedError("the engine resamples 2-D and 3-D variables")
    device = require_device()
    devices = multidevice.active_devices()
    if devices is not None:
        res = _resample_partitioned(data, affine_matrix, output_shape, output_chunks, interp,
                                    agg, recover_nan, fill_value, devices)
        if res is not None:
            return res
    if isinstance(data, np.ndarray) and data.ndim in (2, 3) and \
            data.nbytes >= get_options()["host_streaming_min_bytes"] and \
            not (recover_nan and interp > 0 and np.issubdtype(data.dtype, np.floating)):
        # numpy in, numpy out (affine.py:227-228): band pipeline, no NaN test needed
        arr = data.reshape((1,) + data.shape) if data.ndim == 2 else data
        plan = plan_affine(arr.shape, arr.dtype, affine_matrix, output_shape, output_chunks,
                           interp, agg, False, fill_value)
        res = streaming.affine_host(arr, plan, device)
        if res is not None:
            return res[0] if data.ndim == 2 else res
    src = host_to_device(data, device)
    expanded = src.dim() == 2
    if expanded:
        src = src.unsqueeze(0)
    dtype = np.dtype(str(src.dtype).replace("torch.", ""))
    recover = bool(recover_nan and interp > 0 and np.issubdtype(dtype, np.floating)
                   and kernels.any_nan(src))
    plan = plan_affine(tuple(src.shape), dtype, affine_matrix, output_shape, output_chunks,
                       interp, agg, recover, fill_value)
    out = kernels.affine(src, plan)
    if plan.post_agg is not None:
        out = kernels.coarsen(out, plan.post_div[0], plan.post_div[1], plan.post_agg,
                              plan.post_dtype, chunk_ids=plan.post_chunks)
    final_dtype = plan.out_dtype if plan.post_dtype is None else plan.post_dtype
    if np.dtype(final_dtype) == np.uint64:
        out = out.cpu().numpy().view(np.uint64)
        return out[0] if expanded else out
    return out[0] if expanded else out


def _resample_partitioned(data, affine_matrix, output_shape, output_chunks, interp, agg,
                          recover_nan, fill_value, devices):
    """K2 / K3 over several devices (``multidevice``): output chunk row bands
    (``sharding.coarsen_shard``), each device holding only the source rows its
    chunks' dask-image footprints read (affine.py:336-343: the footprint
    carries the order-1 halo and the NaN dilation), one host thread and
    stream per device.  ``da.any(mask)`` (affine.py:347-349) is the whole
    array's: every device tests its rows, the rows no band reads are tested
    too.  Returns None for plans that cannot be split (a separate coarsen
    pass, chunks without whole windows, uint64 sums): those run whole on the
    current device."""
    from .sharding import coarsen_shard

    expanded = data.ndim == 2
    on_device = is_device_array(data)
    arr = (data.unsqueeze(0) if on_device else np.asarray(data).reshape((1,) + data.shape)) \
        if expanded else (data if on_device else np.asarray(data))
    if on_device:
        from .device import numpy_dtype
        dtype = numpy_dtype(arr.dtype)
    else:
        dtype = np.dtype(arr.dtype)
    shape = tuple(arr.shape)
    plan = plan_affine(shape, dtype, affine_matrix, output_shape, output_chunks, interp, agg,
                       False, fill_value)
    if plan.post_agg is not None or plan.chunk_y % plan.div_y != 0 or \
            np.dtype(plan.out_dtype) == np.uint64:
        return None
    world = len(devices)
    shards = [coarsen_shard(plan, world, i) for i in range(world)]

    def upload(i, dev):
        sh = shards[i]
        if sh.chunk1 <= sh.chunk0:
            return None
        return multidevice.rows_to_device(arr, sh.src_row0, sh.src_row1, dev)

    bands = multidevice.run_parts(devices, upload, sources=[arr])
    if recover_nan and interp > 0 and np.issubdtype(dtype, np.floating):
        if on_device:
            recover = kernels.any_nan(arr.contiguous())
        else:
            def test(i, dev):
                return bands[i] is not None and kernels.any_nan(bands[i].contiguous())
            recover = any(multidevice.run_parts(devices, test))
            if not recover:   # rows no band reads are part of the reference's test
                read = np.zeros(shape[1], bool)
                for sh in shards:
                    read[sh.src_row0:sh.src_row1] = True
                rest = np.flatnonzero(~read)
                if rest.size:
                    recover = kernels.any_nan(host_to_device(
                        np.ascontiguousarray(arr[:, rest]), require_device()))
        if recover:
            plan = plan_affine(shape, dtype, affine_matrix, output_shape, output_chunks, interp,
                               agg, True, fill_value)
            shards = [coarsen_shard(plan, world, i) for i in range(world)]
    out = multidevice.output_like(arr, (shape[0], plan.out_h, plan.out_w), plan.out_dtype)

    def part(i, dev):
        sh = shards[i]
        if bands[i] is None:
            return
        res = kernels.affine(bands[i], sh.plan)
        multidevice.put_rows(out, sh.row0, sh.row1, res)

    multidevice.run_parts(devices, part)
    return out[0] if expanded else out


def resample_dataset(dataset, affine_matrix, yx_dims: tuple[str, str], target_size,
                     target_tile_size, interp_methods=None, agg_methods=None,
                     recover_nans=False, fill_values=None, devices=None) -> Dataset:
    """affine.py:140-240 (``devices``: see affine_transform_dataset)."""
    with multidevice.use_devices(devices):
        return _resample_dataset(dataset, affine_matrix, yx_dims, target_size, target_tile_size,
                                 interp_methods, agg_methods, recover_nans, fill_values)


def _resample_dataset(dataset, affine_matrix, yx_dims, target_size, target_tile_size,
                      interp_methods, agg_methods, recover_nans, fill_values) -> Dataset:
    dataset = as_dataset(dataset)
    data_vars, coords = {}, {}
    for var_name, data_array in dataset.variables.items():
        new = None
        if data_array.dims[-2:] == yx_dims:
            on_device = is_device_array(data_array.data)
            if data_array.chunks is not None:
                lead_chunks = tuple(c[0] for c in data_array.chunks[:-2])
            else:
                auto = dask_auto_chunks(data_array.shape, data_array.dtype.itemsize)
                lead_chunks = tuple(auto[:-2])
            output_shape = data_array.shape[:-2] + (target_size[1], target_size[0])
            output_chunks = lead_chunks + (target_tile_size[1], target_tile_size[0])
            res = _resample_array(
                data_array.data, data_array.dims, data_array.chunks, affine_matrix, output_shape,
                output_chunks,
                _get_interp_method_int(interp_methods, var_name, data_array),
                _get_agg_method(agg_methods, var_name, data_array),
                _get_recover_nan(recover_nans, var_name, data_array),
                _get_fill_value(fill_values, var_name, data_array))
            if not on_device and not isinstance(res, np.ndarray):
                res = device_to_host(res)
            new = DataArray(res, data_array.dims, data_array.attrs)
        elif yx_dims[0] not in data_array.dims and yx_dims[1] not in data_array.dims:
            new = data_array
        if new is not None:
            if var_name in dataset.coords:
                coords[var_name] = new
            elif var_name in dataset.data_vars:
                data_vars[var_name] = new
    return Dataset(data_vars=data_vars, coords=coords, attrs=dataset.attrs)


def affine_transform_dataset(source_ds, target_gm: GridMapping,
                             source_gm: GridMapping | None = None,
                             variables: str | Iterable[str] | None = None, interp_methods=None,
                             agg_methods=None, recover_nans=False, fill_values=None,
                             devices=None) -> Dataset:
    """affine.py:52-137.  ``devices`` (engine extension): split every
    variable's output chunk rows over these GPUs (``multidevice``)."""
    with multidevice.use_devices(devices):
        return _affine_transform_dataset(source_ds, target_gm, source_gm, variables,
                                         interp_methods, agg_methods, recover_nans, fill_values)


def _affine_transform_dataset(source_ds, target_gm, source_gm, variables, interp_methods,
                              agg_methods, recover_nans, fill_values) -> Dataset:
    source_ds = as_dataset(source_ds)
    if source_gm is None:
        source_gm = GridMapping.from_dataset(source_ds)
    source_ds = normalize_grid_mapping(source_ds, source_gm)
    assert _can_apply_affine_transform(source_gm, target_gm), (
        f"Affine transformation cannot be applied to source CRS "
        f"{source_gm.crs.name!r} and target CRS {target_gm.crs.name!r}"
    )
    source_ds = _select_variables(source_ds, variables)
    target_ds = _resample_dataset(
        source_ds, target_gm.ij_transform_to(source_gm),
        (source_gm.xy_dim_names[1], source_gm.xy_dim_names[0]), target_gm.size,
        target_gm.tile_size, interp_methods, agg_methods, recover_nans, fill_values)
    x_name, y_name = target_gm.xy_var_names
    return target_ds.assign_coords({
        x_name: DataArray(target_gm.x_coords.values, target_gm.x_coords.dims),
        y_name: DataArray(target_gm.y_coords.values, target_gm.y_coords.dims),
    })

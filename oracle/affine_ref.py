"""ORACLE (test infrastructure only) — the reference's affine / coarsen path.

Follows xcube_resampling/affine.py:
  _resample_array  243-274   resample_array()
  _downscale       277-313   (divisor, div-x upscale, da.coarsen)
  _upscale         316-362   (order 0/1, recover_nans)
and the third-party code it delegates to, which is not in the reference tree:

* dask-image ``ndinterp.affine_transform`` (dask-image >= 0.6, unpinned in
  pyproject.toml:43-52; not installed here).  Restated from its published
  algorithm: per output chunk, the footprint of the chunk corners maps to an
  input slice ``[rel_i, rel_f + 2)`` and scipy runs on that slice with the
  re-based offset ``offset + M @ chunk_offset - rel_i``.  The per-chunk call
  itself is the REAL ``scipy.ndimage.affine_transform`` (scipy 1.15.3 here and
  on the GPU box), i.e. the reference's actual engine.
* dask ``da.coarsen`` -> ``chunk.coarsen`` (reshape to (h/d, d, w/d, d), reduce
  over the window axes) with the reducers of coarsen.py:50-155 (numpy nan-
  reducers, executed with numpy itself).

``scipy_diag_model`` is an independent pure-numpy model of scipy's order-0/1
NI_GeometricTransform for diagonal matrices (the semantics the HIP kernel
implements); tests check it against scipy itself.
"""

from __future__ import annotations

import math
import warnings
from itertools import product

import numpy as np
import scipy.ndimage as ndi


# --------------------------------------------------------------------------
# dask.array chunk arithmetic
# --------------------------------------------------------------------------

def normalize_chunks(chunks, shape):
    out = []
    for c, s in zip(chunks, shape):
        if isinstance(c, (tuple, list)):
            out.append(tuple(c))
        else:
            c = s if c in (None, -1) else int(c)
            n, r = divmod(s, c)
            out.append((c,) * n + ((r,) if r else ()))
    return tuple(out)


# --------------------------------------------------------------------------
# dask_image.ndinterp.affine_transform (per output chunk -> scipy)
# --------------------------------------------------------------------------

def chunk_params(matrix_diag, offset, output_shape, output_chunks, input_shape, order):
    """Per output chunk and dimension: (rel_i, slice_stop, offset_prime).

    Restates dask_image's footprint computation with a diagonal matrix."""
    n = len(input_shape)
    matrix = np.diag(matrix_diag)
    offset = np.asarray(offset, dtype=np.float64)
    nchunks = normalize_chunks(output_chunks, output_shape)
    offsets = [np.cumsum((0,) + bds[:-1]) for bds in nchunks]
    params = {}
    for block in product(*(range(len(b)) for b in nchunks)):
        shp = [nchunks[d][block[d]] for d in range(n)]
        off = [offsets[d][block[d]] for d in range(n)]
        edges = np.array(list(np.ndindex(tuple([2] * n)))) * np.array(shp) + np.array(off)
        rel_edges = np.dot(matrix, edges.T).T + offset
        rel_i = np.min(rel_edges, 0)
        rel_f = np.max(rel_edges, 0)
        for d in range(n):
            if order % 2 == 0:
                rel_i[d] += 0.5
                rel_f[d] += 0.5
            rel_i[d] = np.floor(rel_i[d]) - order // 2
            rel_f[d] = np.floor(rel_f[d]) - order // 2 + order
            if order == 0:
                rel_i[d] -= 1
        for d, s in enumerate(input_shape):
            rel_i[d] = np.clip(rel_i[d], 0, s - 1)
            rel_f[d] = np.clip(rel_f[d], 0, s - 1)
        sl = tuple(slice(int(rel_i[d]), int(rel_f[d]) + 2) for d in range(n))
        offset_prime = offset + np.dot(matrix, off) - rel_i
        params[block] = (shp, off, sl, offset_prime)
    return nchunks, params


def dask_image_affine_transform(image, matrix_diag, offset, output_shape, output_chunks, order,
                                cval):
    """dask_image.ndinterp.affine_transform(image, np.diag(matrix_diag), offset,
    order=order, output_shape, output_chunks, mode="constant", cval=cval)."""
    image = np.asarray(image)
    nchunks, params = chunk_params(matrix_diag, offset, output_shape, output_chunks, image.shape,
                                   order)
    out = np.empty(tuple(output_shape), dtype=image.dtype)
    matrix = np.diag(matrix_diag)
    for block, (shp, off, sl, offset_prime) in params.items():
        res = ndi.affine_transform(image[sl], matrix, offset=offset_prime, output_shape=tuple(shp),
                                   order=order, mode="constant", cval=cval, prefilter=False)
        out[tuple(slice(o, o + s) for o, s in zip(off, shp))] = res
    return out


# --------------------------------------------------------------------------
# coarsen reducers (coarsen.py:50-155) under dask chunk.coarsen
# --------------------------------------------------------------------------

def _reduce(reducer, nan_reducer, block, axis):
    if np.issubdtype(block.dtype, np.floating):
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", category=RuntimeWarning)
            return nan_reducer(block, axis)
    a = reducer(block, axis)
    if np.issubdtype(a.dtype, np.floating):
        return np.rint(a).astype(block.dtype)
    return a


def _pick(block, axis, which):
    idx = tuple((which(block.shape[i]) if i in axis else slice(None)) for i in range(block.ndim))
    return block[idx]


def _mode(block, axis):
    nd = len(axis)
    block = np.moveaxis(block, axis, range(-nd, 0))
    flat = block.reshape(-1, np.prod(block.shape[-nd:]))
    min_val = int(flat.min())
    max_val = int(flat.max())
    rng = max_val - min_val + 1
    norm = (flat - min_val).astype(np.int64)
    out = np.empty(norm.shape[0], dtype=np.int64)
    for i in range(norm.shape[0]):
        counts = np.bincount(norm[i], minlength=rng)
        out[i] = int(np.argmax(counts)) + min_val  # first maximum, as the numba loop
    return out.reshape(block.shape[:-nd])


AGGS = {
    "center": lambda b, a: _pick(b, a, lambda s: s // 2),
    "count": np.count_nonzero,
    "first": lambda b, a: _pick(b, a, lambda s: 0),
    "last": lambda b, a: _pick(b, a, lambda s: -1),
    "prod": np.nanprod,
    "max": np.nanmax,
    "mean": lambda b, a: _reduce(np.mean, np.nanmean, b, a),
    "median": lambda b, a: _reduce(np.median, np.nanmedian, b, a),
    "min": np.nanmin,
    "mode": _mode,
    "std": lambda b, a: _reduce(np.std, np.nanstd, b, a),
    "sum": np.nansum,
    "var": lambda b, a: _reduce(np.var, np.nanvar, b, a),
}


def aligned_coarsen_chunks(chunks, multiple):
    """dask/array/routines.py:2194-2229 (dask 2021.10)."""
    overflow = np.array(chunks) % multiple
    excess = overflow.sum()
    new_chunks = np.array(chunks) - overflow
    validity = new_chunks == chunks
    valid_inds, invalid_inds = np.where(validity)[0], np.where(~validity)[0]
    order = [*invalid_inds[np.argsort(new_chunks[invalid_inds])],
             *valid_inds[np.argsort(new_chunks[valid_inds])]]
    multiples = (multiple,) * (excess // multiple)
    remainder = (excess % multiple,) if excess % multiple > 0 else ()
    for idx, extra in enumerate(multiples):
        new_chunks[order[idx]] += extra
    new_chunks = np.array([*new_chunks, *remainder])
    return tuple(int(c) for c in new_chunks[new_chunks > 0])


def coarsen_chunked(agg, array, axes, chunks):
    """dask.array.routines.coarsen (routines.py:2233-2261): rechunk to
    aligned_coarsen_chunks, then chunk.coarsen per block (the block matters
    for `mode`, whose offset is the block minimum, coarsen.py:133)."""
    chunks = list(normalize_chunks(chunks, array.shape))
    for i, div in axes.items():
        aligned = aligned_coarsen_chunks(chunks[i], div)
        if aligned != tuple(chunks[i]):
            chunks[i] = aligned
    starts = [np.cumsum((0,) + tuple(c[:-1])) for c in chunks]
    out = None
    for block in product(*(range(len(c)) for c in chunks)):
        sl = tuple(slice(int(starts[d][b]), int(starts[d][b]) + chunks[d][b])
                   for d, b in enumerate(block))
        res = np.asarray(coarsen(agg, array[sl], dict(axes)))
        if out is None:
            out = np.empty(tuple(s // axes.get(i, 1) for i, s in enumerate(array.shape)),
                           dtype=res.dtype)
        osl = tuple(slice(s.start // axes.get(i, 1), s.stop // axes.get(i, 1))
                    for i, s in enumerate(sl))
        out[osl] = res
    return out


def coarsen(agg, array, axes):
    """dask.array.coarsen(reduction, x, axes) on one numpy block (chunk.coarsen)."""
    axes = {i: axes.get(i, 1) for i in range(array.ndim)}
    for i, d in axes.items():
        if array.shape[i] % d:
            raise ValueError(f"Coarsening factors {axes} do not align with array shape {array.shape}.")
    newshape = tuple(v for i in range(array.ndim) for v in (array.shape[i] // axes[i], axes[i]))
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", category=RuntimeWarning)
        return AGGS[agg](array.reshape(newshape), tuple(range(1, array.ndim * 2, 2)))


# --------------------------------------------------------------------------
# affine.py:243-362
# --------------------------------------------------------------------------

def upscale(array, affine_matrix, output_shape, output_chunks, interp, recover_nan, fill):
    """affine.py:316-362."""
    ((i_scale, _, i_off), (_, j_scale, j_off)) = affine_matrix
    nd = array.ndim
    offset = (0,) * (nd - 2) + (j_off, i_off)
    scale = (1,) * (nd - 2) + (j_scale, i_scale)
    if interp > 1:
        raise ValueError(
            "interp_methods must be one of 0, 1, 'nearest', 'bilinear'. "
            "Higher order is not supported for 3D arrays in affine transforms, "
            "as it causes unintended blending across the non-spatial (e.g., time) "
            "dimension.")
    if recover_nan and interp > 0:
        mask = np.isnan(array)
        if np.any(mask):
            filled = np.where(mask, 0.0, array)
            scaled_im = dask_image_affine_transform(filled, scale, offset, output_shape,
                                                    output_chunks, interp, fill)
            scaled_norm = dask_image_affine_transform(1.0 - mask, scale, offset, output_shape,
                                                      output_chunks, interp, fill)
            with warnings.catch_warnings():
                warnings.simplefilter("ignore", category=RuntimeWarning)
                return np.where(np.isclose(scaled_norm, 0.0), np.nan, scaled_im / scaled_norm)
    return dask_image_affine_transform(array, scale, offset, output_shape, output_chunks, interp,
                                       fill)


def resample_array(array, affine_matrix, output_shape, output_chunks, interp, agg, recover_nan,
                   fill):
    """affine.py:243-313 (note the reference's `affine_matrix[1][0] > 1` test)."""
    if (affine_matrix[0][0] > 1 or affine_matrix[1][0] > 1) and interp != 0:
        ((i_scale, _, i_off), (_, j_scale, j_off)) = affine_matrix
        j_div = math.ceil(abs(j_scale))
        i_div = math.ceil(abs(i_scale))
        m = ((i_scale / i_div, affine_matrix[0][1], affine_matrix[0][2]),
             (affine_matrix[1][0], j_scale / j_div, affine_matrix[1][2]))
        shape = tuple(output_shape[:-2]) + (output_shape[-2] * j_div, output_shape[-1] * i_div)
        up = upscale(array, m, shape, output_chunks, interp, recover_nan, fill)
        return coarsen_chunked(agg, up, {up.ndim - 2: j_div, up.ndim - 1: i_div},
                               output_chunks)
    return upscale(array, affine_matrix, output_shape, output_chunks, interp, recover_nan, fill)


# --------------------------------------------------------------------------
# independent model of scipy order-0/1 geometric transform (diagonal matrix)
# --------------------------------------------------------------------------

def _mirror(idx, n):
    """scipy map_coordinate, NI_EXTEND_MIRROR (spline footprint of mode constant)."""
    if n <= 1:
        return 0
    s2 = 2 * n - 2
    if idx < 0:
        idx = s2 * int(-idx / s2) + idx
        return idx + s2 if idx <= 1 - n else -idx
    if idx >= n:
        idx -= s2 * int(idx / s2)
        if idx >= n:
            idx = s2 - idx
    return idx


def scipy_diag_model(image, scale, offset, output_shape, order, cval):
    """Per-axis model: c = offset + scale*o; OOB iff c < 0 or c > n-1 -> cval;
    order 1: start=floor(c), w0=1-(c-start), w1=1-w0, neighbours mirrored;
    order 0: start=floor(c+0.5).  Sum over corners (last dim fastest) of
    ((v*w_0)*w_1)..., starting from 0.0; cast to the image dtype."""
    image = np.asarray(image)
    nd = image.ndim
    axes = []
    for d in range(nd):
        n = image.shape[d]
        entries = []
        for o in range(output_shape[d]):
            c = offset[d] + float(o) * scale[d]
            if c < 0 or c > n - 1:
                entries.append(None)
                continue
            if order == 1:
                s = math.floor(c)
                x = c - s
                w0 = 1.0 - x
                w1 = 1.0 - w0
                entries.append(((_mirror(s, n), w0), (_mirror(s + 1, n), w1)))
            else:
                entries.append(((math.floor(c + 0.5), 1.0),))
        axes.append(entries)
    out = np.empty(output_shape, dtype=image.dtype)
    for o in np.ndindex(*output_shape):
        es = [axes[d][o[d]] for d in range(nd)]
        if any(e is None for e in es):
            t = cval
        else:
            t = 0.0
            for corner in product(*es):
                coeff = float(image[tuple(idx for idx, _ in corner)])
                if order > 0:
                    for _, w in corner:
                        coeff *= w
                t += coeff
        out[o] = t
    return out

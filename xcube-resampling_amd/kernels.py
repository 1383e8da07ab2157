"""Device-level seams: one Python function per C-ABI entry point.

Each function takes device tensors (torch CUDA tensors = HIP allocations) and
host-side plan objects, launches the libxrs kernel on the current HIP stream
and returns device tensors.  These are the functions a dask/xarray
orchestration would call per chunk in place of the reference's block
callables; the Dataset-level API in reproject.py / affine.py /
rectify.py is built on them.
"""

from __future__ import annotations

import collections
import ctypes
import threading

import numpy as np

from . import _native
from .device import empty, ptr, require_device, stream_handle, to_device, torch


class ErrorFlags:
    """Device word the kernels OR data-dependent error bits into."""

    def __init__(self, device):
        self.tensor = torch().zeros(1, dtype=torch().int32, device=device)

    @property
    def ptr(self) -> int:
        return ptr(self.tensor)

    def raise_if_set(self, what: str) -> None:
        bits = int(self.tensor.item())  # synchronises the stream
        if bits & _native.XRS_EFLAG_INDEX:
            raise IndexError(f"{what}: index out of bounds for the source window")
        if bits & _native.XRS_EFLAG_BAND:
            raise _native.NativeLibraryError(f"{what}: read outside the device's source band")
        # coarsen.py:133-134: int(flat.min()) / int(flat.max()) on a float chunk
        if bits & _native.XRS_EFLAG_NAN_TO_INT:
            raise ValueError("cannot convert float NaN to integer")
        if bits & _native.XRS_EFLAG_INF_TO_INT:
            raise OverflowError("cannot convert float infinity to integer")
        if bits & _native.XRS_EFLAG_STATE:
            raise _native.NativeLibraryError(
                f"{what}: inconsistent rectify state (a tile record, claim key or source "
                f"position outside its raster was skipped)")


def reproject(src, plan, interp: str, fill: float, out_dtype=None, rows=None, out=None,
              src_row0: int = 0, flags: ErrorFlags | None = None, check: bool = True,
              stream=None):
    """K1 — reproject all tiles (or target rows `rows=(r0, r1)`) of `src`.

    src: device tensor (n, H_band, W) holding global source rows
         [src_row0, src_row0 + H_band) of the (H, W) source (after the
         reference's j-axis flip, see reproject.py:115-118).
    plan: ReprojectPlan (host tables are uploaded and cached per device).
    Returns the device tensor (n, r1 - r0, target width).
    """
    device = src.device
    if src.dim() != 3:
        raise ValueError("src must have shape (n, height, width)")
    n, h_band, w = src.shape
    if w != plan.src_width:
        raise ValueError(f"source width {w} does not match the plan ({plan.src_width})")
    src_dtype = _native.DTYPE_CODES[_np_dtype(src)]
    interp_code = _native.INTERP_CODES.get(interp)
    if interp_code is None:
        raise NotImplementedError(
            f"interp_methods must be one of 0, 1, 'nearest', 'bilinear', 'triangular', "
            f"was '{interp}'."
        )
    if out_dtype is None:
        out_dtype = np.float64 if interp == "bilinear" else _np_dtype(src)
    r0, r1 = (0, plan.dst_height) if rows is None else rows
    if h_band == 0:
        # a band that reads no source row (all taps in the padding): K1 still
        # addresses element 0 of the band for out-of-source taps
        src = torch().zeros((n, 1, w), dtype=src.dtype, device=device)
    if out is None:
        out = empty((n, r1 - r0, plan.dst_width), out_dtype, device)
    if plan.fused_transform(device):
        return _reproject_proj(src, h_band, plan, interp_code, fill, out_dtype, r0, r1, out,
                               src_row0, flags, check, stream)
    tables = plan.device_tables(device)
    lib = _native.lib()
    ws_bytes = lib.xrs_reproject_workspace_size(plan.dst_height, plan.dst_width, plan.tile_height,
                                                plan.tile_width, plan.coord_mode)
    ws = plan.workspace(device, ws_bytes)
    own_flags = flags is None
    if own_flags:
        flags = ErrorFlags(device)
    sn, sy, sx = src.stride()
    dn, dy, dx = out.stride()
    if sx != 1 or dx != 1:
        raise ValueError("innermost dimension must be contiguous")
    # coord_mode 2: the separable plan's column coordinates generated in K1
    gen = plan.coord_mode == 0 and "x_gen" in tables
    rc = lib.xrs_reproject(
        ptr(src), src_dtype, n, plan.src_height, plan.src_width, src_row0, h_band, sn, sy,
        ptr(out), _native.dtype_code(out_dtype), plan.dst_height, plan.dst_width, r0, r1,
        dn, dy, plan.tile_height, plan.tile_width,
        ptr(tables["x_gen"] if gen else tables["src_x"]), ptr(tables["src_y"]),
        2 if gen else plan.coord_mode,
        ptr(tables["tile_x0"]), ptr(tables["tile_y0"]), ptr(tables["tile_win"]),
        plan.win_height, plan.win_width, float(plan.x_res), float(plan.y_res),
        interp_code, float(fill), ptr(ws) if ws is not None else None, ws_bytes, flags.ptr,
        stream_handle(device, stream))
    _native.check(rc, "xrs_reproject")
    if own_flags and check:
        flags.raise_if_set("reproject")
    return out


def _reproject_proj(src, h_band, plan, interp_code, fill, out_dtype, r0, r1, out, src_row0,
                    flags, check, stream):
    """xrs_reproject_proj: the non-separable plan's transformation fused into
    the gather (reproject.py:472-496 + 268-335 per target pixel, no 2-D
    coordinate tables).  h_band: the caller's band height (0 for a band that
    reads no source row; src is then a one-row placeholder, never a row)."""
    device = src.device
    n = src.shape[0]
    tabs = plan.device_grid(device)
    steps, nsteps = plan.transformer.device_steps()
    own_flags = flags is None
    if own_flags:
        flags = ErrorFlags(device)
    sn, sy, _ = src.stride()
    dn, dy, _ = out.stride()
    rc = _native.lib().xrs_reproject_proj(
        ptr(src), _native.DTYPE_CODES[_np_dtype(src)], n, plan.src_height, plan.src_width,
        src_row0, h_band, sn, sy, ptr(out), _native.dtype_code(out_dtype), plan.dst_height,
        plan.dst_width, r0, r1, dn, dy, plan.tile_height, plan.tile_width,
        ptr(tabs["grid_x"]), ptr(tabs["grid_y"]), ctypes.cast(steps, ctypes.c_void_p), nsteps,
        ptr(tabs["tile_x0"]), ptr(tabs["tile_y0"]), ptr(tabs["tile_win"]),
        plan.win_height, plan.win_width, float(plan.x_res), float(plan.y_res), interp_code,
        float(fill), flags.ptr, stream_handle(device, stream))
    _native.check(rc, "xrs_reproject_proj")
    if own_flags and check:
        flags.raise_if_set("reproject")
    return out


def _np_dtype(t) -> np.dtype:
    from .device import numpy_dtype
    return numpy_dtype(t.dtype)


TILE_INFO_DTYPE = np.dtype([("r0", np.int32), ("c0", np.int32), ("th", np.int32),
                            ("tw", np.int32), ("si0", np.int32), ("sj0", np.int32),
                            ("swin", np.int32), ("shin", np.int32), ("x_off", np.float64),
                            ("y_off", np.float64)])


def _upload_small(arr: np.ndarray, device, stream):
    """A small host array on the device.  On the current stream it is staged
    in page-locked memory and copied asynchronously, so the host does not wait
    for the work already queued (a pageable copy would drain the queue before
    every K4); for a side stream the copy stays synchronous, as the kernel on
    that stream does not wait for the current one."""
    if stream is None:
        return torch().from_numpy(np.ascontiguousarray(arr)).pin_memory().to(
            device, non_blocking=True)
    return to_device(np.ascontiguousarray(arr), device)


def _box_grid(xy_bboxes, xy_border, grid):
    """(bordered boxes (n, 4), ntx, nty): the boxes with the border applied
    (bboxes.py:60-63), and the grid shape when they are the tiles of a
    regular grid — every tile column shares its x bounds and every tile row
    its y bounds — else (0, 0) (K4 then tests every box)."""
    boxes = np.asarray(xy_bboxes, dtype=np.float64).reshape(-1, 4)
    b = np.stack([boxes[:, 0] - xy_border, boxes[:, 1] - xy_border,
                  boxes[:, 2] + xy_border, boxes[:, 3] + xy_border], axis=1)
    if grid is not None:
        ntx, nty = grid
        if ntx * nty == b.shape[0]:
            bb = b.reshape(nty, ntx, 4)
            if np.all(bb[:, :, [0, 2]] == bb[:1, :, [0, 2]]) and \
                    np.all(bb[:, :, [1, 3]] == bb[:, :1, [1, 3]]):
                return b, ntx, nty
    return b, 0, 0


def _ij_bboxes_launch(x_image, y_image, xy_bboxes, xy_border, grid, device, stream, fill=None):
    """Launch K4; returns (device int32 accumulators (n, 4), n, (w, h), grid
    mode used).  ``fill``: a contiguous 4-byte tensor K4's grid sets to ~0
    (the claim-key scratch of the K5 call that follows, xrs_ij_bboxes_fill)."""
    device = require_device(device if device is not None else getattr(x_image, "device", None))
    x = to_device(x_image, device, np.float64)
    y = to_device(y_image, device, np.float64)
    h, w = x.shape
    b, ntx, nty = _box_grid(xy_bboxes, xy_border, grid)
    n = b.shape[0]
    if ntx > 0:
        bb = b.reshape(nty, ntx, 4)
    # one upload for the boxes and the accumulators' initial values (each
    # small copy is a blit of ~6 us on the stream ahead of K4): float64 box
    # bounds first, the int32 (i_min, j_min, i_max, j_max) after them
    if ntx > 0:
        parts = [bb[0, :, [0, 2]].T.reshape(-1), bb[:, 0, [1, 3]].reshape(-1)]
    else:
        parts = [b.reshape(-1)]
    acc0 = np.tile(np.array([[2**31 - 1, 2**31 - 1, -1, -1]], np.int32), (n, 1))
    blob = np.concatenate([np.concatenate(parts).astype(np.float64).view(np.uint8),
                           acc0.reshape(-1).view(np.uint8)])
    dev_blob = _upload_small(blob, device, stream)
    nbx = parts[0].size
    nb = sum(p.size for p in parts)
    bx = dev_blob[:8 * nbx].view(torch().float64)
    by = dev_blob[8 * nbx:8 * nb].view(torch().float64) if ntx > 0 else bx
    acc = dev_blob[8 * nb:].view(torch().int32).view(n, 4)
    if fill is not None and (not fill.is_contiguous() or fill.element_size() != 4):
        raise ValueError("fill must be a contiguous tensor of 4-byte words")
    rc = _native.lib().xrs_ij_bboxes_fill(
        ptr(x), ptr(y), h, w, x.stride(0), n, ntx, nty, ptr(bx), ptr(by), ptr(acc),
        ptr(fill) if fill is not None else None, fill.numel() if fill is not None else 0,
        stream_handle(device, stream))
    _native.check(rc, "xrs_ij_bboxes")
    if stream is not None:
        # made on the current stream, read (acc: written) by K4 on `stream`:
        # bx / by (and uploaded coordinates) are freed when this returns, so
        # keep their memory from the allocator until `stream` is past K4
        for t in (x, y, dev_blob) + ((fill,) if fill is not None else ()):
            t.record_stream(stream)
    return acc, n, (w, h), ntx > 0


def ij_bboxes(x_image, y_image, xy_bboxes, xy_border: float = 0.0, ij_border: int = 0,
              grid: tuple[int, int] | None = None, device=None, stream=None) -> np.ndarray:
    """K4 — gridmapping/bboxes.py:28-106 (compute_ij_bboxes) on the device.

    x_image, y_image: (h, w) source coordinates (numpy or device tensors).
    grid: (ntx, nty) when the boxes are the tiles of a regular grid (box k =
    ty*ntx + tx); enables the per-pixel candidate search over tile columns and
    rows instead of testing every box.
    Returns the (n, 4) int64 ij bboxes [i_min, j_min, i_max, j_max] (-1 = none).
    """
    acc, n, (w, h), _ = _ij_bboxes_launch(x_image, y_image, xy_bboxes, xy_border, grid, device,
                                          stream)
    acc = acc.cpu().numpy().astype(np.int64)
    out = np.full((n, 4), -1, dtype=np.int64)
    found = acc[:, 2] >= 0
    out[found] = np.stack([acc[found, 0], acc[found, 1], acc[found, 2] + 1, acc[found, 3] + 1],
                          axis=1)
    if ij_border != 0:  # bboxes.py:90-106
        f = out[:, 0] != -1
        out[f, 0] = np.maximum(out[f, 0] - ij_border, 0)
        out[f, 1] = np.maximum(out[f, 1] - ij_border, 0)
        out[f, 2] = np.minimum(out[f, 2] + ij_border, w)
        out[f, 3] = np.minimum(out[f, 3] + ij_border, h)
    return out


class DeviceTiles:
    """rectify_tiles_device's result: the tile records (uint8 tensor of
    TILE_INFO records) and chunk offsets (int64 tensor) on the device —
    unpacks as ``tiles, offs`` — and the claim-key scratch K4 filled beside
    them.  The scratch serves the first K5 call given these tiles (its claim
    pass consumes the fill); later calls fill their own."""

    __slots__ = ("tiles", "offs", "_keys", "ready", "made_on")

    def __init__(self, tiles, offs, keys, ready=None, made_on=None):
        self.tiles, self.offs, self._keys = tiles, offs, keys
        self.ready = ready       # event after K4 + xrs_rectify_tiles ...
        self.made_on = made_on   # ... on this stream (handle)

    def wait(self, stream) -> None:
        """Order `stream` after the launches that made these records and
        filled the key scratch, when they ran on another stream (on the same
        stream the order is given)."""
        if self.ready is not None and int(stream.cuda_stream) != self.made_on:
            stream.wait_event(self.ready)

    def __iter__(self):
        return iter((self.tiles, self.offs))

    def take_keys(self, dst_h: int, dst_w: int):
        """The pre-filled (dst_h, dst_w) key scratch, once; else None."""
        k, self._keys = self._keys, None
        return k if k is not None and tuple(k.shape) == (dst_h, dst_w) else None


def rectify_tiles_device(x_image, y_image, target_xy_bboxes, xy_border: float, ij_border: int,
                         grid: tuple[int, int], tile_size: tuple[int, int],
                         dst_size: tuple[int, int], dst_xy_min_max: tuple, dst_res: tuple,
                         j_axis_up: bool, device=None, stream=None):
    """K4 + xrs_rectify_tiles: the per-tile records and chunk offsets of
    rectify.py:312-419 computed and left on the device (no host round trip).
    Returns a DeviceTiles (K4 also fills the K5 claim-key scratch), or None
    when the boxes are not a regular tile grid."""
    dev = require_device(device if device is not None else getattr(x_image, "device", None))
    if _box_grid(target_xy_bboxes, xy_border, grid)[1] == 0:
        return None   # decided on the host: no K4 launch, no key scratch
    keys = torch().empty((dst_size[1], dst_size[0]), dtype=torch().int32, device=dev)
    acc, n, (w, h), is_grid = _ij_bboxes_launch(x_image, y_image, target_xy_bboxes, xy_border,
                                                grid, device, stream, fill=keys)
    assert is_grid
    device = acc.device
    ntx, nty = grid
    tiles = torch().empty(n * TILE_INFO_DTYPE.itemsize, dtype=torch().uint8, device=device)
    offs = torch().empty(n + 1, dtype=torch().int64, device=device)
    x_min, y_min, y_max = dst_xy_min_max
    rc = _native.lib().xrs_rectify_tiles(
        ptr(acc), ntx, nty, tile_size[0], tile_size[1], dst_size[0], dst_size[1], w, h,
        int(ij_border), float(x_min), float(y_min), float(y_max), float(dst_res[0]),
        float(dst_res[1]), int(bool(j_axis_up)), ptr(tiles), ptr(offs),
        stream_handle(device, stream))
    _native.check(rc, "xrs_rectify_tiles")
    s = stream if stream is not None else torch().cuda.current_stream(device)
    ready = torch().cuda.Event()
    ready.record(s)
    return DeviceTiles(tiles, offs, keys, ready, int(s.cuda_stream))


def transform(transformer, x, y, grid: bool, device=None, stream=None):
    """xrs_transform: the transformer's pipeline on the device
    (reproject.py:472-496 / rectify.py:182-231 per-point pyproj calls).

    grid=True: x (W,), y (H,) axes of a regular grid -> (H, W) images of the
    transformed pixel centres; grid=False: x, y (H, W) images.  Returns two
    float64 device tensors (H, W)."""
    device = require_device(device if device is not None else getattr(x, "device", None))
    xd = to_device(x, device, np.float64)
    yd = to_device(y, device, np.float64)
    if stream is not None:
        # uploads made on the current stream, read on `stream`: keep their
        # memory out of the allocator's reach until that stream has read it
        for t in (xd, yd):
            t.record_stream(stream)
    if grid:
        h, w = yd.numel(), xd.numel()
    else:
        h, w = xd.shape
    ox = torch().empty((h, w), dtype=torch().float64, device=device)
    oy = torch().empty((h, w), dtype=torch().float64, device=device)
    steps, nsteps = transformer.device_steps()
    rc = _native.lib().xrs_transform(ptr(xd), ptr(yd), w, h, 1 if grid else 0,
                                     ctypes.cast(steps, ctypes.c_void_p), nsteps, ptr(ox),
                                     ptr(oy), stream_handle(device, stream))
    _native.check(rc, "xrs_transform")
    return ox, oy


# K5a work list: strips of STRIP_H quad rows x STRIP_W quads per tile window
# (xrs_rectify.hip kStripW / kStripH, one wave per strip)
STRIP_W, STRIP_H = 63, 16


def strip_counts(swin, shin):
    """Number of K5a strips over tile windows of swin x shin source pixels."""
    nqi = np.maximum(np.asarray(swin, np.int64) - 1, 0)
    nqj = np.maximum(np.asarray(shin, np.int64) - 1, 0)
    return (nqi + STRIP_W - 1) // STRIP_W * ((nqj + STRIP_H - 1) // STRIP_H)


def _claim_keys(tiles, dst_h, dst_w, device):
    """K5's claim-key scratch and keys_ready: the one K4 filled (DeviceTiles,
    first use), else a fresh one the call fills."""
    k = tiles.take_keys(dst_h, dst_w) if isinstance(tiles, DeviceTiles) else None
    if k is not None and k.device == device:
        return k, 1
    return torch().empty((dst_h, dst_w), dtype=torch().int32, device=device), 0


def _rect_inputs(x_image, y_image, tiles, device, stream=None):
    """Device x/y images, tile records, chunk offsets and the strip count
    of a K5 call (host tiles get their offsets computed here).  Device tiles
    made on another stream are waited for on the K5 stream."""
    x = to_device(x_image, device, np.float64)
    y = to_device(y_image, device, np.float64)
    if isinstance(tiles, np.ndarray):   # host tiles: offsets computed here
        tiles = np.ascontiguousarray(tiles, dtype=TILE_INFO_DTYPE)
        nch = np.where(tiles["si0"] >= 0, strip_counts(tiles["swin"], tiles["shin"]), 0)
        offs_h = np.concatenate([[0], np.cumsum(nch)]).astype(np.int64)
        ntiles, max_chunks = len(tiles), int(offs_h[-1])
        t_dev = torch().from_numpy(tiles.view(np.uint8).copy()).to(device)
        offs = to_device(offs_h, device)
    else:                                 # device tiles from rectify_tiles_device
        t_dev, offs = tiles
        ntiles, max_chunks = offs.numel() - 1, 0
        if isinstance(tiles, DeviceTiles):
            tiles.wait(stream if stream is not None else torch().cuda.current_stream(device))
    return x, y, t_dev, offs, ntiles, max_chunks


def rectify_ij(x_image, y_image, tiles: np.ndarray, ntiles_x: int, dst_h: int, dst_w: int,
               x_scale: float, y_scale: float, uv_delta: float, device=None, stream=None,
               flags: ErrorFlags | None = None, init_nan: bool = False):
    """K5 — per target pixel the fractional source (i, j) (rectify.py:373-576).

    tiles: structured array of TILE_INFO_DTYPE (row-major tile order), or
    the (tiles, chunk offsets) device pair of rectify_tiles_device.
    Returns a device tensor (2, dst_h, dst_w) float64 (NaN = no source pixel).
    An inconsistent tile record or claim key (skipped, never dereferenced)
    raises; with a caller's ``flags`` the caller checks them (no sync here).
    ``init_nan``: the tiles are a subset of the grid (a rank's share,
    sharding.rectify_shard): pixels of the other tiles are NaN, not garbage.
    """
    device = require_device(device)
    x, y, t_dev, offs, ntiles, max_chunks = _rect_inputs(x_image, y_image, tiles, device, stream)
    h, w = x.shape
    keys, keys_ready = _claim_keys(tiles, dst_h, dst_w, device)
    ij = (torch().full((2, dst_h, dst_w), float("nan"), dtype=torch().float64, device=device)
          if init_nan else torch().empty((2, dst_h, dst_w), dtype=torch().float64, device=device))
    own_flags = flags is None
    if own_flags:
        flags = ErrorFlags(device)
    rc = _native.lib().xrs_rectify_ij(ptr(x), ptr(y), h, w, x.stride(0), ptr(t_dev), ntiles,
                                      ntiles_x, ptr(offs), max_chunks, dst_h, dst_w,
                                      float(x_scale), float(y_scale), float(uv_delta),
                                      ptr(keys), keys_ready, ptr(ij), flags.ptr,
                                      stream_handle(device, stream))
    _native.check(rc, "xrs_rectify_ij")
    if own_flags:
        flags.raise_if_set("xrs_rectify_ij")
    return ij


def rectify_ij_var(x_image, y_image, tiles, dst_h: int, dst_w: int, x_scale: float,
                   y_scale: float, uv_delta: float, src, interp: str, fill,
                   keep_ij: bool = True, stream=None, flags: ErrorFlags | None = None):
    """K5 with K6 fused into its resolve pass: the target positions (as
    rectify_ij) and the first variable ``src`` (n, H, W) sampled at them (as
    rectify_var) in one pass — the ij image never makes the HBM round trip
    for that variable.  Returns (ij or None when not ``keep_ij``, out
    (n, dst_h, dst_w) in src dtype); bit-identical to rectify_ij followed by
    rectify_var.  The tiles must cover the whole target grid."""
    device = src.device
    code = _native.INTERP_CODES.get(interp)
    if code is None:
        raise NotImplementedError(
            f"interp_methods must be one of 0, 1, 'nearest', 'bilinear', "
            f"'triangular', was '{interp}'.")
    if src.dim() != 3 or src.stride(2) != 1:
        raise ValueError("src must be (n, H, W) with contiguous rows")
    x, y, t_dev, offs, ntiles, max_chunks = _rect_inputs(x_image, y_image, tiles, device, stream)
    h, w = x.shape
    n, sh, sw = src.shape
    keys, keys_ready = _claim_keys(tiles, dst_h, dst_w, device)
    ij = (torch().empty((2, dst_h, dst_w), dtype=torch().float64, device=device)
          if keep_ij else None)
    out = torch().empty((n, dst_h, dst_w), dtype=src.dtype, device=device)
    own_flags = flags is None
    if own_flags:
        flags = ErrorFlags(device)
    rc = _native.lib().xrs_rectify_ij_var(
        ptr(x), ptr(y), h, w, x.stride(0), ptr(t_dev), ntiles, ptr(offs), max_chunks, dst_h,
        dst_w, float(x_scale), float(y_scale), float(uv_delta), ptr(keys), keys_ready,
        ptr(ij) if ij is not None else None, ptr(src), _native.DTYPE_CODES[_np_dtype(src)], n,
        sh, sw, src.stride(0), src.stride(1), ptr(out), out.stride(0), code, float(fill),
        flags.ptr, stream_handle(device, stream))
    _native.check(rc, "xrs_rectify_ij_var")
    if own_flags:
        flags.raise_if_set("xrs_rectify_ij_var")
    return ij, out


def rectify_var(ij, src, interp: str, fill, stream=None, rows=None, out=None,
                flags: ErrorFlags | None = None):
    """K6 — sample one variable (n, H, W) at the fractional source positions
    `ij` (2, H', W') (rectify.py:605-734).  Returns (n, H', W') in src dtype,
    or with ``rows=(r0, r1)`` the target rows [r0, r1) into ``out`` (n, r1-r0,
    W') (default: a new tensor).  Positions outside the source (never made
    by K5) raise; with a caller's ``flags`` the caller checks them."""
    device = src.device
    code = _native.INTERP_CODES.get(interp)
    if code is None:
        raise NotImplementedError(
            f"interp_methods must be one of 0, 1, 'nearest', 'bilinear', "
            f"'triangular', was '{interp}'.")
    n, h, w = src.shape
    _, dh, dw = ij.shape
    r0, r1 = rows if rows is not None else (0, dh)
    if not 0 <= r0 < r1 <= dh:
        raise ValueError(f"rows {rows} outside the target's {dh} rows")
    if out is None:
        out = torch().empty((n, r1 - r0, dw), dtype=src.dtype, device=device)
    elif tuple(out.shape) != (n, r1 - r0, dw) or out.dtype != src.dtype or \
            out.stride()[1:] != (dw, 1):
        raise ValueError("out must be (n, rows, W') in the source dtype, rows contiguous")
    ij = ij.contiguous()
    own_flags = flags is None
    if own_flags:
        flags = ErrorFlags(device)
    rc = _native.lib().xrs_rectify_var(
        ptr(ij) + r0 * dw * 8, dh * dw, r1 - r0, dw, ptr(src),
        _native.DTYPE_CODES[_np_dtype(src)], n, h, w, src.stride(0), src.stride(1), ptr(out),
        out.stride(0), code, float(fill), flags.ptr, stream_handle(device, stream))
    _native.check(rc, "xrs_rectify_var")
    if own_flags:
        flags.raise_if_set("xrs_rectify_var")
    return out


_WORKSPACES: "collections.OrderedDict" = collections.OrderedDict()
_WORKSPACES_MAX = 8          # (device, stream) entries kept (least recently used dropped)
_WORKSPACES_LOCK = threading.Lock()


def _workspace(device, nbytes: int, stream=None):
    """K2/K3's scratch for launches on `stream` (default: the current stream),
    reused across calls.  Keyed by (device, stream) and allocated on that
    stream: launches of one stream are ordered, so they may share it, while
    partitions running on other streams of the same device (multidevice,
    a threaded chunk scheduler) each get their own.  At most _WORKSPACES_MAX
    entries are kept, least recently used dropped first (the band pipelines
    and multi-device parts take a fresh pool stream per call): a
    dropped workspace returns to torch's caching allocator in the pool of the
    stream it was allocated on, so only later work on that same stream — ordered
    after the launches that used it — can reuse its memory."""
    t = torch()
    s = stream if stream is not None else t.cuda.current_stream(device)
    key = (str(device), int(s.cuda_stream))
    with _WORKSPACES_LOCK:
        ws = _WORKSPACES.get(key)
        if ws is not None:
            _WORKSPACES.move_to_end(key)
    if ws is None or ws.numel() < nbytes:
        with t.cuda.stream(s):
            ws = t.empty(max(nbytes, 1), dtype=t.uint8, device=device)
        with _WORKSPACES_LOCK:
            _WORKSPACES[key] = ws
            _WORKSPACES.move_to_end(key)
            while len(_WORKSPACES) > _WORKSPACES_MAX:
                _WORKSPACES.popitem(last=False)
    return ws


def reserve_affine_workspace(device, ih: int, iw: int, stream=None) -> None:
    """Allocate the K2/K3 workspace of `stream` for an (ih, iw) intermediate
    up front (a band pipeline must not reallocate it while launches are in
    flight)."""
    _workspace(device, _native.lib().xrs_affine_workspace_size(ih, iw), stream)


def any_nan(src, stream=None) -> bool:
    """da.any(da.isnan(array)) on the device (affine.py:347-349)."""
    device = src.device
    flag = torch().zeros(1, dtype=torch().int32, device=device)
    rc = _native.lib().xrs_any_nan(ptr(src), _native.DTYPE_CODES[_np_dtype(src)], src.numel(),
                                   ptr(flag), stream_handle(device, stream))
    _native.check(rc, "xrs_any_nan")
    return bool(flag.item())


def affine(src, plan, out=None, stream=None):
    """K2/K3 — scipy order-0/1 affine resampling per dask-image chunk, fused
    with the coarsen reducer when ``plan.div`` > 1.

    src: device tensor (nt, H, W); plan: affine.AffinePlan.
    Returns the device tensor (nt, out_h, out_w) in ``plan.out_dtype``.
    """
    device = src.device
    nt, h, w = src.shape
    if out is None:
        out = empty((nt, plan.out_h, plan.out_w), plan.out_dtype, device)
    tabs = plan.device_tables(device)
    lib = _native.lib()
    ih, iw = plan.out_h * plan.div_y, plan.out_w * plan.div_x
    nbytes = lib.xrs_affine_workspace_size(ih, iw)
    ws = _workspace(device, nbytes, stream)
    st, sy, sx = src.stride()
    dt, dy, dx = out.stride()
    if sx != 1 or dx != 1:
        raise ValueError("innermost dimension must be contiguous")
    out_code = _native.dtype_code(np.int64 if np.dtype(plan.out_dtype) == np.uint64
                                  else plan.out_dtype)
    rc = lib.xrs_affine(
        ptr(src), _native.DTYPE_CODES[_np_dtype(src)], nt, h, w, st, sy,
        ptr(out), out_code, plan.out_h, plan.out_w, dt, dy, plan.div_y, plan.div_x,
        plan.agg_code, plan.order, float(plan.scale_y), float(plan.scale_x),
        plan.chunk_y, ptr(tabs["rel_y"]), ptr(tabs["len_y"]), ptr(tabs["off_y"]),
        plan.chunk_x, ptr(tabs["rel_x"]), ptr(tabs["len_x"]), ptr(tabs["off_x"]),
        ptr(tabs["t_next"]) if tabs["t_next"] is not None else None,
        float(plan.cval), int(plan.recover_nan), 1 if plan.run_weights else 0, ptr(ws), nbytes,
        stream_handle(device, stream))
    _native.check(rc, "xrs_affine")
    return out


def coarsen(src, div_y: int, div_x: int, agg: str, out_dtype, chunk_ids=None, out=None,
            stream=None):
    """K7 — da.coarsen(agg, src, {1: div_y, 2: div_x}) on a device tensor
    (nt, H, W) (affine.py:308-310 -> dask chunk.coarsen -> coarsen.py).

    chunk_ids: for ``mode`` on float data, the dask chunk id of every slice,
    row and column: ``(ct, cy, cx)`` int32 numpy arrays (coarsen.py:133 takes
    the offset from the chunk minimum).  Returns (nt, H/div_y, W/div_x) in
    ``out_dtype`` (uint64 results are produced as int64 bits).
    """
    device = src.device
    code = _native.AGG_CODES.get(agg)
    if code is None:
        raise NotImplementedError(f"aggregation method {agg!r} is not supported")
    nt, h, w = src.shape
    if h % div_y or w % div_x:
        raise ValueError(f"Coarsening factors {{1: {div_y}, 2: {div_x}}} do not align with "
                         f"array shape {tuple(src.shape)}.")
    if out is None:
        out = empty((nt, h // div_y, w // div_x), out_dtype, device)
    st, sy, sx = src.stride()
    dt, dy, dx = out.stride()
    if sx != 1 or dx != 1:
        raise ValueError("innermost dimension must be contiguous")
    out_code = _native.dtype_code(np.int64 if np.dtype(out_dtype) == np.uint64 else out_dtype)
    lib = _native.lib()
    flags = ErrorFlags(device)
    ct = cy = cx = None
    ncounts = (0, 0, 0)
    ws, ws_bytes = None, 0
    if chunk_ids is not None:
        ct, cy, cx = (to_device(np.ascontiguousarray(c, np.int32), device) for c in chunk_ids)
        ncounts = tuple(int(np.max(c)) + 1 for c in chunk_ids)
        ws_bytes = lib.xrs_coarsen_workspace_size(ncounts[0] * ncounts[1] * ncounts[2])
        ws = torch().empty(max(ws_bytes, 1), dtype=torch().uint8, device=device)
    rc = lib.xrs_coarsen(
        ptr(src), _native.DTYPE_CODES[_np_dtype(src)], nt, h, w, st, sy, ptr(out), out_code, dt,
        dy, div_y, div_x, code, ptr(ct) if ct is not None else None,
        ptr(cy) if cy is not None else None, ptr(cx) if cx is not None else None, *ncounts,
        ptr(ws) if ws is not None else None, ws_bytes, flags.ptr, stream_handle(device, stream))
    _native.check(rc, "xrs_coarsen")
    if code == _native.AGG_CODES["mode"]:
        flags.raise_if_set("coarsen")
    return out

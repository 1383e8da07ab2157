"""Device-level seams: one Python function per C-ABI entry point.

Each function takes device tensors (torch CUDA tensors = HIP allocations) and
host-side plan objects, launches the libxrs kernel on the current HIP stream
and returns device tensors.  These are the functions a dask/xarray
orchestration would call per chunk in place of the reference's block
callables; the Dataset-level API in reproject.py / affine.py /
rectify.py is built on them.
"""

from __future__ import annotations

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
    if out is None:
        out = empty((n, r1 - r0, plan.dst_width), out_dtype, device)
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
    rc = lib.xrs_reproject(
        ptr(src), src_dtype, n, plan.src_height, plan.src_width, src_row0, h_band, sn, sy,
        ptr(out), _native.dtype_code(out_dtype), plan.dst_height, plan.dst_width, r0, r1,
        dn, dy, plan.tile_height, plan.tile_width,
        ptr(tables["src_x"]), ptr(tables["src_y"]), plan.coord_mode,
        ptr(tables["tile_x0"]), ptr(tables["tile_y0"]), ptr(tables["tile_win"]),
        plan.win_height, plan.win_width, float(plan.x_res), float(plan.y_res),
        interp_code, float(fill), ptr(ws) if ws is not None else None, ws_bytes, flags.ptr,
        stream_handle(device, stream))
    _native.check(rc, "xrs_reproject")
    if own_flags and check:
        flags.raise_if_set("reproject")
    return out


def _np_dtype(t) -> np.dtype:
    from .device import numpy_dtype
    return numpy_dtype(t.dtype)


def ij_bboxes(x_image, y_image, xy_bboxes, xy_border, ij_border):  # K4 (rectify path)
    raise NotImplementedError("ij_bboxes kernel not built yet")

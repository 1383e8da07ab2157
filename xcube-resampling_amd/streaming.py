"""Host-resident rasters: band-wise H2D -> kernel -> D2H pipeline.

The reference takes numpy arrays and returns computed numpy arrays
(reproject.py:208-213, 254-255).  A device round trip of a whole raster
through pageable memory serialises three steps that each take far longer than
the kernel (40960^2 f32: 6.7 GB in, 6.7 GB out, ~2.6 ms of K1).  Here the
source and result arrays are page-locked in place (``xrs_host_register``) and
the target is processed in bands of target rows on three HIP streams:

    copy-in  : source rows a band needs that are not yet resident -> HBM
    kernel   : K1 over the band's target rows (waits for its rows)
    copy-out : the band's result -> the host array (waits for the kernel)

so the PCIe transfers in both directions overlap each other and the kernels.
The device holds the whole source (288 GB of HBM per MI355X; a 40960^2 f32
raster is 6.7 GB) and two band-sized result buffers.  Results are bit-identical
to the resident path: the same K1 launch, restricted to the band's rows.
"""

from __future__ import annotations

import ctypes

import numpy as np

from . import _native, kernels
from .constants import LOG
from .device import empty, numpy_dtype, require_device, stream_handle, to_device, torch
from .options import get_options


class HostPin:
    """Page-lock a C-contiguous numpy array in place for the lifetime of the
    context (no copy).  Memory that is already registered stays as it is;
    memory the runtime refuses to lock (e.g. a file-backed np.memmap) stays
    pageable — the copies are then staged by the runtime: slower, same bytes."""

    def __init__(self, array: np.ndarray):
        if not array.flags.c_contiguous:
            raise ValueError("HostPin needs a C-contiguous array")
        self.array = array
        self._registered = False

    def __enter__(self):
        if self.array.nbytes:
            rc = _native.lib().xrs_host_register(
                ctypes.c_void_p(self.array.ctypes.data), self.array.nbytes)
            if rc == _native.XRS_ERR_ARG:
                _native.check(rc, "xrs_host_register")
            if rc == _native.XRS_ERR_HIP:
                LOG.debug("host array not page-locked (%s); copies are staged",
                          _native.last_error())
            self._registered = rc == _native.XRS_OK
        return self.array

    def __exit__(self, *exc):
        if self._registered:
            self._registered = False
            _native.check(_native.lib().xrs_host_unregister(
                ctypes.c_void_p(self.array.ctypes.data)), "xrs_host_unregister")
        return False


def _copy(dst_ptr: int, src_ptr: int, nbytes: int, stream) -> None:
    rc = _native.lib().xrs_copy_async(ctypes.c_void_p(dst_ptr), ctypes.c_void_p(src_ptr),
                                      int(nbytes), stream_handle(stream=stream))
    _native.check(rc, "xrs_copy_async")


def host_to_device(arr, device, dtype=None):
    """numpy -> device tensor.  Arrays of at least ``host_streaming_min_bytes``
    are page-locked in place and copied by DMA (no pageable staging copy);
    smaller ones take torch's copy."""
    if not isinstance(arr, np.ndarray):
        return to_device(arr, device, dtype)
    arr = np.ascontiguousarray(arr if dtype is None else arr.astype(dtype, copy=False))
    if arr.nbytes < max(1, get_options()["host_streaming_min_bytes"]) or \
            arr.dtype not in _native.DTYPE_CODES:
        return to_device(arr, device)
    dst = empty(arr.shape, arr.dtype, device)
    stream = torch().cuda.current_stream(device)
    with HostPin(arr):
        try:
            _copy(dst.data_ptr(), arr.ctypes.data, arr.nbytes, stream)
        finally:   # the copy has landed before the array is unpinned
            stream.synchronize()
    return dst


def device_to_host(x) -> np.ndarray:
    """device tensor -> numpy, by DMA into a page-locked result for tensors of
    at least ``host_streaming_min_bytes``."""
    nbytes = x.numel() * x.element_size()
    if nbytes < max(1, get_options()["host_streaming_min_bytes"]):
        return x.cpu().numpy()
    x = x.contiguous()
    out = np.empty(tuple(x.shape), numpy_dtype(x.dtype))
    stream = torch().cuda.current_stream(x.device)
    with HostPin(out):
        try:
            _copy(out.ctypes.data, x.data_ptr(), nbytes, stream)
        finally:
            stream.synchronize()
    return out


def band_ranges(height: int, band_rows: int) -> list[tuple[int, int]]:
    """Target row bands [r0, r1) of `band_rows` rows (the last one shorter)."""
    if band_rows < 1:
        raise ValueError("band_rows must be >= 1")
    return [(r0, min(height, r0 + band_rows)) for r0 in range(0, height, band_rows)]


def band_source_rows(plan, bands) -> list[tuple[int, int]]:
    """Source rows [j0, j1) each band reads (the union of its tiles' windows,
    ReprojectPlan.source_rows_for), with j1 made non-decreasing: band b is
    computed once rows [0, j1_b) are resident."""
    out, hi = [], 0
    for r0, r1 in bands:
        j0, j1 = plan.source_rows_for(r0, r1)
        hi = max(hi, j1)
        out.append((j0, hi))
    return out


def reproject_host(src: np.ndarray, plan, interp: str, fill: float, out_dtype=None,
                   band_rows: int | None = None, device=None,
                   out: np.ndarray | None = None) -> np.ndarray:
    """K1 over a host-resident (n, H, W) source into a host (n, H', W') result,
    streamed band by band (see the module docstring).  Same values as
    ``kernels.reproject`` on a resident copy of `src`."""
    t = torch()
    device = require_device(device)
    if src.ndim != 3:
        raise ValueError("src must have shape (n, height, width)")
    src = np.ascontiguousarray(src)
    n, h, w = src.shape
    if w != plan.src_width or h != plan.src_height:
        raise ValueError(f"source shape {src.shape[1:]} does not match the plan "
                         f"({plan.src_height}, {plan.src_width})")
    if interp not in _native.INTERP_CODES:
        raise NotImplementedError(
            f"interp_methods must be one of 0, 1, 'nearest', 'bilinear', 'triangular', "
            f"was '{interp}'.")
    if out_dtype is None:
        out_dtype = np.float64 if interp == "bilinear" else src.dtype
    out_dtype = np.dtype(out_dtype)
    hd, wd = plan.dst_height, plan.dst_width
    if out is None:
        out = np.empty((n, hd, wd), out_dtype)
    elif out.shape != (n, hd, wd) or out.dtype != out_dtype or not out.flags.c_contiguous:
        raise ValueError("out must be a C-contiguous (n, H', W') array of the output dtype")
    band_rows = int(band_rows or plan.tile_height)
    bands = band_ranges(hd, band_rows)
    src_rows = band_source_rows(plan, bands)

    dsrc = empty((n, h, w), src.dtype, device)
    bufs = [empty((n, min(band_rows, hd), wd), out_dtype, device) for _ in range(2)]
    cur = t.cuda.current_stream(device)
    s_in, s_k, s_out = (t.cuda.Stream(device) for _ in range(3))
    flags = kernels.ErrorFlags(device)
    plan.device_tables(device)   # uploaded on the current stream, before the others start
    for s in (s_in, s_k, s_out):
        s.wait_stream(cur)
    row_src, row_dst = w * src.itemsize, wd * out_dtype.itemsize
    freed: list = [None, None]
    with HostPin(src), HostPin(out):
        try:
            hi = 0
            for b, ((r0, r1), (_, j1)) in enumerate(zip(bands, src_rows)):
                if j1 > hi:   # rows [hi, j1) of every slice (contiguous per slice)
                    for s in range(n):
                        _copy(dsrc[s, hi].data_ptr(), src[s, hi:j1].ctypes.data,
                              (j1 - hi) * row_src, s_in)
                    hi = j1
                ev_in = t.cuda.Event()
                ev_in.record(s_in)
                s_k.wait_event(ev_in)
                if freed[b % 2] is not None:   # the copy-out of band b-2 has drained
                    s_k.wait_event(freed[b % 2])
                buf = bufs[b % 2][:, :r1 - r0]
                kernels.reproject(dsrc, plan, interp, fill, out_dtype=out_dtype, rows=(r0, r1),
                                  out=buf, flags=flags, stream=s_k)
                ev_k = t.cuda.Event()
                ev_k.record(s_k)
                s_out.wait_event(ev_k)
                for s in range(n):
                    _copy(out[s, r0:r1].ctypes.data, buf[s].data_ptr(), (r1 - r0) * row_dst,
                          s_out)
                freed[b % 2] = t.cuda.Event()
                freed[b % 2].record(s_out)
        finally:   # never unpin (or free) while a copy may still be in flight
            s_in.synchronize()
            s_k.synchronize()
            s_out.synchronize()
    flags.raise_if_set("reproject")
    return out

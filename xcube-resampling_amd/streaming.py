"""Host-resident rasters: band-wise H2D -> kernel -> D2H pipeline.

The reference takes numpy arrays and returns computed numpy arrays
(reproject.py:208-213, 254-255).  A device round trip of a whole raster
through pageable memory serialises three steps that each take far longer than
the kernel (40960^2 f32: 6.7 GB in, 6.7 GB out, ~2.6 ms of K1).  Here every
host <-> device copy goes through two page-locked staging buffers (the host
copies one chunk while the DMA engine moves the other, `_Staging`) and the
target is processed in bands of target rows on three HIP streams:

    copy-in  : source rows a band needs that are not yet resident -> HBM
    kernel   : K1 over the band's target rows (waits for its rows)
    copy-out : the band's result -> the host array (waits for the kernel)

so the PCIe transfers in both directions overlap each other and the kernels.
The device holds the whole source (288 GB of HBM per MI355X; a 40960^2 f32
raster is 6.7 GB) and two band-sized result buffers.  Results are bit-identical
to the resident path: the same K1 launch, restricted to the band's rows.
"""

from __future__ import annotations

import contextlib
import ctypes
import threading

import numpy as np

from . import _native, kernels
from .constants import LOG
from .device import empty, numpy_dtype, require_device, stream_handle, to_device, torch
from .options import get_options


def _copy(dst_ptr: int, src_ptr: int, nbytes: int, stream) -> None:
    rc = _native.lib().xrs_copy_async(ctypes.c_void_p(dst_ptr), ctypes.c_void_p(src_ptr),
                                      int(nbytes), stream_handle(stream=stream))
    _native.check(rc, "xrs_copy_async")


_STAGE_BYTES = 16 << 20     # one staging buffer
_COPY_PART = 2 << 20        # host copies are split over threads in parts of this size
_COPY_POOL = None


def _host_copy(dst: np.ndarray, src: np.ndarray) -> None:
    """dst[:] = src for flat uint8 views, over a small thread pool (numpy's
    contiguous copy releases the GIL): the staging copies run at several
    times one thread's memcpy rate."""
    global _COPY_POOL
    n = dst.size
    if n <= _COPY_PART:
        dst[:] = src
        return
    if _COPY_POOL is None:
        from concurrent.futures import ThreadPoolExecutor
        _COPY_POOL = ThreadPoolExecutor(max_workers=8, thread_name_prefix="xrs-stage")
    parts = [(o, min(n, o + _COPY_PART)) for o in range(0, n, _COPY_PART)]

    def one(p):
        dst[p[0]:p[1]] = src[p[0]:p[1]]

    list(_COPY_POOL.map(one, parts))


class _Staging:
    """Two page-locked host buffers (torch's pinned allocator: allocated once
    per process, never registered / unregistered per call) through which the
    streamed host <-> device copies go: the host copies a chunk into (out of)
    one buffer while the DMA engine moves the other.  Arrays of the caller
    are never page-locked in place: after hipHostRegister / hipHostUnregister
    of arrays the caller then freed, a later pageable copy from a new array
    faulted with an illegal address (twice in the GPU suite, at the first
    copy after such a sequence) — staging removes that pattern."""

    def __init__(self):
        t = torch()
        self.bufs = [t.empty(_STAGE_BYTES, dtype=t.uint8, pin_memory=True) for _ in range(2)]
        self.views = [b.numpy() for b in self.bufs]
        self.events = [None, None]   # the last DMA that used each buffer
        self.k = 0

    def _take(self) -> int:
        i, self.k = self.k, self.k ^ 1
        if self.events[i] is not None:
            self.events[i].synchronize()
            self.events[i] = None
        return i

    def _record(self, i: int, stream) -> None:
        ev = torch().cuda.Event()
        ev.record(stream)
        self.events[i] = ev

    def h2d(self, dst_ptr: int, src: np.ndarray, stream) -> None:
        """C-contiguous host array -> device bytes at dst_ptr, on `stream`.
        Returns once every chunk is queued (a buffer is refilled only after
        its previous DMA has completed)."""
        flat = np.ascontiguousarray(src).reshape(-1).view(np.uint8)
        for off in range(0, flat.size, _STAGE_BYTES):
            nb = min(_STAGE_BYTES, flat.size - off)
            i = self._take()
            _host_copy(self.views[i][:nb], flat[off:off + nb])
            _copy(dst_ptr + off, self.bufs[i].data_ptr(), nb, stream)
            self._record(i, stream)

    def d2h(self, dst: np.ndarray, src_ptr: int, stream) -> None:
        """Device bytes at src_ptr -> C-contiguous host array `dst`, on
        `stream`; returns when they have landed in `dst`."""
        flat = dst.reshape(-1).view(np.uint8)
        pending = None
        for off in range(0, flat.size, _STAGE_BYTES):
            nb = min(_STAGE_BYTES, flat.size - off)
            i = self._take()
            _copy(self.bufs[i].data_ptr(), src_ptr + off, nb, stream)
            self._record(i, stream)
            if pending is not None:
                self._drain(flat, *pending)
            pending = (i, off, nb)
        if pending is not None:
            self._drain(flat, *pending)

    def _drain(self, flat: np.ndarray, i: int, off: int, nb: int) -> None:
        self.events[i].synchronize()
        self.events[i] = None
        _host_copy(flat[off:off + nb], self.views[i][:nb])

    def drain(self) -> None:
        """Wait for every DMA still using a buffer."""
        for i in range(2):
            if self.events[i] is not None:
                self.events[i].synchronize()
                self.events[i] = None


_POOL_MAX = 8                # staging pairs a process keeps at most (8 x 32 MiB page-locked)
_POOL_COND = threading.Condition()
_POOL_FREE: list = []
_POOL_MADE = 0


@contextlib.contextmanager
def _staging():
    """A pair of staging buffers, borrowed for one streamed transfer.  A
    _Staging holds state (the buffer index, the events of the DMAs still using
    each buffer) that two threads must not interleave, so a thread takes a
    pair from a small process-wide pool and returns it drained; at most
    _POOL_MAX pairs are ever allocated (a threaded chunk scheduler with many
    workers waits for a free pair instead of pinning 32 MiB per thread,
    ADVICE r04)."""
    global _POOL_MADE
    with _POOL_COND:
        while not _POOL_FREE and _POOL_MADE >= _POOL_MAX:
            _POOL_COND.wait()
        if _POOL_FREE:
            st = _POOL_FREE.pop()
        else:
            _POOL_MADE += 1
            st = None
    if st is None:
        try:
            st = _Staging()
        except BaseException:
            with _POOL_COND:
                _POOL_MADE -= 1
                _POOL_COND.notify()
            raise
    try:
        yield st
    finally:
        try:
            st.drain()
        finally:
            with _POOL_COND:
                _POOL_FREE.append(st)
                _POOL_COND.notify()


def _small(nbytes: int) -> bool:
    return nbytes < max(1, get_options()["host_streaming_min_bytes"])


def host_to_device(arr, device, dtype=None):
    """numpy -> device tensor.  Arrays of at least ``host_streaming_min_bytes``
    go through the page-locked staging buffers (DMA overlapped with the host
    copy); smaller ones take torch's copy."""
    if not isinstance(arr, np.ndarray):
        return to_device(arr, device, dtype)
    arr = np.ascontiguousarray(arr if dtype is None else arr.astype(dtype, copy=False))
    if _small(arr.nbytes) or arr.dtype not in _native.DTYPE_CODES:
        return to_device(arr, device)
    dst = empty(arr.shape, arr.dtype, device)
    with _staging() as st:
        st.h2d(dst.data_ptr(), arr, torch().cuda.current_stream(device))
    return dst


def host_rows_to_device(arr: np.ndarray, j0: int, j1: int, device):
    """Rows [j0, j1) of every slice of a host (n, H, W) array as a contiguous
    device tensor (n, j1 - j0, W), slice by slice through the staging buffers
    (no host copy of the strided band first)."""
    n, _, w = arr.shape
    rows = max(0, j1 - j0)
    dst = empty((n, rows, w), arr.dtype, device)
    if rows == 0:
        return dst
    if _small(n * rows * w * arr.itemsize) or arr.dtype not in _native.DTYPE_CODES:
        dst.copy_(torch().from_numpy(np.ascontiguousarray(arr[:, j0:j1])))
        return dst
    stream = torch().cuda.current_stream(device)
    with _staging() as st:
        for s in range(n):
            st.h2d(dst[s].data_ptr(), arr[s, j0:j1], stream)
    return dst


def device_to_host(x) -> np.ndarray:
    """device tensor -> numpy through the page-locked staging buffers, for
    tensors of at least ``host_streaming_min_bytes``."""
    if _small(x.numel() * x.element_size()):
        return x.cpu().numpy()
    out = np.empty(tuple(x.shape), numpy_dtype(x.dtype))
    device_to_host_into(out, x)
    return out


def device_to_host_into(out: np.ndarray, x) -> None:
    """out[...] = x (device tensor of out's shape), slice by slice through the
    staging buffers; `out` may be a strided view of a C-contiguous array whose
    last two axes are contiguous per slice (a row band of a result)."""
    if _small(x.numel() * x.element_size()) or out.ndim != 3:
        out[...] = x.cpu().numpy()
        return
    x = x.contiguous()
    stream = torch().cuda.current_stream(x.device)
    with _staging() as st:
        for s in range(out.shape[0]):
            dst = out[s]
            if dst.flags.c_contiguous:
                st.d2h(dst, x[s].data_ptr(), stream)
            else:
                tmp = np.empty(dst.shape, dst.dtype)
                st.d2h(tmp, x[s].data_ptr(), stream)
                dst[...] = tmp


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
    # the plan's device inputs are uploaded on the current stream, before the
    # others start: the grid axes when the transformation is fused into the
    # gather (no 2-D coordinate tables: reproject_table_max_bytes holds here
    # too), else the coordinate tables
    if plan.fused_transform(device):
        plan.device_grid(device)
    else:
        plan.device_tables(device)
    for s in (s_in, s_k, s_out):
        s.wait_stream(cur)
    with _staging() as st:
        prev = None   # the band whose copy-out is pending: it overlaps the next kernel
        try:
            hi = 0
            for b, ((r0, r1), (_, j1)) in enumerate(zip(bands, src_rows)):
                if j1 > hi:   # rows [hi, j1) of every slice (contiguous per slice)
                    for s in range(n):
                        st.h2d(dsrc[s, hi].data_ptr(), src[s, hi:j1], s_in)
                    hi = j1
                ev_in = t.cuda.Event()
                ev_in.record(s_in)
                s_k.wait_event(ev_in)
                # bufs[b % 2] held band b - 2, whose copy-out has landed (d2h returns
                # when the bytes are in `out`)
                buf = bufs[b % 2][:, :r1 - r0]
                kernels.reproject(dsrc, plan, interp, fill, out_dtype=out_dtype, rows=(r0, r1),
                                  out=buf, flags=flags, stream=s_k)
                ev_k = t.cuda.Event()
                ev_k.record(s_k)
                if prev is not None:
                    _copy_out(st, out, prev, s_out)
                prev = (r0, r1, buf, ev_k)
            if prev is not None:
                _copy_out(st, out, prev, s_out)
        finally:   # nothing may still use the device buffers when they are freed
            st.drain()
            s_in.synchronize()
            s_k.synchronize()
            s_out.synchronize()
    flags.raise_if_set("reproject")
    return out


def _copy_out(st: _Staging, out: np.ndarray, band, s_out) -> None:
    """The result rows [r0, r1) of every slice: device band buffer -> `out`,
    after the band's kernel (event ev_k)."""
    r0, r1, buf, ev_k = band
    s_out.wait_event(ev_k)
    for s in range(out.shape[0]):
        st.d2h(out[s, r0:r1], buf[s].data_ptr(), s_out)


# ---- generic band pipeline (affine / rectify host paths) --------------------------
class _SourceRows:
    """Host -> device copies of source rows on demand: only rows not yet
    resident are copied (in contiguous runs, every dim-0 slice), on `stream`."""

    def __init__(self, src: np.ndarray, dsrc, stream, staging: _Staging):
        self.src, self.dsrc, self.stream, self.staging = src, dsrc, stream, staging
        self.resident = np.zeros(src.shape[1], bool)

    def need(self, j0: int, j1: int) -> None:
        j0, j1 = max(0, int(j0)), min(len(self.resident), int(j1))
        if j1 <= j0:
            return
        missing = np.concatenate([[0], (~self.resident[j0:j1]).astype(np.int8), [0]])
        edges = np.flatnonzero(np.diff(missing))
        for a, b in zip(edges[0::2], edges[1::2]):
            ra, rb = j0 + int(a), j0 + int(b)
            for s in range(self.src.shape[0]):
                self.staging.h2d(self.dsrc[s, ra].data_ptr(), self.src[s, ra:rb], self.stream)
        self.resident[j0:j1] = True


def band_pipeline(src: np.ndarray, dsrc, out: np.ndarray, bands, src_rows, launch,
                  device, poison: bool = False) -> np.ndarray:
    """The three-stream pattern of `reproject_host` for any kernel whose target
    row band [r0, r1) reads only source rows [j0, j1):

        copy-in  : the band's source rows not yet resident -> dsrc
        kernel   : launch(b, r0, r1, buf, stream) writes the band into buf
        copy-out : buf -> out[:, r0:r1]

    `src` / `out` are C-contiguous host arrays (n, H, W) / (n, H', W'), moved
    through the page-locked staging buffers.  ``poison`` (tests): fill the device
    source with NaN bytes first, so a kernel that read a row outside its band's
    [j0, j1) would not match the resident result."""
    t = torch()
    n, hd, wd = out.shape
    band_max = max(r1 - r0 for r0, r1 in bands)
    out_dtype = out.dtype
    bufs = [empty((n, band_max, wd), out_dtype, device) for _ in range(2)]
    if poison:
        dsrc.view(t.uint8).fill_(0xFF)
    cur = t.cuda.current_stream(device)
    s_in, s_k, s_out = (t.cuda.Stream(device) for _ in range(3))
    for s in (s_in, s_k, s_out):
        s.wait_stream(cur)
    with _staging() as st:
        rows = _SourceRows(src, dsrc, s_in, st)
        prev = None   # the band whose copy-out is pending: it overlaps the next kernel
        try:
            for b, ((r0, r1), (j0, j1)) in enumerate(zip(bands, src_rows)):
                rows.need(j0, j1)
                ev_in = t.cuda.Event()
                ev_in.record(s_in)
                s_k.wait_event(ev_in)
                buf = bufs[b % 2][:, :r1 - r0]   # band b - 2's copy-out has landed
                launch(b, r0, r1, buf, s_k)
                ev_k = t.cuda.Event()
                ev_k.record(s_k)
                if prev is not None:
                    _copy_out(st, out, prev, s_out)
                prev = (r0, r1, buf, ev_k)
            if prev is not None:
                _copy_out(st, out, prev, s_out)
        finally:   # nothing may still use the device buffers when they are freed
            st.drain()
            s_in.synchronize()
            s_k.synchronize()
            s_out.synchronize()
    return out


def _band_rows(height: int, row_bytes: int, unit: int, target_bytes: int = 64 << 20) -> int:
    """Rows per band: about `target_bytes` of output, a multiple of `unit`."""
    rows = max(unit, (target_bytes // max(1, row_bytes)) // unit * unit)
    return min(rows, -(-height // unit) * unit)


def rectify_host(src: np.ndarray, ij, interp: str, fill, device=None,
                 band_rows: int | None = None, out: np.ndarray | None = None,
                 poison: bool = False) -> np.ndarray:
    """K6 over a host-resident (n, H, W) variable into a host (n, H', W')
    result, streamed in target row bands (rectify.py:297-298: numpy in, numpy
    out).  Each band needs the source rows its positions ij read: K6 reads rows
    int(j) and int(j) + 1 (rectify.py:663-734), bounded per target row from ij
    on the device.  Same values as ``kernels.rectify_var`` on a resident copy."""
    t = torch()
    device = require_device(device)
    src = np.ascontiguousarray(src)
    n, h, w = src.shape
    _, hd, wd = ij.shape
    if out is None:
        out = np.empty((n, hd, wd), src.dtype)
    jf = ij[1]
    nan = t.isnan(jf)
    lo = t.where(nan, t.full_like(jf, np.inf), jf).amin(dim=1)
    hi = t.where(nan, t.full_like(jf, -np.inf), jf).amax(dim=1)
    lo, hi = lo.cpu().numpy(), hi.cpu().numpy()
    rows = int(band_rows or _band_rows(hd, n * wd * src.itemsize, 8))
    bands = band_ranges(hd, rows)
    src_rows = []
    for r0, r1 in bands:
        blo, bhi = lo[r0:r1].min(), hi[r0:r1].max()
        if not np.isfinite(blo):   # nothing to sample: fill only
            src_rows.append((0, 0))
        else:
            src_rows.append((int(np.floor(blo)), int(np.floor(bhi)) + 2))
    dsrc = empty((n, h, w), src.dtype, device)
    flags = kernels.ErrorFlags(device)

    def launch(b, r0, r1, buf, stream):
        kernels.rectify_var(ij, dsrc, interp, fill, stream=stream, rows=(r0, r1), out=buf,
                            flags=flags)

    band_pipeline(src, dsrc, out, bands, src_rows, launch, device, poison)
    flags.raise_if_set("rectify")
    return out


def affine_host(src: np.ndarray, plan, device=None, band_chunks: int | None = None,
                out: np.ndarray | None = None, poison: bool = False) -> np.ndarray | None:
    """K2 / K3 over a host-resident (nt, H, W) array into a host result,
    streamed in bands of whole output chunk rows (affine.py:227-228: numpy in,
    numpy out).  A band of y-chunks [k0, k1) reads only the dask-image input
    slices of those chunks, rows [rel_y[k], rel_y[k] + len_y[k]); its launch is
    the plan restricted to those chunks (every output pixel depends only on its
    chunk's tables, so the values equal the whole launch's).  Returns None when
    the plan cannot be banded (a separate coarsen pass, or chunks that do not
    hold whole coarsen windows)."""
    import dataclasses

    if plan.post_agg is not None or plan.chunk_y % plan.div_y != 0:
        return None
    device = require_device(device)
    src = np.ascontiguousarray(src)
    nt, h, w = src.shape
    out_dtype = np.dtype(plan.out_dtype)
    if out_dtype == np.uint64:
        return None
    if out is None:
        out = np.empty((nt, plan.out_h, plan.out_w), out_dtype)
    nchunks = len(plan.rel_y)
    rows_per_chunk = plan.chunk_y // plan.div_y        # output rows of a full y-chunk
    per = int(band_chunks or max(1, _band_rows(plan.out_h, nt * plan.out_w * out_dtype.itemsize,
                                               rows_per_chunk) // rows_per_chunk))
    bands, src_rows, plans = [], [], []
    for k0 in range(0, nchunks, per):
        k1 = min(nchunks, k0 + per)
        r0 = k0 * rows_per_chunk
        r1 = min(plan.out_h, k1 * rows_per_chunk)
        bands.append((r0, r1))
        src_rows.append((int(plan.rel_y[k0:k1].min()),
                         int((plan.rel_y[k0:k1] + plan.len_y[k0:k1]).max())))
        plans.append(dataclasses.replace(plan, out_h=r1 - r0, rel_y=plan.rel_y[k0:k1],
                                         len_y=plan.len_y[k0:k1], off_y=plan.off_y[k0:k1],
                                         _cache={}))
    for p in plans:   # small tables, uploaded before the streams start
        p.device_tables(device)
    dsrc = empty((nt, h, w), src.dtype, device)

    def launch(b, r0, r1, buf, stream):
        if b == 0:   # the kernel stream's workspace, sized for the tallest band
            kernels.reserve_affine_workspace(device, max(p.out_h for p in plans) * plan.div_y,
                                             plan.out_w * plan.div_x, stream)
        kernels.affine(dsrc, plans[b], out=buf, stream=stream)

    return band_pipeline(src, dsrc, out, bands, src_rows, launch, device, poison)

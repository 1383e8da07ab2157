"""Several GPUs from one process, behind the dataset API.

The reference cuts a variable into dask chunks and runs the per-chunk inner
loop as independent tasks on dask's threads: ``da.map_blocks(_reproject_block)``
(reproject.py:230-252), the per-tile ``_compute_target_source_ij_block`` and
``_compute_var_image`` blocks (rectify.py:347-370), dask-image's per-chunk
``affine_transform`` (affine.py:336-362).  Here a variable is cut into the
engine's independent partitions —

* reproject: target row bands (``sharding.band_shard``, cost-balanced), each
  device holding only the source rows its band reads;
* affine / coarsen: output chunk row bands (``sharding.coarsen_shard``), each
  device holding only the source rows its chunks' footprints read;
* rectify: runs of target tiles (``sharding.rectify_shard``); coordinates and
  variables are replicated (a tile's source window can lie anywhere);

— and partition i runs on ``devices[i]`` from its own host thread, on its own
HIP stream (``run_parts``).  The C-ABI is re-entrant and stream-ordered, and
no two threads share a stream, a workspace (``kernels._workspace`` is keyed by
stream) or an error-flag word.  Partitions write disjoint target pixels, so
there is no exchange: results are copied into the caller's output, a numpy
array (numpy in, numpy out) or a tensor on the source's device.

The device list comes from the ``devices=`` keyword of the dataset functions
(``use_devices``: this call and the calls it makes, in this thread) or from
``set_options(devices=[...])``.  Repeating a device (``[0, 0]``) runs two
partitions on one GPU from two threads, which is how the one-GPU test box
exercises this code.
"""

from __future__ import annotations

import contextlib
import contextvars

import numpy as np

from .device import empty, is_device_array, torch
from .options import _valid_devices, get_options

_ACTIVE = contextvars.ContextVar("xrs_devices", default=None)


def normalize(devices):
    """The device list as torch devices (None stays None: one device)."""
    if devices is None:
        return None
    if not _valid_devices(devices):
        raise ValueError(f"devices must be a non-empty list of device ordinals or 'cuda:k' "
                         f"strings, was {devices!r}")
    t = torch()
    out = []
    for d in devices:
        if isinstance(d, int):
            out.append(t.device("cuda", d))
        else:
            d = t.device(d)
            # an index-less "cuda" is torch's current device, resolved now (under
            # torch.cuda.set_device(k) it is GPU k, not 0 — ADVICE r05)
            out.append(d if d.index is not None else t.device("cuda", t.cuda.current_device()))
    return out


@contextlib.contextmanager
def use_devices(devices):
    """Run the enclosed calls over `devices` (no-op for None: the option
    ``devices`` then decides).  Context-local, so threads of a chunk
    scheduler calling the dataset functions do not see each other's lists."""
    if devices is None:
        yield
        return
    token = _ACTIVE.set(normalize(devices))
    try:
        yield
    finally:
        _ACTIVE.reset(token)


def active_devices():
    """The device list in force here: the enclosing ``use_devices``, else the
    ``devices`` option, else None (run on the current device)."""
    v = _ACTIVE.get()
    if v is not None:
        return v
    return normalize(get_options()["devices"])


def run_parts(devices, fn, sources=()):
    """``fn(i, device)`` for every part i on ``devices[i]``, each from its own
    host thread with its own HIP stream current; returns the results in part
    order.  Work queued on the current streams of the `sources`' devices (the
    inputs) is complete before any part starts, and every part's stream has
    drained before this returns (results complete, nothing left in flight on
    the parts' memory).  The first exception of any part is re-raised after
    all parts have ended."""
    from concurrent.futures import ThreadPoolExecutor

    for dev in {x.device for x in sources if is_device_array(x)}:
        torch().cuda.current_stream(dev).synchronize()

    def one(i):
        with _part_context(devices[i]):
            return fn(i, devices[i])

    if len(devices) == 1:
        return [one(0)]
    with ThreadPoolExecutor(max_workers=len(devices), thread_name_prefix="xrs-dev") as ex:
        futs = [ex.submit(one, i) for i in range(len(devices))]
        errs = [f.exception() for f in futs]
    for e in errs:
        if e is not None:
            raise e
    return [f.result() for f in futs]


@contextlib.contextmanager
def _part_context(dev):
    """A part's device and stream: `dev` current for this thread, a fresh HIP
    stream current on it (ordered after the thread's default stream), drained
    on exit whatever happened inside."""
    t = torch()
    with t.cuda.device(dev):
        s = t.cuda.Stream(dev)
        s.wait_stream(t.cuda.current_stream(dev))
        try:
            with t.cuda.stream(s):
                yield s
        finally:
            s.synchronize()


def rows_to_device(arr, j0: int, j1: int, device):
    """Rows [j0, j1) of every slice of an (n, H, W) numpy array or device
    tensor, on `device` (a view when the tensor already lives there)."""
    if is_device_array(arr):
        band = arr[:, j0:j1]
        return band if band.device == device else band.to(device)
    from .streaming import host_rows_to_device

    return host_rows_to_device(arr, j0, j1, device)


def output_like(src, shape, dtype):
    """The result of a partitioned call: numpy for numpy sources, a tensor
    on the source's device for device sources."""
    if is_device_array(src):
        return empty(shape, dtype, src.device)
    return np.empty(shape, np.dtype(dtype))


def put_rows(out, r0: int, r1: int, band) -> None:
    """out[:, r0:r1] = band (a device tensor of this part's stream)."""
    if isinstance(out, np.ndarray) and isinstance(band, np.ndarray):
        out[:, r0:r1] = band
    elif isinstance(out, np.ndarray):
        from .streaming import device_to_host_into

        device_to_host_into(out[:, r0:r1], band)
    else:
        out[:, r0:r1].copy_(band)


def put_tiles(out, band, tiles, row0: int) -> None:
    """The pixels of `tiles` (TILE_INFO records) from a band of target rows
    starting at row0 into out (numpy or tensor) — the other tiles of the
    band's rows belong to other parts."""
    if isinstance(out, np.ndarray) and not isinstance(band, np.ndarray):
        from .streaming import device_to_host

        band = device_to_host(band)
    for rec in tiles:
        r, c, th, tw = int(rec["r0"]), int(rec["c0"]), int(rec["th"]), int(rec["tw"])
        src = band[:, r - row0:r - row0 + th, c:c + tw]
        if isinstance(out, np.ndarray):
            out[:, r:r + th, c:c + tw] = src
        else:
            out[:, r:r + th, c:c + tw].copy_(src)

"""Device plumbing: torch-ROCm tensors as device memory, HIP stream handles.

PyTorch is used only as an allocator / stream / collective provider; all pixel
work runs in libxrs.so.  Nothing here computes results on the host.
"""

from __future__ import annotations

import numpy as np

from ._native import NativeLibraryError

_TORCH_DTYPES = None


def torch():
    import torch as _torch
    return _torch


def _torch_dtypes():
    global _TORCH_DTYPES
    if _TORCH_DTYPES is None:
        t = torch()
        _TORCH_DTYPES = {
            np.dtype(np.uint8): t.uint8, np.dtype(np.int8): t.int8,
            np.dtype(np.uint16): t.uint16, np.dtype(np.int16): t.int16,
            np.dtype(np.uint32): t.uint32, np.dtype(np.int32): t.int32,
            np.dtype(np.int64): t.int64, np.dtype(np.float32): t.float32,
            np.dtype(np.float64): t.float64,
        }
    return _TORCH_DTYPES


def torch_dtype(dtype):
    return _torch_dtypes()[np.dtype(dtype)]


def numpy_dtype(tdtype) -> np.dtype:
    for k, v in _torch_dtypes().items():
        if v == tdtype:
            return k
    raise TypeError(f"unsupported torch dtype {tdtype}")


def is_device_array(x) -> bool:
    return type(x).__module__.startswith("torch") and x.is_cuda


def require_device(device=None):
    """The HIP device to run on; raises if none is available (no CPU fallback)."""
    t = torch()
    if not t.cuda.is_available():
        raise NativeLibraryError(
            "xcube_resampling_amd: no HIP device available; the engine runs only "
            "on AMD GPUs (MI355X / gfx950) and has no CPU fallback"
        )
    if device is not None:
        device = t.device(device) if not isinstance(device, t.device) else device
        if device.type == "cuda":
            return device
    # host arrays (numpy's ``.device`` is "cpu") run on the current HIP device
    return t.device("cuda", t.cuda.current_device())


def to_device(x, device, dtype=None):
    """numpy array / torch tensor -> contiguous device tensor."""
    t = torch()
    if isinstance(x, np.ndarray):
        if dtype is not None:
            x = x.astype(dtype, copy=False)
        x = np.ascontiguousarray(x)
        return t.from_numpy(x).to(device, non_blocking=False)
    if type(x).__module__.startswith("torch"):
        x = x.to(device)
        if dtype is not None:
            x = x.to(torch_dtype(dtype))
        return x.contiguous()
    return to_device(np.asarray(x), device, dtype)


def empty(shape, dtype, device):
    if np.dtype(dtype) == np.uint64:  # no torch uint64 arithmetic needed: bits only
        return torch().empty(tuple(shape), dtype=torch().int64, device=device)
    return torch().empty(tuple(shape), dtype=torch_dtype(dtype), device=device)


def stream_handle(device=None, stream=None) -> int:
    """hipStream_t of `stream` (default: torch's current stream on `device`)."""
    t = torch()
    if stream is None:
        stream = t.cuda.current_stream(device)
    return int(stream.cuda_stream)


def ptr(x) -> int:
    return int(x.data_ptr())

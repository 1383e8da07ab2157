"""Engine options (not part of the reference API).

``reproject_bilinear_dtype``:
    "float64" (default) — bilinear reprojection returns float64, exactly what
    the reference returns (float32 values times float64 weights, see
    reproject.py:326-328; dask's declared dtype is not enforced);
    "source" — store the float64 result in the (floating) source dtype, the
    dtype the reference *declares* (reproject.py:241): half the output bytes.

``host_streaming_min_bytes``:
    numpy (host-resident) sources at least this large are reprojected by the
    band-wise H2D -> K1 -> D2H pipeline of ``streaming.reproject_host``
    (page-locked in place, transfers overlapped with the kernels); smaller
    ones are copied whole.  Default 64 MiB; 0 streams every host array.
"""

from __future__ import annotations

import contextlib

_OPTIONS = {"reproject_bilinear_dtype": "float64", "host_streaming_min_bytes": 64 << 20}
_ALLOWED = {"reproject_bilinear_dtype": ("float64", "source"),
            "host_streaming_min_bytes": lambda v: isinstance(v, int) and v >= 0}


def get_options() -> dict:
    return dict(_OPTIONS)


@contextlib.contextmanager
def set_options(**kwargs):
    old = dict(_OPTIONS)
    for k, v in kwargs.items():
        if k not in _OPTIONS:
            raise KeyError(k)
        allowed = _ALLOWED[k]
        if not (allowed(v) if callable(allowed) else v in allowed):
            raise ValueError(f"invalid value {v!r} for option {k}")
        _OPTIONS[k] = v
    try:
        yield
    finally:
        _OPTIONS.clear()
        _OPTIONS.update(old)

"""Engine options (not part of the reference API).

``reproject_bilinear_dtype``:
    "float64" (default) — bilinear reprojection returns float64, exactly what
    the reference returns (float32 values times float64 weights, see
    reproject.py:326-328; dask's declared dtype is not enforced);
    "source" — store the float64 result in the (floating) source dtype, the
    dtype the reference *declares* (reproject.py:241): half the output bytes.
"""

from __future__ import annotations

import contextlib

_OPTIONS = {"reproject_bilinear_dtype": "float64"}
_ALLOWED = {"reproject_bilinear_dtype": ("float64", "source")}


def get_options() -> dict:
    return dict(_OPTIONS)


@contextlib.contextmanager
def set_options(**kwargs):
    old = dict(_OPTIONS)
    for k, v in kwargs.items():
        if k not in _OPTIONS:
            raise KeyError(k)
        if v not in _ALLOWED[k]:
            raise ValueError(f"{k} must be one of {_ALLOWED[k]}")
        _OPTIONS[k] = v
    try:
        yield
    finally:
        _OPTIONS.clear()
        _OPTIONS.update(old)

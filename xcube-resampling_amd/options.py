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

``reproject_table_max_bytes``:
    non-separable CRS pairs (UTM, LAEA, ...): the target pixel centres are
    transformed on the device into 2-D coordinate tables (16 B per target
    pixel) that every variable of the plan reuses — measured faster than
    evaluating the projection inside the gather (8192^2 UTM -> LAEA: 2.95 vs
    3.26 ms for one variable: the projection is f64-compute bound and the
    table traffic overlaps it).  Plans whose tables would exceed this many
    bytes fuse the projection into the gather instead (xrs_reproject_proj: no
    tables, the same values bit for bit).  Default 16 GiB; 0 always fuses.
"""

from __future__ import annotations

import contextlib

_OPTIONS = {"reproject_bilinear_dtype": "float64", "host_streaming_min_bytes": 64 << 20,
            "reproject_table_max_bytes": 16 << 30}
_ALLOWED = {"reproject_bilinear_dtype": ("float64", "source"),
            "host_streaming_min_bytes": lambda v: isinstance(v, int) and v >= 0,
            "reproject_table_max_bytes": lambda v: isinstance(v, int) and v >= 0}


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

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

``devices``:
    None (default) — every call runs on the current HIP device;
    a list of devices (ordinals or "cuda:k" strings, repeats allowed) —
    reproject_dataset / rectify_dataset / affine_transform_dataset (and
    resample_in_space) split each variable's independent partitions over them
    from this one process: one host thread and HIP stream per entry, each
    device holding only the source rows its partition reads
    (``multidevice``).  The dataset functions also take ``devices=`` as a
    keyword (it applies to that call and the calls it makes, in its thread).
"""

from __future__ import annotations

import contextlib

_OPTIONS = {"reproject_bilinear_dtype": "float64", "host_streaming_min_bytes": 64 << 20,
            "reproject_table_max_bytes": 16 << 30, "devices": None}
_ALLOWED = {"reproject_bilinear_dtype": ("float64", "source"),
            "host_streaming_min_bytes": lambda v: isinstance(v, int) and v >= 0,
            "reproject_table_max_bytes": lambda v: isinstance(v, int) and v >= 0,
            "devices": lambda v: v is None or _valid_devices(v)}


def _valid_devices(v) -> bool:
    """A non-empty list / tuple of device ordinals (int >= 0) or "cuda[:k]"
    strings (torch.device objects of type cuda are accepted too)."""
    if isinstance(v, (str, bytes)) or not isinstance(v, (list, tuple)) or len(v) == 0:
        return False
    for d in v:
        if isinstance(d, bool):
            return False
        if isinstance(d, int):
            if d < 0:
                return False
        elif isinstance(d, str):
            if not (d == "cuda" or (d.startswith("cuda:") and d[5:].isdigit())):
                return False
        elif getattr(d, "type", None) != "cuda":
            return False
    return True


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

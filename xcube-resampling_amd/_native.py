"""ctypes binding of libxrs.so (the HIP kernels behind include/xrs.h).

The library is the product: there is no CPU fallback.  If it is missing, or
no HIP device is present, every compute call raises ``NativeLibraryError``.

Load order matters: ``torch`` is imported first so that the process holds ONE
HIP runtime.  libxrs.so's DT_NEEDED ``libamdhip64.so.7`` then resolves to the
runtime torch already loaded (same SONAME), so device pointers and streams
created by torch are valid in the kernels' runtime.
"""

from __future__ import annotations

import ctypes
import os
import re
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PRODUCT_LIB = os.path.join(_HERE, "lib", "libxrs.so")
PROBE_DIR = os.path.join(os.path.dirname(_HERE), "probe")


def _library_path() -> str:
    """The product library, or — for A/B timing scripts only — an arm built
    under the repository's probe/ directory named by XRS_LIBRARY (any other
    path is refused: the environment cannot substitute a product binary)."""
    path = os.environ.get("XRS_LIBRARY")
    if not path:
        return PRODUCT_LIB
    real = os.path.realpath(path)
    if real == os.path.realpath(PRODUCT_LIB) or \
            real.startswith(os.path.realpath(PROBE_DIR) + os.sep):
        return real
    raise NativeLibraryError(
        f"XRS_LIBRARY={path!r}: only the product library or an A/B arm under "
        f"{PROBE_DIR} may be loaded")


_LIB_PATH_ERROR = None
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "xrs.h")

XRS_OK = 0
XRS_ERR_ARG = -1
XRS_ERR_HIP = -2
XRS_ERR_NOTIMPL = -3

XRS_EFLAG_INDEX = 1
XRS_EFLAG_BAND = 2
XRS_EFLAG_NAN_TO_INT = 4
XRS_EFLAG_INF_TO_INT = 8
XRS_EFLAG_STATE = 16

INTERP_CODES = {"nearest": 0, "bilinear": 1, "triangular": 2}

DTYPE_CODES = {
    np.dtype(np.uint8): 1,
    np.dtype(np.int8): 2,
    np.dtype(np.uint16): 3,
    np.dtype(np.int16): 4,
    np.dtype(np.uint32): 5,
    np.dtype(np.int32): 6,
    np.dtype(np.int64): 7,
    np.dtype(np.float32): 10,
    np.dtype(np.float64): 11,
}


class NativeLibraryError(RuntimeError):
    """libxrs.so could not be loaded or a HIP call failed."""


try:   # the library this process loads (XRS_LIBRARY: probe arms only)
    LIB_PATH = _library_path()
except NativeLibraryError as _e:
    LIB_PATH, _LIB_PATH_ERROR = None, _e


_c_i64 = ctypes.c_int64
_c_int = ctypes.c_int
_c_dbl = ctypes.c_double
_c_ptr = ctypes.c_void_p

# argument lists, in declaration order of include/xrs.h
_SIGNATURES = {
    "xrs_version": (ctypes.c_char_p, []),
    "xrs_last_error": (ctypes.c_char_p, []),
    "xrs_host_register": (_c_int, [_c_ptr, _c_i64]),
    "xrs_host_unregister": (_c_int, [_c_ptr, _c_ptr, _c_i64]),
    "xrs_copy_async": (_c_int, [_c_ptr, _c_ptr, _c_i64, _c_ptr]),
    "xrs_reproject": (_c_int, [
        _c_ptr, _c_int, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64,  # src
        _c_ptr, _c_int, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64,          # dst
        _c_i64, _c_i64,                                                          # tile
        _c_ptr, _c_ptr, _c_int,                                                  # coords
        _c_ptr, _c_ptr, _c_ptr, _c_i64, _c_i64,                                  # tile tables
        _c_dbl, _c_dbl, _c_int, _c_dbl,                                          # res, interp, fill
        _c_ptr, _c_i64, _c_ptr, _c_ptr,                                          # ws, flags, stream
    ]),
    "xrs_reproject_workspace_size": (_c_i64, [_c_i64, _c_i64, _c_i64, _c_i64, _c_int]),
    "xrs_affine_workspace_size": (_c_i64, [_c_i64, _c_i64]),
    "xrs_affine": (_c_int, [
        _c_ptr, _c_int, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64,                  # src
        _c_ptr, _c_int, _c_i64, _c_i64, _c_i64, _c_i64,                          # dst
        _c_i64, _c_i64, _c_int, _c_int, _c_dbl, _c_dbl,                          # div, agg, order, scale
        _c_i64, _c_ptr, _c_ptr, _c_ptr,                                          # y chunks
        _c_i64, _c_ptr, _c_ptr, _c_ptr,                                          # x chunks
        _c_ptr, _c_dbl, _c_int, _c_int, _c_ptr, _c_i64, _c_ptr,                  # t_next .. stream
    ]),
    "xrs_coarsen_workspace_size": (_c_i64, [_c_i64]),
    "xrs_coarsen": (_c_int, [
        _c_ptr, _c_int, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64,                  # src
        _c_ptr, _c_int, _c_i64, _c_i64,                                          # dst
        _c_i64, _c_i64, _c_int,                                                  # div, agg
        _c_ptr, _c_ptr, _c_ptr, _c_i64, _c_i64, _c_i64,                          # chunk ids
        _c_ptr, _c_i64, _c_ptr, _c_ptr,                                          # ws, flags, stream
    ]),
    "xrs_any_nan": (_c_int, [_c_ptr, _c_int, _c_i64, _c_ptr, _c_ptr]),
    "xrs_ij_bboxes": (_c_int, [_c_ptr, _c_ptr, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64,
                               _c_ptr, _c_ptr, _c_ptr, _c_ptr]),
    "xrs_ij_bboxes_fill": (_c_int, [_c_ptr, _c_ptr, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64,
                                    _c_i64, _c_ptr, _c_ptr, _c_ptr, _c_ptr, _c_i64, _c_ptr]),
    "xrs_rectify_ij": (_c_int, [_c_ptr, _c_ptr, _c_i64, _c_i64, _c_i64, _c_ptr, _c_i64, _c_i64,
                                _c_ptr, _c_i64, _c_i64, _c_i64, _c_dbl, _c_dbl, _c_dbl,
                                _c_ptr, _c_int, _c_ptr, _c_ptr, _c_ptr]),   # keys, keys_ready, ij
    "xrs_rectify_ij_var": (_c_int, [_c_ptr, _c_ptr, _c_i64, _c_i64, _c_i64, _c_ptr, _c_i64,
                                    _c_ptr, _c_i64, _c_i64, _c_i64, _c_dbl, _c_dbl, _c_dbl,
                                    _c_ptr, _c_int, _c_ptr,                # keys, keys_ready, ij
                                    _c_ptr, _c_int, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64,
                                    _c_ptr, _c_i64, _c_int, _c_dbl, _c_ptr, _c_ptr]),
    "xrs_rectify_tiles": (_c_int, [_c_ptr, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64,
                                   _c_i64, _c_i64, _c_i64, _c_dbl, _c_dbl, _c_dbl, _c_dbl,
                                   _c_dbl, _c_int, _c_ptr, _c_ptr, _c_ptr]),
    "xrs_testing_set": (_c_i64, [_c_int, _c_i64]),
    "xrs_rectify_var": (_c_int, [_c_ptr, _c_i64, _c_i64, _c_i64, _c_ptr, _c_int, _c_i64, _c_i64,
                                 _c_i64, _c_i64, _c_i64, _c_ptr, _c_i64, _c_int, _c_dbl, _c_ptr,
                                 _c_ptr]),
    "xrs_transform": (_c_int, [_c_ptr, _c_ptr, _c_i64, _c_i64, _c_int, _c_ptr, _c_int, _c_ptr,
                               _c_ptr, _c_ptr]),
    "xrs_reproject_proj": (_c_int, [
        _c_ptr, _c_int, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64,  # src
        _c_ptr, _c_int, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64,          # dst
        _c_i64, _c_i64,                                                          # tile
        _c_ptr, _c_ptr, _c_ptr, _c_int,                                          # grid axes, steps
        _c_ptr, _c_ptr, _c_ptr, _c_i64, _c_i64,                                  # tile tables
        _c_dbl, _c_dbl, _c_int, _c_dbl,                                          # res, interp, fill
        _c_ptr, _c_ptr,                                                          # flags, stream
    ]),
}


class ProjStep(ctypes.Structure):
    """XrsProjStep (include/xrs.h): one PROJ operation of an xrs_transform pipeline."""

    _fields_ = [("kind", ctypes.c_int32), ("mode", ctypes.c_int32),
                ("a", _c_dbl), ("ra", _c_dbl), ("x0", _c_dbl), ("y0", _c_dbl),
                ("lam0", _c_dbl), ("phi0", _c_dbl), ("e", _c_dbl), ("es", _c_dbl),
                ("one_es", _c_dbl), ("c", _c_dbl * 24), ("Qn", _c_dbl), ("Zb", _c_dbl),
                ("qp", _c_dbl), ("mmf", _c_dbl), ("apa", _c_dbl * 3), ("rq", _c_dbl),
                ("dd", _c_dbl), ("xmf", _c_dbl), ("ymf", _c_dbl), ("sinb1", _c_dbl),
                ("cosb1", _c_dbl)]


PROJ_KINDS = {"webmerc_fwd": 1, "webmerc_inv": 2, "tmerc_fwd": 3, "tmerc_inv": 4,
              "laea_fwd": 5, "laea_inv": 6}
MAX_PROJ_STEPS = 4

TESTING_KNOBS = {"reproject_band": 1, "reproject_blocks_per_cu": 2, "affine_generic": 3,
                 "rectify_exact": 4, "rectify_margin": 5,
                 "rectify_plain_keys": 7, "proj_two_step": 8,
                 "rectify_compact": 9}   # 6: retired (K1's column-group deal, round 5)


class testing_knob:
    """Context manager forcing one test-only path knob (xrs_testing_set):
    ``with testing_knob("rectify_exact", 1): ...``.  Tests only."""

    def __init__(self, name: str, value: int):
        self.knob = TESTING_KNOBS[name]
        self.value = int(value)
        self.prev = None

    def __enter__(self):
        self.prev = lib().xrs_testing_set(self.knob, self.value)
        return self

    def __exit__(self, *exc):
        lib().xrs_testing_set(self.knob, self.prev)
        return False


AGG_CODES = {"mean": 1, "sum": 2, "max": 3, "min": 4, "prod": 5, "count": 6, "first": 7,
             "last": 8, "center": 9, "median": 10, "mode": 11, "std": 12, "var": 13}
# reducers the fused K3 (xrs_affine) evaluates; the others run as K2 at the
# div-x grid followed by K7 (xrs_coarsen)
FUSED_AGGS = ("mean", "sum", "max", "min", "prod", "count", "first", "last", "center")

_lib = None
_lock = threading.Lock()


def declared_symbols(header: str = HEADER_PATH) -> list[str]:
    """Names of all functions declared in include/xrs.h."""
    with open(header) as f:
        text = f.read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\**\s+\**(xrs_\w+)\s*\(", text, re.M)))


def load_library(path: str | None = None):
    """Load libxrs.so without requiring a GPU (symbol checks, CPU tests)."""
    if path is None:
        if LIB_PATH is None:
            raise _LIB_PATH_ERROR
        path = LIB_PATH
    if not os.path.exists(path):
        raise NativeLibraryError(
            f"libxrs.so not found at {path}: build it with "
            f"`make -C xcube-resampling_amd/csrc` (or __graft_entry__.build())"
        )
    lib = ctypes.CDLL(path)
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def lib():
    """The loaded library, bound to torch's HIP runtime."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                import torch  # noqa: F401  (must precede the CDLL: one HIP runtime)
                _lib = load_library()
    return _lib


def last_error() -> str:
    msg = lib().xrs_last_error()
    return msg.decode() if msg else ""


def check(rc: int, what: str) -> None:
    if rc == XRS_OK:
        return
    msg = last_error()
    if rc == XRS_ERR_NOTIMPL:
        raise NotImplementedError(msg)
    if rc == XRS_ERR_ARG:
        raise ValueError(f"{what}: {msg}")
    raise NativeLibraryError(f"{what}: {msg}")


def dtype_code(dtype) -> int:
    try:
        return DTYPE_CODES[np.dtype(dtype)]
    except KeyError:
        raise TypeError(f"unsupported dtype {dtype!r}") from None

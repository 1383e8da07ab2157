"""Load individual functions of the reference implementation by AST, for
GENERATING golden fixtures in the development container only.

The reference package cannot be imported here (xarray, dask, numba, pyproj,
dask_image are absent).  Its numeric functions only need numpy, so we compile
just the requested function definitions from the reference source files and
execute them with stand-ins for the missing modules — exactly the mode the
reference's own tests use for numba (tests/conftest.py:1-3 disables the JIT):

* ``numba``: ``njit``/``jit`` are identity decorators, ``prange`` is ``range``;
* ``dask.array``: the few calls used on these paths (from_array, zeros, pad)
  are mapped to numpy.

Nothing produced by this module is shipped: only the resulting input/output
arrays are committed under tests/golden/ (see make_goldens.py).  The GPU box
never reads /root/reference.
"""

from __future__ import annotations

import ast
import math
import os
import types

import numpy as np

REFERENCE_ROOT = os.environ.get("XRS_REFERENCE_ROOT", "/root/reference")


class _NumbaStub(types.SimpleNamespace):
    @staticmethod
    def njit(*args, **kwargs):
        if len(args) == 1 and callable(args[0]) and not kwargs:
            return args[0]
        return lambda f: f

    jit = njit
    prange = range


class _ChunkedArray(np.ndarray):
    """numpy array carrying a dask-like ``chunks`` attribute."""

    chunks = None


def chunked(a, chunks):
    out = np.asarray(a).view(_ChunkedArray)
    out.chunks = chunks
    return out


class _DaskArrayStub(types.SimpleNamespace):
    @staticmethod
    def from_array(x, chunks=None):
        return np.asarray(x)

    @staticmethod
    def zeros(shape, chunks=None, dtype=float):
        return np.zeros(shape, dtype=dtype)

    @staticmethod
    def pad(array, pad_width, mode="constant", constant_values=0):
        return np.pad(np.asarray(array), pad_width, mode=mode, constant_values=constant_values)


def load_functions(relpath: str, names: list[str], extra: dict | None = None) -> dict:
    path = os.path.join(REFERENCE_ROOT, relpath)
    with open(path) as f:
        tree = ast.parse(f.read(), filename=path)
    wanted = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in names]
    missing = set(names) - {n.name for n in wanted}
    if missing:
        raise KeyError(f"{missing} not found in {relpath}")
    for fn in wanted:  # annotations name modules we do not have (pyproj, xr, ...)
        fn.returns = None
        for a in fn.args.args + fn.args.kwonlyargs + fn.args.posonlyargs:
            a.annotation = None
    mod = ast.Module(body=wanted, type_ignores=[])
    ns = dict(np=np, math=math, nb=_NumbaStub(), da=_DaskArrayStub(),
              __name__=f"refload:{relpath}")
    ns.update(extra or {})
    exec(compile(mod, path, "exec"), ns)
    return {n: ns[n] for n in names}

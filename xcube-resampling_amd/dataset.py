"""A minimal, dependency-free labelled-array model (Dataset / DataArray).

The reference's public functions take and return ``xarray.Dataset`` objects
(spatial.py:40, affine.py:52, reproject.py:51, rectify.py:54).  ``xarray`` and
``dask`` are not installed in this image, so the engine ships this small model
with the subset of the xarray API the reference relies on: named dimensions,
coordinate and data variables, attributes, positional selection (``isel``),
``assign_coords`` / ``drop_vars`` and dask-style chunk metadata (``chunks``,
``chunk()``), which drives the tile geometry exactly like dask chunks do in the
reference (coords.py:166-171, 266-283; affine.py:212-216; reproject.py:230).

Array payloads may be numpy arrays (host) or torch CUDA tensors (device); the
engine keeps device payloads on the device.  Real ``xarray`` objects are
accepted by the public API through duck typing (they expose the same names).
"""

from __future__ import annotations

import copy as _copy
from collections.abc import Hashable, Iterable, Mapping
from typing import Any

import numpy as np


def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch")


def to_numpy(x) -> np.ndarray:
    """Host numpy view/copy of a payload (numpy array, torch tensor, scalar)."""
    if isinstance(x, np.ndarray):
        return x
    if _is_torch(x):
        return x.detach().cpu().numpy()
    values = getattr(x, "values", None)
    if isinstance(values, np.ndarray):
        return values
    return np.asarray(x)


def normalize_chunks(chunks, shape) -> tuple[tuple[int, ...], ...] | None:
    """dask.array.core.normalize_chunks for int / tuple-of-int / tuple-of-tuples."""
    if chunks is None:
        return None
    if isinstance(chunks, int):
        chunks = (chunks,) * len(shape)
    out = []
    for c, s in zip(chunks, shape):
        if c is None or c == -1:
            out.append((s,) if s > 0 else (0,))
        elif isinstance(c, int):
            n, r = divmod(s, c)
            out.append((c,) * n + ((r,) if r else ()) or (0,))
        else:
            out.append(tuple(int(v) for v in c))
    return tuple(out)


class DataArray:
    """Labelled n-d array (subset of ``xarray.DataArray``)."""

    def __init__(self, data: Any, dims: Iterable[Hashable] | str | None = None,
                 attrs: Mapping | None = None, name: Hashable | None = None,
                 chunks=None, coords: Mapping | None = None):
        if isinstance(data, DataArray):
            dims = data.dims if dims is None else dims
            attrs = dict(data.attrs) if attrs is None else attrs
            name = data.name if name is None else name
            chunks = data.chunks if chunks is None else chunks
            data = data.data
        if not (isinstance(data, np.ndarray) or _is_torch(data)):
            data = np.asarray(data)
        if dims is None:
            dims = tuple(f"dim_{i}" for i in range(data.ndim))
        elif isinstance(dims, str):
            dims = (dims,)
        self._data = data
        self._dims = tuple(dims)
        if len(self._dims) != data.ndim:
            raise ValueError(
                f"different number of dimensions on data and dims: "
                f"{data.ndim} vs {len(self._dims)}"
            )
        self.attrs = dict(attrs or {})
        self.name = name
        self._chunks = normalize_chunks(chunks, data.shape) if chunks is not None else None
        self._coords = dict(coords or {})

    # ---- array-like ------------------------------------------------------
    @property
    def data(self):
        return self._data

    @property
    def values(self) -> np.ndarray:
        return to_numpy(self._data)

    @property
    def dims(self) -> tuple:
        return self._dims

    @property
    def shape(self) -> tuple:
        return tuple(self._data.shape)

    @property
    def ndim(self) -> int:
        return len(self._dims)

    @property
    def size(self) -> int:
        return int(np.prod(self.shape)) if self.shape else 1

    @property
    def dtype(self) -> np.dtype:
        if _is_torch(self._data):
            return np.dtype(str(self._data.dtype).replace("torch.", ""))
        return self._data.dtype

    @property
    def sizes(self) -> dict:
        return dict(zip(self._dims, self.shape))

    @property
    def coords(self) -> dict:
        return self._coords

    @property
    def chunks(self):
        return self._chunks

    @property
    def chunksize(self):
        if self._chunks is None:
            return None
        return tuple(max(c) if c else 0 for c in self._chunks)

    def chunk(self, chunks=None) -> "DataArray":
        if isinstance(chunks, Mapping):
            spec = [chunks.get(d, self._chunks[i] if self._chunks else -1)
                    for i, d in enumerate(self._dims)]
        elif chunks is None:
            spec = [-1] * self.ndim
        else:
            spec = chunks
        return DataArray(self._data, self._dims, self.attrs, self.name, chunks=spec)

    def __array__(self, dtype=None, copy=None):
        v = self.values
        return v.astype(dtype) if dtype is not None else v

    def __len__(self) -> int:
        return self.shape[0]

    def __repr__(self) -> str:
        return f"<DataArray {self.name!r} {dict(zip(self.dims, self.shape))} {self.dtype}>"

    def astype(self, dtype) -> "DataArray":
        return DataArray(self.values.astype(dtype), self._dims, self.attrs, self.name,
                         chunks=self._chunks)

    def copy(self, deep: bool = True) -> "DataArray":
        data = self._data.clone() if _is_torch(self._data) else self._data.copy()
        return DataArray(data, self._dims, _copy.deepcopy(self.attrs), self.name,
                         chunks=self._chunks)

    # ---- selection ----------------------------------------------------------
    def isel(self, indexers: Mapping | None = None, **kw) -> "DataArray":
        indexers = dict(indexers or {}, **kw)
        key = tuple(indexers.get(d, slice(None)) for d in self._dims)
        return self[key]

    def __getitem__(self, key) -> "DataArray":
        if not isinstance(key, tuple):
            key = (key,)
        if any(k is Ellipsis for k in key):
            i = key.index(Ellipsis)
            key = key[:i] + (slice(None),) * (self.ndim - len(key) + 1) + key[i + 1:]
        key = key + (slice(None),) * (self.ndim - len(key))
        data = self._data[key]
        dims = tuple(d for d, k in zip(self._dims, key) if not isinstance(k, (int, np.integer)))
        chunks = None
        if self._chunks is not None:
            chunks = []
            for d, k, c, s in zip(self._dims, key, self._chunks, self.shape):
                if isinstance(k, (int, np.integer)):
                    continue
                if isinstance(k, slice) and k == slice(None):
                    chunks.append(c)
                else:  # dask keeps the chunk size; good enough for tiling decisions
                    n = len(range(*k.indices(s))) if isinstance(k, slice) else len(k)
                    cs = max(c) if c else n
                    chunks.append(cs if n else 0)
            chunks = tuple(chunks)
            if any(c == 0 for c in chunks):
                chunks = None
        return DataArray(data, dims, self.attrs, self.name, chunks=chunks)

    def diff(self, dim: Hashable) -> "DataArray":
        axis = self._dims.index(dim)
        return DataArray(np.diff(self.values, axis=axis), self._dims, name=self.name)

    def expand_dims(self, dims: Mapping) -> "DataArray":
        (name, size), = dict(dims).items()
        data = self._data[None]
        if size != 1:
            data = np.repeat(data, size, axis=0)
        chunks = None if self._chunks is None else ((size,),) + self._chunks
        return DataArray(data, (name,) + self._dims, self.attrs, self.name, chunks=chunks)


class Dataset:
    """Collection of named DataArrays split into coordinates and data variables."""

    def __init__(self, data_vars: Mapping | None = None, coords: Mapping | None = None,
                 attrs: Mapping | None = None):
        self._coords: dict[Hashable, DataArray] = {}
        self._data_vars: dict[Hashable, DataArray] = {}
        self.attrs = dict(attrs or {})
        for k, v in (coords or {}).items():
            self._coords[k] = self._as_var(k, v, coord=True)
        for k, v in (data_vars or {}).items():
            self._data_vars[k] = self._as_var(k, v)

    @staticmethod
    def _as_var(name, value, coord: bool = False) -> DataArray:
        if isinstance(value, DataArray):
            da = DataArray(value)
        elif hasattr(value, "dims") and hasattr(value, "values"):  # foreign (xarray) DataArray
            da = DataArray(value.values, tuple(value.dims), dict(getattr(value, "attrs", {})))
        elif isinstance(value, tuple):
            dims, data = value[0], value[1]
            attrs = value[2] if len(value) > 2 else None
            da = DataArray(data, dims, attrs)
        else:
            arr = value if _is_torch(value) else np.asarray(value)
            dims = (name,) if arr.ndim == 1 else ()
            if arr.ndim > 1:
                raise ValueError(f"cannot infer dims for variable {name!r}")
            da = DataArray(arr, dims)
        da.name = name
        return da

    # ---- mapping API ------------------------------------------------------
    @property
    def coords(self) -> dict:
        return self._coords

    @property
    def data_vars(self) -> dict:
        return self._data_vars

    @property
    def variables(self) -> dict:
        out = dict(self._coords)
        out.update(self._data_vars)
        return out

    def items(self):
        return self._data_vars.items()

    def keys(self):
        return self._data_vars.keys()

    def __iter__(self):
        return iter(self._data_vars)

    def __len__(self) -> int:
        return len(self._data_vars)

    def __contains__(self, name) -> bool:
        return name in self._coords or name in self._data_vars

    def __getitem__(self, name):
        if isinstance(name, (list, tuple)) and not isinstance(name, str):
            ds = Dataset(coords=self._coords, attrs=self.attrs)
            for n in name:
                ds._data_vars[n] = self._data_vars[n]
            return ds
        if name in self._data_vars:
            return self._data_vars[name]
        if name in self._coords:
            return self._coords[name]
        raise KeyError(name)

    def __setitem__(self, name, value) -> None:
        self._data_vars[name] = self._as_var(name, value)
        self._coords.pop(name, None)

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        try:
            return self[name]
        except KeyError:
            raise AttributeError(name) from None

    @property
    def dims(self) -> dict:
        out: dict = {}
        for v in self.variables.values():
            out.update(v.sizes)
        return out

    sizes = dims

    def __repr__(self) -> str:
        return (f"<Dataset dims={self.dims} coords={list(self._coords)} "
                f"data_vars={list(self._data_vars)}>")

    # ---- transformations ---------------------------------------------------
    def copy(self) -> "Dataset":
        ds = Dataset(attrs=_copy.deepcopy(self.attrs))
        ds._coords = {k: DataArray(v) for k, v in self._coords.items()}
        ds._data_vars = {k: DataArray(v) for k, v in self._data_vars.items()}
        for k in ds._coords:
            ds._coords[k].attrs = dict(self._coords[k].attrs)
        for k in ds._data_vars:
            ds._data_vars[k].attrs = dict(self._data_vars[k].attrs)
        return ds

    def isel(self, indexers: Mapping | None = None, **kw) -> "Dataset":
        indexers = dict(indexers or {}, **kw)
        ds = Dataset(attrs=self.attrs)
        for k, v in self._coords.items():
            ds._coords[k] = v.isel({d: s for d, s in indexers.items() if d in v.dims})
            ds._coords[k].name = k
        for k, v in self._data_vars.items():
            ds._data_vars[k] = v.isel({d: s for d, s in indexers.items() if d in v.dims})
            ds._data_vars[k].name = k
        return ds

    def assign_coords(self, coords: Mapping | None = None, **kw) -> "Dataset":
        ds = self.copy()
        for k, v in dict(coords or {}, **kw).items():
            ds._coords[k] = self._as_var(k, v, coord=True)
            ds._data_vars.pop(k, None)
        return ds

    def drop_vars(self, names) -> "Dataset":
        if isinstance(names, str) or not isinstance(names, Iterable):
            names = [names]
        names = set(names)
        ds = self.copy()
        for n in names:
            if n not in ds:
                raise ValueError(f"variable {n!r} not found")
            ds._coords.pop(n, None)
            ds._data_vars.pop(n, None)
        return ds

    def chunk(self, chunks: Mapping) -> "Dataset":
        ds = self.copy()
        for store in (ds._coords, ds._data_vars):
            for k, v in store.items():
                spec = {d: c for d, c in chunks.items() if d in v.dims}
                if spec and v.ndim:
                    store[k] = v.chunk(spec)
                    store[k].name = k
        return ds

"""Per-variable parameter resolution and dataset helpers (utils.py of the
reference, lines quoted per function).  Same defaults, same warnings on the
``xcube.resampling`` logger, same exceptions."""

from __future__ import annotations

from collections.abc import Hashable, Iterable, Mapping, Sequence

import numpy as np

from .constants import (
    AGG_METHOD_NAMES,
    FILLVALUE_FLOAT,
    FILLVALUE_INT,
    FILLVALUE_UINT8,
    FILLVALUE_UINT16,
    INTERP_METHOD_MAPPING,
    LOG,
)
from .dataset import DataArray, Dataset
from .gridmapping import GridMapping


def get_spatial_dims(ds) -> tuple[str, str]:
    """utils.py:47-74."""
    if "lat" in ds and "lon" in ds:
        return "lon", "lat"
    if "y" in ds and "x" in ds:
        return "x", "y"
    raise KeyError(
        "No standard spatial dimensions found in dataset. "
        f"Expected pairs ('lon', 'lat') or ('x', 'y'), but found: {list(ds.dims)}."
    )


def clip_dataset_by_bbox(ds, bbox: Sequence, spatial_dims: tuple[str, str] | None = None):
    """utils.py:77-124 — label-based clip (xarray ``sel`` slice semantics on
    monotonic 1-D coordinates: inclusive bounds)."""
    if len(bbox) != 4:
        raise ValueError(f"Expected bbox of length 4, got: {bbox}")
    if spatial_dims is None:
        spatial_dims = get_spatial_dims(ds)
    x_dim, y_dim = spatial_dims
    x = ds[x_dim].values
    y = ds[y_dim].values
    xs = _label_slice(x, bbox[0], bbox[2])
    if y[-1] - y[0] < 0:
        ys = _label_slice(y, bbox[3], bbox[1])
    else:
        ys = _label_slice(y, bbox[1], bbox[3])
    ds = ds.isel({x_dim: xs, y_dim: ys})
    if any(size == 0 for size in ds.sizes.values()):
        LOG.warning(
            "Clipped dataset contains at least one zero-sized dimension. "
            f"Check if the bounding box {bbox} overlaps with the dataset extent."
        )
    return ds


def _label_slice(coord: np.ndarray, start, stop) -> slice:
    """pandas Index.slice_indexer for a monotonic index (inclusive labels)."""
    if coord.size < 2 or coord[-1] >= coord[0]:
        i0 = int(np.searchsorted(coord, start, side="left"))
        i1 = int(np.searchsorted(coord, stop, side="right"))
    else:
        r = coord[::-1]
        i0 = coord.size - int(np.searchsorted(r, start, side="right"))
        i1 = coord.size - int(np.searchsorted(r, stop, side="left"))
    return slice(i0, max(i0, i1))


def normalize_grid_mapping(ds, gm: GridMapping):
    """utils.py:127-151 — standard ``spatial_ref`` grid-mapping coordinate."""
    gm_name = _get_grid_mapping_name(ds)
    if gm_name is not None:
        ds = ds.drop_vars(gm_name)
    ds = ds.assign_coords(spatial_ref=DataArray(np.array(0), (), gm.crs.to_cf()))
    for var in ds.data_vars:
        ds[var].attrs["grid_mapping"] = "spatial_ref"
    return ds


def _select_variables(ds, variables: str | Iterable[str] | None = None):
    """utils.py:154-161."""
    if variables is not None:
        if isinstance(variables, str):
            variables = [variables]
        ds = ds[list(variables)]
    return ds


def _get_grid_mapping_name(ds) -> str | None:
    """utils.py:164-178."""
    names = []
    for var in ds.data_vars:
        if "grid_mapping" in ds[var].attrs:
            names.append(ds[var].attrs["grid_mapping"])
    if "crs" in ds:
        names.append("crs")
    if "spatial_ref" in ds.coords:
        names.append("spatial_ref")
    names = np.unique(names)
    assert len(names) <= 1, "Multiple grid mapping names found."
    return str(names[0]) if len(names) == 1 else None


def _can_apply_affine_transform(source_gm: GridMapping, target_gm: GridMapping) -> bool:
    """utils.py:181-184."""
    GridMapping.assert_regular(source_gm, name="source_gm")
    GridMapping.assert_regular(target_gm, name="target_gm")
    return _is_equal_crs(source_gm, target_gm)


def _is_equal_crs(source_gm: GridMapping, target_gm: GridMapping) -> bool:
    """utils.py:187-189."""
    geographic = source_gm.crs.is_geographic and target_gm.crs.is_geographic
    return geographic or source_gm.crs.equals(target_gm.crs)


def _get_interp_method(interp_methods, key: Hashable, var):
    """utils.py:192-214."""
    def assign_defaults(data_type):
        return 0 if np.issubdtype(data_type, np.integer) else 1

    if isinstance(interp_methods, Mapping):
        interp_method = interp_methods.get(str(key), interp_methods.get(var.dtype))
        if interp_method is None:
            LOG.warning(
                f"Interpolation method could not be derived from the mapping "
                f"`interp_methods` for data variable {key!r} with data type "
                f"{var.dtype!r}. Defaults are assigned."
            )
            interp_method = assign_defaults(var.dtype)
    elif isinstance(interp_methods, (int, str)):
        interp_method = interp_methods
    else:
        interp_method = assign_defaults(var.dtype)
    return interp_method


def _get_interp_method_int(interp_methods, key: Hashable, var):
    """utils.py:217-225."""
    m = _get_interp_method(interp_methods, key, var)
    if isinstance(m, str):
        m = INTERP_METHOD_MAPPING[m]
    return m


def _get_interp_method_str(interp_methods, key: Hashable, var):
    """utils.py:228-236."""
    m = _get_interp_method(interp_methods, key, var)
    if isinstance(m, int):
        m = INTERP_METHOD_MAPPING[m]
    return m


def _prep_interp_methods_downscale(interp_methods):
    """utils.py:239-251."""
    if interp_methods == "triangular":
        return "bilinear"
    if isinstance(interp_methods, Mapping) and "triangular" in interp_methods.values():
        return {k: ("bilinear" if v == "triangular" else v) for k, v in interp_methods.items()}
    return interp_methods


def _get_agg_method(agg_methods, key: Hashable, var) -> str:
    """utils.py:254-276 (returns the method NAME; the reducer runs on device)."""
    def assign_defaults(data_type):
        return "center" if np.issubdtype(data_type, np.integer) else "mean"

    if isinstance(agg_methods, Mapping):
        agg_method = agg_methods.get(str(key), agg_methods.get(var.dtype))
        if agg_method is None:
            LOG.warning(
                f"Aggregation method could not be derived from the mapping `agg_methods` "
                f"for data variable {key!r} with data type {var.dtype!r}. Defaults "
                f"are assigned."
            )
            agg_method = assign_defaults(var.dtype)
    elif isinstance(agg_methods, str):
        agg_method = agg_methods
    else:
        agg_method = assign_defaults(var.dtype)
    if agg_method not in AGG_METHOD_NAMES:
        raise KeyError(agg_method)  # reference: AGG_METHODS[agg_method]
    return agg_method


def _get_recover_nan(recover_nans, key: Hashable, var) -> bool:
    """utils.py:279-298."""
    if isinstance(recover_nans, Mapping):
        recover_nan = recover_nans.get(str(key), recover_nans.get(var.dtype))
        if recover_nan is None:
            LOG.warning(
                f"The method to recover nan could not be derived from the mapping "
                f"`recover_nans`  for data variable {key!r} with data type "
                f"{var.dtype!r}. Defaults are assigned."
            )
            recover_nan = False
    elif isinstance(recover_nans, bool):
        recover_nan = recover_nans
    else:
        recover_nan = False
    return recover_nan


def _get_fill_value(fill_values, key: Hashable, var):
    """utils.py:301-332."""
    def assign_defaults(data_type):
        if data_type == np.uint8:
            return FILLVALUE_UINT8
        if data_type == np.uint16:
            return FILLVALUE_UINT16
        if np.issubdtype(data_type, np.integer):
            return FILLVALUE_INT
        return FILLVALUE_FLOAT

    if isinstance(fill_values, Mapping):
        fill_value = fill_values.get(str(key), fill_values.get(var.dtype))
        if fill_value is None:
            LOG.warning(
                f"Fill value could not be derived from the mapping `fill_values` "
                f"for data variable {key!r} with data type {var.dtype!r}. Defaults "
                f"are assigned."
            )
            fill_value = assign_defaults(var.dtype)
    elif fill_values is not None:
        fill_value = fill_values
    else:
        fill_value = assign_defaults(var.dtype)
    return fill_value


def as_dataset(ds) -> Dataset:
    """Accept the engine's Dataset or a foreign (xarray) dataset."""
    if isinstance(ds, Dataset):
        return ds
    if hasattr(ds, "data_vars") and hasattr(ds, "coords"):
        out = Dataset(attrs=dict(getattr(ds, "attrs", {})))
        for k, v in ds.coords.items():
            out.coords[k] = Dataset._as_var(k, v, coord=True)
        for k, v in ds.data_vars.items():
            out.data_vars[k] = Dataset._as_var(k, v)
        return out
    raise TypeError("source_ds must be a Dataset")

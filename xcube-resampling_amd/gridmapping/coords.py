"""Grid mappings from 1-D / 2-D coordinate arrays (gridmapping/coords.py:49-472)."""

from __future__ import annotations

import math

import numpy as np

from ..crs import normalize_crs
from ..dataset import DataArray
from .base import DEFAULT_TOLERANCE, GridMapping, _assert
from .helpers import (
    _default_xy_var_names,
    _normalize_int_pair,
    _normalize_number_pair,
    _to_int_or_float,
    from_lon_360,
    round_to_fraction,
    to_lon_360,
)

_ER = 6371000


class CoordsGridMapping(GridMapping):
    @property
    def x_coords(self):
        assert isinstance(self._x_coords, DataArray)
        return self._x_coords

    @property
    def y_coords(self):
        assert isinstance(self._y_coords, DataArray)
        return self._y_coords

    def _new_x_coords(self):
        return self._x_coords

    def _new_y_coords(self):
        return self._y_coords


class Coords1DGridMapping(CoordsGridMapping):
    def _new_xy_coords(self) -> DataArray:
        x = self._x_coords.values
        y = self._y_coords.values
        xy = np.empty((2, y.size, x.size), dtype=np.result_type(x, y))
        xy[0] = x[None, :]
        xy[1] = y[:, None]
        return DataArray(xy, ("coord", self._y_coords.dims[0], self._x_coords.dims[0]),
                         chunks=self.xy_coords_chunks)


class Coords2DGridMapping(CoordsGridMapping):
    def _new_xy_coords(self) -> DataArray:
        x = self._x_coords.data
        y = self._y_coords.data
        if type(x).__module__.startswith("torch"):
            import torch
            xy = torch.stack([x, y])
        else:
            xy = np.stack([np.asarray(x), np.asarray(y)])
        return DataArray(xy, ("coord",) + tuple(self._x_coords.dims), chunks=None)


def _abs_no_zero(array):
    """coords.py:330-332."""
    array = np.fabs(np.asarray(array))
    return np.where(np.isclose(array, 0), np.nan, array)


def _abs_no_nan(array):
    """coords.py:335-337."""
    array = np.fabs(np.asarray(array))
    return np.where(np.logical_or(np.isnan(array), np.isclose(array, 0)), 0, array)


def _as_data_array(c, name) -> DataArray:
    if isinstance(c, DataArray):
        return c
    if hasattr(c, "dims") and hasattr(c, "values"):
        return DataArray(c.values, tuple(c.dims), dict(getattr(c, "attrs", {})),
                         name=getattr(c, "name", None), chunks=getattr(c, "chunks", None))
    raise TypeError(f"{name} must be an instance of DataArray")


def new_grid_mapping_from_coords(x_coords, y_coords, crs, *, xy_res=None, xy_bbox=None,
                                 tile_size=None, tolerance: float = DEFAULT_TOLERANCE
                                 ) -> GridMapping:
    """coords.py:99-327."""
    crs = normalize_crs(crs)
    x_coords = _as_data_array(x_coords, "x_coords")
    y_coords = _as_data_array(y_coords, "y_coords")
    _assert(x_coords.ndim in (1, 2), "x_coords and y_coords must be either 1D or 2D arrays")
    if not isinstance(tolerance, float):
        raise TypeError("tolerance must be an instance of float")
    _assert(tolerance > 0.0, "tolerance must be greater zero")

    if x_coords.name and y_coords.name:
        xy_var_names = str(x_coords.name), str(y_coords.name)
    else:
        xy_var_names = _default_xy_var_names(crs)

    tile_size = _normalize_int_pair(tile_size, default=None)
    is_lon_360 = None
    if crs.is_geographic:
        is_lon_360 = bool(np.any(x_coords.values > 180))

    if x_coords.ndim == 1:
        cls = Coords1DGridMapping
        _assert(x_coords.size >= 2 and y_coords.size >= 2,
                "sizes of x_coords and y_coords 1D arrays must be >= 2")
        size = x_coords.size, y_coords.size
        x_dim, y_dim = x_coords.dims[0], y_coords.dims[0]
        x_diff = _abs_no_zero(np.diff(x_coords.values))
        y_diff = _abs_no_zero(np.diff(y_coords.values))
        if not is_lon_360 and crs.is_geographic:
            if np.any(np.nanmax(x_diff) > 180):
                x_coords = DataArray(to_lon_360(x_coords.values), x_coords.dims,
                                     x_coords.attrs, x_coords.name, chunks=x_coords.chunks)
                x_diff = _abs_no_zero(np.diff(x_coords.values))
                is_lon_360 = True
        if xy_res is not None:
            x_res, y_res = _normalize_number_pair(xy_res)
            is_regular = True
        else:
            x_res = x_diff[0]
            y_res = y_diff[0]
            is_regular = bool(np.allclose(x_diff, x_res, atol=tolerance)
                              and np.allclose(y_diff, y_res, atol=tolerance))
            if is_regular:
                x_res = round_to_fraction(float(x_res), 5, 0.25)
                y_res = round_to_fraction(float(y_res), 5, 0.25)
            else:
                x_res = round_to_fraction(float(np.nanmedian(x_diff, axis=0)), 2, 0.5)
                y_res = round_to_fraction(float(np.nanmedian(y_diff, axis=0)), 2, 0.5)
        if tile_size is None and x_coords.chunks is not None and y_coords.chunks is not None:
            tile_size = (max(0, *x_coords.chunks[0]), max(0, *y_coords.chunks[0]))
        yv = y_coords.values
        is_j_axis_up = bool(yv[0] < yv[-1])
    else:
        cls = Coords2DGridMapping
        _assert(x_coords.shape == y_coords.shape,
                "shapes of x_coords and y_coords 2D arrays must be equal")
        _assert(x_coords.dims == y_coords.dims,
                "dimensions of x_coords and y_coords 2D arrays must be equal")
        y_dim, x_dim = x_coords.dims
        height, width = x_coords.shape
        size = width, height
        x = x_coords.values
        y = y_coords.values
        # the reference restricts these probes to the first dask chunk
        # (coords.py:197-200); numpy-backed coordinates form a single chunk
        cs = x_coords.chunksize or x.shape
        x_x_diff = _abs_no_nan(np.diff(x[0, :cs[1]]))
        x_y_diff = _abs_no_nan(np.diff(x[:cs[0], 0]))
        y_x_diff = _abs_no_nan(np.diff(y[0, :cs[0]]))
        y_y_diff = _abs_no_nan(np.diff(y[:cs[1], 0]))
        if not is_lon_360 and crs.is_geographic:
            if np.max(x_x_diff) > 180 or np.max(x_y_diff) > 180:
                x = to_lon_360(x)
                x_coords = DataArray(x, x_coords.dims, x_coords.attrs, x_coords.name,
                                     chunks=x_coords.chunks)
                x_x_diff = _abs_no_nan(np.diff(x[0, :]))
                x_y_diff = _abs_no_nan(np.diff(x[:, 0]))
                is_lon_360 = True
        if xy_res is not None:
            x_res, y_res = _normalize_number_pair(xy_res)
        else:
            x_res = x_x_diff[0]
            y_res = y_y_diff[0]
        is_regular = bool(np.allclose(x_x_diff, x_res, atol=tolerance)
                          and np.allclose(y_y_diff, y_res, atol=tolerance)
                          and np.allclose(x_y_diff, 0, atol=tolerance)
                          and np.allclose(y_x_diff, 0, atol=tolerance))
        if not is_regular and xy_res is None:
            x_res, y_res = _estimate_2d_resolution(x, y, crs)
        if tile_size is None and x_coords.chunks is not None:
            j_chunks, i_chunks = x_coords.chunks
            tile_size = max(0, *i_chunks), max(0, *j_chunks)
        if tile_size is not None:
            tile_width, tile_height = tile_size
            x_coords = x_coords.chunk({x_coords.dims[0]: tile_height, x_coords.dims[1]: tile_width})
            y_coords = y_coords.chunk({y_coords.dims[0]: tile_height, y_coords.dims[1]: tile_width})
        ycs = (y_coords.chunksize or y.shape)[1]
        is_j_axis_up = bool(np.all(y[0, :ycs] < y[-1, :ycs]))

    _assert(x_res > 0 and y_res > 0, "internal error: x_res and y_res could not be determined",
            exception_type=RuntimeError)
    x_res, y_res = _to_int_or_float(x_res), _to_int_or_float(y_res)
    if xy_bbox is None:
        xv = x_coords.values
        yv = y_coords.values
        x_res_05, y_res_05 = x_res / 2, y_res / 2
        x_min = _to_int_or_float(np.min(xv[..., 0]) - x_res_05)
        x_max = _to_int_or_float(np.max(xv[..., -1]) + x_res_05)
        if is_j_axis_up:
            y_min = _to_int_or_float(float(np.min(yv[0, ...])) - y_res_05)
            y_max = _to_int_or_float(float(np.max(yv[-1, ...])) + y_res_05)
        else:
            y_min = _to_int_or_float(float(np.min(yv[-1, ...])) - y_res_05)
            y_max = _to_int_or_float(float(np.max(yv[0, ...])) + y_res_05)
        xy_bbox = (x_min, y_min, x_max, y_max)

    if cls is Coords1DGridMapping and is_regular:
        from .regular import RegularGridMapping
        cls = RegularGridMapping

    return cls(x_coords=x_coords, y_coords=y_coords, crs=crs, size=size, tile_size=tile_size,
               xy_bbox=xy_bbox, xy_res=(x_res, y_res), xy_var_names=xy_var_names,
               xy_dim_names=(str(x_dim), str(y_dim)), is_regular=is_regular,
               is_lon_360=is_lon_360, is_j_axis_up=is_j_axis_up)


def _estimate_2d_resolution(x: np.ndarray, y: np.ndarray, crs):
    """coords.py:226-264 — area-based resolution estimate of irregular 2-D coords."""
    x_x_diff = _abs_no_nan(np.diff(x, axis=1))
    x_y_diff = _abs_no_nan(np.diff(x, axis=0))
    y_x_diff = _abs_no_nan(np.diff(y, axis=1))
    y_y_diff = _abs_no_nan(np.diff(y, axis=0))
    x_x_diff_c = np.concatenate([x_x_diff, x_x_diff[:, -1:]], axis=1)
    y_x_diff_c = np.concatenate([y_x_diff, y_x_diff[:, -1:]], axis=1)
    x_y_diff_c = np.concatenate([x_y_diff, x_y_diff[-1:, :]], axis=0)
    y_y_diff_c = np.concatenate([y_y_diff, y_y_diff[-1:, :]], axis=0)
    x_abs_diff = np.sqrt(np.square(x_x_diff_c) + np.square(x_y_diff_c))
    y_abs_diff = np.sqrt(np.square(y_x_diff_c) + np.square(y_y_diff_c))
    if crs.is_geographic:
        x_abs_diff_r = np.radians(x_abs_diff)
        y_abs_diff_r = np.radians(y_abs_diff)
        x_abs_diff = _ER * np.cos(x_abs_diff_r) * y_abs_diff_r
        y_abs_diff = _ER * y_abs_diff_r
    xy_areas = (x_abs_diff * y_abs_diff).flatten()
    xy_areas = np.where(xy_areas > 0, xy_areas, np.nan)
    xy_res_min = math.sqrt(xy_areas[np.nanargmin(xy_areas)])
    xy_res_max = math.sqrt(xy_areas[np.nanargmax(xy_areas)])
    xy_res = 0.7 * xy_res_min + 0.3 * xy_res_max
    if crs.is_geographic:
        xy_res = math.degrees(xy_res / _ER)
    xy_res = round_to_fraction(xy_res, digits=1, resolution=0.5)
    return float(xy_res), float(xy_res)


def grid_mapping_to_coords(grid_mapping: GridMapping, xy_var_names=None, xy_dim_names=None,
                           reuse_coords: bool = False, exclude_bounds: bool = False) -> dict:
    """coords.py:340-472 — CF axis + bounds coordinate variables."""
    if reuse_coords:
        try:
            x, y = grid_mapping.x_coords, grid_mapping.y_coords
        except AttributeError:
            x, y = None, None
        if (isinstance(x, DataArray) and isinstance(y, DataArray) and x.ndim == 1
                and y.ndim == 1 and x.size == grid_mapping.width
                and y.size == grid_mapping.height):
            return {name: DataArray(coord.values, dim, coord.attrs)
                    for name, dim, coord in zip(xy_var_names, xy_dim_names, (x, y))}
    x_name, y_name = xy_var_names or grid_mapping.xy_var_names
    x_dim_name, y_dim_name = xy_dim_names or grid_mapping.xy_dim_names
    w, h = grid_mapping.size
    x1, y1, x2, y2 = grid_mapping.xy_bbox
    x_res, y_res = grid_mapping.xy_res
    x_res_05 = x_res / 2
    y_res_05 = y_res / 2
    x_data = np.linspace(x1 + x_res_05, x2 - x_res_05, w, dtype=np.float64)
    if grid_mapping.is_lon_360:
        x_data = from_lon_360(x_data)
    if grid_mapping.is_j_axis_up:
        y_data = np.linspace(y1 + y_res_05, y2 - y_res_05, h, dtype=np.float64)
    else:
        y_data = np.linspace(y2 - y_res_05, y1 + y_res_05, h, dtype=np.float64)
    if grid_mapping.crs.is_geographic:
        x_attrs = dict(long_name="longitude coordinate", standard_name="longitude",
                       units="degrees_east")
        y_attrs = dict(long_name="latitude coordinate", standard_name="latitude",
                       units="degrees_north")
    else:
        x_attrs = dict(long_name="x coordinate of projection",
                       standard_name="projection_x_coordinate")
        y_attrs = dict(long_name="y coordinate of projection",
                       standard_name="projection_y_coordinate")
    coords = {x_name: DataArray(x_data, x_dim_name, x_attrs, name=x_name),
              y_name: DataArray(y_data, y_dim_name, y_attrs, name=y_name)}
    if not exclude_bounds:
        x_b0 = np.linspace(x1, x2 - x_res, w, dtype=np.float64)
        x_b1 = np.linspace(x1 + x_res, x2, w, dtype=np.float64)
        if grid_mapping.is_lon_360:
            x_b0, x_b1 = from_lon_360(x_b0), from_lon_360(x_b1)
        if grid_mapping.is_j_axis_up:
            y_b0 = np.linspace(y1, y2 - y_res, h, dtype=np.float64)
            y_b1 = np.linspace(y1 + y_res, y2, h, dtype=np.float64)
        else:
            y_b0 = np.linspace(y2, y1 + y_res, h, dtype=np.float64)
            y_b1 = np.linspace(y2 - y_res, y1, h, dtype=np.float64)
        x_bnds_name, y_bnds_name = f"{x_name}_bnds", f"{y_name}_bnds"
        coords[x_name].attrs.update(bounds=x_bnds_name)
        coords[y_name].attrs.update(bounds=y_bnds_name)
        coords[x_bnds_name] = DataArray(np.stack([x_b0, x_b1], axis=1), (x_dim_name, "bnds"))
        coords[y_bnds_name] = DataArray(np.stack([y_b0, y_b1], axis=1), (y_dim_name, "bnds"))
    return coords

"""Regular grid mappings (restates gridmapping/regular.py:38-166)."""

from __future__ import annotations

import numpy as np

from ..crs import normalize_crs
from ..dataset import DataArray
from .base import GridMapping, _assert
from .helpers import (
    _default_xy_dim_names,
    _default_xy_var_names,
    _normalize_int_pair,
    _normalize_number_pair,
    _to_int_or_float,
    dask_linspace,
)


class RegularGridMapping(GridMapping):
    def __init__(self, **kwargs):
        kwargs.pop("is_regular", None)
        super().__init__(is_regular=True, **kwargs)
        self._xy_coords = None

    def _new_x_coords(self) -> DataArray:
        """regular.py:44-52 — blockwise dask linspace of the pixel centres."""
        self._assert_regular()
        x_res = self.x_res
        x1, x2 = self.x_min + x_res / 2, self.x_max - x_res / 2
        return DataArray(dask_linspace(x1, x2, self.width, self.tile_width),
                         dims=self.xy_dim_names[0], chunks=(self.tile_width,))

    def _new_y_coords(self) -> DataArray:
        """regular.py:54-63."""
        self._assert_regular()
        y_res = self.y_res
        y1, y2 = self.y_min + y_res / 2, self.y_max - y_res / 2
        if not self.is_j_axis_up:
            y1, y2 = y2, y1
        return DataArray(dask_linspace(y1, y2, self.height, self.tile_height),
                         dims=self.xy_dim_names[1], chunks=(self.tile_height,))

    def _new_xy_coords(self) -> DataArray:
        """regular.py:65-84 — broadcast to (2, height, width)."""
        self._assert_regular()
        x = self.x_coords.values
        y = self.y_coords.values
        xy = np.empty((2, y.size, x.size), dtype=np.float64)
        xy[0] = x[None, :]
        xy[1] = y[:, None]
        return DataArray(xy, dims=("coord", self.y_coords.dims[0], self.x_coords.dims[0]),
                         name="xy_coords",
                         chunks=(2, self.tile_height, self.tile_width))


def new_regular_grid_mapping(size, xy_min, xy_res, crs, *, tile_size=None,
                             is_j_axis_up: bool = False) -> GridMapping:
    """regular.py:87-129."""
    width, height = _normalize_int_pair(size, name="size")
    _assert(width > 1 and height > 1, "invalid size")
    x_min, y_min = _normalize_number_pair(xy_min, name="xy_min")
    x_res, y_res = _normalize_number_pair(xy_res, name="xy_res")
    _assert(x_res > 0 and y_res > 0, "invalid xy_res")
    crs = normalize_crs(crs)
    x_min = _to_int_or_float(x_min)
    y_min = _to_int_or_float(y_min)
    x_max = _to_int_or_float(x_min + x_res * width)
    y_max = _to_int_or_float(y_min + y_res * height)
    if crs.is_geographic:
        if y_min < -90:
            raise ValueError("invalid y_min")
        if y_max > 90:
            raise ValueError("invalid size, y_min combination")
    return RegularGridMapping(
        crs=crs,
        size=(width, height),
        tile_size=tile_size or (width, height),
        xy_bbox=(x_min, y_min, x_max, y_max),
        xy_res=(x_res, y_res),
        xy_var_names=_default_xy_var_names(crs),
        xy_dim_names=_default_xy_dim_names(crs),
        is_lon_360=(x_max > 180) and crs.is_geographic,
        is_j_axis_up=is_j_axis_up,
    )


def to_regular_grid_mapping(grid_mapping: GridMapping, *, tile_size=None,
                            is_j_axis_up: bool = False) -> GridMapping:
    """regular.py:132-166."""
    if grid_mapping.is_regular:
        if tile_size is not None or is_j_axis_up != grid_mapping.is_j_axis_up:
            return grid_mapping.derive(tile_size=tile_size, is_j_axis_up=is_j_axis_up)
        return grid_mapping
    x_min, y_min, x_max, y_max = grid_mapping.xy_bbox
    x_res, y_res = grid_mapping.xy_res
    xy_res = min(x_res, y_res) or max(x_res, y_res)
    width = round((x_max - x_min + xy_res) / xy_res)
    height = round((y_max - y_min + xy_res) / xy_res)
    width = width if width >= 2 else 2
    height = height if height >= 2 else 2
    if tile_size is None:
        tile_size = grid_mapping.tile_size
    return new_regular_grid_mapping(size=(width, height), xy_min=(x_min, y_min), xy_res=xy_res,
                                    crs=grid_mapping.crs, tile_size=tile_size,
                                    is_j_axis_up=is_j_axis_up)

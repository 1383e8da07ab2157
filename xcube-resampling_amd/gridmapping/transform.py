"""GridMapping.transform — restates gridmapping/transform.py:57-125.

The target-CRS coordinates of every source pixel centre are computed with
the engine's Transformer (PROJ's formulas for the supported CRS families,
crs.py / projections.py), eagerly in numpy instead of a dask ufunc; the
result is a 2-D coordinate grid mapping (new_grid_mapping_from_coords), as
in the reference.
"""

from __future__ import annotations

from ..crs import Transformer, normalize_crs
from ..dataset import DataArray
from .base import DEFAULT_TOLERANCE, GridMapping
from .coords import new_grid_mapping_from_coords
from .helpers import _assert_valid_xy_names, _normalize_number_pair


def transform_grid_mapping(grid_mapping: GridMapping, crs, *, xy_res=None, tile_size=None,
                           xy_var_names=None, tolerance: float = DEFAULT_TOLERANCE
                           ) -> GridMapping:
    """transform.py:57-125."""
    target_crs = normalize_crs(crs)
    if xy_var_names:
        _assert_valid_xy_names(xy_var_names, name="xy_var_names")
    source_crs = grid_mapping.crs
    if source_crs == target_crs:
        if tile_size is not None or xy_var_names is not None:
            return grid_mapping.derive(tile_size=tile_size, xy_var_names=xy_var_names)
        return grid_mapping

    transformer = Transformer.from_crs(source_crs, target_crs, always_xy=True)
    xy = grid_mapping.xy_coords
    x2, y2 = transformer.transform(xy.values[0], xy.values[1])

    if xy_res is not None:
        bbox = transformer.transform_bounds(*grid_mapping.xy_bbox, densify_pts=101)
        x_res, y_res = _normalize_number_pair(xy_res)
        x_res_05, y_res_05 = x_res / 2, y_res / 2
        xy_bbox = (bbox[0] - x_res_05, bbox[1] - y_res_05, bbox[2] + x_res_05,
                   bbox[3] + y_res_05)
    else:
        xy_bbox = None

    xy_var_names = xy_var_names or ("transformed_x", "transformed_y")
    if tile_size is None:
        tile_size = grid_mapping.tile_size
    dims = xy.dims[1:]
    return new_grid_mapping_from_coords(
        x_coords=DataArray(x2, dims, name=xy_var_names[0]),
        y_coords=DataArray(y2, dims, name=xy_var_names[1]),
        crs=target_crs, xy_res=xy_res, xy_bbox=xy_bbox, tile_size=tile_size,
        tolerance=tolerance)

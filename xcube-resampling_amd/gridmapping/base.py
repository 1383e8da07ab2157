"""GridMapping: image grid + its mapping to CRS coordinates.

Restates gridmapping/base.py:59-913 of the reference on top of the engine's
own CRS registry and Dataset model (no pyproj / xarray / dask).  The public
surface (factories, properties, affine transforms, tile bounding boxes,
``is_close``) keeps the reference's names, argument meaning and errors.
``ij_bboxes_from_xy_bboxes`` runs the K4 HIP kernel (``xrs_ij_bboxes``) on the
device: the brute-force per-tile bbox scan the reference runs as a parallel
numba kernel (bboxes.py:28-106).
"""

from __future__ import annotations

import abc
import copy
import math
import threading
from typing import Any, Callable

import numpy as np

from ..crs import CRS, CRS_CRS84, CRS_WGS84, normalize_crs
from ..dataset import DataArray
from .helpers import (
    _assert_valid_xy_names,
    _from_affine,
    _normalize_int_pair,
    _normalize_number_pair,
    _to_affine,
    chunk_sizes,
    scale_xy_res_and_size,
)

CRS84 = "OGC:CRS84"
DEFAULT_TOLERANCE = 1.0e-5


def _assert(cond: bool, message: str, exception_type=ValueError):
    if not cond:
        raise exception_type(message)


class GridMapping(abc.ABC):
    """Abstract grid mapping (base.py:59-80).  Use the factories
    :meth:`regular`, :meth:`from_dataset`, :meth:`from_coords`."""

    def __init__(self, /, size, tile_size, xy_bbox, xy_res, crs: CRS,
                 xy_var_names: tuple[str, str], xy_dim_names: tuple[str, str],
                 is_regular: bool | None = None, is_lon_360: bool | None = None,
                 is_j_axis_up: bool | None = None, x_coords: DataArray | None = None,
                 y_coords: DataArray | None = None):
        width, height = _normalize_int_pair(size, name="size")
        _assert(width > 1 and height > 1, "invalid size")
        tile_width, tile_height = _normalize_int_pair(tile_size, default=(width, height))
        _assert(tile_width > 1 and tile_height > 1, "invalid tile_size")
        _assert(xy_bbox is not None, "xy_bbox must be given")
        _assert(xy_res is not None, "xy_res must be given")
        _assert_valid_xy_names(xy_var_names, name="xy_var_names")
        _assert_valid_xy_names(xy_dim_names, name="xy_dim_names")
        if not isinstance(crs, CRS):
            raise TypeError("crs must be an instance of CRS")
        for c, n in ((x_coords, "x_coords"), (y_coords, "y_coords")):
            if c is not None:
                _assert(c.ndim in (1, 2), f"{n}.ndim must be 1 or 2, was {c.ndim}")
        x_min, y_min, x_max, y_max = xy_bbox
        x_res, y_res = _normalize_number_pair(xy_res, name="xy_res")
        _assert(x_res > 0 and y_res > 0, "invalid xy_res")
        self._lock = threading.RLock()
        self._size = width, height
        self._tile_size = tile_width, tile_height
        self._xy_bbox = x_min, y_min, x_max, y_max
        self._xy_res = x_res, y_res
        self._crs = crs
        self._xy_var_names = xy_var_names
        self._xy_dim_names = xy_dim_names
        self._is_regular = is_regular
        self._is_lon_360 = is_lon_360
        self._is_j_axis_up = is_j_axis_up
        self._x_coords = x_coords
        self._y_coords = y_coords
        self._xy_coords = None

    # ---- derivation (base.py:145-246) ------------------------------------
    def derive(self, /, xy_var_names=None, xy_dim_names=None, tile_size=None,
               is_j_axis_up=None) -> "GridMapping":
        other = copy.copy(self)
        other._lock = threading.RLock()
        if xy_var_names is not None:
            _assert_valid_xy_names(xy_var_names, name="xy_var_names")
            other._xy_var_names = xy_var_names
        if xy_dim_names is not None:
            _assert_valid_xy_names(xy_dim_names, name="xy_dim_names")
            other._xy_dim_names = xy_dim_names
        if tile_size is not None:
            tile_width, tile_height = _normalize_int_pair(tile_size, name="tile_size")
            _assert(tile_width > 1 and tile_height > 1, "invalid tile_size")
            if other.tile_size != (tile_width, tile_height):
                # As in the reference, coordinates already computed are kept
                # (a dask rechunk does not change values); coordinates not yet
                # computed will use the new tile size (blockwise linspace).
                other._tile_size = tile_width, tile_height
        if is_j_axis_up is not None and is_j_axis_up != other._is_j_axis_up:
            other._is_j_axis_up = is_j_axis_up
            if other._y_coords is not None:
                other._y_coords = other._y_coords[::-1]
            if other._xy_coords is not None:
                other._xy_coords = other._xy_coords[:, ::-1, :]
        return other

    def scale(self, xy_scale, tile_size=None) -> "GridMapping":
        self._assert_regular()
        x_scale, y_scale = _normalize_number_pair(xy_scale)
        new_xy_res, new_size = scale_xy_res_and_size(self.xy_res, self.size, (x_scale, y_scale))
        if tile_size is not None:
            tile_width, tile_height = _normalize_int_pair(tile_size, name="tile_size")
        else:
            tile_width, tile_height = self.tile_size
        tile_width = min(new_size[0], tile_width)
        tile_height = min(new_size[1], tile_height)
        return self.regular(new_size, (self.x_min, self.y_min), new_xy_res, self.crs,
                            tile_size=(tile_width, tile_height),
                            is_j_axis_up=self.is_j_axis_up).derive(
            xy_dim_names=self.xy_dim_names, xy_var_names=self.xy_var_names)

    # ---- properties (base.py:248-434) -------------------------------------
    size = property(lambda self: self._size)
    width = property(lambda self: self._size[0])
    height = property(lambda self: self._size[1])
    tile_size = property(lambda self: self._tile_size)
    tile_width = property(lambda self: self._tile_size[0])
    tile_height = property(lambda self: self._tile_size[1])
    is_tiled = property(lambda self: self._size != self._tile_size)
    xy_var_names = property(lambda self: self._xy_var_names)
    xy_dim_names = property(lambda self: self._xy_dim_names)
    xy_bbox = property(lambda self: self._xy_bbox)
    x_min = property(lambda self: self._xy_bbox[0])
    y_min = property(lambda self: self._xy_bbox[1])
    x_max = property(lambda self: self._xy_bbox[2])
    y_max = property(lambda self: self._xy_bbox[3])
    xy_res = property(lambda self: self._xy_res)
    x_res = property(lambda self: self._xy_res[0])
    y_res = property(lambda self: self._xy_res[1])
    crs = property(lambda self: self._crs)
    is_lon_360 = property(lambda self: self._is_lon_360)
    is_regular = property(lambda self: self._is_regular)
    is_j_axis_up = property(lambda self: self._is_j_axis_up)

    @property
    def spatial_unit_name(self) -> str:
        return self._crs.axis_info[0].unit_name

    @property
    def x_coords(self) -> DataArray:
        return self._get_computed_attribute("_x_coords", self._new_x_coords)

    @property
    def y_coords(self) -> DataArray:
        return self._get_computed_attribute("_y_coords", self._new_y_coords)

    @property
    def xy_coords(self) -> DataArray:
        xy = self._get_computed_attribute("_xy_coords", self._new_xy_coords)
        _assert(xy.ndim == 3 and xy.shape[0] == 2 and xy.shape[1] >= 2 and xy.shape[2] >= 2,
                "xy_coords must have dimensions (2, height, width) with height >= 2 and width >= 2")
        return xy

    @property
    def xy_coords_chunks(self) -> tuple[int, int, int]:
        return 2, self.tile_height, self.tile_width

    @abc.abstractmethod
    def _new_x_coords(self) -> DataArray: ...

    @abc.abstractmethod
    def _new_y_coords(self) -> DataArray: ...

    @abc.abstractmethod
    def _new_xy_coords(self) -> DataArray: ...

    def _get_computed_attribute(self, name: str, computer: Callable[[], Any]) -> Any:
        value = getattr(self, name)
        if value is not None:
            return value
        with self._lock:
            value = getattr(self, name)
            if value is not None:
                return value
            value = computer()
            setattr(self, name, value)
            return value

    # ---- affine transforms (base.py:436-496) ------------------------------
    @property
    def ij_to_xy_transform(self):
        self._assert_regular()
        if self.is_j_axis_up:
            return (self.x_res, 0.0, self.x_min), (0.0, self.y_res, self.y_min)
        return (self.x_res, 0.0, self.x_min), (0.0, -self.y_res, self.y_max)

    @property
    def xy_to_ij_transform(self):
        self._assert_regular()
        return _from_affine(~_to_affine(self.ij_to_xy_transform))

    def ij_transform_to(self, other: "GridMapping"):
        self._assert_regular()
        self.assert_regular(other, name="other")
        a = _to_affine(self.ij_to_xy_transform)
        b = _to_affine(other.xy_to_ij_transform)
        return _from_affine(b * a)

    def ij_transform_from(self, other: "GridMapping"):
        self._assert_regular()
        self.assert_regular(other, name="other")
        a = _to_affine(self.ij_transform_to(other))
        return _from_affine(~a)

    # ---- tile boxes (base.py:498-533) --------------------------------------
    @property
    def ij_bbox(self) -> tuple[int, int, int, int]:
        return 0, 0, self.width, self.height

    @property
    def ij_bboxes(self) -> np.ndarray:
        ys = chunk_sizes(self.height, self.tile_height)
        xs = chunk_sizes(self.width, self.tile_width)
        y0 = np.concatenate([[0], np.cumsum(ys)])
        x0 = np.concatenate([[0], np.cumsum(xs)])
        out = np.ndarray((len(ys) * len(xs), 4), dtype=np.int64)
        k = 0
        for j in range(len(ys)):
            for i in range(len(xs)):
                out[k] = (x0[i], y0[j], x0[i + 1], y0[j + 1])
                k += 1
        return out

    @property
    def xy_bboxes(self) -> np.ndarray:
        if self.is_j_axis_up:
            xy_offset = np.array([self.x_min, self.y_min, self.x_min, self.y_min])
            xy_scale = np.array([self.x_res, self.y_res, self.x_res, self.y_res])
            return xy_offset + xy_scale * self.ij_bboxes
        xy_offset = np.array([self.x_min, self.y_max, self.x_min, self.y_max])
        xy_scale = np.array([self.x_res, -self.y_res, self.x_res, -self.y_res])
        xy_bboxes = xy_offset + xy_scale * self.ij_bboxes
        xy_bboxes[:, [1, 3]] = xy_bboxes[:, [3, 1]]
        return xy_bboxes

    def ij_bbox_from_xy_bbox(self, xy_bbox, xy_border: float = 0.0, ij_border: int = 0):
        xy_bboxes = np.array([xy_bbox], dtype=np.float64)
        ij_bboxes = np.full_like(xy_bboxes, -1, dtype=np.int64)
        self.ij_bboxes_from_xy_bboxes(xy_bboxes, xy_border=xy_border, ij_border=ij_border,
                                      ij_bboxes=ij_bboxes)
        return tuple(map(int, ij_bboxes[0]))

    def ij_bboxes_from_xy_bboxes(self, xy_bboxes: np.ndarray, xy_border: float = 0.0,
                                 ij_border: int = 0, ij_bboxes: np.ndarray | None = None,
                                 grid: tuple[int, int] | None = None):
        """base.py:565-629 — per-box source ij bbox via the K4 HIP kernel.

        ``grid=(ntx, nty)``: the boxes are the tiles of a regular grid (engine
        extension; enables the per-pixel tile search)."""
        from ..kernels import ij_bboxes as _k4

        xy_bboxes = np.asarray(xy_bboxes, dtype=np.float64)
        if ij_bboxes is None:
            ij_bboxes = np.full_like(xy_bboxes, -1, dtype=np.int64)
        xy = self.xy_coords.data
        ij_bboxes[:, :] = _k4(xy[0], xy[1], xy_bboxes, xy_border, ij_border, grid=grid)
        return ij_bboxes

    # ---- misc ------------------------------------------------------------
    def to_coords(self, xy_var_names=None, xy_dim_names=None, exclude_bounds: bool = False,
                  reuse_coords: bool = False):
        self._assert_regular()
        from .coords import grid_mapping_to_coords
        return grid_mapping_to_coords(self, xy_var_names=xy_var_names, xy_dim_names=xy_dim_names,
                                      exclude_bounds=exclude_bounds, reuse_coords=reuse_coords)

    def transform(self, crs, *, xy_res=None, tile_size=None, xy_var_names=None,
                  tolerance: float = DEFAULT_TOLERANCE) -> "GridMapping":
        from .transform import transform_grid_mapping
        return transform_grid_mapping(self, crs, xy_res=xy_res, tile_size=tile_size,
                                      xy_var_names=xy_var_names, tolerance=tolerance)

    @classmethod
    def regular(cls, size, xy_min, xy_res, crs, *, tile_size=None,
                is_j_axis_up: bool = False) -> "GridMapping":
        from .regular import new_regular_grid_mapping
        return new_regular_grid_mapping(size=size, xy_min=xy_min, xy_res=xy_res, crs=crs,
                                        tile_size=tile_size, is_j_axis_up=is_j_axis_up)

    def to_regular(self, tile_size=None, is_j_axis_up: bool = False) -> "GridMapping":
        from .regular import to_regular_grid_mapping
        return to_regular_grid_mapping(self, tile_size=tile_size, is_j_axis_up=is_j_axis_up)

    @classmethod
    def from_dataset(cls, dataset, *, crs=None, tile_size=None, prefer_is_regular: bool = True,
                     prefer_crs=None, emit_warnings: bool = False,
                     tolerance: float = DEFAULT_TOLERANCE) -> "GridMapping":
        from .dataset import new_grid_mapping_from_dataset
        return new_grid_mapping_from_dataset(dataset=dataset, crs=crs, tile_size=tile_size,
                                             prefer_is_regular=prefer_is_regular,
                                             prefer_crs=prefer_crs,
                                             emit_warnings=emit_warnings, tolerance=tolerance)

    @classmethod
    def from_coords(cls, x_coords, y_coords, crs, *, tile_size=None,
                    tolerance: float = DEFAULT_TOLERANCE) -> "GridMapping":
        from .coords import new_grid_mapping_from_coords
        return new_grid_mapping_from_coords(x_coords=x_coords, y_coords=y_coords, crs=crs,
                                            tile_size=tile_size, tolerance=tolerance)

    def is_close(self, other: "GridMapping", tolerance: float = DEFAULT_TOLERANCE) -> bool:
        """base.py:839-876."""
        if self is other:
            return True
        if (self.is_j_axis_up == other.is_j_axis_up and self.is_lon_360 == other.is_lon_360
                and self.is_regular == other.is_regular and self.size == other.size
                and self.tile_size == other.tile_size and self.crs == other.crs):
            sxr, syr = self.xy_res
            oxr, oyr = other.xy_res
            if math.isclose(sxr, oxr, abs_tol=tolerance) and math.isclose(syr, oyr, abs_tol=tolerance):
                sx1, sy1, sx2, sy2 = self.xy_bbox
                ox1, oy1, ox2, oy2 = other.xy_bbox
                return (math.isclose(sx1, ox1, abs_tol=tolerance)
                        and math.isclose(sy1, oy1, abs_tol=tolerance)
                        and math.isclose(sx2, ox2, abs_tol=tolerance)
                        and math.isclose(sy2, oy2, abs_tol=tolerance))
        return False

    @classmethod
    def assert_regular(cls, value: Any, name: str | None = None):
        if not isinstance(value, GridMapping):
            raise TypeError(f"{name or 'value'} must be an instance of GridMapping")
        if not value.is_regular:
            raise ValueError(f"{name or 'value'} must be a regular grid mapping")

    def _assert_regular(self):
        if not self.is_regular:
            raise NotImplementedError("Operation not implemented for non-regular grid mappings")

    def __repr__(self) -> str:
        return (f"{type(self).__name__}(size={self.size}, tile_size={self.tile_size}, "
                f"xy_bbox={self.xy_bbox}, xy_res={self.xy_res}, crs={self.crs.srs}, "
                f"is_regular={self.is_regular}, is_j_axis_up={self.is_j_axis_up})")

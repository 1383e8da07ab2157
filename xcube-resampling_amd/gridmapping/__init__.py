"""GridMapping API (mirrors xcube_resampling.gridmapping)."""

from ..crs import CRS_CRS84, CRS_WGS84
from .base import CRS84, DEFAULT_TOLERANCE, GridMapping
from .coords import Coords1DGridMapping, Coords2DGridMapping
from .regular import RegularGridMapping

__all__ = [
    "CRS84",
    "CRS_CRS84",
    "CRS_WGS84",
    "DEFAULT_TOLERANCE",
    "Coords1DGridMapping",
    "Coords2DGridMapping",
    "GridMapping",
    "RegularGridMapping",
]

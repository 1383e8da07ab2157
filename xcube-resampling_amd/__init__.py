"""xcube_resampling_amd — MI355X-native engine for xcube-resampling's hot path.

Drop-in API of xcube_resampling (spatial.py, affine.py, reproject.py,
rectify.py, gridmapping/): the pixel work runs in hand-written HIP kernels for
gfx950 (libxrs.so, C-ABI in include/xrs.h); the host code restates the
reference's orchestration, tiling math and parameter semantics.
"""

from .version import version as __version__
from .constants import LOG
from .crs import CRS, CRS_CRS84, CRS_WEBMERC, CRS_WGS84, Transformer
from .dataset import DataArray, Dataset
from .gridmapping import GridMapping
from .options import get_options, set_options
from .affine import affine_transform_dataset, resample_dataset
from .reproject import plan_reproject, reproject_dataset
from .rectify import rectify_dataset
from .spatial import resample_in_space

__all__ = [
    "CRS",
    "CRS_CRS84",
    "CRS_WEBMERC",
    "CRS_WGS84",
    "DataArray",
    "affine_transform_dataset",
    "resample_dataset",
    "Dataset",
    "GridMapping",
    "LOG",
    "Transformer",
    "get_options",
    "plan_reproject",
    "rectify_dataset",
    "reproject_dataset",
    "resample_in_space",
    "set_options",
]

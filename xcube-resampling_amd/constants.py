"""Types and constants (mirrors xcube_resampling/constants.py:30-82)."""

from __future__ import annotations

import logging
from collections.abc import Hashable, Mapping
from typing import Literal, TypeAlias

import numpy as np

FloatInt = int | float
AffineTransformMatrix = tuple[tuple[FloatInt, FloatInt, FloatInt],
                              tuple[FloatInt, FloatInt, FloatInt]]
AggMethod: TypeAlias = Literal["center", "count", "first", "last", "max", "mean", "median",
                               "mode", "min", "prod", "std", "sum", "var"]
AggMethods: TypeAlias = AggMethod | Mapping[np.dtype | str, AggMethod]
# The engine's aggregation methods run on the device (xrs_affine_coarsen); the
# names are the reference's keys of AGG_METHODS (constants.py:51-65).
AGG_METHOD_NAMES = ("center", "count", "first", "last", "prod", "max", "mean", "median",
                    "min", "mode", "std", "sum", "var")
InterpMethodInt = Literal[0, 1]
InterpMethodStr = Literal["nearest", "triangular", "bilinear"]
InterpMethod = InterpMethodInt | InterpMethodStr
InterpMethods: TypeAlias = InterpMethod | Mapping[np.dtype | Hashable, InterpMethod]
INTERP_METHOD_MAPPING = {0: "nearest", 1: "bilinear", "nearest": 0, "bilinear": 1}
RecoverNans: TypeAlias = bool | Mapping[np.dtype | str, bool]
FillValues: TypeAlias = FloatInt | Mapping[np.dtype | str, FloatInt]

FILLVALUE_UINT8 = 255
FILLVALUE_UINT16 = 65535
FILLVALUE_INT = -1
FILLVALUE_FLOAT = np.nan

SCALE_LIMIT = 0.95
UV_DELTA = 1e-3

LOG = logging.getLogger("xcube.resampling")

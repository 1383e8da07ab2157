"""Numeric helpers of the grid-mapping layer.

Restates gridmapping/helpers.py of the reference (numbers quoted below), the
``affine`` package arithmetic it delegates to (helpers.py:51-56) and dask's
blockwise ``linspace`` (regular.py:50,61 call ``da.linspace(..., chunks=tile)``).
These functions define every sample position of the hot path, so they are
restated operation by operation (same float64 operations in the same order).
"""

from __future__ import annotations

import math
from fractions import Fraction
from typing import Any

import numpy as np

FloatInt = int | float

_UNDEFINED = object()


def _to_int_or_float(x: FloatInt) -> FloatInt:
    """helpers.py:39-48 — snap values within 1e-5 (relative) of an int."""
    if isinstance(x, int):
        return x
    xf = float(x)
    xi = round(xf)
    return xi if math.isclose(xi, xf, rel_tol=1e-5) else xf


def _normalize_int_pair(value: Any, name: str | None = None,
                        default: Any = _UNDEFINED) -> tuple[int, int]:
    """helpers.py:66-78."""
    if isinstance(value, int):
        return value, value
    elif value is not None:
        x, y = value
        return int(x), int(y)
    elif default is not _UNDEFINED:
        return default
    raise ValueError(f"{name} must be an int or a sequence of two ints")


def _normalize_number_pair(value: Any, name: str | None = None,
                           default: Any = _UNDEFINED) -> tuple[FloatInt, FloatInt]:
    """helpers.py:81-94."""
    if isinstance(value, (float, int)):
        return _to_int_or_float(value), _to_int_or_float(value)
    elif value is not None:
        x, y = value
        return _to_int_or_float(x), _to_int_or_float(y)
    elif default is not _UNDEFINED:
        return default
    raise ValueError(f"{name} must be a number or a sequence of two numbers")


_RESOLUTIONS = {10: (1, 0), 20: (2, 0), 25: (25, 1), 50: (5, 0), 100: (1, -1)}
_RESOLUTION_SET = {k / 100 for k in _RESOLUTIONS}


def round_to_fraction(value: float, digits: int = 2, resolution: float = 1) -> Fraction:
    """helpers.py:203-239 — round at `digits` significant digits, as Fraction."""
    if digits < 1:
        raise ValueError("digits must be a positive integer")
    resolution_key = round(100 * resolution)
    if resolution_key not in _RESOLUTIONS or not math.isclose(100 * resolution, resolution_key):
        raise ValueError(f"resolution must be one of {_RESOLUTION_SET}")
    if value == 0:
        return Fraction(0, 1)
    sign = 1
    if value < 0:
        sign = -1
        value = -value
    resolution, resolution_digits = _RESOLUTIONS[resolution_key]
    exponent = math.floor(math.log10(value)) - digits - resolution_digits
    if exponent >= 0:
        magnitude = Fraction(10**exponent, 1)
    else:
        magnitude = Fraction(1, 10**-exponent)
    scaled_value = value / magnitude
    discrete_value = resolution * round(scaled_value / resolution)
    return (sign * discrete_value) * magnitude


def scale_xy_res_and_size(xy_res, size, xy_scale):
    """helpers.py:242-255."""
    x_res, y_res = xy_res
    x_scale, y_scale = xy_scale
    w, h = size
    w, h = round(x_scale * w), round(y_scale * h)
    return (x_res / x_scale, y_res / y_scale), (w if w >= 2 else 2, h if h >= 2 else 2)


def to_lon_360(lon):
    """helpers.py:97-102."""
    lon = np.asarray(lon)
    return np.where(lon >= 0.0, lon, lon + 360.0)


def from_lon_360(lon):
    """helpers.py:105-110."""
    lon = np.asarray(lon)
    return np.where(lon <= 180.0, lon, lon - 360.0)


def _default_xy_var_names(crs) -> tuple[str, str]:
    """helpers.py:164-165."""
    return ("lon", "lat") if crs.is_geographic else ("x", "y")


def _default_xy_dim_names(crs) -> tuple[str, str]:
    return _default_xy_var_names(crs)


def _assert_valid_xy_names(value: Any, name: str | None = None):
    """helpers.py:172-177."""
    if not isinstance(value, tuple):
        raise TypeError(f"{name or 'value'} must be an instance of tuple")
    if not (len(value) == 2 and all(value) and value[0] != value[1]):
        raise ValueError(f"invalid {name or 'value'}")


# --------------------------------------------------------------------------
# affine package arithmetic (affine>=2.2, Affine.__mul__ / __invert__)
# --------------------------------------------------------------------------

class Affine(tuple):
    """3x3 affine matrix (a, b, c, d, e, f, 0, 0, 1) with the affine package's
    multiplication and inversion formulas (evaluated in the same order)."""

    def __new__(cls, a, b, c, d, e, f, g=0.0, h=0.0, i=1.0):
        return tuple.__new__(cls, (a, b, c, d, e, f, g, h, i))

    a = property(lambda s: s[0])
    b = property(lambda s: s[1])
    c = property(lambda s: s[2])
    d = property(lambda s: s[3])
    e = property(lambda s: s[4])
    f = property(lambda s: s[5])

    @property
    def determinant(self):
        a, b, _, d, e, _ = self[:6]
        return a * e - b * d

    def __mul__(self, other):
        sa, sb, sc, sd, se, sf = self[:6]
        if isinstance(other, Affine):
            oa, ob, oc, od, oe, of = other[:6]
            return Affine(sa * oa + sb * od, sa * ob + sb * oe, sa * oc + sb * of + sc,
                          sd * oa + se * od, sd * ob + se * oe, sd * oc + se * of + sf)
        vx, vy = other
        return (vx * sa + vy * sb + sc, vx * sd + vy * se + sf)

    def __invert__(self):
        if self.determinant == 0:
            raise ZeroDivisionError("Cannot invert degenerate transform")
        idet = 1.0 / self.determinant
        sa, sb, sc, sd, se, sf = self[:6]
        ra = se * idet
        rb = -sb * idet
        rd = -sd * idet
        re = sa * idet
        return Affine(ra, rb, -sc * ra - sf * rb, rd, re, -sc * rd - sf * re)


def _from_affine(matrix: Affine):
    """helpers.py:51-52."""
    return (matrix.a, matrix.b, matrix.c), (matrix.d, matrix.e, matrix.f)


def _to_affine(matrix) -> Affine:
    """helpers.py:55-56."""
    return Affine(*matrix[0], *matrix[1])


# --------------------------------------------------------------------------
# dask.array.linspace (blockwise) — coordinates of regular grid mappings
# --------------------------------------------------------------------------

def dask_linspace(start: float, stop: float, num: int, chunk: int | None) -> np.ndarray:
    """Values of ``dask.array.linspace(start, stop, num, chunks=chunk)``.

    dask computes a float step once, then every block independently with
    ``np.linspace(blockstart, blockstart + (bs-1)*step, bs)`` where
    ``blockstart`` accumulates ``step * bs`` block by block.
    """
    num = int(num)
    chunk = num if not chunk else int(chunk)
    div = num - 1
    step = float(stop - start) / div
    out = np.empty(num, dtype=np.float64)
    blockstart = start
    pos = 0
    while pos < num:
        bs = min(chunk, num - pos)
        blockstop = blockstart + ((bs - 1) * step)
        out[pos:pos + bs] = np.linspace(blockstart, blockstop, bs)
        blockstart = blockstart + (step * bs)
        pos += bs
    return out


def chunk_sizes(size: int, chunk: int) -> tuple[int, ...]:
    """dask.py:138-144 (`get_chunk_sizes` for one dimension)."""
    n = size // chunk
    return (chunk,) * n + ((size % chunk,) if n * chunk < size else ())

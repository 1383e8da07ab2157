"""Coordinate reference systems and transformations for the resampling engine.

The reference reaches PROJ through ``pyproj`` (``pyproj.CRS``,
``pyproj.Transformer.from_crs(..., always_xy=True)``; call sites
reproject.py:124-126,347,398,483 and rectify.py:196-203).  Neither pyproj nor
PROJ's database is available here or on the GPU box, so this module restates
the small part of PROJ the engine needs:

* a registry of the CRSs the engine supports (geographic WGS 84 in both axis
  orders, Web Mercator, the UTM zones EPSG:326xx/327xx, LAEA Europe
  EPSG:3035, and transverse Mercator / LAEA CRSs given by CF parameters), with
  the attributes the reference reads (``is_geographic``, ``name``, ``equals``,
  ``to_cf``, ``axis_info``);
* ``Transformer`` with ``transform`` and ``transform_bounds`` following PROJ's
  formulas: spherical Mercator (``webmerc``: merc_s_forward / merc_s_inverse
  with ``a = 6378137``; coordinates de-scaled by the reciprocal ``ra = 1/a``;
  radians <-> degrees through a precomputed ``unitconvert`` factor), the
  ellipsoidal ``tmerc`` and ``laea`` of projections.py, and PROJ's
  ``proj_trans_bounds`` edge densification (21 points per edge by default).

If ``pyproj`` is importable, ``CRS.from_pyproj`` accepts pyproj objects for the
supported codes.  Transformations between unsupported CRS pairs raise
``NotImplementedError`` instead of silently approximating.
"""

from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

# PROJ constants (proj_internal.h / unitconvert.cpp)
_DEG_TO_RAD = 0.017453292519943296
_RAD_TO_DEG_FACTOR = 1.0 / _DEG_TO_RAD   # unitconvert xy_factor rad -> deg
_WGS84_A = 6378137.0
_WGS84_RF = 298.257223563


@dataclass(frozen=True)
class AxisInfo:
    name: str
    abbrev: str
    direction: str
    unit_name: str


@dataclass(frozen=True, eq=False)
class CRS:
    """A coordinate reference system known to the engine.

    Mirrors the subset of ``pyproj.CRS`` the reference uses
    (gridmapping/base.py:398-404, utils.py:187-189, cfconv.py).
    """

    authority: str          # "EPSG", "OGC" or "CF" (defined by CF parameters)
    code: str               # "4326", "CRS84", "3857", "32632", "3035", ...
    name: str
    kind: str               # "geographic" | "webmerc" | "tmerc" | "laea"
    axis_order: str         # "latlon" | "lonlat" | "en"
    cf: dict = field(default_factory=dict)
    # projection parameters (tmerc / laea): ellipsoid name, lon_0, lat_0, k0,
    # false easting, false northing
    params: tuple = ()

    # ---- pyproj-like API ------------------------------------------------
    @property
    def is_geographic(self) -> bool:
        # a rotated-pole grid is a derived geographic CRS (pyproj: is_geographic)
        return self.kind in ("geographic", "rotated")

    @property
    def is_projected(self) -> bool:
        return not self.is_geographic

    @property
    def type_name(self) -> str:
        """pyproj's CRS.type_name for the kinds the engine knows (the
        reference's tests and dataset.py pick grid mappings by it)."""
        if self.kind == "rotated":
            return "Derived Geographic 2D CRS"
        return "Geographic 2D CRS" if self.is_geographic else "Projected CRS"

    @property
    def srs(self) -> str:
        return f"{self.authority}:{self.code}"

    def to_string(self) -> str:
        return self.srs

    def to_epsg(self) -> int | None:
        return int(self.code) if self.authority == "EPSG" else None

    @property
    def axis_info(self) -> list[AxisInfo]:
        if self.is_geographic:
            lat = AxisInfo("Geodetic latitude", "Lat", "north", "degree")
            lon = AxisInfo("Geodetic longitude", "Lon", "east", "degree")
            return [lat, lon] if self.axis_order == "latlon" else [lon, lat]
        return [
            AxisInfo("Easting", "X", "east", "metre"),
            AxisInfo("Northing", "Y", "north", "metre"),
        ]

    def to_cf(self) -> dict:
        return dict(self.cf)

    def equals(self, other, ignore_axis_order: bool = False) -> bool:
        other = _as_crs(other)
        if other is None:
            return False
        if self.kind != other.kind or self.params != other.params:
            return False
        if ignore_axis_order:
            return True
        return self.axis_order == other.axis_order

    def __eq__(self, other) -> bool:
        try:
            other = _as_crs(other)
        except (ValueError, TypeError):
            return False
        return other is not None and self.equals(other)

    def __hash__(self) -> int:
        return hash((self.kind, self.axis_order, self.params))

    def __repr__(self) -> str:
        return f"<CRS {self.srs}: {self.name}>"

    __str__ = to_string

    # ---- construction ------------------------------------------------------
    @classmethod
    def from_string(cls, value: str) -> "CRS":
        key = value.strip().upper().replace(" ", "")
        if key in _ALIASES:
            return _REGISTRY[_ALIASES[key]]
        code = key[5:] if key.startswith("EPSG:") else key
        if code.isdigit():
            c = int(code)
            if 32601 <= c <= 32660 or 32701 <= c <= 32760:
                return utm_crs(c % 100, south=c > 32700)
        raise ValueError(f"unsupported CRS: {value!r}")

    @classmethod
    def from_epsg(cls, code: int | str) -> "CRS":
        return cls.from_string(f"EPSG:{int(code)}")

    @classmethod
    def from_user_input(cls, value) -> "CRS":
        crs = _as_crs(value)
        if crs is None:
            raise ValueError(f"unsupported CRS: {value!r}")
        return crs

    @classmethod
    def from_cf(cls, attrs: dict) -> "CRS":
        """Recognise a CRS from CF grid-mapping attributes (cfconv.py:66-212)."""
        for key in ("crs_wkt", "spatial_ref"):
            wkt = attrs.get(key)
            if isinstance(wkt, str):
                for crs in _REGISTRY.values():
                    if crs.cf.get("crs_wkt") == wkt:
                        return crs
                if "Pseudo-Mercator" in wkt or "Popular Visualisation" in wkt:
                    return _REGISTRY["EPSG:3857"]
                if wkt.startswith("GEOGCRS") or wkt.startswith("GEOGCS"):
                    if "CRS84" in wkt:
                        return _REGISTRY["OGC:CRS84"]
                    return _REGISTRY["EPSG:4326"]
        gm_name = attrs.get("grid_mapping_name")
        wkt = attrs.get("crs_wkt") or attrs.get("spatial_ref")
        if isinstance(wkt, str):
            for crs in list(_REGISTRY.values()) + list(_UTM_CACHE.values()):
                if crs.cf.get("crs_wkt") == wkt:
                    return crs
        if gm_name in ("transverse_mercator", "lambert_azimuthal_equal_area"):
            return _projected_from_cf(attrs)
        if gm_name == "latitude_longitude":
            return _REGISTRY["EPSG:4326"]
        if gm_name == "rotated_latitude_longitude":
            return rotated_pole_crs(float(attrs["grid_north_pole_latitude"]),
                                    float(attrs["grid_north_pole_longitude"]),
                                    float(attrs.get("north_pole_grid_longitude", 0.0)))
        if gm_name == "mercator" and float(attrs.get("semi_major_axis", _WGS84_A)) == _WGS84_A \
                and float(attrs.get("inverse_flattening", 0.0)) == 0.0:
            return _REGISTRY["EPSG:3857"]
        raise ValueError(f"unsupported CF grid mapping: {attrs!r}")


def _geographic_cf(name: str, crs_wkt: str) -> dict:
    return dict(
        crs_wkt=crs_wkt,
        semi_major_axis=_WGS84_A,
        semi_minor_axis=6356752.314245179,
        inverse_flattening=_WGS84_RF,
        reference_ellipsoid_name="WGS 84",
        longitude_of_prime_meridian=0.0,
        prime_meridian_name="Greenwich",
        geographic_crs_name=name,
        horizontal_datum_name="World Geodetic System 1984 ensemble",
        grid_mapping_name="latitude_longitude",
    )


_WKT_4326 = 'GEOGCRS["WGS 84",ENSEMBLE["World Geodetic System 1984 ensemble"],ID["EPSG",4326]]'
_WKT_CRS84 = 'GEOGCRS["WGS 84 (CRS84)",ENSEMBLE["World Geodetic System 1984 ensemble"],ID["OGC","CRS84"]]'
_WKT_3857 = 'PROJCRS["WGS 84 / Pseudo-Mercator",BASEGEOGCRS["WGS 84"],CONVERSION["Popular Visualisation Pseudo-Mercator"],ID["EPSG",3857]]'

_REGISTRY: dict[str, CRS] = {
    "EPSG:4326": CRS("EPSG", "4326", "WGS 84", "geographic", "latlon",
                     _geographic_cf("WGS 84", _WKT_4326)),
    "OGC:CRS84": CRS("OGC", "CRS84", "WGS 84 (CRS84)", "geographic", "lonlat",
                     _geographic_cf("WGS 84 (CRS84)", _WKT_CRS84)),
    "EPSG:3857": CRS("EPSG", "3857", "WGS 84 / Pseudo-Mercator", "webmerc", "en",
                     dict(crs_wkt=_WKT_3857, semi_major_axis=_WGS84_A,
                          semi_minor_axis=6356752.314245179,
                          inverse_flattening=_WGS84_RF,
                          reference_ellipsoid_name="WGS 84",
                          longitude_of_prime_meridian=0.0,
                          prime_meridian_name="Greenwich",
                          geographic_crs_name="WGS 84",
                          horizontal_datum_name="World Geodetic System 1984 ensemble",
                          projected_crs_name="WGS 84 / Pseudo-Mercator",
                          grid_mapping_name="mercator",
                          standard_parallel=0.0,
                          longitude_of_projection_origin=0.0,
                          false_easting=0.0, false_northing=0.0)),
}
_WKT_3035 = ('PROJCRS["ETRS89-extended / LAEA Europe",BASEGEOGCRS["ETRS89"],'
             'CONVERSION["Europe Equal Area 2001"],ID["EPSG",3035]]')
_GRS80_B = 6356752.314140356


def _laea_3035_cf() -> dict:
    return dict(crs_wkt=_WKT_3035, semi_major_axis=_WGS84_A, semi_minor_axis=_GRS80_B,
                inverse_flattening=298.257222101, reference_ellipsoid_name="GRS 1980",
                longitude_of_prime_meridian=0.0, prime_meridian_name="Greenwich",
                geographic_crs_name="ETRS89",
                horizontal_datum_name="European Terrestrial Reference System 1989 ensemble",
                projected_crs_name="ETRS89-extended / LAEA Europe",
                grid_mapping_name="lambert_azimuthal_equal_area",
                latitude_of_projection_origin=52.0, longitude_of_projection_origin=10.0,
                false_easting=4321000.0, false_northing=3210000.0)


_REGISTRY["EPSG:3035"] = CRS("EPSG", "3035", "ETRS89-extended / LAEA Europe", "laea", "en",
                             _laea_3035_cf(),
                             ("GRS 1980", 10.0, 52.0, 1.0, 4321000.0, 3210000.0))

_ALIASES = {
    "EPSG:4326": "EPSG:4326", "WGS84": "EPSG:4326", "4326": "EPSG:4326",
    "OGC:CRS84": "OGC:CRS84", "CRS84": "OGC:CRS84", "OGC:1.3:CRS84": "OGC:CRS84",
    "URN:OGC:DEF:CRS:OGC:1.3:CRS84": "OGC:CRS84",
    "EPSG:3857": "EPSG:3857", "3857": "EPSG:3857", "EPSG:900913": "EPSG:3857",
    "EPSG:3035": "EPSG:3035", "3035": "EPSG:3035",
}
_UTM_CACHE: dict[int, CRS] = {}


def utm_crs(zone: int, south: bool = False) -> CRS:
    """EPSG:326zz / 327zz — WGS 84 / UTM zone zz N|S (PROJ +proj=utm)."""
    if not 1 <= zone <= 60:
        raise ValueError(f"invalid UTM zone {zone}")
    code = (32700 if south else 32600) + zone
    crs = _UTM_CACHE.get(code)
    if crs is None:
        name = f"WGS 84 / UTM zone {zone}{'S' if south else 'N'}"
        lon_0 = 6.0 * zone - 183.0
        fn = 10000000.0 if south else 0.0
        wkt = f'PROJCRS["{name}",BASEGEOGCRS["WGS 84"],CONVERSION["UTM zone {zone}' \
              f'{"S" if south else "N"}"],ID["EPSG",{code}]]'
        cf = dict(crs_wkt=wkt, semi_major_axis=_WGS84_A, semi_minor_axis=6356752.314245179,
                  inverse_flattening=_WGS84_RF, reference_ellipsoid_name="WGS 84",
                  longitude_of_prime_meridian=0.0, prime_meridian_name="Greenwich",
                  geographic_crs_name="WGS 84",
                  horizontal_datum_name="World Geodetic System 1984 ensemble",
                  projected_crs_name=name, grid_mapping_name="transverse_mercator",
                  latitude_of_projection_origin=0.0, longitude_of_central_meridian=lon_0,
                  false_easting=500000.0, false_northing=fn,
                  scale_factor_at_central_meridian=0.9996)
        crs = CRS("EPSG", str(code), name, "tmerc", "en", cf,
                  ("WGS 84", lon_0, 0.0, 0.9996, 500000.0, fn))
        _UTM_CACHE[code] = crs
    return crs


def _projected_from_cf(attrs: dict) -> CRS:
    """A transverse Mercator / LAEA CRS from its CF grid-mapping parameters
    (the EPSG definition when the parameters are those of a UTM zone or of
    EPSG:3035, else a CRS defined by the parameters)."""
    gm = attrs["grid_mapping_name"]
    rf = float(attrs.get("inverse_flattening", _WGS84_RF))
    ell = "GRS 1980" if abs(rf - 298.257222101) < 1e-9 else "WGS 84"
    fe = float(attrs.get("false_easting", 0.0))
    fn = float(attrs.get("false_northing", 0.0))
    lat_0 = float(attrs.get("latitude_of_projection_origin", 0.0))
    if gm == "transverse_mercator":
        lon_0 = float(attrs.get("longitude_of_central_meridian", 0.0))
        k0 = float(attrs.get("scale_factor_at_central_meridian", 1.0))
        zone = (lon_0 + 183.0) / 6.0
        if ell == "WGS 84" and k0 == 0.9996 and fe == 500000.0 and lat_0 == 0.0 \
                and zone == int(zone) and fn in (0.0, 10000000.0):
            return utm_crs(int(zone), south=fn != 0.0)
        params = (ell, lon_0, lat_0, k0, fe, fn)
        return CRS("CF", "tmerc", attrs.get("projected_crs_name", "Transverse Mercator"),
                   "tmerc", "en", dict(attrs), params)
    lon_0 = float(attrs.get("longitude_of_projection_origin", 0.0))
    params = (ell, lon_0, lat_0, 1.0, fe, fn)
    if params == _REGISTRY["EPSG:3035"].params:
        return _REGISTRY["EPSG:3035"]
    return CRS("CF", "laea", attrs.get("projected_crs_name", "Lambert Azimuthal Equal Area"),
               "laea", "en", dict(attrs), params)

def rotated_pole_crs(pole_lat: float, pole_lon: float, pole_grid_lon: float = 0.0) -> CRS:
    """A CF rotated latitude-longitude grid (``rotated_latitude_longitude``,
    PROJ ``ob_tran``): recognised for grid-mapping discovery (cfconv.py:66-212
    assigns rotated coordinates to it); transformations to or from it raise
    ``NotImplementedError`` (no rotated-pole grid is on the hot path)."""
    cf = dict(grid_mapping_name="rotated_latitude_longitude",
              grid_north_pole_latitude=pole_lat, grid_north_pole_longitude=pole_lon,
              north_pole_grid_longitude=pole_grid_lon)
    return CRS("CF", "rotated", "Rotated pole (WGS 84)", "rotated", "lonlat", cf,
               ("WGS 84", pole_lat, pole_lon, pole_grid_lon))


CRS_WGS84 = _REGISTRY["EPSG:4326"]
CRS_CRS84 = _REGISTRY["OGC:CRS84"]
CRS_WEBMERC = _REGISTRY["EPSG:3857"]


def _as_crs(value) -> CRS | None:
    if value is None:
        return None
    if isinstance(value, CRS):
        return value
    if isinstance(value, str):
        return CRS.from_string(value)
    if isinstance(value, int):
        return CRS.from_epsg(value)
    # pyproj.CRS, if pyproj is installed: map by authority code
    to_authority = getattr(value, "to_authority", None)
    if callable(to_authority):
        auth = to_authority()
        if auth:
            return CRS.from_string(f"{auth[0]}:{auth[1]}")
    raise ValueError(f"unsupported CRS: {value!r}")


def normalize_crs(crs) -> CRS:
    """gridmapping/helpers.py:59-63 (`_normalize_crs`)."""
    return CRS.from_user_input(crs)


# --------------------------------------------------------------------------
# Transformations (always_xy=True semantics: x = lon/easting, y = lat/northing)
# --------------------------------------------------------------------------

def webmerc_inverse(x, y):
    """EPSG:3857 -> geographic degrees (PROJ merc_s_inverse, webmerc).

    PROJ de-scales by the reciprocal of the semi-major axis (inv_prepare:
    ``x * ra``) then ``lam = x``, ``phi = atan(sinh(y))`` (k0 = 1), then
    unitconvert multiplies radians by the precomputed rad->deg factor.
    """
    ra = 1.0 / _WGS84_A
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    lam = x * ra
    phi = np.arctan(np.sinh(y * ra))
    return lam * _RAD_TO_DEG_FACTOR, phi * _RAD_TO_DEG_FACTOR


def webmerc_forward(lon, lat):
    """Geographic degrees -> EPSG:3857 (PROJ merc_s_forward, webmerc)."""
    lam = np.asarray(lon, dtype=np.float64) * _DEG_TO_RAD
    phi = np.asarray(lat, dtype=np.float64) * _DEG_TO_RAD
    x = lam
    y = np.arcsinh(np.tan(phi))
    return _WGS84_A * x, _WGS84_A * y


def _ellipsoid(name: str):
    from .projections import GRS80, WGS84
    return GRS80 if name == "GRS 1980" else WGS84


def _adjlon(lam):
    """PROJ adjlon: wrap to [-pi, pi] when outside by more than the tolerance."""
    lam = np.asarray(lam, dtype=np.float64)
    out = np.abs(lam) >= math.pi + 1e-12
    if not np.any(out):
        return lam
    wrapped = lam + math.pi
    wrapped = wrapped - 2 * math.pi * np.floor(wrapped / (2 * math.pi)) - math.pi
    return np.where(out, wrapped, lam)


_PROJ_CACHE: dict = {}


def _projection(crs: CRS):
    """(forward, inverse) in degrees <-> metres for a projected CRS, following
    PROJ's pj_fwd / pj_inv around the restated projection (lam0 subtraction +
    adjlon, unit-ellipsoid scaling by a / ra, false easting / northing)."""
    key = (crs.kind, crs.params)
    hit = _PROJ_CACHE.get(key)
    if hit is not None:
        return hit
    if crs.kind == "webmerc":
        hit = (webmerc_forward, webmerc_inverse)
    else:
        from .projections import LambertAzimuthalEqualArea, TransverseMercator
        ell_name, lon_0, lat_0, k0, x_0, y_0 = crs.params
        ell = _ellipsoid(ell_name)
        lam0 = lon_0 * _DEG_TO_RAD
        phi0 = lat_0 * _DEG_TO_RAD
        proj = (TransverseMercator(ell, k0, phi0) if crs.kind == "tmerc"
                else LambertAzimuthalEqualArea(ell, phi0))
        a, ra = ell.a, 1.0 / ell.a

        def forward(lon, lat, proj=proj, lam0=lam0, a=a, x_0=x_0, y_0=y_0):
            lam = _adjlon(np.asarray(lon, dtype=np.float64) * _DEG_TO_RAD - lam0)
            phi = np.asarray(lat, dtype=np.float64) * _DEG_TO_RAD
            x, y = proj.forward(lam, phi)
            return a * x + x_0, a * y + y_0

        def inverse(x, y, proj=proj, lam0=lam0, ra=ra, x_0=x_0, y_0=y_0):
            xx = (np.asarray(x, dtype=np.float64) - x_0) * ra
            yy = (np.asarray(y, dtype=np.float64) - y_0) * ra
            lam, phi = proj.inverse(xx, yy)
            lam = _adjlon(lam + lam0)
            return lam * _RAD_TO_DEG_FACTOR, phi * _RAD_TO_DEG_FACTOR

        hit = (forward, inverse)
    _PROJ_CACHE[key] = hit
    return hit


def _proj_step(crs: CRS, inverse: bool):
    """The xrs_transform record (include/xrs.h XrsProjStep) of crs._projection
    forward / inverse: the same constants the numpy restatement uses."""
    from ._native import PROJ_KINDS, ProjStep

    st = ProjStep()
    if crs.kind == "webmerc":
        st.kind = PROJ_KINDS["webmerc_inv" if inverse else "webmerc_fwd"]
        st.a, st.ra = _WGS84_A, 1.0 / _WGS84_A
        return st
    from .projections import LambertAzimuthalEqualArea, TransverseMercator
    ell_name, lon_0, lat_0, k0, x_0, y_0 = crs.params
    ell = _ellipsoid(ell_name)
    st.a, st.ra, st.x0, st.y0 = ell.a, 1.0 / ell.a, x_0, y_0
    st.lam0, st.phi0 = lon_0 * _DEG_TO_RAD, lat_0 * _DEG_TO_RAD
    st.e, st.es, st.one_es = ell.e, ell.es, ell.one_es
    if crs.kind == "tmerc":
        proj = TransverseMercator(ell, k0, st.phi0)
        st.kind = PROJ_KINDS["tmerc_inv" if inverse else "tmerc_fwd"]
        for k, v in enumerate(list(proj.cgb) + list(proj.cbg) + list(proj.utg) + list(proj.gtu)):
            st.c[k] = v
        st.Qn, st.Zb = proj.Qn, proj.Zb
    else:
        proj = LambertAzimuthalEqualArea(ell, st.phi0)
        st.kind = PROJ_KINDS["laea_inv" if inverse else "laea_fwd"]
        st.mode = {"npole": 0, "spole": 1, "equit": 2, "obliq": 3}[proj.mode]
        st.qp, st.mmf = proj.qp, proj.mmf
        for k in range(3):
            st.apa[k] = proj.apa[k]
        st.dd = proj.dd
        for name in ("rq", "xmf", "ymf", "sinb1", "cosb1"):
            if hasattr(proj, name):
                setattr(st, name, getattr(proj, name))
    return st


class Transformer:
    """Subset of ``pyproj.Transformer`` used by the reference (always_xy).

    Pipelines are source -> geographic -> target; geographic CRSs on WGS 84 and
    ETRS89 are related by PROJ's null (ballpark) datum transformation."""

    def __init__(self, crs_from: CRS, crs_to: CRS):
        self.source_crs = crs_from
        self.target_crs = crs_to
        same = crs_from.kind == crs_to.kind and crs_from.params == crs_to.params
        if same:
            self._fn = None
            self._separable = True
            self._step_crs = []
            return
        if "rotated" in (crs_from.kind, crs_to.kind):
            raise NotImplementedError(
                f"transformations to or from a rotated-pole grid are not supported "
                f"({crs_from!r} -> {crs_to!r})")
        steps = []
        self._step_crs = []   # (crs, inverse) per step: the device pipeline (xrs_transform)
        if not crs_from.is_geographic:
            steps.append(_projection(crs_from)[1])
            self._step_crs.append((crs_from, True))
        if not crs_to.is_geographic:
            steps.append(_projection(crs_to)[0])
            self._step_crs.append((crs_to, False))

        def fn(xx, yy, steps=tuple(steps)):
            for step in steps:
                xx, yy = step(xx, yy)
            return xx, yy

        self._fn = fn
        # x' depends only on x and y' only on y: geographic <-> web Mercator
        kinds = {crs_from.kind, crs_to.kind}
        self._separable = kinds <= {"geographic", "webmerc"}

    @classmethod
    def from_crs(cls, crs_from, crs_to, always_xy: bool = False) -> "Transformer":
        if not always_xy:
            raise NotImplementedError("only always_xy=True is supported")
        return cls(normalize_crs(crs_from), normalize_crs(crs_to))

    @property
    def is_identity(self) -> bool:
        return self._fn is None

    @property
    def is_separable(self) -> bool:
        """x' depends only on x and y' only on y (identity, geographic <-> web
        Mercator); other pairs need 2-D coordinate tables."""
        return self._separable

    def separable_x_scales(self):
        """(m1, m2) with x' = (x * m1) * m2 in this transformer's operation
        order, for the separable pipelines made of scalings (identity,
        geographic <-> geographic, web Mercator inverse or forward; PROJ
        webmerc's x: ``lam = x * ra`` then the rad -> deg factor, or
        ``a * (lon * deg -> rad)``); None otherwise.  Used only through
        reproject.column_generators, which checks the result bit for bit."""
        if not self._separable:
            return None
        if not self._step_crs:
            return (1.0, 1.0)
        if len(self._step_crs) == 1 and self._step_crs[0][0].kind == "webmerc":
            if self._step_crs[0][1]:
                return (1.0 / _WGS84_A, _RAD_TO_DEG_FACTOR)
            return (_DEG_TO_RAD, _WGS84_A)
        return None

    def device_steps(self):
        """The pipeline as a ctypes array of XrsProjStep records for
        xrs_transform (kernels.transform)."""
        from ._native import ProjStep

        arr = (ProjStep * max(1, len(self._step_crs)))()
        for k, (crs, inverse) in enumerate(self._step_crs):
            arr[k] = _proj_step(crs, inverse)
        return arr, len(self._step_crs)

    def transform(self, xx, yy):
        xx = np.asarray(xx, dtype=np.float64)
        yy = np.asarray(yy, dtype=np.float64)
        if self._fn is None:
            return xx.copy(), yy.copy()
        return self._fn(xx, yy)

    def transform_x(self, x):
        """Separable x part: x' for a vector of x (y is irrelevant)."""
        return self.transform(x, np.zeros_like(np.asarray(x, dtype=np.float64)))[0]

    def transform_y(self, y):
        """Separable y part: y' for a vector of y (x is irrelevant)."""
        return self.transform(np.zeros_like(np.asarray(y, dtype=np.float64)), y)[1]

    def transform_bounds(self, left, bottom, right, top, densify_pts: int = 21):
        """PROJ proj_trans_bounds: densify the four edges, transform, min/max."""
        side = densify_pts + 1
        dx = (right - left) / side
        dy = (top - bottom) / side
        xs = np.empty(4 * side)
        ys = np.empty(4 * side)
        k = np.arange(side, dtype=np.float64)
        xs[0:side], ys[0:side] = left, top - k * dy
        xs[side:2 * side], ys[side:2 * side] = left + k * dx, bottom
        xs[2 * side:3 * side], ys[2 * side:3 * side] = right, bottom + k * dy
        xs[3 * side:], ys[3 * side:] = right - k * dx, top
        tx, ty = self.transform(xs, ys)
        ok = np.isfinite(tx) & np.isfinite(ty)
        if not np.any(ok):
            return (math.inf, math.inf, math.inf, math.inf)
        tx, ty = tx[ok], ty[ok]
        return (float(tx.min()), float(ty.min()), float(tx.max()), float(ty.max()))

    def transform_bounds_many(self, bboxes, densify_pts: int = 21):
        """transform_bounds for an (N, 4) array of (left, bottom, right, top),
        in one vectorised pass: the same densified points (element for
        element the same float64 operations) and the same min / max, as an
        (N, 4) array; rows with no finite point are inf."""
        b = np.asarray(bboxes, dtype=np.float64).reshape(-1, 4)
        left, bottom, right, top = (b[:, i:i + 1] for i in range(4))
        side = densify_pts + 1
        dx = (right - left) / side
        dy = (top - bottom) / side
        k = np.arange(side, dtype=np.float64)[None, :]
        n = len(b)
        xs = np.empty((n, 4 * side))
        ys = np.empty((n, 4 * side))
        xs[:, 0:side], ys[:, 0:side] = left, top - k * dy
        xs[:, side:2 * side], ys[:, side:2 * side] = left + k * dx, bottom
        xs[:, 2 * side:3 * side], ys[:, 2 * side:3 * side] = right, bottom + k * dy
        xs[:, 3 * side:], ys[:, 3 * side:] = right - k * dx, top
        tx, ty = self.transform(xs.ravel(), ys.ravel())
        tx, ty = tx.reshape(n, -1), ty.reshape(n, -1)
        ok = np.isfinite(tx) & np.isfinite(ty)
        out = np.stack([np.where(ok, tx, np.inf).min(axis=1), np.where(ok, ty, np.inf).min(axis=1),
                        np.where(ok, tx, -np.inf).max(axis=1),
                        np.where(ok, ty, -np.inf).max(axis=1)], axis=1)
        out[~ok.any(axis=1)] = np.inf
        return out

"""CPU tests of the CRS registry and the restated PROJ projections
(xcube_resampling_amd/crs.py, projections.py).  Their PROJ parity is pinned on
the GPU by the reference's PROJ-dependent goldens (test_crs_gpu.py); here:
round trips, CF discovery, separability and known closed-form values."""

from __future__ import annotations

import math

import numpy as np
import pytest

import xcube_resampling_amd as xrs


@pytest.mark.parametrize("code", ["EPSG:32632", "EPSG:32601", "EPSG:32760", "EPSG:3035"])
def test_cf_round_trip_and_names(code):
    crs = xrs.CRS.from_string(code)
    assert xrs.CRS.from_cf(crs.to_cf()) == crs
    assert crs.is_projected and not crs.is_geographic
    assert xrs.CRS.from_string(code.lower()) == crs
    if code == "EPSG:3035":
        assert crs.name == "ETRS89-extended / LAEA Europe"
    else:
        assert crs.name.startswith("WGS 84 / UTM zone ")


def test_generic_cf_transverse_mercator():
    attrs = dict(xrs.CRS.from_string("EPSG:32632").to_cf())
    attrs.pop("crs_wkt")
    attrs["scale_factor_at_central_meridian"] = 1.0   # not a UTM zone any more
    crs = xrs.CRS.from_cf(attrs)
    assert crs.kind == "tmerc" and crs.to_epsg() is None
    assert crs != xrs.CRS.from_string("EPSG:32632")


@pytest.mark.parametrize("src,dst", [("EPSG:4326", "EPSG:32632"), ("EPSG:4326", "EPSG:3035"),
                                     ("EPSG:3035", "EPSG:32632"), ("EPSG:3857", "EPSG:32633"),
                                     ("EPSG:4326", "EPSG:32733")])
def test_round_trips(src, dst):
    rng = np.random.default_rng(3)
    lon = rng.uniform(5.0, 13.0, 500)
    lat = rng.uniform(-60.0, 70.0, 500) if dst.startswith("EPSG:327") else \
        rng.uniform(40.0, 68.0, 500)
    x, y = xrs.Transformer.from_crs("EPSG:4326", src, always_xy=True).transform(lon, lat)
    fwd = xrs.Transformer.from_crs(src, dst, always_xy=True)
    inv = xrs.Transformer.from_crs(dst, src, always_xy=True)
    assert not fwd.is_separable
    u, v = fwd.transform(x, y)
    x2, y2 = inv.transform(u, v)
    scale = 1e-6 if src == "EPSG:4326" else 1e-3     # degrees / metres
    np.testing.assert_allclose(x2, x, atol=scale * 1e-3)
    np.testing.assert_allclose(y2, y, atol=scale * 1e-3)


def test_closed_form_values():
    t = xrs.Transformer.from_crs("EPSG:4326", "EPSG:32632", always_xy=True)
    x, y = t.transform(np.array([9.0]), np.array([0.0]))
    assert x[0] == pytest.approx(500000.0, abs=1e-9) and y[0] == pytest.approx(0.0, abs=1e-9)
    # along the central meridian the northing is k0 times the meridian arc
    x, y = t.transform(np.array([9.0]), np.array([45.0]))
    assert x[0] == pytest.approx(500000.0, abs=1e-6)
    assert y[0] == pytest.approx(0.9996 * 4984944.377977, abs=1e-3)  # WGS 84 arc to 45 deg
    t = xrs.Transformer.from_crs("EPSG:4326", "EPSG:3035", always_xy=True)
    x, y = t.transform(np.array([10.0]), np.array([52.0]))
    assert (x[0], y[0]) == (pytest.approx(4321000.0, abs=1e-6), pytest.approx(3210000.0, abs=1e-6))
    # equal-area: the area of a small lon/lat cell is preserved
    lon = np.array([20.0, 20.001, 20.0]), np.array([60.0, 60.0, 60.001])
    x, y = t.transform(*lon)
    area = abs((x[1] - x[0]) * (y[2] - y[0]) - (x[2] - x[0]) * (y[1] - y[0]))
    a, f = 6378137.0, 1 / 298.257222101
    e2 = f * (2 - f)
    phi = math.radians(60.0005)
    m = a * (1 - e2) / (1 - e2 * math.sin(phi) ** 2) ** 1.5
    n = a / math.sqrt(1 - e2 * math.sin(phi) ** 2)
    cell = (m * math.radians(0.001)) * (n * math.cos(phi) * math.radians(0.001))
    assert area == pytest.approx(cell, rel=1e-4)


def test_geographic_and_webmerc_stay_separable():
    for a, b in [("EPSG:4326", "EPSG:3857"), ("EPSG:3857", "OGC:CRS84"),
                 ("EPSG:4326", "EPSG:4326")]:
        assert xrs.Transformer.from_crs(a, b, always_xy=True).is_separable


def test_discovery_from_dataset():
    from fixtures import dataset_5x5_regular_utm

    gm = xrs.GridMapping.from_dataset(dataset_5x5_regular_utm())
    assert gm.crs == xrs.CRS.from_epsg(32632)
    assert gm.xy_res == (100, 100) and gm.is_regular


def test_webmerc_matches_published_epsg3857_constants():
    """EPSG:3857 has no reference test (PROJ is absent and the reference's
    tests never use it), so the spherical web Mercator restatement is checked
    against constants published independently of this code: the EPSG
    registry's projected bounds of EPSG:3857 (x = +-20037508.34 m at
    lon = +-180, y = +-20048966.10 m at lat = +-85.06) and the square-world
    latitude 85.0511287798066 deg, whose y equals pi * a = 20037508.342789244 m."""
    from xcube_resampling_amd import crs

    x, y = crs.webmerc_forward(np.array([180.0, -180.0, 0.0, 0.0, 0.0]),
                               np.array([0.0, 0.0, 85.06, -85.06, 85.0511287798066]))
    assert abs(x[0] - 20037508.34) < 0.005 and abs(x[1] + 20037508.34) < 0.005
    assert abs(y[2] - 20048966.10) < 0.005 and abs(y[3] + 20048966.10) < 0.005
    assert abs(y[4] - math.pi * 6378137.0) < 1e-6
    assert x[2] == 0.0 and y[0] == 0.0
    lon, lat = crs.webmerc_inverse(np.array([20037508.342789244]), np.array([20037508.342789244]))
    assert abs(lon[0] - 180.0) < 1e-12 and abs(lat[0] - 85.0511287798066) < 1e-12
    # the separable transformer of the bench pair (3857 -> 4326) uses these
    tr = xrs.Transformer.from_crs("EPSG:3857", "EPSG:4326", always_xy=True)
    assert tr.is_separable
    np.testing.assert_array_equal(tr.transform_x(np.array([20037508.342789244])), [180.0])

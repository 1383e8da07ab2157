"""Input datasets of the reference's unit tests (tests/sampledata.py of the
reference), rebuilt as data with the engine's Dataset model."""

from __future__ import annotations

import numpy as np

import xcube_resampling_amd as xrs

nan = np.nan

REFL_8X6 = np.array(
    [[0, 1, 0, 2, 0, 3, 0, 4],
     [2, 0, 3, 0, 4, 0, 1, 0],
     [0, 4, 0, nan, 0, 2, 0, 3],
     [1, 0, 2, 0, 3, 0, 4, 0],
     [0, 3, 0, 4, 0, 1, 0, 2],
     [4, 0, 1, 0, 2, 0, 3, 0]], dtype=np.float64)


def dataset_8x6_regular():
    """sampledata.py:60-83."""
    res = 0.1
    return xrs.Dataset(
        data_vars={"refl": (("lat", "lon"), REFL_8X6.copy())},
        coords={"lon": ("lon", 50.0 + res * np.arange(0, 8) + 0.5 * res),
                "lat": ("lat", 10.6 - res * np.arange(0, 6) - 0.5 * res)})


def dataset_2x8x6_regular():
    """sampledata.py:86-92 (time as int64 day numbers instead of datetime64)."""
    ds = dataset_8x6_regular()
    arr = np.repeat(REFL_8X6[np.newaxis], 2, axis=0)
    return xrs.Dataset(data_vars={"refl": (("time", "lat", "lon"), arr)},
                       coords={"time": ("time", np.array([0, 1])), "lat": ds["lat"],
                               "lon": ds["lon"]})


def dataset_2x2_irregular():
    """sampledata.py:29-39."""
    return xrs.Dataset(
        data_vars={"rad": (("y", "x"), np.array([[1.0, 2.0], [3.0, 4.0]]))},
        coords={"lon": (("y", "x"), np.array([[1.0, 6.0], [0.0, 2.0]])),
                "lat": (("y", "x"), np.array([[56.0, 53.0], [52.0, 50.0]]))})


def dataset_2x2x2_irregular():
    """sampledata.py:42-57."""
    rad = np.array([[[1.0, 2.0], [3.0, 4.0]], [[1.0, 2.0], [3.0, 4.0]]])
    ds = dataset_2x2_irregular()
    return xrs.Dataset(
        data_vars={"rad": (("time", "y", "x"), rad),
                   "time_series": (("time",), np.array([1, 2]))},
        coords={"lon": ds["lon"], "lat": ds["lat"], "time": ("time", np.array([0, 1]))})


def dataset_2x2_irregular_antimeridian():
    """sampledata.py:160-172."""
    return xrs.Dataset(
        data_vars={"rad": (("y", "x"), np.array([[1.0, 2.0], [3.0, 4.0]]))},
        coords={"lon": (("y", "x"), np.array([[+179.0, -176.0], [+178.0, +180.0]])),
                "lat": (("y", "x"), np.array([[56.0, 53.0], [52.0, 50.0]]))})


def dataset_4x4_irregular():
    """sampledata.py:175-208."""
    lon = np.array([[1.0, 2.0, 3.0, 4.0], [0.0, 1.0, 2.0, 3.0], [-1.0, 0.0, 1.0, 2.0],
                    [-2.0, -1.0, 0.0, 1.0]])
    lat = np.array([[56.0, 55.0, 54.0, 53.0], [55.0, 54.0, 53.0, 52.0],
                    [54.0, 53.0, 52.0, 51.0], [53.0, 52.0, 51.0, 50.0]])
    rad = np.arange(1.0, 17.0).reshape(4, 4)
    return xrs.Dataset(data_vars={"rad": (("y", "x"), rad)},
                       coords={"lon": (("y", "x"), lon), "lat": (("y", "x"), lat)})


def reference_goldens(module: str) -> dict:
    import json
    import os

    from conftest import GOLDEN

    with open(os.path.join(GOLDEN, "reference_test_goldens.json")) as f:
        d = json.load(f)[module]
    out = {}
    for k, v in d.items():
        if k == "__helpers__":
            out[k] = {n: np.array(a, dtype=float) for n, a in v.items()}
            continue
        out[k] = [(np.array(e["expected"], dtype=float), e["decimal"]) for e in v]
    return out


def _spatial_ref(code: str):
    return xrs.DataArray(np.array(0), (), xrs.CRS.from_string(code).to_cf())


def dataset_5x5_regular_utm():
    """sampledata.py:95-109 (EPSG:32632)."""
    x = np.arange(565300.0, 565800.0, 100.0)
    y = np.arange(5934300.0, 5933800.0, -100.0)
    return xrs.Dataset(
        data_vars={"band_1": xrs.DataArray(np.arange(25).reshape((5, 5)), ("y", "x"),
                                           {"grid_mapping": "spatial_ref"})},
        coords={"x": ("x", x), "y": ("y", y), "spatial_ref": _spatial_ref("EPSG:32632")})


def dataset_2x5x5_regular_utm():
    """sampledata.py:112-128 (time as int64 day numbers instead of datetime64)."""
    ds = dataset_5x5_regular_utm()
    band = np.repeat(np.arange(25).reshape((5, 5))[np.newaxis], 2, axis=0)
    return xrs.Dataset(
        data_vars={"band_1": xrs.DataArray(band, ("time", "y", "x"),
                                           {"grid_mapping": "spatial_ref"})},
        coords={"time": ("time", np.array([0, 1])), "x": ds["x"], "y": ds["y"],
                "spatial_ref": _spatial_ref("EPSG:32632")})


def dataset_large_for_reproject():
    """sampledata.py:131-157 (EPSG:3035; eager instead of dask-chunked)."""
    nt, nx, ny = 10, 100, 100
    x = np.linspace(3900000, 4500000, nx)
    y = np.linspace(2600000, 3200000, ny)
    temp = np.arange(nt * nx * ny, dtype=np.float32).reshape(nt, nx, ny)
    return xrs.Dataset(
        data_vars={"temperature": xrs.DataArray(temp, ("time", "y", "x"),
                                                {"grid_mapping": "spatial_ref"}),
                   "onedim_data": xrs.DataArray(np.arange(nt), ("time",))},
        coords={"time": ("time", np.arange(nt)), "x": ("x", x), "y": ("y", y),
                "spatial_ref": _spatial_ref("EPSG:3035")})

"""Shared test helpers."""

from __future__ import annotations

import os

import numpy as np

from conftest import GOLDEN


def load_golden(name: str) -> dict:
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def assert_bitwise_equal(actual, expected, msg=""):
    """Equal in dtype, shape and bits (NaN == NaN, -0 != +0)."""
    actual = np.ascontiguousarray(actual)
    expected = np.ascontiguousarray(expected)
    assert actual.dtype == expected.dtype, f"{msg} dtype {actual.dtype} != {expected.dtype}"
    assert actual.shape == expected.shape, f"{msg} shape {actual.shape} != {expected.shape}"
    a = actual.view(np.uint8).reshape(actual.shape + (-1,))
    e = expected.view(np.uint8).reshape(expected.shape + (-1,))
    same = np.all(a == e, axis=-1)
    if np.issubdtype(actual.dtype, np.floating):
        same |= np.isnan(actual) & np.isnan(expected)
    bad = np.argwhere(~same)
    assert bad.size == 0, (
        f"{msg} {len(bad)} of {actual.size} elements differ; first at {tuple(bad[0])}: "
        f"{actual[tuple(bad[0])]!r} vs {expected[tuple(bad[0])]!r}"
    )


def reproject_golden_inputs(g: dict):
    """(source Dataset, target GridMapping) of a reproject golden fixture."""
    import xcube_resampling_amd as xrs

    data = g["data"]
    ds = xrs.Dataset(
        data_vars={"v": (("time", "lat", "lon"), data)},
        coords={"lon": ("lon", g["src_lon"]), "lat": ("lat", g["src_lat"])},
    )
    tsize = tuple(int(v) for v in g["tsize"])
    ttile = tuple(int(v) for v in g["ttile"])
    tgm = xrs.GridMapping.regular(tsize, tuple(g["txy_min"]), tuple(g["tres"]), "EPSG:3857",
                                  tile_size=ttile)
    return ds, tgm

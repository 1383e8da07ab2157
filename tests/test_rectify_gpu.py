"""GPU parity tests of the rectify path: K4 (xrs_ij_bboxes), K5
(xrs_rectify_ij) and K6 (xrs_rectify_var).

Bar: bit-exact against fixtures made by executing the reference's own numba
kernels (tests/golden/rectify_*.npz), the reference's own test goldens
(tests/test_rectify.py, tests/gridmapping/test_bboxes.py) through the Dataset
API, and bit-exact against the C oracle (oracle/rectify_ref.c) on larger
seeded swaths that the fixtures cannot hold."""

from __future__ import annotations

import numpy as np
import pytest

from fixtures import (
    dataset_2x2_irregular,
    dataset_2x2_irregular_antimeridian,
    dataset_2x2x2_irregular,
    reference_goldens,
)
from helpers import assert_bitwise_equal, load_golden
from oracle import rectify_ref
from test_rectify_cpu import BORDER_BOX, CASES, _geometry

pytestmark = pytest.mark.gpu
GOLD = reference_goldens("tests/test_rectify.py")
RAD13 = GOLD["__helpers__"]["expected_rad_13x13"]


def _device_ij(lon, lat, size, tile, xy_min, res, j_up):
    import xcube_resampling_amd as xrs
    from xcube_resampling_amd import rectify as R

    tgm = xrs.GridMapping.regular(size, xy_min, res, "EPSG:4326", tile_size=tile,
                                  is_j_axis_up=j_up)
    sgm = xrs.GridMapping.from_coords(xrs.DataArray(lon, ("y", "x"), name="lon"),
                                      xrs.DataArray(lat, ("y", "x"), name="lat"), "EPSG:4326")
    tiles, ntx, bb, _ = R.rectify_tiles(sgm, tgm)
    ij = R._compute_target_source_ij(sgm, tgm, 1e-3)
    return ij, bb


# ---------------------------------------------------------------- K4 ---------
def test_k4_bboxes_reference_test_goldens():
    """tests/gridmapping/test_bboxes.py goldens, generic (box list) mode."""
    from xcube_resampling_amd import kernels

    gold = reference_goldens("tests/gridmapping/test_bboxes.py")
    lon, lat = np.meshgrid(np.linspace(10.0, 20.0, 11), np.linspace(50.0, 60.0, 11))
    a0, a1, a2 = 0.0, 5.0, 10.0
    tiles = np.array([[10.0 + a0, 50.0 + a0, 10.0 + a1, 50.0 + a1],
                      [10.0 + a1, 50.0 + a0, 10.0 + a2, 50.0 + a1],
                      [10.0 + a0, 50.0 + a1, 10.0 + a1, 50.0 + a2],
                      [10.0 + a1, 50.0 + a1, 10.0 + a2, 50.0 + a2]])
    cases = [("test_all_included", [(np.array([[10.0, 50.0, 20.0, 60.0]]), 0.0, 0, None)]),
             ("test_tiles", [(tiles, 0.0, 0, None), (tiles, 0.0, 0, (2, 2))]),
             ("test_none_found", [(tiles + 11.0, 0.0, 0, None), (tiles + 11.0, 0.0, 0, (2, 2))]),
             ("test_with_border", [(BORDER_BOX, 0.0, 0, None), (BORDER_BOX, 0.5, 0, None),
                                   (BORDER_BOX, 1.0, 0, None), (BORDER_BOX, 2.0, 0, None),
                                   (BORDER_BOX, 2.0, 2, None)])]
    for name, calls in cases:
        exp_list = gold[name]
        for k, (boxes, xb, ib, grid) in enumerate(calls):
            exp = exp_list[min(k, len(exp_list) - 1)][0] if name != "test_with_border" \
                else exp_list[k][0]
            got = kernels.ij_bboxes(lon, lat, boxes, xb, ib, grid=grid)
            np.testing.assert_array_equal(got, exp.astype(np.int64), err_msg=f"{name} {k}")


@pytest.mark.parametrize("seed", range(6))
def test_k4_grid_and_generic_modes_match_oracle(seed):
    from oracle import gridmapping_ref as gref
    from xcube_resampling_amd import kernels

    rng = np.random.default_rng(seed)
    h, w = int(rng.integers(30, 300)), int(rng.integers(30, 300))
    lon = 5 + 0.01 * np.arange(w)[None, :] + 0.003 * np.arange(h)[:, None] \
        + rng.normal(0, 0.002, (h, w))
    lat = 60 - 0.008 * np.arange(h)[:, None] - 0.001 * np.arange(w)[None, :] \
        + rng.normal(0, 0.002, (h, w))
    if seed % 2:
        lon.ravel()[rng.choice(lon.size, 20, replace=False)] = np.nan
    size = (int(rng.integers(10, 90)), int(rng.integers(10, 90)))
    tile = (int(rng.integers(3, 40)), int(rng.integers(3, 40)))
    boxes = gref.xy_bboxes(size, tile, (5.2, 58.4, 5.2 + size[0] * 0.02, 58.4 + size[1] * 0.02),
                           (0.02, 0.02), bool(seed % 3 == 0))
    ntx, nty = -(-size[0] // tile[0]), -(-size[1] // tile[1])
    for xb, ib in ((0.0, 0), (0.05, 1), (0.3, 2)):
        exp = rectify_ref.compute_ij_bboxes(lon, lat, boxes, xb, ib)
        np.testing.assert_array_equal(kernels.ij_bboxes(lon, lat, boxes, xb, ib), exp)
        np.testing.assert_array_equal(
            kernels.ij_bboxes(lon, lat, boxes, xb, ib, grid=(ntx, nty)), exp)


# ------------------------------------------------------------- K5 + K6 -------
@pytest.mark.parametrize("case", CASES)
def test_rectify_kernels_match_reference_kernels(case):
    """Fixtures from the reference's own numba kernels: ij positions and all
    three interpolations bit for bit."""
    from xcube_resampling_amd import kernels

    g = load_golden(f"rectify_{case}.npz")
    size, tile, geo = _geometry(g)
    ij, bb = _device_ij(g["lon"], g["lat"], size, tile, tuple(g["xy_min"]), float(g["res"]),
                        bool(g["j_up"]))
    np.testing.assert_array_equal(bb, g["ij_bboxes"])
    assert_bitwise_equal(ij.cpu().numpy(), g["ij"], "ij")
    import torch

    src = torch.from_numpy(g["var"]).cuda()
    for interp in ("nearest", "bilinear", "triangular"):
        out = kernels.rectify_var(ij, src, interp, g["fill"].item())
        assert_bitwise_equal(out.cpu().numpy(), g[f"out_{interp}"], interp)


def _olci_like(rng, h, w, nan_px=0):
    i = np.arange(w)[None, :]
    j = np.arange(h)[:, None]
    lon = 5.0 + 0.0045 * i + 0.0009 * j + rng.normal(0, 0.0002, (h, w))
    lat = 60.0 - 0.0027 * j - 0.0004 * i + 1e-8 * (i - w / 2) ** 2 \
        + rng.normal(0, 0.0001, (h, w))
    if nan_px:
        lat.ravel()[rng.choice(lat.size, nan_px, replace=False)] = np.nan
    return lon, lat


@pytest.mark.parametrize("dtype,j_up,tile", [(np.float32, False, (256, 256)),
                                             (np.uint16, True, (100, 64)),
                                             (np.float64, False, (512, 128))])
def test_rectify_kernels_match_oracle_swath(dtype, j_up, tile):
    """A 700x900 jittered swath (NaN holes) rectified to a 1000x760 target:
    device == C oracle of the numba kernels, bit for bit."""
    from xcube_resampling_amd import kernels
    import torch

    rng = np.random.default_rng(7)
    h, w = 700, 900
    lon, lat = _olci_like(rng, h, w, nan_px=40)
    size, xy_min, res = (1000, 760), (5.3, 58.3), 0.0025
    if np.issubdtype(dtype, np.floating):
        var = rng.random((2, h, w)).astype(dtype)
        var[0].ravel()[rng.choice(h * w, 500, replace=False)] = np.nan
        fill = np.nan
    else:
        var = rng.integers(0, 60000, (2, h, w)).astype(dtype)
        fill = 65535
    from oracle import gridmapping_ref as gref

    geo = gref.regular_geometry(size, xy_min, res, tile_size=tile, is_j_axis_up=j_up)
    exp_ij, exp_bb = rectify_ref.compute_target_source_ij(lon, lat, size, tile, geo["xy_bbox"],
                                                          geo["xy_res"], j_up, threads=8)
    ij, bb = _device_ij(lon, lat, size, tile, xy_min, res, j_up)
    np.testing.assert_array_equal(bb, exp_bb)
    assert_bitwise_equal(ij.cpu().numpy(), exp_ij, "ij")
    assert np.sum(~np.isnan(exp_ij[0])) > size[0] * size[1] // 3
    src = torch.from_numpy(var).cuda()
    for interp in ("nearest", "bilinear", "triangular"):
        exp = rectify_ref.compute_var_image(exp_ij, var, fill, interp, tile, threads=8)
        out = kernels.rectify_var(ij, src, interp, fill)
        assert_bitwise_equal(out.cpu().numpy(), exp, interp)


# ------------------------------------------------------- Dataset API ---------
def _rect(ds, size, xy_min, res, interp=0, **kw):
    import xcube_resampling_amd as xrs

    tgm = xrs.GridMapping.regular(size, xy_min, res, "EPSG:4326", **kw)
    return xrs.rectify_dataset(ds, target_gm=tgm, interp_methods=interp)


def test_rectify_dataset_2x2_goldens():
    import xcube_resampling_amd as xrs

    out = _rect(dataset_2x2_irregular(), (4, 4), (-1, 49), 2)
    np.testing.assert_almost_equal(out["rad"].values, GOLD["test_rectify_2x2_to_default"][0][0])
    out = xrs.rectify_dataset(dataset_2x2_irregular(), interp_methods=0)
    np.testing.assert_almost_equal(out["rad"].values, GOLD["test_rectify_2x2_to_regular"][0][0])
    src = dataset_2x2x2_irregular()
    out = _rect(src, (4, 4), (-1, 49), 2)
    assert set(out.variables) == set(src.variables) | {"spatial_ref"}
    np.testing.assert_almost_equal(out["rad"].values, GOLD["test_rectify_2x2x2_to_default"][0][0])


def _offset_2x2():
    ds = dataset_2x2_irregular()
    ds["rad"] = type(ds["rad"])(ds["rad"].values + np.array([[0.0, 0.0], [0.0, 1.0]]),
                                ds["rad"].dims)
    return ds


@pytest.mark.parametrize("name,interp", [("test_rectify_2x2_to_7x7", 0),
                                         ("test_rectify_2x2_to_7x7_interp_methods_1",
                                          "triangular"),
                                         ("test_rectify_2x2_to_7x7_bilinear_interpol",
                                          "bilinear")])
def test_rectify_dataset_7x7_goldens(name, interp):
    out = _rect(_offset_2x2(), (7, 7), (-0.5, 49.5), 1.0, interp)
    exp, dec = GOLD[name][0]
    np.testing.assert_almost_equal(out["lon"].values, np.arange(0, 6.1))
    np.testing.assert_almost_equal(out["lat"].values, np.arange(56, 49.9, -1))
    assert out["rad"].dims == ("lat", "lon") and out["rad"].shape == (7, 7)
    np.testing.assert_almost_equal(out["rad"].values, exp, decimal=dec)


def test_rectify_dataset_7x7_subset_and_invalid():
    out = _rect(dataset_2x2_irregular(), (7, 7), (1.5, 50.5), 1.0, "nearest")
    np.testing.assert_almost_equal(out["lon"].values, np.arange(2, 8.1))
    np.testing.assert_almost_equal(out["rad"].values, GOLD["test_rectify_2x2_to_7x7_subset"][0][0])
    with pytest.raises(NotImplementedError):
        _rect(dataset_2x2_irregular(), (7, 7), (-0.5, 49.5), 1.0, "cubic")


@pytest.mark.parametrize("tile,j_up", [(None, False), (None, True), (5, True), (7, False),
                                       (5, False), ((3, 13), False), ((13, 3), False)])
def test_rectify_dataset_13x13_goldens(tile, j_up):
    kw = {"is_j_axis_up": j_up}
    if tile is not None:
        kw["tile_size"] = tile
    out = _rect(dataset_2x2_irregular(), (13, 13), (-0.25, 49.75), 0.5, **kw)
    np.testing.assert_almost_equal(out["lon"].values, np.arange(0, 6.1, 0.5))
    lat = np.arange(50, 56.1, 0.5) if j_up else np.arange(56, 49.9, -0.5)
    np.testing.assert_almost_equal(out["lat"].values, lat)
    np.testing.assert_almost_equal(out["rad"].values, RAD13[::-1] if j_up else RAD13)


def test_rectify_dataset_antimeridian_and_none():
    import xcube_resampling_amd as xrs

    tgm = xrs.GridMapping.regular((13, 13), (177.75, 49.75), 0.5, "EPSG:4326")
    assert tgm.is_lon_360
    out = xrs.rectify_dataset(dataset_2x2_irregular_antimeridian(), target_gm=tgm,
                              interp_methods=0)
    np.testing.assert_almost_equal(out["lon"].values,
                                   GOLD["test_rectify_2x2_to_13x13_antimeridian"][0][0])
    np.testing.assert_almost_equal(out["rad"].values, RAD13)
    for xy_min in ((10.0, 50.0), (-10.0, 50.0), (0.0, 58.0), (0.0, 42.0)):
        out = _rect(dataset_2x2_irregular(), (13, 13), xy_min, 0.5)
        assert np.all(np.isnan(out["rad"].values))


def test_resample_in_space_dispatches_rectify():
    import xcube_resampling_amd as xrs

    tgm = xrs.GridMapping.regular((13, 13), (-0.25, 49.75), 0.5, "EPSG:4326")
    out = xrs.resample_in_space(dataset_2x2_irregular(), target_gm=tgm, interp_methods=0)
    np.testing.assert_almost_equal(out["rad"].values, RAD13)


@pytest.mark.parametrize("j_up", [False, True])
@pytest.mark.parametrize("tile", [(5, 7), (16, 16), (64, 32)])
def test_device_tiling_matches_host_tiling(j_up, tile):
    """xrs_rectify_tiles (K4 accumulators -> tile records + chunk offsets on the
    device) reproduces the host tiling byte for byte, and K5 driven by it gives
    the same ij image as K5 driven by host tiles."""
    import torch

    import xcube_resampling_amd as xrs
    from xcube_resampling_amd import kernels
    from xcube_resampling_amd import rectify as R

    rng = np.random.default_rng(21)
    h, w = 60, 50
    jj, ii = np.mgrid[0:h, 0:w].astype(np.float64)
    lon = 10.0 + 0.02 * ii + 0.004 * jj + rng.normal(0, 0.001, (h, w))
    lat = 50.0 - 0.015 * jj + 0.003 * ii + rng.normal(0, 0.001, (h, w))
    sgm = xrs.GridMapping.from_coords(xrs.DataArray(lon, ("y", "x"), name="lon"),
                                      xrs.DataArray(lat, ("y", "x"), name="lat"), "EPSG:4326")
    res = 0.012
    x0, y0 = float(np.floor(lon.min() / res) * res), float(np.floor(lat.min() / res) * res)
    size = (int(np.ceil((lon.max() - x0) / res)), int(np.ceil((lat.max() - y0) / res)))
    tgm = xrs.GridMapping.regular(size, (x0, y0), res, "EPSG:4326", tile_size=tile,
                                  is_j_axis_up=j_up)
    xy = (torch.from_numpy(lon).cuda(), torch.from_numpy(lat).cuda())
    tiles, ntx, _, _ = R.rectify_tiles(sgm, tgm, xy=xy)
    t_dev, offs = R._device_tiles(sgm, tgm, xy)
    assert np.array_equal(t_dev.cpu().numpy(), tiles.view(np.uint8).ravel())
    nqi = np.maximum(tiles["swin"] - 1, 0).astype(np.int64)
    nqj = np.maximum(tiles["shin"] - 1, 0).astype(np.int64)
    nch = np.where(tiles["si0"] >= 0, (nqi + 62) // 63 * ((nqj + 15) // 16), 0)
    exp_offs = np.concatenate([[0], np.cumsum(nch)])
    np.testing.assert_array_equal(offs.cpu().numpy(), exp_offs)
    ysc = tgm.y_res if j_up else -tgm.y_res
    a = kernels.rectify_ij(xy[0], xy[1], tiles, ntx, tgm.height, tgm.width, tgm.x_res, ysc, 1e-3)
    b = kernels.rectify_ij(xy[0], xy[1], (t_dev, offs), ntx, tgm.height, tgm.width, tgm.x_res,
                           ysc, 1e-3)
    assert_bitwise_equal(b.cpu().numpy(), a.cpu().numpy(), "device vs host tiles")


@pytest.mark.parametrize("dtype,interp,n,keep_ij", [
    (np.float32, "nearest", 1, False), (np.float32, "bilinear", 2, True),
    (np.float64, "triangular", 1, True), (np.uint8, "nearest", 3, False),
    (np.int16, "bilinear", 1, False), (np.float32, "triangular", 2, False)])
def test_fused_resolve_sampling_equals_k5_then_k6(dtype, interp, n, keep_ij):
    """xrs_rectify_ij_var (K6 sampled inside K5's resolve pass) == K5 then K6
    bit for bit, and the ij image it keeps == K5's; device and host tiles,
    a swath with NaN coordinates and degenerate quads."""
    import torch

    import xcube_resampling_amd as xrs
    from xcube_resampling_amd import kernels
    from xcube_resampling_amd import rectify as R

    rng = np.random.default_rng(17)
    h, w = 110, 95
    jj, ii = np.mgrid[0:h, 0:w].astype(np.float64)
    lon = 3.0 + 0.01 * ii + 0.002 * jj + rng.normal(0, 0.002, (h, w))
    lat = 40.0 - 0.008 * jj + 0.001 * ii + rng.normal(0, 0.002, (h, w))
    lat[40:42, 20] = np.nan
    lon[60, 5] = lon[60, 4]
    sgm = xrs.GridMapping.from_coords(xrs.DataArray(lon, ("y", "x"), name="lon"),
                                      xrs.DataArray(lat, ("y", "x"), name="lat"), "EPSG:4326")
    res = 0.006
    x0 = float(np.floor(np.nanmin(lon) / res) * res)
    y0 = float(np.floor(np.nanmin(lat) / res) * res)
    size = (int(np.ceil((np.nanmax(lon) - x0) / res)), int(np.ceil((np.nanmax(lat) - y0) / res)))
    tgm = xrs.GridMapping.regular(size, (x0, y0), res, "EPSG:4326", tile_size=(40, 36))
    xy = (torch.from_numpy(lon).cuda(), torch.from_numpy(lat).cuda())
    if np.issubdtype(dtype, np.integer):
        var = rng.integers(0, 200, (n, h, w)).astype(dtype)
        fill = 0
    else:
        var = rng.random((n, h, w)).astype(dtype)
        fill = float("nan")
    src = torch.from_numpy(var).cuda()
    tiles, ntx, _, _ = R.rectify_tiles(sgm, tgm, xy=xy)
    for t in (tiles, R._device_tiles(sgm, tgm, xy)):
        ij = kernels.rectify_ij(xy[0], xy[1], t, ntx, tgm.height, tgm.width, tgm.x_res,
                                -tgm.y_res, 1e-3)
        exp = kernels.rectify_var(ij, src, interp, fill).cpu().numpy()
        ij2, got = kernels.rectify_ij_var(xy[0], xy[1], t, tgm.height, tgm.width, tgm.x_res,
                                          -tgm.y_res, 1e-3, src, interp, fill, keep_ij=keep_ij)
        assert_bitwise_equal(got.cpu().numpy(), exp, f"fused {interp}")
        if keep_ij:
            assert_bitwise_equal(ij2.cpu().numpy(), ij.cpu().numpy(), "fused ij")
        else:
            assert ij2 is None
    assert np.isfinite(ij.cpu().numpy()).sum() > 0.4 * ij[0].numel() * 2


@pytest.mark.parametrize("interp", ["nearest", "bilinear", "triangular"])
def test_triangle_keys_equal_plain_keys(interp):
    """The claim records the reference's triangle in the key's low bit and the
    resolve evaluates that triangle only; swaths of 2^31 points or more keep
    plain raster keys and test both triangles (forced here by the test knob).
    Both paths give the same ij image and samples bit for bit, fused and
    unfused, on a jittered swath with degenerate and NaN-cornered quads, and
    on a lattice whose points sit on pixel centres (exact edge cases)."""
    import torch

    import xcube_resampling_amd as xrs
    from xcube_resampling_amd import kernels
    from xcube_resampling_amd import rectify as R
    from xcube_resampling_amd._native import testing_knob

    rng = np.random.default_rng(23)
    for lattice in (False, True):
        h, w = 96, 88
        jj, ii = np.mgrid[0:h, 0:w].astype(np.float64)
        if lattice:
            lon = 3.0 + 0.01 * ii + 0.005
            lat = 40.0 - 0.01 * jj - 0.005
        else:
            lon = 3.0 + 0.01 * ii + 0.002 * jj + rng.normal(0, 0.002, (h, w))
            lat = 40.0 - 0.008 * jj + 0.001 * ii + rng.normal(0, 0.002, (h, w))
            lon[10, 10:14] = lon[10, 10]
            lat[50:52, 30] = np.nan
        sgm = xrs.GridMapping.from_coords(xrs.DataArray(lon, ("y", "x"), name="lon"),
                                          xrs.DataArray(lat, ("y", "x"), name="lat"),
                                          "EPSG:4326")
        res = 0.01 if lattice else 0.006
        x0 = float(np.floor(np.nanmin(lon) / res) * res)
        y0 = float(np.floor(np.nanmin(lat) / res) * res)
        size = (int(np.ceil((np.nanmax(lon) - x0) / res)),
                int(np.ceil((np.nanmax(lat) - y0) / res)))
        tgm = xrs.GridMapping.regular(size, (x0, y0), res, "EPSG:4326", tile_size=(40, 36))
        xy = (torch.from_numpy(lon).cuda(), torch.from_numpy(lat).cuda())
        src = torch.from_numpy(rng.random((2, h, w)).astype(np.float32)).cuda()
        tiles = R._device_tiles(sgm, tgm, xy)

        def run():
            ij = kernels.rectify_ij(xy[0], xy[1], tiles, 0, tgm.height, tgm.width, tgm.x_res,
                                    -tgm.y_res, 1e-3)
            ij2, out = kernels.rectify_ij_var(xy[0], xy[1], tiles, tgm.height, tgm.width,
                                              tgm.x_res, -tgm.y_res, 1e-3, src, interp,
                                              float("nan"), keep_ij=True)
            return ij.cpu().numpy(), ij2.cpu().numpy(), out.cpu().numpy()

        got = run()
        with testing_knob("rectify_plain_keys", 1):
            exp = run()
        for g, e, what in zip(got, exp, ("ij", "fused ij", "fused samples")):
            assert_bitwise_equal(g, e, f"{what} lattice={lattice}")
        assert np.isfinite(got[0]).sum() > 0.3 * got[0].size


def test_k4_filled_claim_keys_equal_in_call_fill():
    """K4 fills the claim-key scratch beside the coordinate scan
    (xrs_ij_bboxes_fill; DeviceTiles hands it to the first K5 call, which
    passes keys_ready = 1); later calls with the same tiles fill their own.
    Same ij and fused samples bit for bit; the fill itself sets every word,
    16-byte body and word tail, and leaves K4's accumulators unchanged."""
    import torch

    import xcube_resampling_amd as xrs
    from xcube_resampling_amd import kernels
    from xcube_resampling_amd import rectify as R

    rng = np.random.default_rng(31)
    h, w = 140, 121
    jj, ii = np.mgrid[0:h, 0:w].astype(np.float64)
    lon = 3.0 + 0.01 * ii + 0.002 * jj + rng.normal(0, 0.002, (h, w))
    lat = 40.0 - 0.008 * jj + 0.001 * ii + rng.normal(0, 0.002, (h, w))
    sgm = xrs.GridMapping.from_coords(xrs.DataArray(lon, ("y", "x"), name="lon"),
                                      xrs.DataArray(lat, ("y", "x"), name="lat"), "EPSG:4326")
    res = 0.006
    x0 = float(np.floor(lon.min() / res) * res)
    y0 = float(np.floor(lat.min() / res) * res)
    size = (int(np.ceil((lon.max() - x0) / res)), int(np.ceil((lat.max() - y0) / res)))
    tgm = xrs.GridMapping.regular(size, (x0, y0), res, "EPSG:4326", tile_size=(48, 40))
    xy = (torch.from_numpy(lon).cuda(), torch.from_numpy(lat).cuda())
    src = torch.from_numpy(rng.random((1, h, w)).astype(np.float32)).cuda()

    def ij_of(t):
        return kernels.rectify_ij(xy[0], xy[1], t, 0, tgm.height, tgm.width, tgm.x_res,
                                  -tgm.y_res, 1e-3).cpu().numpy()

    def fused_of(t):
        return kernels.rectify_ij_var(xy[0], xy[1], t, tgm.height, tgm.width, tgm.x_res,
                                      -tgm.y_res, 1e-3, src, "bilinear", float("nan"),
                                      keep_ij=False)[1].cpu().numpy()

    for run in (ij_of, fused_of):
        t = R._device_tiles(sgm, tgm, xy)
        assert isinstance(t, kernels.DeviceTiles) and t._keys is not None
        got = run(t)               # K4's fill (keys_ready = 1)
        assert t._keys is None     # consumed
        again = run(t)             # the call's own fill
        assert_bitwise_equal(got, again, run.__name__)
    assert np.isfinite(ij_of(R._device_tiles(sgm, tgm, xy))).mean() > 0.3

    # K5 on a side stream right after K4 + records on the current stream
    # (ADVICE r04): the records' event orders it, with the K4-filled keys
    ref = ij_of(R._device_tiles(sgm, tgm, xy))
    side = torch.cuda.Stream()
    for _ in range(3):
        t = R._device_tiles(sgm, tgm, xy)
        out = kernels.rectify_ij(xy[0], xy[1], t, 0, tgm.height, tgm.width, tgm.x_res,
                                 -tgm.y_res, 1e-3, stream=side)
        side.synchronize()
        assert_bitwise_equal(out.cpu().numpy(), ref, "side stream")

    # the fill: odd word counts (16-byte body + tail), accumulators as without
    boxes = np.asarray(tgm.xy_bboxes, np.float64)
    grid = (len(range(0, tgm.width, tgm.tile_width)), len(range(0, tgm.height, tgm.tile_height)))
    plain, _, _, _ = kernels._ij_bboxes_launch(xy[0], xy[1], boxes, 0.01, grid, None, None)
    for words in (1, 5, 4099):
        buf = torch.zeros(words + 8, dtype=torch.int32, device="cuda")
        acc, _, _, _ = kernels._ij_bboxes_launch(xy[0], xy[1], boxes, 0.01, grid, None, None,
                                                 fill=buf[4:4 + words])
        b = buf.cpu().numpy()
        assert (b[4:4 + words] == -1).all() and (b[:4] == 0).all() and (b[4 + words:] == 0).all()
        assert_bitwise_equal(acc.cpu().numpy(), plain.cpu().numpy(), f"acc fill={words}")


def test_rectify_dataset_fused_first_variable():
    """rectify_dataset samples its first device variable inside K5's resolve
    pass whatever its interpolation (rectify.py fuses nearest, bilinear and
    triangular alike): one and two variables, nearest, bilinear and mixed,
    give the same values as each variable rectified alone."""
    import xcube_resampling_amd as xrs

    rng = np.random.default_rng(3)
    h, w = 70, 64
    jj, ii = np.mgrid[0:h, 0:w].astype(np.float64)
    lon = 10.0 + 0.02 * ii + 0.004 * jj + rng.normal(0, 0.001, (h, w))
    lat = 50.0 - 0.015 * jj + 0.003 * ii + rng.normal(0, 0.001, (h, w))
    a = rng.random((h, w)).astype(np.float32)
    b = rng.random((2, h, w))
    coords = {"lon": xrs.DataArray(lon, ("y", "x")), "lat": xrs.DataArray(lat, ("y", "x"))}
    both = xrs.Dataset(data_vars={"a": xrs.DataArray(a, ("y", "x")),
                                  "b": xrs.DataArray(b, ("t", "y", "x"))}, coords=coords)
    only_a = xrs.Dataset(data_vars={"a": xrs.DataArray(a, ("y", "x"))}, coords=coords)
    only_b = xrs.Dataset(data_vars={"b": xrs.DataArray(b, ("t", "y", "x"))}, coords=coords)
    for interp in ("nearest", "bilinear", {"a": "nearest", "b": "bilinear"}):
        kw = dict(interp_methods=interp, tile_size=32)
        r2 = xrs.rectify_dataset(both, **kw)
        ra = xrs.rectify_dataset(only_a, **kw)
        rb = xrs.rectify_dataset(only_b, **kw)
        assert_bitwise_equal(np.asarray(r2["a"].values), np.asarray(ra["a"].values), f"a {interp}")
        assert_bitwise_equal(np.asarray(r2["b"].values), np.asarray(rb["b"].values), f"b {interp}")
        assert isinstance(r2["a"].values, np.ndarray) and r2["b"].dims[0] == "t"
        assert np.isfinite(r2["a"].values).mean() > 0.5


def test_claim_fast_decisions_equal_exact_divisions():
    """K5a decides pixel windows and triangle hits by reciprocal
    multiplication with an exact-division fallback near every boundary; forcing
    the exact path everywhere (test-only knob XRS_TESTING_RECTIFY_EXACT) gives the same ij image on
    a jittered swath with degenerate (duplicate) and NaN coordinates."""
    import torch

    import xcube_resampling_amd as xrs
    from xcube_resampling_amd import kernels
    from xcube_resampling_amd import rectify as R

    rng = np.random.default_rng(5)
    h, w = 120, 90
    jj, ii = np.mgrid[0:h, 0:w].astype(np.float64)
    lon = 3.0 + 0.01 * ii + 0.002 * jj + rng.normal(0, 0.002, (h, w))
    lat = 40.0 - 0.008 * jj + 0.001 * ii + rng.normal(0, 0.002, (h, w))
    lon[10, 10:14] = lon[10, 10]                  # degenerate quads
    lat[50:52, 30] = np.nan                       # missing coordinates
    lon[70, 5] = lon[70, 4]
    sgm = xrs.GridMapping.from_coords(xrs.DataArray(lon, ("y", "x"), name="lon"),
                                      xrs.DataArray(lat, ("y", "x"), name="lat"), "EPSG:4326")
    res = 0.005
    x0 = float(np.floor(np.nanmin(lon) / res) * res)
    y0 = float(np.floor(np.nanmin(lat) / res) * res)
    size = (int(np.ceil((np.nanmax(lon) - x0) / res)), int(np.ceil((np.nanmax(lat) - y0) / res)))
    tgm = xrs.GridMapping.regular(size, (x0, y0), res, "EPSG:4326", tile_size=(48, 40))
    xy = (torch.from_numpy(lon).cuda(), torch.from_numpy(lat).cuda())
    tiles, ntx, _, _ = R.rectify_tiles(sgm, tgm, xy=xy)
    run = lambda: kernels.rectify_ij(xy[0], xy[1], tiles, ntx, tgm.height, tgm.width,  # noqa
                                     tgm.x_res, -tgm.y_res, 1e-3).cpu().numpy()
    fast = run()
    from xcube_resampling_amd._native import testing_knob

    with testing_knob("rectify_exact", 1):
        exact = run()
    assert_bitwise_equal(fast, exact, "fast vs exact decisions")
    assert np.isfinite(fast).sum() > 0.5 * fast.size


def test_config4_full_size_matches_oracle():
    """BASELINE config 4 at full size: the 4000x4800 jittered swath (f64
    lon/lat) rectified to the ~8266x5392 EPSG:4326 grid in 512^2 tiles — K4
    bboxes, K5 source positions and K6 samples (nearest, bilinear,
    triangular — rectify.py:663-734), unfused and fused into the resolve pass
    with and without the ij image, == the C oracle of the numba kernels on
    the whole swath, bit for bit."""
    import torch

    from oracle import gridmapping_ref as gref
    from xcube_resampling_amd import kernels

    w, h = 4000, 4800
    rng = np.random.default_rng(20250905)
    i = np.arange(w)[None, :].astype(np.float64)
    j = np.arange(h)[:, None].astype(np.float64)
    lat = 60 - 0.0027 * j - 0.0004 * i + 1e-9 * (i - 2000) ** 2 \
        + rng.normal(0, 0.05 * 0.0027, (h, w))
    lon = 5 + 0.0045 * i + 0.0009 * j + rng.normal(0, 0.05 * 0.0045, (h, w))
    var = rng.random((1, h, w), dtype=np.float32)
    res = 0.0027
    x0, y0 = float(np.floor(lon.min() / res) * res), float(np.floor(lat.min() / res) * res)
    size = (int(np.ceil((lon.max() - x0) / res)), int(np.ceil((lat.max() - y0) / res)))
    tile = (512, 512)
    geo = gref.regular_geometry(size, (x0, y0), res, tile_size=tile)
    exp_ij, exp_bb = rectify_ref.compute_target_source_ij(lon, lat, size, tile, geo["xy_bbox"],
                                                          geo["xy_res"], False, threads=16)
    ij, bb = _device_ij(lon, lat, size, tile, (x0, y0), res, False)
    np.testing.assert_array_equal(bb, exp_bb)
    assert_bitwise_equal(ij.cpu().numpy(), exp_ij, "ij")
    assert np.sum(~np.isnan(exp_ij[0])) > 30_000_000
    from xcube_resampling_amd._native import testing_knob

    with testing_knob("rectify_compact", 1):   # the wave-compacted claim walk on every tile
        ij_c, _ = _device_ij(lon, lat, size, tile, (x0, y0), res, False)
    assert_bitwise_equal(ij_c.cpu().numpy(), exp_ij, "ij (compacted walk)")
    del ij_c
    src = torch.from_numpy(var).cuda()
    # the fused pass (K6 inside K5's resolve) is what rectify_dataset runs for
    # its first variable and what the config-4 line times: oracle-pinned here
    # on the whole swath too, keeping the ij image and not
    import xcube_resampling_amd as xrs
    from xcube_resampling_amd import rectify as R

    tgm = xrs.GridMapping.regular(size, (x0, y0), res, "EPSG:4326", tile_size=tile)
    sgm = xrs.GridMapping.from_coords(xrs.DataArray(lon, ("y", "x"), name="lon"),
                                      xrs.DataArray(lat, ("y", "x"), name="lat"), "EPSG:4326")
    xy = (torch.from_numpy(lon).cuda(), torch.from_numpy(lat).cuda())
    dev_tiles = R._device_tiles(sgm, tgm, xy)
    for interp in ("nearest", "bilinear", "triangular"):
        exp = rectify_ref.compute_var_image(exp_ij, var, np.nan, interp, tile, threads=16)
        assert_bitwise_equal(kernels.rectify_var(ij, src, interp, np.nan).cpu().numpy(), exp,
                             interp)
        for keep_ij in (False, True):
            ij2, got = kernels.rectify_ij_var(xy[0], xy[1], dev_tiles, tgm.height, tgm.width,
                                              tgm.x_res, -tgm.y_res, 1e-3, src, interp, np.nan,
                                              keep_ij=keep_ij)
            assert_bitwise_equal(got.cpu().numpy(), exp, f"fused {interp} keep_ij={keep_ij}")
            if keep_ij:
                assert_bitwise_equal(ij2.cpu().numpy(), exp_ij, "fused ij")
            del ij2, got


def test_nan_cornered_quads_on_untiled_large_target():
    """A NaN source coordinate makes the quads that have it as corner p0 / p3
    span their whole tile (floor(NaN) -> INT64_MIN clamps to 0,
    rectify.py:500-526) and test only the other triangle.  On an untiled
    ~9 Mpx target (the reference's default tiling for numpy swaths) each such
    window holds millions of (quad, pixel) tests: K5's test numbering (int64
    prefix sums) and (row, column) decomposition must stay exact there.  ij
    == the C oracle bit for bit."""
    w, h = 1600, 1400
    jj, ii = np.mgrid[0:h, 0:w].astype(np.float64)
    lon = 10.0 + 0.002 * ii + 0.0004 * jj
    lat = 50.0 - 0.002 * jj + 0.0003 * ii
    for j, i in [(1390, 1590), (1395, 20), (700, 1500)]:
        lat[j, i] = np.nan
    res = 0.001
    x0 = float(np.floor(np.nanmin(lon) / res) * res)
    y0 = float(np.floor(np.nanmin(lat) / res) * res)
    size = (int(np.ceil((np.nanmax(lon) - x0) / res)), int(np.ceil((np.nanmax(lat) - y0) / res)))
    assert size[0] * size[1] >= 8_500_000
    from oracle import gridmapping_ref as gref

    geo = gref.regular_geometry(size, (x0, y0), res, tile_size=size)
    exp_ij, exp_bb = rectify_ref.compute_target_source_ij(lon, lat, size, size, geo["xy_bbox"],
                                                          geo["xy_res"], False)
    ij, bb = _device_ij(lon, lat, size, size, (x0, y0), res, False)
    np.testing.assert_array_equal(bb, exp_bb)
    assert_bitwise_equal(ij.cpu().numpy(), exp_ij, "ij")
    assert np.isfinite(exp_ij[0]).sum() > 0.5 * size[0] * size[1]


def _device_ij_crs(x, y, size, tile, xy_min, res, j_up, crs, names):
    import xcube_resampling_amd as xrs
    from xcube_resampling_amd import rectify as R

    tgm = xrs.GridMapping.regular(size, xy_min, res, crs, tile_size=tile, is_j_axis_up=j_up)
    sgm = xrs.GridMapping.from_coords(xrs.DataArray(x, ("y", "x"), name=names[0]),
                                      xrs.DataArray(y, ("y", "x"), name=names[1]), crs)
    _, _, bb, _ = R.rectify_tiles(sgm, tgm)
    return R._compute_target_source_ij(sgm, tgm, 1e-3), bb


# quads covering ~0.3 to ~8 target pixels per side, rotated and sheared, in
# degrees near (5, 60) and in UTM metres near (5e5, 6.6e6) with 20-30 m pixels
FORM_CASES = [
    # (seed, scale, angle_deg, projected, jitter, j_up)
    (0, 0.35, 0.0, False, 0.05, False),
    (1, 0.9, 17.0, False, 0.2, True),
    (2, 1.6, -33.0, True, 0.05, False),
    (3, 2.4, 61.0, True, 0.3, False),
    (4, 3.7, 5.0, False, 0.0, False),
    (5, 1.0, 0.0, True, 0.0, True),    # lattice: source points on target pixel centres
    # quads of 30-90 target pixels: windows above kLaneWindow, walked by the
    # whole wave on the quad's forms
    (6, 5.5, 23.0, False, 0.1, False),
    (7, 8.0, -47.0, True, 0.2, True),
]


def _form_case_geometry(seed, scale, angle, projected, jitter):
    rng = np.random.default_rng(100 + seed)
    h, w = 150, 170
    res = 25.0 if projected else 0.0025
    src_res = res * scale
    jj, ii = np.mgrid[0:h, 0:w].astype(np.float64)
    c, s = np.cos(np.radians(angle)), np.sin(np.radians(angle))
    u = (ii + 0.5) * src_res
    v = (jj + 0.5) * src_res
    x0, y0 = (500000.0, 6600000.0) if projected else (5.0, 60.0)
    x = x0 + c * u + s * v + rng.normal(0, jitter * src_res, (h, w))
    y = y0 - (-s * u + c * v) + rng.normal(0, jitter * src_res, (h, w))
    gx0 = float(np.floor(np.nanmin(x) / res) * res)
    gy0 = float(np.floor(np.nanmin(y) / res) * res)
    if jitter == 0.0 and angle == 0.0 and scale == 1.0:   # lattice: centres coincide
        x = gx0 + (ii + 0.5) * res
        y = gy0 + (h - jj - 0.5) * res
    size = (int(np.ceil((np.nanmax(x) - gx0) / res)) + 1,
            int(np.ceil((np.nanmax(y) - gy0) / res)) + 1)
    return x, y, size, (gx0, gy0), res


@pytest.mark.parametrize("seed,scale,angle,projected,jitter,j_up", FORM_CASES)
def test_claim_forms_match_oracle_geometries(seed, scale, angle, projected, jitter, j_up):
    """K5a decides each (quad, pixel) test from float32 affine forms with a
    per-quad error bound and the reference's exact float64 test inside the
    band: over quads from 0.35 to 8 target pixels wide (the widest walked by
    the whole wave), rotated, jittered,
    in degrees and in UTM metres (large coordinates, small pixels), and a
    lattice whose source points sit on target pixel centres, ij == the C
    oracle bit for bit — and again with the band widened 3000-fold (the
    exact-test path taken by a large share of the tests), and with every tile
    forced through the wave-compacted walk and through the per-lane walk."""
    from oracle import gridmapping_ref as gref
    from xcube_resampling_amd._native import testing_knob

    x, y, size, xy_min, res = _form_case_geometry(seed, scale, angle, projected, jitter)
    tile = (64, 48)
    crs, names = ("EPSG:32632", ("x", "y")) if projected else ("EPSG:4326", ("lon", "lat"))
    geo = gref.regular_geometry(size, xy_min, res, tile_size=tile, is_j_axis_up=j_up)
    exp_ij, exp_bb = rectify_ref.compute_target_source_ij(x, y, size, tile, geo["xy_bbox"],
                                                          geo["xy_res"], j_up, threads=8)
    assert np.isfinite(exp_ij[0]).sum() > 0.3 * size[0] * size[1]
    ij, bb = _device_ij_crs(x, y, size, tile, xy_min, res, j_up, crs, names)
    np.testing.assert_array_equal(bb, exp_bb)
    assert_bitwise_equal(ij.cpu().numpy(), exp_ij, "ij")
    with testing_knob("rectify_margin", 3000):
        ij_w, _ = _device_ij_crs(x, y, size, tile, xy_min, res, j_up, crs, names)
    assert_bitwise_equal(ij_w.cpu().numpy(), exp_ij, "ij (widened band)")
    # every tile through the wave-compacted walk, and every tile per lane
    for mode, name in ((1, "compacted"), (2, "per-lane")):
        with testing_knob("rectify_compact", mode):
            ij_c, _ = _device_ij_crs(x, y, size, tile, xy_min, res, j_up, crs, names)
            assert_bitwise_equal(ij_c.cpu().numpy(), exp_ij, f"ij ({name} walk)")
            with testing_knob("rectify_margin", 3000):
                ij_c, _ = _device_ij_crs(x, y, size, tile, xy_min, res, j_up, crs, names)
            assert_bitwise_equal(ij_c.cpu().numpy(), exp_ij, f"ij ({name} walk, widened band)")

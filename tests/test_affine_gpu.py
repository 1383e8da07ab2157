"""GPU parity tests of K2/K3 (xrs_affine): the reference's affine path
(dask-image -> scipy order 0/1 + coarsen reducers).

Bar: the reference's own test goldens (tests/test_affine.py, decimal 7 as
there) through the Dataset API, and bit-exact equality with the oracle
(dask-image restatement calling scipy itself + numpy reducers) on seeded
random inputs covering upscale/downscale, 2-D/3-D, NaN/Inf, chunk edges,
integer dtypes, every implemented reducer and recover_nans."""

from __future__ import annotations

import numpy as np
import pytest

from fixtures import dataset_2x8x6_regular, dataset_8x6_regular, reference_goldens
from helpers import assert_bitwise_equal
from test_affine_cpu import CASES, RES

pytestmark = pytest.mark.gpu
GOLD = reference_goldens("tests/test_affine.py")


@pytest.mark.parametrize("name,idx,size,xy_min,res,recover", CASES)
def test_affine_transform_dataset_reference_goldens(name, idx, size, xy_min, res, recover):
    import xcube_resampling_amd as xrs

    ds = dataset_8x6_regular()
    tgm = xrs.GridMapping.regular(size, xy_min, res, "EPSG:4326")
    out = xrs.affine_transform_dataset(ds, tgm, interp_methods=1, recover_nans=recover)
    exp, dec = GOLD[name][idx]
    np.testing.assert_almost_equal(out["refl"].values, exp, decimal=dec)
    assert set(out.variables) == set(ds.variables) | {"spatial_ref"}
    assert out["refl"].shape == (size[1], size[0])


def test_affine_3d_and_interp_forms():
    import xcube_resampling_amd as xrs

    ds3 = dataset_2x8x6_regular()
    tgm = xrs.GridMapping.regular((3, 3), (50.0, 10.0), RES, "EPSG:4326")
    out = xrs.affine_transform_dataset(ds3, tgm, interp_methods=1)
    exp, dec = GOLD["test_subset_3d"][0]
    np.testing.assert_almost_equal(out["refl"].values, exp, decimal=dec)
    ds = dataset_8x6_regular()
    for im in ("bilinear", {"refl": "bilinear"}, {"refl": 1}):
        o = xrs.affine_transform_dataset(ds, tgm, source_gm=xrs.GridMapping.from_dataset(ds),
                                         interp_methods=im)
        np.testing.assert_almost_equal(o["refl"].values, GOLD["test_subset_with_source_gm"][0][0])


def test_affine_errors():
    import xcube_resampling_amd as xrs

    ds = dataset_8x6_regular()
    sgm = xrs.GridMapping.from_dataset(ds)
    tgm = xrs.GridMapping.regular((8, 6), (50.2, 10.1), RES, sgm.crs)
    with pytest.raises(ValueError, match="Higher order is not supported"):
        xrs.affine_transform_dataset(ds, tgm, source_gm=sgm, interp_methods=3)
    tgm = xrs.GridMapping.regular((3, 3), (50.05, 10.05), RES, "EPSG:3857")
    with pytest.raises(AssertionError, match="Affine transformation cannot be applied"):
        xrs.affine_transform_dataset(ds, tgm, source_gm=sgm)


def _random_case(rng, dtype, nd, nan_frac):
    shp = (int(rng.integers(1, 4)),) if nd == 3 else ()
    shp += (int(rng.integers(20, 90)), int(rng.integers(20, 90)))
    if np.issubdtype(dtype, np.floating):
        a = (rng.random(shp) * 10 - 5).astype(dtype)
        a.ravel()[rng.random(a.size) < nan_frac] = np.nan
        if nan_frac:
            a.ravel()[rng.integers(0, a.size)] = np.inf
        a.ravel()[rng.integers(0, a.size, max(1, a.size // 50))] = -0.0   # order 0: -> +0.0
    else:
        a = rng.integers(0, 200, shp).astype(dtype)
    return a


@pytest.mark.parametrize("seed", range(24))
def test_kernel_matches_oracle_random(seed):
    """Random affine matrices (up/down-scale, shifts), chunkings, dtypes and
    reducers: engine == oracle bit for bit."""
    import xcube_resampling_amd.affine as A
    from oracle import affine_ref

    rng = np.random.default_rng(1000 + seed)
    dtype = [np.float32, np.float64, np.uint8, np.int16][seed % 4]
    nd = 3 if seed % 3 == 0 else 2
    a = _random_case(rng, dtype, nd, 0.02 if seed % 2 else 0.0)
    h, w = a.shape[-2:]
    interp = int(seed % 5 != 0)
    s_i = float(rng.choice([0.5, 0.75, 1.0, 1.5, 2.0, 2.5, 4.0, 1 / 3]))
    s_j = float(rng.choice([0.5, 0.9216, 1.0, 2.0, 3.0, 4.0]))
    o_i, o_j = float(rng.uniform(-3, 3)), float(rng.choice([0.0, 0.5, -1.25, 2.0]))
    matrix = ((s_i, 0.0, o_i), (0.0, s_j, o_j))
    out_h, out_w = int(rng.integers(5, 40)), int(rng.integers(5, 40))
    tile = (int(rng.integers(2, 20)), int(rng.integers(2, 20)))
    lead = a.shape[:-2]
    agg = ["mean", "sum", "max", "min", "count", "first", "last", "center", "prod"][seed % 9]
    recover = bool(seed % 6 == 1)
    fill = np.nan if np.issubdtype(dtype, np.floating) else 7
    oshape = lead + (out_h, out_w)
    ochunks = tuple(int(rng.integers(1, 3)) for _ in lead) + tile
    ref = affine_ref.resample_array(a, matrix, oshape, ochunks, interp, agg, recover, fill)
    got = A._resample_array(a, None, None, matrix, oshape, ochunks, interp, agg, recover, fill)
    got = got if isinstance(got, np.ndarray) else got.cpu().numpy()
    assert_bitwise_equal(got, np.asarray(ref), f"seed {seed} {dtype} {agg} interp={interp}")


@pytest.mark.parametrize("agg", ["mean", "sum", "max", "min", "count", "first", "last",
                                 "center", "prod"])
def test_coarsen_4x4_matches_oracle(agg):
    """Config-3 shape in miniature: 1024^2 f32 (0.1 % NaN) -> 256^2, scale 4."""
    import xcube_resampling_amd.affine as A
    from oracle import affine_ref

    rng = np.random.default_rng(5)
    a = rng.random((1024, 1024), dtype=np.float32)
    a.ravel()[rng.choice(a.size, a.size // 1000, replace=False)] = np.nan
    m = ((4.0, 0.0, 0.0), (0.0, 4.0, 0.0))
    ref = affine_ref.resample_array(a, m, (256, 256), (128, 128), 1, agg, False, np.nan)
    got = A._resample_array(a, None, None, m, (256, 256), (128, 128), 1, agg, False, np.nan)
    assert_bitwise_equal(got.cpu().numpy(), np.asarray(ref), agg)


def test_coarsen_via_dataset_api():
    import xcube_resampling_amd as xrs
    from oracle import affine_ref

    rng = np.random.default_rng(9)
    n = 512
    a = rng.random((n, n), dtype=np.float32)
    res = 2.0 ** -10
    ds = xrs.Dataset(data_vars={"v": (("lat", "lon"), a)},
                     coords={"lon": ("lon", (np.arange(n) + 0.5) * res),
                             "lat": ("lat", 0.5 - (np.arange(n) + 0.5) * res)})
    tgm = xrs.GridMapping.regular((n // 4, n // 4), (0, 0), 2.0 ** -8, "EPSG:4326", tile_size=64)
    out = xrs.affine_transform_dataset(ds, tgm)  # float default: bilinear + mean
    sgm = xrs.GridMapping.from_dataset(ds)
    m = tgm.ij_transform_to(sgm)
    assert m == ((4.0, 0.0, 0.0), (0.0, 4.0, 0.0))
    ref = affine_ref.resample_array(a, m, (n // 4, n // 4), (64, 64), 1, "mean", False, np.nan)
    assert_bitwise_equal(out["v"].values, ref)


@pytest.mark.parametrize("dtype,nd", [(np.float32, 2), (np.float64, 3), (np.float32, 3),
                                      (np.uint8, 2), (np.int16, 3)])
@pytest.mark.parametrize("agg", ["mean", "sum", "max", "min", "count", "prod", "center"])
@pytest.mark.parametrize("order", [1, 0])
def test_integral_grid_coarsen_special_values(dtype, nd, agg, order):
    """Integer scales with integral offsets hit the kernel's exact shortcut for
    integral sample positions: NaN, +-inf and -0.0 around the taps (zero-weight
    neighbours included), the zero-weight time neighbour of 3-D inputs, and
    chunk edges; order 0 too (scipy's order-0 value is 0.0 + v, so -0.0 comes
    out as +0.0) — engine == oracle bit for bit."""
    import xcube_resampling_amd.affine as A
    from oracle import affine_ref

    rng = np.random.default_rng(77)
    shp = ((3,) if nd == 3 else ()) + (96, 80)
    if np.issubdtype(dtype, np.floating):
        a = (rng.random(shp) * 4 - 2).astype(dtype)
        flat = a.reshape(-1)
        idx = rng.choice(flat.size, 60, replace=False)
        flat[idx[:20]] = np.nan
        flat[idx[20:30]] = np.inf
        flat[idx[30:40]] = -np.inf
        flat[idx[40:]] = -0.0
        fill = np.nan
    else:
        a = rng.integers(0, 120, shp).astype(dtype)
        fill = 3
    lead = shp[:-2]
    for m, oshape, tile in [(((4.0, 0.0, 0.0), (0.0, 4.0, 0.0)), (24, 20), (8, 10)),
                            (((2.0, 0.0, 2.0), (0.0, 3.0, -3.0)), (30, 38), (7, 16)),
                            (((1.0, 0.0, 1.0), (0.0, 1.0, 0.0)), (90, 76), (45, 76))]:
        ochunks = tuple(1 for _ in lead) + tile
        ref = affine_ref.resample_array(a, m, lead + oshape, ochunks, order, agg, False, fill)
        got = A._resample_array(a, None, None, m, lead + oshape, ochunks, order, agg, False,
                                fill)
        got = got if isinstance(got, np.ndarray) else got.cpu().numpy()
        assert_bitwise_equal(got, np.asarray(ref), f"{dtype} {agg} order={order} {m}")


@pytest.mark.parametrize("k3i", ["1", "0"])
@pytest.mark.parametrize("dtype,nd", [(np.float32, 2), (np.float64, 2), (np.float32, 3),
                                      (np.float64, 3)])
def test_integral_coarsen_k3i_matches_oracle(k3i, dtype, nd):
    """K3i (the integral-grid coarsen kernel: square factors 2/4/8 whose div-x
    grid sits on source pixels) and the generic K3 (forced by the test-only
    knob xrs_testing_set(XRS_TESTING_AFFINE_GENERIC, 1)) are
    both bit-exact with the oracle: order 0 and 1, integral offsets incl.
    misaligned vector starts and targets reaching past the source (cval /
    exact path at the edges), NaN / +-inf / -0.0 in the taps, the zero-weight
    time neighbour of 3-D inputs, chunk edges (mirrored taps), widths that
    are not a multiple of the 256-column block; a fractional offset (tables
    not integral) routes to the generic K3."""
    import xcube_resampling_amd.affine as A
    from oracle import affine_ref

    from xcube_resampling_amd._native import testing_knob

    rng = np.random.default_rng(4242)
    lead = (3,) if nd == 3 else ()
    cases = [(4, (0.0, 0.0), (70, 300), (32, 128), 1, "mean"),
             (4, (1.0, 3.0), (64, 270), (17, 270), 1, "mean"),
             (2, (-2.0, 5.0), (90, 140), (30, 64), 1, "sum"),
             (8, (8.0, -1.0), (20, 40), (8, 40), 1, "max"),
             (4, (0.0, 2.0), (50, 66), (25, 33), 0, "mean"),
             (2, (3.0, 0.0), (33, 515), (33, 515), 0, "min"),
             (4, (0.5, 0.0), (40, 60), (20, 60), 1, "mean")]
    for d, (ox, oy), oshape, tile, order, agg in cases:
        shp = lead + (oshape[0] * d + 6, oshape[1] * d + 3)
        a = (rng.random(shp) * 4 - 2).astype(dtype)
        flat = a.reshape(-1)
        idx = rng.choice(flat.size, max(4, flat.size // 400), replace=False)
        q = idx.size // 4
        flat[idx[:q]] = np.nan
        flat[idx[q:2 * q]] = np.inf
        flat[idx[2 * q:3 * q]] = -np.inf
        flat[idx[3 * q:]] = -0.0
        m = ((float(d), 0.0, ox), (0.0, float(d), oy))
        ochunks = tuple(1 for _ in lead) + tile
        ref = affine_ref.resample_array(a, m, lead + oshape, ochunks, order, agg, False, np.nan)
        with testing_knob("affine_generic", 0 if k3i == "1" else 1):
            got = A._resample_array(a, None, None, m, lead + oshape, ochunks, order, agg, False,
                                    np.nan)
        got = got if isinstance(got, np.ndarray) else got.cpu().numpy()
        assert_bitwise_equal(got, np.asarray(ref), f"k3i={k3i} {dtype} d={d} off={ox},{oy} "
                                                   f"order={order} {agg}")


@pytest.mark.parametrize("nan_frac", [0.002, 0.05, 0.3])
@pytest.mark.parametrize("order", [1, 0])
def test_integral_coarsen_slow_list(nan_frac, order):
    """K3i hands pixels with non-finite taps (order 1) or non-integral columns
    to its slow-pixel list (exact path in integral_slow_kernel); a list longer
    than the workspace holds (nan_frac 0.3, 3 slices) hands the whole launch to
    the generic K3.  Every regime is bit-exact with the oracle."""
    import xcube_resampling_amd.affine as A
    from oracle import affine_ref

    rng = np.random.default_rng(int(nan_frac * 1000) + order)
    for dtype, d, lead in [(np.float32, 4, (3,)), (np.float64, 2, ()), (np.float32, 8, ())]:
        oshape = (60, 70)
        shp = lead + (oshape[0] * d + 2, oshape[1] * d + 5)
        a = (rng.random(shp) * 4 - 2).astype(dtype)
        flat = a.reshape(-1)
        idx = rng.choice(flat.size, int(flat.size * nan_frac), replace=False)
        flat[idx[: idx.size // 2]] = np.nan
        flat[idx[idx.size // 2: 3 * idx.size // 4]] = np.inf
        flat[idx[3 * idx.size // 4:]] = -0.0
        m = ((float(d), 0.0, 0.0), (0.0, float(d), 0.0))
        ochunks = tuple(1 for _ in lead) + (30, 70)
        for agg in ("mean", "max"):
            ref = affine_ref.resample_array(a, m, lead + oshape, ochunks, order, agg, False,
                                            np.nan)
            got = A._resample_array(a, None, None, m, lead + oshape, ochunks, order, agg, False,
                                    np.nan)
            got = got if isinstance(got, np.ndarray) else got.cpu().numpy()
            assert_bitwise_equal(got, np.asarray(ref), f"{dtype} d={d} {agg} nan={nan_frac}")


def test_config3_full_size_sampled_blocks():
    """BASELINE config 3 at full size — coarsen mean 4x4 of a 16384^2 float32
    raster with 0.1 % NaN (K3i, one launch): 1024^2-source blocks at the
    corners, the centre and across an output-chunk seam == the oracle
    (dask-image chunk footprint + scipy order 1 + numpy nanmean in dask
    chunk.coarsen order), bit for bit, EVERY output row and column of the block
    included: the oracle runs on the block plus a one-output-pixel source halo
    (4 rows / columns) where the raster continues, so the block's last
    row/column (an interior seam of the full raster) sees the same
    neighbours — including the zero-weight NaN taps of the next block — as the
    one-launch result does."""
    import torch

    import xcube_resampling_amd.affine as A
    from oracle import affine_ref
    from xcube_resampling_amd import kernels

    n, k = 16384, 4
    m = ((4.0, 0.0, 0.0), (0.0, 4.0, 0.0))
    gen = torch.Generator(device="cuda")
    gen.manual_seed(9)
    src = torch.rand((1, n, n), generator=gen, device="cuda", dtype=torch.float32)
    src[torch.rand((1, n, n), generator=gen, device="cuda") < 0.001] = float("nan")
    plan = A.plan_affine(tuple(src.shape), np.dtype(np.float32), m, (1, n // k, n // k),
                         (1, 512, 512), 1, "mean", False, np.nan)
    out = kernels.affine(src, plan)
    c = 1024
    # (1536, 3584): output rows 384-639 straddle the 512-row output chunk seam
    for r0, c0 in [(0, 0), (0, n - c), (n // 2 - c // 2, n // 2 - c // 2), (1536, 3584),
                   (n - c, 0), (n - c, n - c)]:
        r1, c1 = min(n, r0 + c + k), min(n, c0 + c + k)
        a = src[:, r0:r1, c0:c1].cpu().numpy()
        oh, ow = (r1 - r0) // k, (c1 - c0) // k
        ref = affine_ref.resample_array(a, m, (1, oh, ow), (1, oh, ow), 1, "mean", False, np.nan)
        got = out[:, r0 // k:(r0 + c) // k, c0 // k:(c0 + c) // k].cpu().numpy()
        assert np.isnan(a).any(), "the sample must exercise the NaN path"
        assert_bitwise_equal(got, np.asarray(ref)[:, :c // k, :c // k], f"block at ({r0}, {c0})")


@pytest.mark.parametrize("nt,interp,dtype", [(7, 0, np.float32), (64, 0, np.float32),
                                             (5, 0, np.uint8), (1, 1, np.float32),
                                             (1, 1, np.int16), (3, 0, np.float64),
                                             (1, 0, np.float32)])
def test_k2_slice_groups_match_oracle(nt, interp, dtype):
    """K2's grouped items (slices sharing one geometry: order 0, or order 1
    without a time neighbour; S slices per item, the last group short) ==
    the oracle slice by slice — the dask shape of config 1 (many chunks of
    one grid stacked on dim 0)."""
    import torch

    import xcube_resampling_amd.affine as A
    from oracle import affine_ref

    rng = np.random.default_rng(40 + nt)
    n = 96
    a = (rng.random((nt, n, n)) * 200).astype(dtype)
    if np.issubdtype(dtype, np.floating):
        a.ravel()[rng.random(a.size) < 0.01] = np.nan
    m = ((0.9216, 0.0, 7.4), (0.0, 0.9216, 5.0))
    fill = np.nan if np.issubdtype(dtype, np.floating) else 7
    src = a if nt > 1 else a[0]
    oshape = ((nt,) if nt > 1 else ()) + (n, n)
    ochunks = ((1,) if nt > 1 else ()) + (40, 48)
    plan = A.plan_affine((nt, n, n), np.dtype(dtype), m, oshape, ochunks, interp, "first",
                         False, fill)
    assert plan.agg_code == 0 and (interp == 0 or plan.t_next is None)
    got = A._resample_array(src, None, None, m, oshape, ochunks, interp, "first", False, fill)
    got = got.cpu().numpy() if isinstance(got, torch.Tensor) else got
    for t in range(nt):
        ref = affine_ref.resample_array(a[t:t + 1], m, (1, n, n), (1, 40, 48), interp, "first",
                                        False, fill)
        assert_bitwise_equal(got[t] if nt > 1 else got, np.asarray(ref)[0], f"slice {t}")


@pytest.mark.parametrize("dtype,nd", [(np.float32, 2), (np.float64, 2), (np.float32, 3),
                                      (np.float64, 3)])
def test_fractional_coarsen_k3w_matches_oracle(dtype, nd):
    """K3w (square 2/4/8 order-1 coarsens whose div-x grid has scale 1 but a
    fractional offset: contiguous taps, fractional weights — a target grid not
    aligned to the source, affine.py:277-313) is bit-exact with the oracle for
    every fused reducer, NaN / +-inf / -0.0 taps, the zero-weight time
    neighbour of 3-D inputs, targets reaching past the source (cval, mirrored
    last row / column through the exact path) and chunk edges; the plan's
    hint selects it (AffinePlan.run_weights) and the integral-run kernel gives
    the same bits on the same grids."""
    import xcube_resampling_amd.affine as A
    from oracle import affine_ref

    rng = np.random.default_rng(777)
    lead = (2,) if nd == 3 else ()
    cases = [(4, (0.5, 0.25), (40, 60), (20, 60), "mean"),
             (4, (-1.3, 2.7), (33, 70), (33, 35), "sum"),
             (2, (0.3, -0.6), (50, 130), (25, 64), "max"),
             (2, (1.75, 0.5), (21, 90), (21, 90), "min"),
             (8, (0.125, 3.5), (12, 40), (6, 40), "mean"),
             (4, (2.5, 0.5), (30, 50), (30, 50), "prod"),
             (4, (0.5, 1.5), (30, 50), (15, 50), "count")]
    for d, (ox, oy), oshape, tile, agg in cases:
        if d == 8 and dtype == np.float64:
            continue   # (no K3i / K3w instance: 9 rows of 8 doubles)
        shp = lead + (oshape[0] * d + 3, oshape[1] * d + 2)
        a = (rng.random(shp) * 4 - 2).astype(dtype)
        flat = a.reshape(-1)
        idx = rng.choice(flat.size, max(4, flat.size // 300), replace=False)
        q = idx.size // 4
        flat[idx[:q]] = np.nan
        flat[idx[q:2 * q]] = np.inf
        flat[idx[2 * q:3 * q]] = -np.inf
        flat[idx[3 * q:]] = -0.0
        m = ((float(d), 0.0, ox), (0.0, float(d), oy))
        ochunks = tuple(1 for _ in lead) + tile
        plan = A.plan_affine((1,) * (3 - nd) + a.shape, np.dtype(dtype), m,
                             (1,) * (3 - nd) + lead + oshape, (1,) * (3 - nd) + ochunks, 1, agg,
                             False, np.nan)
        assert plan.run_weights, (d, ox, oy)
        ref = affine_ref.resample_array(a, m, lead + oshape, ochunks, 1, agg, False, np.nan)
        got = A._resample_array(a, None, None, m, lead + oshape, ochunks, 1, agg, False, np.nan)
        got = got if isinstance(got, np.ndarray) else got.cpu().numpy()
        assert_bitwise_equal(got, np.asarray(ref), f"k3w {dtype} d={d} off={ox},{oy} {agg}")


@pytest.mark.parametrize("dtype,nd", [(np.float32, 2), (np.float64, 2), (np.float32, 3)])
def test_generic_coarsen_non_integer_factors_matches_oracle(dtype, nd):
    """The generic coarsen (affine.py:277-313 for non-integer factors: scales
    1.7 ... 7.3 give divisors 2 ... 8 with the div-x grid off scale 1, which
    since round 6 skip K3i / K3w and go straight to the LDS-band K3) is
    bit-exact with the oracle (order 1: order 0 never coarsens,
    affine.py:253-263) for several reducers, NaN / +-inf / -0.0 taps, the
    zero-weight time neighbour of 3-D inputs and targets reaching past the
    source."""
    import xcube_resampling_amd.affine as A
    from oracle import affine_ref

    rng = np.random.default_rng(2468)
    lead = (2,) if nd == 3 else ()
    cases = [(1.7, (0.3, 0.2), (40, 70), (20, 70), 1, "mean"),
             (2.5, (1.1, -0.4), (30, 50), (30, 25), 1, "max"),
             (3.5, (0.0, 0.5), (24, 40), (12, 40), 1, "sum"),
             (4.6, (2.2, 0.7), (16, 30), (16, 30), 1, "mean"),
             (5.5, (0.5, 1.5), (14, 25), (7, 25), 1, "min"),
             (3.25, (0.75, 0.25), (20, 33), (20, 33), 1, "count"),
             (7.3, (0.4, 0.6), (10, 18), (10, 18), 1, "mean")]
    for sc, (ox, oy), oshape, tile, order, agg in cases:
        shp = lead + (int(oshape[0] * sc) + 4, int(oshape[1] * sc) + 3)
        a = (rng.random(shp) * 4 - 2).astype(dtype)
        flat = a.reshape(-1)
        idx = rng.choice(flat.size, max(4, flat.size // 250), replace=False)
        q = idx.size // 4
        flat[idx[:q]] = np.nan
        flat[idx[q:2 * q]] = np.inf
        flat[idx[2 * q:3 * q]] = -np.inf
        flat[idx[3 * q:]] = -0.0
        m = ((sc, 0.0, ox), (0.0, sc, oy))
        ochunks = tuple(1 for _ in lead) + tile
        ref = affine_ref.resample_array(a, m, lead + oshape, ochunks, order, agg, False, np.nan)
        got = A._resample_array(a, None, None, m, lead + oshape, ochunks, order, agg, False,
                                np.nan)
        got = got if isinstance(got, np.ndarray) else got.cpu().numpy()
        assert_bitwise_equal(got, np.asarray(ref), f"generic {dtype} scale={sc} off={ox},{oy} "
                                                   f"order={order} {agg}")

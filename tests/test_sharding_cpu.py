"""Multi-process (gloo, world_size 2) tests of the multi-GPU partition on the
CPU: the row-band shard of a reprojection reads only its source rows and the
bands reassemble to the reference's output bit for bit; dim-0 slice shards
cover the cube exactly once; the bench's max-over-ranks clock.

The per-rank compute here is the oracle (tests may use it as the checker);
on the GPU the same partition drives xrs_reproject (test_reproject_gpu.py::
test_row_band_sharding_matches_whole_raster)."""

from __future__ import annotations

import os
import socket

import numpy as np
import pytest

from helpers import load_golden, reproject_golden_inputs

POISON = np.float32(1.0e30)


def _plan(g):
    import xcube_resampling_amd as xrs

    ds, tgm = reproject_golden_inputs(g)
    sgm = xrs.GridMapping.from_dataset(ds)
    return xrs.plan_reproject(sgm, tgm, xrs.Transformer.from_crs(tgm.crs, sgm.crs,
                                                                  always_xy=True))


@pytest.mark.parametrize("balance", ["rows", "bytes", "cost"])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_band_shards_partition_target_rows(world, balance):
    """Row-granular bands cover every target row once; each band's source
    rows are exactly the rows its floor / ceil taps read (a superset of every
    row K1 touches, and inside the tile windows)."""
    from xcube_resampling_amd.sharding import band_shard

    plan = _plan(load_golden("reproject_f32.npz"))
    shards = [band_shard(plan, world, r, balance) for r in range(world)]
    rows = [r for s in shards for r in range(s.row0, s.row1)]
    assert rows == list(range(plan.dst_height))
    lo, hi = plan.row_source_extent()
    for s in shards:
        if s.row1 > s.row0:
            ok = hi[s.row0:s.row1] >= lo[s.row0:s.row1]
            if not ok.any():   # the band reads only padding (fill)
                assert s.src_rows == (0, 0)
                continue
            assert s.src_row0 == lo[s.row0:s.row1][ok].min()
            assert s.src_row1 == hi[s.row0:s.row1][ok].max() + 1
            w0, w1 = plan.source_rows_for(s.row0, s.row1)
            assert w0 <= s.src_row0 and s.src_row1 <= w1


def test_row_extents_match_oracle_taps():
    """plan.row_source_extent == the rows the oracle's _reproject_block reads
    (floor / ceil window indices of reproject.py:286-291 mapped through the
    oracle's windows)."""
    import math

    from oracle import gridmapping_ref as gref
    from oracle import reproject_ref

    g = load_golden("reproject_pad.npz")
    plan = _plan(g)
    tsize = tuple(int(v) for v in g["tsize"])
    ttile = tuple(int(v) for v in g["ttile"])
    geo = gref.regular_geometry(tsize, tuple(g["txy_min"]), tuple(g["tres"]), tile_size=ttile)
    ntx, nty = math.ceil(tsize[0] / ttile[0]), math.ceil(tsize[1] / ttile[1])
    h, w = g["data"].shape[1:]
    b, _, yc, pad = reproject_ref.get_scr_bboxes_indices(
        lambda *bb: gref.transform_bounds(gref.webmerc_inverse, *bb), g["src_lon"], g["src_lat"],
        float(g["x_res"]), float(g["y_res"]), w, h, geo["xy_bboxes"], ntx, nty)
    lo, hi = plan.row_source_extent()
    for r in range(tsize[1]):
        j = r // ttile[1]
        rows = set()
        for i in range(ntx):
            _, sy = gref.webmerc_inverse(geo["x_coords"][:1], geo["y_coords"][r:r + 1])
            iy = (sy[0] - yc[0, j, i]) / -float(g["y_res"])
            for f in (np.floor, np.ceil):
                wi = int(np.int16(f(iy)))
                wi = wi + yc.shape[0] if wi < 0 else wi
                gj = int(b[1, j, i]) - pad[1][0] + wi
                if 0 <= wi < yc.shape[0] and 0 <= gj < h:
                    rows.add(gj)
        if rows:
            assert (lo[r], hi[r]) == (min(rows), max(rows)), r
        else:
            assert lo[r] > hi[r]


@pytest.mark.parametrize("world", [2, 4, 8])
def test_config5_band_balance(world):
    """Config 5 (40960^2, 20 tile rows) split over `world` ranks at row
    granularity: balance="rows" gives equal target rows (max/mean 1.0; whole
    tile rows would give 1.2 at world 8), balance="bytes" equal algorithmic
    bytes within 5 %, balance="cost" equal modelled K1 time within 1 %
    (model fitted to the one-GPU rehearsal); every source row a band holds is
    one it reads."""
    import bench
    from xcube_resampling_amd.sharding import band_shard

    _, _, plan, _, _ = bench.workload(40960, 2048)
    cols = plan.source_cols_read()
    from xcube_resampling_amd.sharding import COST_DUP_ROW_WEIGHT, COST_SRC_ROW_WEIGHT

    lo, hi = plan.row_source_extent()
    valid = hi >= lo
    dup = np.zeros(len(lo), bool)
    dup[1:] = (lo[1:] == lo[:-1]) & valid[1:] & valid[:-1]
    for balance in ("rows", "bytes", "cost"):
        shards = [band_shard(plan, world, r, balance) for r in range(world)]
        nrows = np.array([s.row1 - s.row0 for s in shards], float)
        alg = np.array([4 * 40960 * (s.row1 - s.row0) + 4 * cols * (s.src_row1 - s.src_row0)
                        for s in shards], float)
        cost = np.array([(s.row1 - s.row0) + COST_SRC_ROW_WEIGHT * (s.src_row1 - s.src_row0)
                         + COST_DUP_ROW_WEIGHT * dup[s.row0:s.row1].sum() for s in shards])
        if balance == "rows":
            assert nrows.max() / nrows.mean() <= 1.0 + 1e-9
        elif balance == "bytes":
            assert alg.max() / alg.mean() <= 1.05, alg / alg.mean()
        else:
            assert cost.max() / cost.mean() <= 1.01, cost / cost.mean()
        assert sum(nrows) == 40960
        # source bands are contiguous and overlap their neighbours by at most
        # the rows two adjacent target rows share
        for a, b in zip(shards, shards[1:]):
            assert b.src_row0 >= a.src_row0 and a.src_row1 - b.src_row0 <= 2


@pytest.mark.parametrize("n,world", [(1, 1), (8, 8), (5, 2), (3, 4), (17, 8)])
def test_slice_shards_cover_cube_once(n, world):
    from xcube_resampling_amd.sharding import slice_shard

    got = [i for r in range(world) for i in range(*slice_shard(n, world, r))]
    assert got == list(range(n))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, result_dir, balance="rows"):
    import sys

    import torch
    import torch.distributed as dist

    here = os.path.dirname(os.path.abspath(__file__))
    for p in (here, os.path.dirname(here)):
        if p not in sys.path:
            sys.path.insert(0, p)
    from oracle import gridmapping_ref as gref
    from oracle import reproject_ref
    from xcube_resampling_amd.sharding import band_shard, gather_rows, max_over_ranks

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = load_golden("reproject_f32.npz")
        plan = _plan(g)
        shard = band_shard(plan, world, rank, balance)
        # the rank holds only its source rows: everything else is poison
        data = np.full_like(g["data"], POISON)
        j0, j1 = shard.src_rows
        data[:, j0:j1] = g["data"][:, j0:j1]
        tsize = tuple(int(v) for v in g["tsize"])
        ttile = tuple(int(v) for v in g["ttile"])
        geo = gref.regular_geometry(tsize, tuple(g["txy_min"]), tuple(g["tres"]),
                                    tile_size=ttile)
        ntx = plan.num_tiles[0]
        tiles = [(j, i) for j in range(shard.row0 // ttile[1], -(-shard.row1 // ttile[1]))
                 for i in range(ntx)]
        full = reproject_ref.reproject_array(
            data, gref.webmerc_inverse, lambda *b: gref.transform_bounds(gref.webmerc_inverse, *b),
            g["src_lon"], g["src_lat"], float(g["x_res"]), float(g["y_res"]), geo["x_coords"],
            geo["y_coords"], geo["xy_bboxes"], ttile[0], ttile[1], "bilinear",
            g["fill"].item(), tiles=tiles)
        local = torch.from_numpy(np.ascontiguousarray(full[:, shard.row0:shard.row1]))
        out = gather_rows(local, plan.dst_height)
        clock = max_over_ranks(1.0 + rank)
        if rank == 0:
            np.save(os.path.join(result_dir, f"bands_{balance}.npy"), out.numpy())
            with open(os.path.join(result_dir, "clock.txt"), "w") as f:
                f.write(repr(clock))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("balance", ["rows", "bytes", "cost"])
def test_gloo_band_sharded_reprojection_matches_reference(tmp_path, balance):
    """world_size 2 over gloo: each rank holds only the source rows of its
    row band (everything else poisoned), bands split mid-tile, and the
    gathered raster equals the reference's output bit for bit."""
    import torch.multiprocessing as mp

    world = 2
    mp.spawn(_rank_main, args=(world, _free_port(), str(tmp_path), balance), nprocs=world,
             join=True)
    g = load_golden("reproject_f32.npz")
    got = np.load(tmp_path / f"bands_{balance}.npy")
    assert got.dtype == np.float64
    np.testing.assert_array_equal(got.view(np.uint64), g["out_bilinear"].view(np.uint64))
    assert float((tmp_path / "clock.txt").read_text()) == float(world)


# ---- coarsen / rectify splits (SURVEY §8(e) "Other configs") ------------------------
@pytest.mark.parametrize("world", [1, 2, 3, 5, 8])
def test_cost_splits_partition_and_balance(world):
    from xcube_resampling_amd.sharding import cost_splits

    rng = np.random.default_rng(world)
    costs = rng.random(97) * 10
    cuts = cost_splits(costs, world)
    assert cuts[0] == 0 and cuts[-1] == 97 and all(a <= b for a, b in zip(cuts, cuts[1:]))
    per = [costs[a:b].sum() for a, b in zip(cuts, cuts[1:])]
    assert max(per) <= costs.sum() / world + costs.max() + 1e-9


def _coarsen_plan(n=(1, 160, 176), div=4, chunks=8, agg="mean"):
    import xcube_resampling_amd.affine as A

    m = ((float(div), 0.0, 0.0), (0.0, float(div), 0.0))
    return A.plan_affine(n, np.dtype(np.float32), m, (n[0], n[1] // div, n[2] // div),
                         (1, chunks, n[2] // div), 1, agg, False, np.nan), m


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_coarsen_shards_partition_output_chunks(world):
    """Output chunk rows are split once each; every rank's source rows cover
    its chunks' dask-image footprints, re-based in the rank's plan."""
    from xcube_resampling_amd.sharding import coarsen_shard

    plan, _ = _coarsen_plan()
    shards = [coarsen_shard(plan, world, r) for r in range(world)]
    assert [s.row0 for s in shards if s.row1 > s.row0][0] == 0
    rows = [r for s in shards for r in range(*s.rows)]
    assert rows == list(range(plan.out_h))
    for s in shards:
        if s.row1 == s.row0:
            continue
        rel, ln = plan.rel_y[s.chunk0:s.chunk1], plan.len_y[s.chunk0:s.chunk1]
        assert s.src_row0 == rel.min() and s.src_row1 == (rel + ln).max()
        assert np.array_equal(s.plan.rel_y + s.src_row0, rel) and s.plan.out_h == s.row1 - s.row0


def test_coarsen_shard_refuses_separate_reducer_plans():
    from xcube_resampling_amd.sharding import coarsen_shard

    plan, _ = _coarsen_plan(agg="median")
    with pytest.raises(NotImplementedError):
        coarsen_shard(plan, 2, 0)


def _rect_case(h=150, w=120, tile=32):
    """A jittered swath (the config-4 form, small) and the oracle's tiling."""
    import xcube_resampling_amd as xrs
    import xcube_resampling_amd.rectify as R
    from oracle import rectify_ref

    ii, jj = np.meshgrid(np.arange(w), np.arange(h))
    rng = np.random.default_rng(4)
    lat = 60 - 0.0027 * jj - 0.0004 * ii + rng.normal(0, 1e-4, (h, w))
    lon = 5 + 0.0045 * ii + 0.0009 * jj + rng.normal(0, 1e-4, (h, w))
    res = 0.0027
    x0, y0 = float(np.floor(lon.min() / res) * res), float(np.floor(lat.min() / res) * res)
    size = (int(np.ceil((lon.max() - x0) / res)), int(np.ceil((lat.max() - y0) / res)))
    tgm = xrs.GridMapping.regular(size, (x0, y0), res, "EPSG:4326", tile_size=tile)
    bbox = tuple(tgm.xy_bbox)
    ij, bboxes = rectify_ref.compute_target_source_ij(lon, lat, size, (tile, tile), bbox,
                                                      (res, res), tgm.is_j_axis_up)
    tiles = R.tile_records(tgm, bboxes, w, h)
    var = rng.random((2, h, w)).astype(np.float32)
    return dict(lon=lon, lat=lat, size=size, tile=(tile, tile), bbox=bbox, res=(res, res),
                j_up=tgm.is_j_axis_up, ij=ij, tiles=tiles, var=var, tgm=tgm)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_rectify_shards_partition_tiles(world):
    from xcube_resampling_amd.sharding import rectify_shard, rectify_tile_costs

    c = _rect_case()
    tiles = c["tiles"]
    shards = [rectify_shard(tiles, world, r) for r in range(world)]
    ids = [t for s in shards for t in range(s.tile0, s.tile1)]
    assert ids == list(range(len(tiles)))
    costs = rectify_tile_costs(tiles)
    per = [costs[s.tile0:s.tile1].sum() for s in shards]
    assert max(per) <= costs.sum() / world + costs.max() + 1e-9
    for s in shards:
        for t in range(s.tile0, s.tile1):
            assert s.row0 <= tiles["r0"][t] and tiles["r0"][t] + tiles["th"][t] <= s.row1


def _rank_coarsen(rank, world, port, result_dir):
    import sys

    import torch
    import torch.distributed as dist

    here = os.path.dirname(os.path.abspath(__file__))
    for p in (here, os.path.dirname(here)):
        if p not in sys.path:
            sys.path.insert(0, p)
    from oracle import affine_ref
    from xcube_resampling_amd.sharding import coarsen_shard, gather_rows

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        plan, m = _coarsen_plan()
        shard = coarsen_shard(plan, world, rank)
        a = np.random.default_rng(11).random((1, 160, 176)).astype(np.float32)
        a.ravel()[::97] = np.nan
        held = np.full_like(a, POISON)              # only the rank's source rows are real
        held[:, shard.src_row0:shard.src_row1] = a[:, shard.src_row0:shard.src_row1]
        full = affine_ref.resample_array(held, m, (1, 40, 44), (1, 8, 44), 1, "mean", False,
                                         np.nan)
        local = torch.from_numpy(np.ascontiguousarray(np.asarray(full)[:, shard.row0:shard.row1]))
        out = gather_rows(local, 40)
        if rank == 0:
            np.save(os.path.join(result_dir, "coarsen.npy"), out.numpy())
    finally:
        dist.destroy_process_group()


def test_gloo_coarsen_shards_match_oracle(tmp_path):
    """world_size 2 over gloo: each rank holds only the source rows of its
    output chunk rows (the rest poisoned); the gathered coarsen result equals
    the whole-array oracle bit for bit (the chunk-edge halo is inside the
    footprints: affine.py:336-343)."""
    import torch.multiprocessing as mp

    from helpers import assert_bitwise_equal
    from oracle import affine_ref

    mp.spawn(_rank_coarsen, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    plan, m = _coarsen_plan()
    a = np.random.default_rng(11).random((1, 160, 176)).astype(np.float32)
    a.ravel()[::97] = np.nan
    exp = np.asarray(affine_ref.resample_array(a, m, (1, 40, 44), (1, 8, 44), 1, "mean", False,
                                               np.nan))
    assert_bitwise_equal(np.load(tmp_path / "coarsen.npy"), exp, "coarsen over 2 ranks")


def _rank_rectify(rank, world, port, result_dir):
    import sys

    import torch.distributed as dist

    here = os.path.dirname(os.path.abspath(__file__))
    for p in (here, os.path.dirname(here)):
        if p not in sys.path:
            sys.path.insert(0, p)
    from oracle import rectify_ref
    from xcube_resampling_amd.sharding import merge_tile_runs, rectify_shard

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        c = _rect_case()
        shard = rectify_shard(c["tiles"], world, rank)
        ids = range(shard.tile0, shard.tile1)
        ij, _ = rectify_ref.compute_target_source_ij(c["lon"], c["lat"], c["size"], c["tile"],
                                                     c["bbox"], c["res"], c["j_up"], tile_ids=ids)
        out = rectify_ref.compute_var_image(ij, c["var"], np.nan, "bilinear", c["tile"],
                                            tile_ids=ids)
        parts = [None] * world
        dist.all_gather_object(parts, (shard, out[:, shard.row0:shard.row1]))
        if rank == 0:
            w, h = c["size"]
            np.save(os.path.join(result_dir, "rectify.npy"),
                    merge_tile_runs(parts, c["tiles"], (h, w), np.nan))
    finally:
        dist.destroy_process_group()


def test_gloo_rectify_tile_shards_match_oracle(tmp_path):
    """world_size 2 over gloo: coordinates and data replicated, each rank
    rectifies its cost-balanced run of target tiles; the merged raster equals
    the whole oracle bit for bit."""
    import torch.multiprocessing as mp

    from helpers import assert_bitwise_equal
    from oracle import rectify_ref

    mp.spawn(_rank_rectify, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    c = _rect_case()
    exp = rectify_ref.compute_var_image(c["ij"], c["var"], np.nan, "bilinear", c["tile"])
    got = np.load(tmp_path / "rectify.npy")
    assert np.isfinite(exp).mean() > 0.5
    assert_bitwise_equal(got, exp, "rectify over 2 ranks")

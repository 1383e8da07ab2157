"""Multi-process (gloo, world_size 2) tests of the multi-GPU partition with the
HIP kernels doing the per-rank work: each rank uploads only the source rows
of its target-row band, runs ``kernels.reproject`` (xrs_reproject) on that
band, and the bands gathered over gloo equal the reference's output (golden
fixture) and the oracle (a larger seeded raster) bit for bit.  On a one-GPU
box the two ranks share the device, as the bench rehearsal does; the split,
the source-band upload and the reassembly are the code the driver's 8-GPU run
executes (reference reproject.py:230-252)."""

from __future__ import annotations

import os
import socket

import numpy as np
import pytest

from helpers import assert_bitwise_equal, load_golden, reproject_golden_inputs

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle_case():
    """A 1024x768 seeded source (0.1 % NaN) and a 900x700 EPSG:3857 target in
    128x96 tiles; returns (data, lon, lat, res, target args)."""
    rng = np.random.default_rng(20250905)
    h, w = 768, 1024
    xr, yr = 0.0075, 0.005
    lon = -5.0 + (np.arange(w) + 0.5) * xr
    lat = 55.0 - (np.arange(h) + 0.5) * yr
    data = rng.random((1, h, w), dtype=np.float32)
    data.ravel()[rng.choice(data.size, data.size // 1000, replace=False)] = np.nan
    return data, lon, lat, (xr, yr), ((900, 700), (-540000.0, 6500000.0), (800.0, 840.0),
                                      (128, 96))


def _case(name):
    import xcube_resampling_amd as xrs

    if name == "golden":
        g = load_golden("reproject_f32.npz")
        ds, tgm = reproject_golden_inputs(g)
        sgm = xrs.GridMapping.from_dataset(ds)
        return g["data"], sgm, tgm, g["fill"].item()
    data, lon, lat, _, (tsize, tmin, tres, ttile) = _oracle_case()
    sgm = xrs.GridMapping.from_coords(xrs.DataArray(lon, "lon", name="lon"),
                                      xrs.DataArray(lat, "lat", name="lat"), "EPSG:4326")
    tgm = xrs.GridMapping.regular(tsize, tmin, tres, "EPSG:3857", tile_size=ttile)
    return data, sgm, tgm, np.nan


def _rank_main(rank, world, port, result_dir, case, balance):
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    for p in (here, os.path.dirname(here)):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist

    import xcube_resampling_amd as xrs
    from xcube_resampling_amd import kernels
    from xcube_resampling_amd.sharding import band_shard, gather_rows

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)   # ranks share the box's GPU
        data, sgm, tgm, fill = _case(case)
        plan = xrs.plan_reproject(sgm, tgm, xrs.Transformer.from_crs(tgm.crs, sgm.crs,
                                                                      always_xy=True))
        shard = band_shard(plan, world, rank, balance)
        j0, j1 = shard.src_rows
        band = torch.from_numpy(np.ascontiguousarray(data[:, j0:j1])).cuda()   # its rows only
        out = kernels.reproject(band, plan, "bilinear", fill, rows=shard.rows, src_row0=j0)
        torch.cuda.synchronize()
        local = out.cpu()
        whole = gather_rows(local, plan.dst_height)
        if rank == 0:
            np.save(os.path.join(result_dir, f"{case}_{balance}.npy"), whole.numpy())
            np.save(os.path.join(result_dir, f"{case}_{balance}_cuts.npy"),
                    np.array([shard.row0, shard.row1]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case", ["golden", "oracle"])
@pytest.mark.parametrize("balance", ["rows", "cost"])
def test_gloo_band_sharded_hip_reprojection(tmp_path, case, balance):
    import torch.multiprocessing as mp

    world = 2
    mp.spawn(_rank_main, args=(world, _free_port(), str(tmp_path), case, balance), nprocs=world,
             join=True)
    got = np.load(tmp_path / f"{case}_{balance}.npy")
    r0, r1 = np.load(tmp_path / f"{case}_{balance}_cuts.npy")
    assert r0 == 0 and 0 < r1 < got.shape[1]   # rank 0 holds a real, partial band
    if case == "golden":
        exp = load_golden("reproject_f32.npz")["out_bilinear"]
    else:
        from oracle import gridmapping_ref as gref
        from oracle import reproject_ref

        data, lon, lat, (xr, yr), (tsize, tmin, tres, ttile) = _oracle_case()
        geo = gref.regular_geometry(tsize, tmin, tres, tile_size=ttile)
        exp = reproject_ref.reproject_array(
            data, gref.webmerc_inverse,
            lambda *b: gref.transform_bounds(gref.webmerc_inverse, *b), lon, lat, xr, yr,
            geo["x_coords"], geo["y_coords"], geo["xy_bboxes"], ttile[0], ttile[1], "bilinear",
            np.nan)
    assert got.dtype == exp.dtype == np.float64
    assert_bitwise_equal(got, exp, f"{case}/{balance}")   # NaN == NaN, -0 != +0


# ---- coarsen and rectify splits on the HIP kernels ---------------------------------
def _rank_coarsen_hip(rank, world, port, result_dir):
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    for p in (here, os.path.dirname(here)):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist

    from test_sharding_cpu import _coarsen_plan
    from xcube_resampling_amd import kernels
    from xcube_resampling_amd.sharding import coarsen_shard, gather_rows

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        plan, _ = _coarsen_plan()
        a = np.random.default_rng(11).random((1, 160, 176)).astype(np.float32)
        a.ravel()[::97] = np.nan
        shard = coarsen_shard(plan, world, rank)
        band = torch.from_numpy(np.ascontiguousarray(a[:, shard.src_row0:shard.src_row1])).cuda()
        out = kernels.affine(band, shard.plan)   # the rank's source rows only
        torch.cuda.synchronize()
        whole = gather_rows(out.cpu(), plan.out_h)
        if rank == 0:
            np.save(os.path.join(result_dir, "coarsen.npy"), whole.numpy())
    finally:
        dist.destroy_process_group()


def test_gloo_coarsen_shards_on_hip(tmp_path):
    """Each of 2 ranks runs K3 (xrs_affine) on only the source rows of its
    output chunk rows, with its re-based plan; the gathered result equals the
    whole-array oracle bit for bit (affine.py:277-313)."""
    import torch.multiprocessing as mp

    from oracle import affine_ref
    from test_sharding_cpu import _coarsen_plan

    mp.spawn(_rank_coarsen_hip, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    _, m = _coarsen_plan()
    a = np.random.default_rng(11).random((1, 160, 176)).astype(np.float32)
    a.ravel()[::97] = np.nan
    exp = np.asarray(affine_ref.resample_array(a, m, (1, 40, 44), (1, 8, 44), 1, "mean", False,
                                               np.nan))
    assert_bitwise_equal(np.load(tmp_path / "coarsen.npy"), exp, "coarsen on 2 ranks")


def _rank_rectify_hip(rank, world, port, result_dir):
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    for p in (here, os.path.dirname(here)):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist

    import xcube_resampling_amd as xrs
    from test_sharding_cpu import _rect_case
    from xcube_resampling_amd import rectify as R
    from xcube_resampling_amd.sharding import merge_tile_runs, rectify_shard

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        c = _rect_case()
        sgm = xrs.GridMapping.from_coords(xrs.DataArray(c["lon"], ("y", "x"), name="lon"),
                                          xrs.DataArray(c["lat"], ("y", "x"), name="lat"),
                                          "EPSG:4326")
        tgm = c["tgm"]
        tiles, _, _, _ = R.rectify_tiles(sgm, tgm)
        shard = rectify_shard(tiles, world, rank)
        band = R.rectify_tile_run(sgm, tgm, torch.from_numpy(c["var"]).cuda(), shard,
                                  "bilinear", np.nan, tiles=tiles)
        parts = [None] * world
        dist.all_gather_object(parts, (shard, band.cpu().numpy()))
        if rank == 0:
            w, h = c["size"]
            np.save(os.path.join(result_dir, "rectify.npy"),
                    merge_tile_runs(parts, tiles, (h, w), np.nan))
            np.save(os.path.join(result_dir, "tiles.npy"), tiles.view(np.uint8))
    finally:
        dist.destroy_process_group()


def test_gloo_rectify_tile_shards_on_hip(tmp_path):
    """Each of 2 ranks runs K5 on its cost-balanced run of target tiles and K6
    on the rows they cover; the merged raster equals the oracle bit for bit
    (rectify.py:347-370, 605-734)."""
    import torch.multiprocessing as mp

    from oracle import rectify_ref
    from test_sharding_cpu import _rect_case

    mp.spawn(_rank_rectify_hip, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    c = _rect_case()
    got_tiles = np.load(tmp_path / "tiles.npy").view(c["tiles"].dtype)
    assert np.array_equal(got_tiles.view(np.uint8), c["tiles"].view(np.uint8))   # same tiling
    exp = rectify_ref.compute_var_image(c["ij"], c["var"], np.nan, "bilinear", c["tile"])
    assert np.isfinite(exp).mean() > 0.5
    assert_bitwise_equal(np.load(tmp_path / "rectify.npy"), exp, "rectify on 2 ranks")

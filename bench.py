"""Benchmark: reproject bilinear EPSG:4326 -> EPSG:3857, 40960x40960 float32,
2048x2048 target tiles (BASELINE.json metric / configs[4]).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (driver, N > 1)

One "step" = one pass of the hot path (xrs_reproject, all 400 target tiles of
one 40960x40960 raster in one launch) over one synthetic raster resident in
HBM.  Multi-GPU: the global job is an (N, 40960, 40960) cube (the reference's
dim-0 axis, reproject.py:230-252); rank r reprojects slice r on its own GPU —
independent partitions, no data-path collective ("scaling": "weak").
Rank 0 prints ONE JSON line.
"""

from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)

# config 5 geometry: source EPSG:4326 pixel centres, target EPSG:3857
SRC_X0, SRC_Y0 = -20.0, 70.96
TGT_MIN = (-2226000.0, 3504000.0)


def workload(size: int, tile: int):
    import xcube_resampling_amd as xrs

    scale = 40960 / size
    xres, yres = 0.0015 * scale, 0.001 * scale
    lon = SRC_X0 + (np.arange(size) + 0.5) * xres
    lat = SRC_Y0 - (np.arange(size) + 0.5) * yres
    src_gm = xrs.GridMapping.from_coords(xrs.DataArray(lon, "lon", name="lon"),
                                         xrs.DataArray(lat, "lat", name="lat"), "EPSG:4326")
    tgm = xrs.GridMapping.regular((size, size), TGT_MIN, (166 * scale, 190 * scale), "EPSG:3857",
                                  tile_size=tile)
    tr = xrs.Transformer.from_crs(tgm.crs, src_gm.crs, always_xy=True)
    plan = xrs.plan_reproject(src_gm, tgm, tr)
    return src_gm, tgm, plan, lon, lat


def source_pixels_read(plan, band=None) -> int:
    """Distinct in-bounds source pixels the bilinear gather reads for target
    rows `band` (default all; separable plan: |rows read| x |cols read|); the
    algorithmic read bytes are 4x this."""
    ntx, nty = plan.num_tiles
    b0, b1 = band if band is not None else (0, plan.dst_height)
    cols = np.zeros(plan.src_width, bool)
    rows = np.zeros(plan.src_height, bool)
    for t in range(ntx * nty):
        ty, tx = divmod(t, ntx)
        c = np.arange(tx * plan.tile_width, min(plan.dst_width, (tx + 1) * plan.tile_width))
        r = np.arange(max(b0, ty * plan.tile_height),
                      min(b1, plan.dst_height, (ty + 1) * plan.tile_height))
        if r.size == 0:
            continue
        ix = (plan.src_x[c] - np.float64(plan.tile_x0[t])) / plan.x_res
        iy = (plan.src_y[r] - np.float64(plan.tile_y0[t])) / -plan.y_res
        for idx, base, n, mask in ((ix, plan.tile_win[t, 0], plan.src_width, cols),
                                   (iy, plan.tile_win[t, 1], plan.src_height, rows)):
            for f in (np.floor(idx), np.ceil(idx)):
                g = base + f.astype(np.int64)
                g = g[(g >= 0) & (g < n)]
                mask[g] = True
    return int(rows.sum()) * int(cols.sum())


def cpu_baseline(plan, src_gm, lon, lat, tgm, seconds: float = 12.0):
    """Oracle (numpy restatement of reproject.py:268-335 + the per-tile window
    copy of 499-530) on the host cores, one task per 2048^2 tile on a thread
    pool (dask threaded scheduler style), until `seconds` of work is done."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import reproject_ref

    cores = min(16, len(os.sched_getaffinity(0)))
    ntx, nty = plan.num_tiles
    tiles = [(j, i) for j in range(min(2, nty)) for i in range(ntx)]
    rows = [plan.source_rows_for(j * plan.tile_height, (j + 1) * plan.tile_height) for j, _ in tiles]
    j0, j1 = min(r[0] for r in rows), max(r[1] for r in rows)
    rng = np.random.default_rng(1)
    band = rng.random((1, j1 - j0, plan.src_width), dtype=np.float32)
    xc, yc = tgm.x_coords.values, tgm.y_coords.values
    wy, wx = plan.win_height, plan.win_width

    def run_tile(jt):
        j, i = jt
        t = j * ntx + i
        r0, r1 = j * plan.tile_height, min(plan.dst_height, (j + 1) * plan.tile_height)
        c0, c1 = i * plan.tile_width, min(plan.dst_width, (i + 1) * plan.tile_width)
        xx, yy = np.meshgrid(xc[c0:c1], yc[r0:r1])
        from xcube_resampling_amd.crs import webmerc_inverse  # same formula as the oracle's
        sxx, syy = webmerc_inverse(xx, yy)
        wi0, wj0 = plan.tile_win[t]
        win = np.full((1, wy, wx), np.nan, np.float32)
        sj0, sj1 = max(wj0, 0), min(wj0 + wy, plan.src_height)
        si0, si1 = max(wi0, 0), min(wi0 + wx, plan.src_width)
        win[:, sj0 - wj0:sj1 - wj0, si0 - wi0:si1 - wi0] = band[:, sj0 - j0:sj1 - j0, si0:si1]
        x_coord = np.full((wx, 1, 1), plan.tile_x0[t], np.float32)
        y_coord = np.full((wy, 1, 1), plan.tile_y0[t], np.float32)
        out = reproject_ref.reproject_block(sxx, syy, win, x_coord, y_coord, plan.x_res,
                                            plan.y_res, "bilinear")
        return out.shape[1] * out.shape[2]

    px = 0
    t0 = time.perf_counter()
    with ThreadPoolExecutor(max_workers=cores) as ex:
        k = 0
        while time.perf_counter() - t0 < seconds:
            batch = [tiles[(k + q) % len(tiles)] for q in range(cores)]
            k += cores
            px += sum(ex.map(run_tile, batch))
    dt = time.perf_counter() - t0
    return dict(value=px / dt / 1e6, unit="Mpixels/s", cores=cores, kind="port",
                sample=f"{px // (plan.tile_width * plan.tile_height)} target tiles of "
                       f"{plan.tile_width}x{plan.tile_height} (bilinear, f32 in, f64 out as the "
                       f"reference) in {dt:.1f} s, incl. per-tile coordinate transform and "
                       f"window copy; numpy oracle on a {cores}-thread pool")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--size", type=int, default=40960)
    ap.add_argument("--tile", type=int, default=2048)
    ap.add_argument("--out-dtype", choices=["f32", "f64"], default="f32")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--shard", choices=["slices", "bands"], default="slices",
                    help="slices: rank r reprojects slice r of an (N, S, S) cube (weak); "
                         "bands: the ranks split the target tile rows of ONE SxS raster, "
                         "each holding only the source rows its band reads (strong)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_r01.json"))
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from xcube_resampling_amd import kernels
    from xcube_resampling_amd.sharding import band_shard, env_rank, max_over_ranks

    rank, world, local_rank = env_rank()
    # one GPU per rank; XRS_BENCH_BACKEND=gloo with more ranks than GPUs is only
    # a rehearsal of the multi-rank logic on a smaller box (ranks share GPUs)
    backend = os.environ.get("XRS_BENCH_BACKEND", "nccl")
    dev_index = local_rank % torch.cuda.device_count() if backend == "gloo" else local_rank
    torch.cuda.set_device(dev_index)
    device = torch.device("cuda", dev_index)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)

    src_gm, tgm, plan, lon, lat = workload(args.size, args.tile)
    out_np = np.float32 if args.out_dtype == "f32" else np.float64
    gen = torch.Generator(device=device)
    gen.manual_seed(20250905 + rank)
    if args.shard == "bands":
        shard = band_shard(plan, world, rank)
        rows, (j0, j1) = shard.rows, shard.src_rows
    else:
        rows, (j0, j1) = (0, plan.dst_height), (0, plan.src_height)
    src = torch.rand((1, j1 - j0, args.size), generator=gen, device=device, dtype=torch.float32)
    out = torch.empty((1, rows[1] - rows[0], args.size), device=device,
                      dtype=torch.float32 if args.out_dtype == "f32" else torch.float64)
    flags = kernels.ErrorFlags(device)

    def step():
        if rows[1] > rows[0]:
            kernels.reproject(src, plan, "bilinear", float("nan"), out_dtype=out_np, out=out,
                              rows=rows, src_row0=j0, flags=flags)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            if backend == "nccl":
                dist.barrier(device_ids=[dev_index])
            else:
                dist.barrier()

    barrier()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(device)      # the stream xrs_reproject launches on
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    flags.raise_if_set("bench reproject")

    elapsed = t1 - t0
    kernel_ms = ev0.elapsed_time(ev1) / args.steps
    elapsed = max_over_ranks(elapsed, device)
    ms_per_step = elapsed / args.steps * 1e3
    npx = args.size * args.size
    n_rasters = world if args.shard == "slices" else 1
    value = n_rasters * npx / (ms_per_step / 1e3) / 1e6

    if rank == 0:
        s_read = source_pixels_read(plan, rows)
        out_bytes = (rows[1] - rows[0]) * args.size * np.dtype(out_np).itemsize
        alg_bytes = out_bytes + 4 * s_read
        achieved = alg_bytes / (kernel_ms / 1e3) / 1e9
        traffic = None
        if os.path.exists(args.traffic_json):
            with open(args.traffic_json) as f:
                tj = json.load(f)
            if tj.get("size") == args.size and tj.get("out_dtype") == args.out_dtype \
                    and args.shard == "slices":
                traffic = tj.get("hbm_bytes_per_launch")
        res = {
            "metric": "Mpixels/s reproject bilinear 40960² f32; achieved HBM GB/s vs peak",
            "value": round(value, 1),
            "unit": "Mpixels/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak" if args.shard == "slices" else "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {
                "workload": f"reproject EPSG:4326->EPSG:3857 bilinear {args.size}x{args.size} "
                            f"f32 source, {args.tile}x{args.tile} target tiles (configs[4]); "
                            + (f"{world} slice(s) of an (N,{args.size},{args.size}) cube, 1 per GPU"
                               if args.shard == "slices" else
                               f"one raster split into {world} tile-row band(s), 1 per GPU"),
                "source_dtype": "f32",
                "out_dtype": args.out_dtype,
                "interp": "bilinear",
                "tiles": plan.num_tiles[0] * plan.num_tiles[1],
                "window": [plan.win_height, plan.win_width],
                "parallelism": f"{args.shard}{world}",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "kernel": "gather_separable_mlp_kernel<float,float,1,8,true,2> (+ axis_tables_kernel<1>, <0.6%)",
                "kernel_ms": round(kernel_ms, 4),
                "algorithmic_bytes": int(alg_bytes),
            },
        }
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(plan, src_gm, lon, lat, tgm, args.cpu_seconds)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

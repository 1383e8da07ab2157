"""Secondary measurement lines: BASELINE.json configs 1-4.

    python scripts/bench_configs.py [--configs 1,2,2u,3,3f,4,4f] [--steps K] [--cpu-seconds S]

bench.py measures the headline metric (config 5 on one GPU per slice); this
script measures the other configurations the same way — inputs resident in
HBM, HIP events on the launch stream around K timed launches after a warm-up,
algorithmic bytes per SURVEY.md §8(d) — and times the oracle on a bounded
sample of the same workload beside it.  One JSON line per config.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
HBM_PEAK_GBS = 8000.0


def _timed(fn, steps, warmup, graph=False):
    """(event ms/step, wall ms/step); graph=True replays one captured call
    (no Python/ctypes launch overhead between steps, as bench.py)."""
    import torch

    if graph:   # the K timed steps captured back to back in one graph
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(steps):
                fn()
        for _ in range(max(1, warmup)):
            g.replay()
        torch.cuda.synchronize()
        stream = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        g.replay()
        e1.record(stream)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / steps * 1e3
        return e0.elapsed_time(e1) / steps, wall
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(steps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps * 1e3
    return e0.elapsed_time(e1) / steps, wall


def _line(cfg, workload, npx, ms, wall_ms, alg_bytes, kernel, cpu, extra=None):
    achieved = alg_bytes / (ms / 1e3) / 1e9
    d = {"config": cfg, "workload": workload, "metric": "target Mpixels/s",
         "value": round(npx / (wall_ms / 1e3) / 1e6, 1), "unit": "Mpixels/s",
         "ms_per_step": round(wall_ms, 4),
         "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                      "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                      "kernel": kernel, "kernel_ms": round(ms, 4),
                      "algorithmic_bytes": int(alg_bytes)},
         "cpu_baseline": cpu}
    if extra:
        d.update(extra)
    print(json.dumps(d), flush=True)


def _cpu_whole(run, npx, passes=3):
    """The whole configuration on the host, best of `passes`: run(executor)
    does every task of the raster on a thread pool of all cores of the
    affinity mask.  Returns (Mpx/s of the best pass, its seconds, cores)."""
    from concurrent.futures import ThreadPoolExecutor

    cores = len(os.sched_getaffinity(0))
    best = float("inf")
    with ThreadPoolExecutor(max_workers=cores) as ex:
        for _ in range(passes):
            t0 = time.perf_counter()
            run(ex)
            best = min(best, time.perf_counter() - t0)
    return npx / best / 1e6, best, cores


def _cpu_pool(fn, seconds):
    """Run independent per-chunk tasks `fn()` (-> target pixels) on a thread
    pool over ALL cores of the affinity mask (the dask threaded scheduler's
    shape; scipy.ndimage and numpy release the GIL) for `seconds`."""
    from concurrent.futures import ThreadPoolExecutor

    cores = len(os.sched_getaffinity(0))
    px, t0 = 0, time.perf_counter()
    with ThreadPoolExecutor(max_workers=cores) as ex:
        while time.perf_counter() - t0 < seconds:
            px += sum(ex.map(lambda _: fn(), range(cores)))
    dt = time.perf_counter() - t0
    return px / dt / 1e6, px, dt, cores


# the issue-bound rectify kernels: one rocprofv3 --pmc pass (6 SQ + 2 GRBM
# counters) of scripts/time_rectify.py --fused, reduced per kernel
ISSUE_COUNTERS = ["SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_WAVE_CYCLES",
                  "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "GRBM_GUI_ACTIVE", "GRBM_COUNT"]
N_SIMD = 1024   # 256 CUs x 4 SIMDs
N_XCD = 8


def issue_pmc(kernels=("claim", "resolve", "ij_bboxes"), timeout=150,
              script=("time_rectify.py", "--fused", "--reps", "3")):
    """Per kernel: VALU-issue fraction = 4 x SQ_ACTIVE_INST_VALU (quad-cycles
    of VALU issue, summed over the SIMDs) / (N_SIMD x GRBM_GUI_ACTIVE / N_XCD
    (the dispatch's shader cycles; the GRBM counter sums the 8 XCDs)): the
    share of the SIMDs' cycles spent issuing vector instructions at the
    nominal 4 cycles per wave64 instruction — the roof of an issue-bound
    kernel, as the HBM fraction is of a memory-bound one.  Also the wave
    cycles parked on memory (SQ_WAIT_ANY / SQ_WAVE_CYCLES).  Runs as a child
    process while this one is idle; None when rocprofv3 is absent or fails."""
    import csv
    import shutil
    import subprocess
    import tempfile
    from collections import defaultdict

    prof = shutil.which("rocprofv3")
    if prof is None:
        return None
    d = tempfile.mkdtemp(prefix="xrs_issue_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        cmd = ["timeout", "-s", "KILL", str(timeout), prof, "--pmc", *ISSUE_COUNTERS,
               "--kernel-trace", "--output-format", "csv", "-d", d, "-o", "p", "--",
               sys.executable, os.path.join(ROOT, "scripts", script[0]), *script[1:]]
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        if r.returncode != 0:
            print(f"issue_pmc: rocprofv3 failed (rc {r.returncode}):\n{r.stdout[-1500:]}",
                  file=sys.stderr)
            return None
        acc = defaultdict(float)
        disp = defaultdict(set)
        for path in _find(d, "counter_collection.csv"):
            for row in csv.DictReader(open(path)):
                k = next((n for n in kernels if n in row["Kernel_Name"]), None)
                if k is None:
                    continue
                acc[(k, row["Counter_Name"])] += float(row["Counter_Value"])
                disp[k].add(row["Dispatch_Id"])
        out = {}
        for k in kernels:
            n = len(disp[k])
            if not n:
                continue
            c = {name: acc[(k, name)] / n for name in ISSUE_COUNTERS}
            cyc = c["GRBM_GUI_ACTIVE"] / N_XCD
            out[k] = {"valu_issue_frac": round(4 * c["SQ_ACTIVE_INST_VALU"] / (N_SIMD * cyc), 4)
                      if cyc else None,
                      "valu_wave_insts": int(c["SQ_INSTS_VALU"]),
                      "salu_wave_insts": int(c["SQ_INSTS_SALU"]),
                      "wait_frac": round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 4)
                      if c["SQ_WAVE_CYCLES"] else None,
                      "shader_cycles": int(cyc), "dispatches": n}
        out["method"] = ("rocprofv3 --pmc " + " ".join(ISSUE_COUNTERS) + " on scripts/" +
                         " ".join(script) + ": valu_issue_frac = 4 x "
                         "SQ_ACTIVE_INST_VALU / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs); "
                         "wait_frac = SQ_WAIT_ANY / SQ_WAVE_CYCLES")
        return out
    finally:
        shutil.rmtree(d, ignore_errors=True)


def kernel_times(interp, timeout=150, reps=30, res_div=1.0):
    """The fused config-4 pipeline's own kernels (scripts/time_rectify.py
    --fused: K4 + device tiling + claim + resolve with K6 inside), average
    microseconds per launch from one rocprofv3 --kernel-trace --stats child
    run; None when rocprofv3 is absent or fails."""
    import csv
    import shutil
    import subprocess
    import tempfile

    prof = shutil.which("rocprofv3")
    if prof is None:
        return None
    d = tempfile.mkdtemp(prefix="xrs_kt_", dir=os.environ.get("TMPDIR", "/tmp"))
    cmd = ["timeout", "-s", "KILL", str(timeout), prof, "--kernel-trace", "--stats",
           "--output-format", "csv", "-d", d, "-o", "kt", "--", sys.executable,
           os.path.join(ROOT, "scripts", "time_rectify.py"), "--fused", "--interp", interp,
           "--reps", str(reps), "--res-div", str(res_div)]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        print(f"kernel_times: rocprofv3 failed (rc {r.returncode}):\n{r.stdout[-1500:]}",
              file=sys.stderr)
        return None
    names = {"K4 ij_bboxes": "ij_bboxes", "tiles": "rectify_tiles_kernel",
             "K5a claim": "rectify_claim_kernel", "K5b resolve + K6 (fused)": "rectify_resolve_kernel"}
    out = {}
    for path in _find(d, "kernel_stats.csv"):
        for row in csv.DictReader(open(path)):
            for label, key in names.items():
                if key in row["Name"]:
                    out[label] = out.get(label, 0.0) + float(row["AverageNs"]) / 1e3
    return {k: round(v, 1) for k, v in out.items()} or None


def _find(root, suffix):
    for dp, _, files in os.walk(root):
        for f in files:
            if f.endswith(suffix):
                yield os.path.join(dp, f)


# ------------------------------------------------------------------ config 1
def config1(args):
    """Affine nearest 1024^2 f32, EPSG:4326 -> EPSG:4326 (scale 0.9216)."""
    import torch

    import xcube_resampling_amd as xrs
    import xcube_resampling_amd.affine as A
    from xcube_resampling_amd import kernels
    from oracle import affine_ref

    n = 1024
    res = 2.0 ** -10
    lon = 10 + (np.arange(n) + 0.5) * res
    lat = 51 - (np.arange(n) + 0.5) * res
    sgm = xrs.GridMapping.from_coords(xrs.DataArray(lon, "lon", name="lon"),
                                      xrs.DataArray(lat, "lat", name="lat"), "EPSG:4326")
    tgm = xrs.GridMapping.regular((n, n), (10.1, 50.05), 0.0009, "EPSG:4326")
    m = tgm.ij_transform_to(sgm)
    a = np.random.default_rng(20250905).random((1, n, n), dtype=np.float32)
    plan = A.plan_affine(a.shape, a.dtype, m, (1, n, n), (1, tgm.tile_height, tgm.tile_width),
                         0, "first", False, np.nan)
    src = torch.from_numpy(a).cuda()
    out = kernels.affine(src, plan)
    ref = affine_ref.resample_array(a, m, (1, n, n), (1, tgm.tile_height, tgm.tile_width), 0,
                                    "first", False, np.nan)
    assert np.array_equal(out.cpu().numpy(), ref, equal_nan=True), "config 1 parity"
    ms, wall = _timed(lambda: kernels.affine(src, plan, out), args.steps, args.warmup, graph=True)
    s_read = n * n  # every source pixel is read at most once (scale < 1)
    # many small chunks (the dask shape): 64 independent 1024^2 chunks with
    # one geometry stacked on dim 0 -> ONE launch instead of 64 latency-bound
    # ones; slice 5 checked against the oracle of that chunk alone
    nb_ = 64
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    srcb = torch.rand((nb_, n, n), generator=g, device="cuda", dtype=torch.float32)
    planb = A.plan_affine(tuple(srcb.shape), np.dtype(np.float32), m, (nb_, n, n),
                          (1, tgm.tile_height, tgm.tile_width), 0, "first", False, np.nan)
    outb = kernels.affine(srcb, planb)
    refb = affine_ref.resample_array(srcb[5:6].cpu().numpy(), m, (1, n, n),
                                     (1, tgm.tile_height, tgm.tile_width), 0, "first", False,
                                     np.nan)
    assert np.array_equal(outb[5:6].cpu().numpy(), refb, equal_nan=True), "batched parity"
    bms, bwall = _timed(lambda: kernels.affine(srcb, planb, outb), args.steps, args.warmup,
                        graph=True)
    batched = {"batched": {"chunks": nb_, "ms_per_launch": round(bwall, 4),
                           "value": round(nb_ * n * n / (bwall / 1e3) / 1e6, 1),
                           "achieved_GBs": round(nb_ * 8 * n * n / (bms / 1e3) / 1e9, 1),
                           "note": "64 independent 1024^2 chunks of one geometry stacked on "
                                   "dim 0, one launch (slice 5 == the oracle of that chunk)"}}
    del srcb, outb
    cpu_v, px, dt, cores = _cpu_pool(lambda: affine_ref.resample_array(
        a, m, (1, n, n), (1, n, n), 0, "first", False, np.nan).size, args.cpu_seconds)
    _line(1, "affine nearest 1024x1024 f32 EPSG:4326 (scale 0.9216, offset 102.4 px)", n * n,
          ms, wall, 4 * n * n + 4 * s_read, "affine_direct_kernel<float,float,0,false>",
          dict(value=round(cpu_v, 2), unit="Mpixels/s", cores=cores, kind="port",
               sample=f"{px // (n * n)} independent 1024^2 single-chunk resamples in {dt:.1f} s "
                      f"on a {cores}-thread pool (dask-image chunk restatement calling "
                      "scipy.ndimage.affine_transform)"), batched)


# ------------------------------------------------------------------ config 2
def config2(args):
    """Reproject bilinear 8192^2 f32 EPSG:4326 -> EPSG:3857, 2048^2 tiles."""
    import torch

    import bench
    from xcube_resampling_amd import kernels

    size = 8192
    src_gm, tgm, plan, lon, lat = bench.workload(size, 2048)
    src = torch.rand((1, size, size), device="cuda", dtype=torch.float32)
    out = torch.empty((1, size, size), device="cuda", dtype=torch.float64)
    flags = kernels.ErrorFlags(src.device)
    ms, wall = _timed(lambda: kernels.reproject(src, plan, "bilinear", float("nan"), out=out,
                                                flags=flags, check=False),
                      args.steps, args.warmup, graph=True)
    flags.raise_if_set("config 2")
    s_read = bench.source_pixels_read(plan)
    cpu = bench.cpu_baseline(plan, tgm, args.cpu_seconds)
    _line(2, "reproject bilinear 8192x8192 f32 EPSG:4326->EPSG:3857, 2048^2 tiles, f64 out "
             "(the reference's bilinear dtype)", size * size, ms, wall,
          8 * size * size + 4 * s_read, "gather_separable_kernel<float,double,1>", cpu)


# ------------------------------------------------------ config 2u
def config2u(args):
    """Reproject bilinear 8192^2 f32 UTM 32N (EPSG:32632) -> LAEA Europe
    (EPSG:3035), 2048^2 tiles: a non-separable pair, per-pixel transform on
    the device (xrs_transform) + K1 on the 2-D coordinate tables."""
    import torch

    import xcube_resampling_amd as xrs
    from xcube_resampling_amd import kernels

    size, res = 8192, 30.0
    sgm = xrs.GridMapping.regular((size, size), (400000.0, 5400000.0), res, "EPSG:32632",
                                  tile_size=2048)
    tgm = xrs.GridMapping.regular((size, size), (4180000.0, 2870000.0), res, "EPSG:3035",
                                  tile_size=2048)
    tr = xrs.Transformer.from_crs(tgm.crs, sgm.crs, always_xy=True)
    plan = xrs.plan_reproject(sgm, tgm, tr)
    assert plan.coord_mode == 1
    g = torch.Generator(device="cuda")
    g.manual_seed(20250905)
    src = torch.rand((1, size, size), generator=g, device="cuda", dtype=torch.float32)
    out = torch.empty((1, size, size), device="cuda", dtype=torch.float64)
    flags = kernels.ErrorFlags(src.device)

    def end_to_end():   # coordinate tables rebuilt every step, then K1
        plan._device_cache.clear()
        kernels.reproject(src, plan, "bilinear", float("nan"), out=out, flags=flags)

    gx = torch.from_numpy(plan.grid_x).cuda()
    gy = torch.from_numpy(plan.grid_y).cuda()
    t_ms, _ = _timed(lambda: kernels.transform(tr, gx, gy, True), args.steps, args.warmup)
    plan.device_tables(src.device)
    k_ms, _ = _timed(lambda: kernels.reproject(src, plan, "bilinear", float("nan"), out=out,
                                               flags=flags), args.steps, args.warmup)
    e_ms, wall = _timed(end_to_end, max(3, args.steps // 4), 1)
    flags.raise_if_set("config 2u")
    covered = int(torch.isfinite(out).sum().item())
    # CPU: the numpy restatement of the per-pixel transformation, one 512^2
    # block per task on a pool over all cores (the reference's
    # _transform_gridpoints per dask block, its dominant per-block cost)
    xx, yy = np.meshgrid(plan.grid_x[:512], plan.grid_y[:512])
    cpu_v, px, dt, cores = _cpu_pool(lambda: (tr.transform(xx, yy), xx.size)[1],
                                     args.cpu_seconds)
    # algorithmic bytes of the end-to-end step: tables written + read (32 B/px),
    # f64 out, f32 source reads (<= the source once)
    alg = 16 * size * size + 16 * size * size + 8 * size * size + 4 * size * size
    _line("2u", "reproject bilinear 8192x8192 f32 UTM 32N (EPSG:32632) -> LAEA Europe "
                "(EPSG:3035) 30 m, 2048^2 tiles, f64 out; per-pixel transform on the device "
                "(xrs_transform: laea inverse + tmerc forward) then K1 on 2-D tables, end to end",
          size * size, e_ms, wall, alg,
          f"transform_kernel<true> {t_ms:.3f} ms + gather K1 (2-D tables) {k_ms:.3f} ms",
          dict(value=round(cpu_v, 2), unit="Mpixels/s", cores=cores, kind="port",
               sample=f"numpy restatement of the per-pixel LAEA -> UTM transform "
                      f"(projections.py) over {px // xx.size} 512^2 blocks in {dt:.1f} s on "
                      f"{cores} threads (the transform alone; the block gather is not "
                      "included; numpy's ufuncs hold the GIL between calls)"),
          {"transform_ms": round(t_ms, 4), "k1_ms": round(k_ms, 4), "covered_px": covered,
           "transform_gpts_s": round(size * size / (t_ms / 1e3) / 1e9, 2)})

    # the same step with the transformation fused into the gather
    # (xrs_reproject_proj, what reproject_dataset runs for ONE variable)
    import dataclasses
    fplan = dataclasses.replace(plan, fuse_transform=True, _device_cache={})
    fout = torch.empty_like(out)
    f_ms, f_wall = _timed(lambda: kernels.reproject(src, fplan, "bilinear", float("nan"), out=fout,
                                                    flags=flags, check=False),
                          args.steps, args.warmup, graph=True)
    flags.raise_if_set("config 2u fused")
    assert torch.equal(torch.nan_to_num(fout, nan=-7.0), torch.nan_to_num(out, nan=-7.0)), \
        "config 2u: fused gather differs from the tables path"
    torch.cuda.synchronize()
    # the transformation is f64-VALU bound: its issue fractions (2u-fused's roof)
    issue = issue_pmc(kernels=("gather_proj_kernel", "transform_kernel", "gather_2d_kernel"),
                      script=("time_2u.py", "--reps", "3"))
    _line("2u-fused", "reproject bilinear 8192x8192 f32 UTM 32N (EPSG:32632) -> LAEA Europe "
                      "(EPSG:3035) 30 m, 2048^2 tiles, f64 out; transformation fused into the "
                      "gather (xrs_reproject_proj), bit-identical to the tables path",
          size * size, f_ms, f_wall, 8 * size * size + 4 * size * size,
          "gather_proj_kernel<LAEA_INV, TMERC_FWD>",
          dict(value=round(cpu_v, 2), unit="Mpixels/s", cores=cores, kind="port",
               sample="as the 2u line"), {"covered_px": covered, "issue": issue})


# ------------------------------------------------------------------ config 3
def config3f(args):
    """Config 3 with the target grid shifted by 0.3 / 0.6 source pixels (a
    target not aligned to the source: the div-x grid has scale 1 and
    fractional offsets, K3w)."""
    config3(args, frac=True)


def config3(args, frac=False):
    """Coarsen mean 4x4: 16384^2 f32 -> 4096^2 (bilinear upscale at scale 1 + nanmean)."""
    import torch

    import xcube_resampling_amd as xrs
    import xcube_resampling_amd.affine as A
    from xcube_resampling_amd import kernels
    from oracle import affine_ref

    n, k = 16384, 4
    res = 2.0 ** -10
    lon = (np.arange(n) + 0.5) * res
    lat = n * res - (np.arange(n) + 0.5) * res
    sgm = xrs.GridMapping.from_coords(xrs.DataArray(lon, "lon", name="lon"),
                                      xrs.DataArray(lat, "lat", name="lat"), "EPSG:4326")
    if frac:   # shifted by (0.3, 0.6) source pixels, one output pixel short of the edge
        tgm = xrs.GridMapping.regular((n // k - 1, n // k - 1), (0.3 * res, 0.6 * res), res * k,
                                      "EPSG:4326")
    else:
        tgm = xrs.GridMapping.regular((n // k, n // k), (0, 0), res * k, "EPSG:4326")
    m = tgm.ij_transform_to(sgm)
    if not frac:
        assert m == ((4.0, 0.0, 0.0), (0.0, 4.0, 0.0)), m
    no = tgm.width
    g = torch.Generator(device="cuda")
    g.manual_seed(20250905)
    src = torch.rand((1, n, n), generator=g, device="cuda", dtype=torch.float32)
    oc = (1, tgm.tile_height, tgm.tile_width)
    plan = A.plan_affine(tuple(src.shape), np.dtype(np.float32), m, (1, no, no), oc, 1,
                         "mean", False, np.nan)
    assert plan.run_weights == frac
    out = kernels.affine(src, plan)
    # parity on a corner (the oracle on the full 1 GiB raster takes minutes)
    c = 1024
    a = src[:, :c, :c].cpu().numpy()
    ref = affine_ref.resample_array(a, m, (1, c // k, c // k), (1, c // k, c // k), 1, "mean",
                                    False, np.nan)
    assert np.array_equal(out[:, :c // k - 1, :c // k - 1].cpu().numpy(),
                          ref[:, :-1, :-1]), "config 3 parity"
    ms, wall = _timed(lambda: kernels.affine(src, plan, out), args.steps, args.warmup, graph=True)
    # CPU baseline on the whole raster: the reference's 64 per-chunk tasks (a
    # 2048^2 source chunk -> a 512^2 output chunk each) over the whole 16384^2
    # source on a thread pool of all cores, best of 3 passes
    cs = 2048
    host = src.cpu().numpy()
    chunks = [(cj, ci) for cj in range(n // cs) for ci in range(n // cs)]

    def task(c):
        cj, ci = c
        blk = host[:, cj * cs:(cj + 1) * cs, ci * cs:(ci + 1) * cs]
        return affine_ref.resample_array(blk, m, (1, cs // k, cs // k), (1, cs // k, cs // k), 1,
                                         "mean", False, np.nan).size   # (frac: same work)

    cpu_v, dt, cores = _cpu_whole(lambda ex: sum(ex.map(task, chunks)), (n // k) ** 2)
    del host
    _line("3f" if frac else 3,
          ("coarsen mean 4x4, target shifted by (0.3, 0.6) source px: 16384x16384 f32 -> "
           "4095x4095 (affine bilinear at the 4x grid with fractional weights + nanmean)")
          if frac else ("coarsen mean 4x4: 16384x16384 f32 -> 4096x4096 (affine bilinear at the "
                        "4x grid + nanmean)"), no * no, ms, wall, 4 * n * n + 4 * no * no,
          ("K3w affine_reduce_integral_kernel<float,1,4,false,true> (contiguous runs, fractional "
           "weights; edge pixels via integral_slow_kernel)") if frac else
          ("K3i affine_reduce_integral_kernel<float,1,4> (fused upscale+coarsen; edge pixels "
           "via integral_slow_kernel)"),
          dict(value=round(cpu_v, 3), unit="Mpixels/s", cores=cores, kind="port",
               sample=f"the whole 16384^2 raster: its {len(chunks)} per-chunk tasks (a 2048^2 "
                      f"source chunk -> 512^2 each; scipy affine_transform + numpy nanmean in "
                      f"dask chunk.coarsen order) on a {cores}-thread pool, best of 3 passes: "
                      f"{dt:.2f} s"))


# ------------------------------------------------------------------ config 4
def config4(args, div=1.0):
    """Rectify a 4000x4800 jittered swath to a ~8.3k x 5.4k EPSG:4326 grid, 512^2 tiles
    (div > 1: onto a grid div-fold finer, line "4f": the claim's compacted walk)."""
    import torch

    import xcube_resampling_amd as xrs
    from xcube_resampling_amd import kernels
    from xcube_resampling_amd import rectify as R
    from oracle import gridmapping_ref as gref
    from oracle import rectify_ref

    w, h = 4000, 4800
    rng = np.random.default_rng(20250905)
    i = np.arange(w)[None, :].astype(np.float64)
    j = np.arange(h)[:, None].astype(np.float64)
    lat = 60 - 0.0027 * j - 0.0004 * i + 1e-9 * (i - 2000) ** 2 \
        + rng.normal(0, 0.05 * 0.0027, (h, w))
    lon = 5 + 0.0045 * i + 0.0009 * j + rng.normal(0, 0.05 * 0.0045, (h, w))
    var = rng.random((1, h, w), dtype=np.float32)
    res = 0.0027 / div
    x0, y0 = float(np.floor(lon.min() / res) * res), float(np.floor(lat.min() / res) * res)
    tw, th = int(np.ceil((lon.max() - x0) / res)), int(np.ceil((lat.max() - y0) / res))
    tgm = xrs.GridMapping.regular((tw, th), (x0, y0), res, "EPSG:4326", tile_size=512)
    geo = gref.regular_geometry((tw, th), (x0, y0), res, tile_size=(512, 512))
    sgm = xrs.GridMapping.from_coords(xrs.DataArray(lon, ("y", "x"), name="lon"),
                                      xrs.DataArray(lat, ("y", "x"), name="lat"), "EPSG:4326")
    dlon, dlat = torch.from_numpy(lon).cuda(), torch.from_numpy(lat).cuda()
    src = torch.from_numpy(var).cuda()
    xy = (dlon, dlat)

    tiles, ntx, bb, _ = R.rectify_tiles(sgm, tgm, xy=xy)
    dst_y_scale = -tgm.y_res
    flags = kernels.ErrorFlags(src.device)   # checked once at the end (no sync per call)

    def k5():
        return kernels.rectify_ij(xy[0], xy[1], tiles, ntx, tgm.height, tgm.width, tgm.x_res,
                                  dst_y_scale, 1e-3, flags=flags)

    ij = k5()
    covered = int(torch.sum(~torch.isnan(ij[0])).item())
    k5_ms, _ = _timed(k5, args.steps, args.warmup)
    lines = {}
    for interp in ("nearest", "bilinear"):
        k6_ms, _ = _timed(lambda: kernels.rectify_var(ij, src, interp, float("nan"),
                                                      flags=flags),
                          args.steps, args.warmup)
        lines[interp] = k6_ms

    def separate(interp):   # K4 -> device tiling -> K5 -> K6, no host round trip
        t = R._device_tiles(sgm, tgm, xy)
        ij_ = kernels.rectify_ij(xy[0], xy[1], t, ntx, tgm.height, tgm.width, tgm.x_res,
                                 dst_y_scale, 1e-3, flags=flags)
        return kernels.rectify_var(ij_, src, interp, float("nan"), flags=flags)

    def pipeline(interp):   # rectify_dataset's single-variable path: K6 inside K5b
        t = R._device_tiles(sgm, tgm, xy)
        return kernels.rectify_ij_var(xy[0], xy[1], t, tgm.height, tgm.width, tgm.x_res,
                                      dst_y_scale, 1e-3, src, interp, float("nan"),
                                      keep_ij=False, flags=flags)[1]

    # the device tiling reproduces the host tiling byte for byte
    t_dev, offs = R._device_tiles(sgm, tgm, xy)
    assert np.array_equal(t_dev.cpu().numpy(), tiles.view(np.uint8).ravel()), "device tiles"
    assert torch.equal(torch.nan_to_num(pipeline("nearest"), 12345.0),
                       torch.nan_to_num(kernels.rectify_var(ij, src, "nearest", float("nan")),
                                        12345.0)), "device-tiled pipeline"
    for interp in ("nearest", "bilinear"):
        assert torch.equal(torch.nan_to_num(pipeline(interp), 12345.0),
                           torch.nan_to_num(separate(interp), 12345.0)), "fused K5+K6"


    npx = tgm.width * tgm.height
    S = w * h
    torch.cuda.synchronize()
    issue = issue_pmc()   # the claim is VALU-issue bound, the resolve waits on memory
    for interp in ("nearest", "bilinear") if div == 1.0 else ("nearest",):
        # 20 steps after 5 warm-up passes (5 after 1 let the shader clock's
        # ramp into the timed steps: 0.97 vs 0.90 ms for the same kernels)
        ms, wall = _timed(lambda: pipeline(interp), args.steps, max(5, args.warmup))
        sep_ms, _ = _timed(lambda: separate(interp), args.steps, max(5, args.warmup))
        cores = len(os.sched_getaffinity(0))
        # CPU baseline on the config itself: the C restatement of the numba
        # kernels (K4 bboxes + K5 + K6, tiles on a thread pool of all cores)
        # over the whole 4000x4800 swath -> the whole target grid, best of 3
        best = float("inf")
        for _ in range(3):
            t0 = time.perf_counter()
            ij_c, _ = rectify_ref.compute_target_source_ij(lon, lat, (tw, th), (512, 512),
                                                           geo["xy_bbox"], geo["xy_res"], False,
                                                           threads=cores)
            rectify_ref.compute_var_image(ij_c, var, np.nan, interp, (512, 512), threads=cores)
            best = min(best, time.perf_counter() - t0)
            del ij_c
        cpu_v, dt = npx / best / 1e6, best
        kt = kernel_times(interp, res_div=div)
        kern = ("fused pipeline: " + ", ".join(f"{k} {v:.1f} us" for k, v in kt.items()) +
                f" (sum {sum(kt.values()) / 1e3:.3f} ms)") if kt else "fused pipeline"
        _line(4 if div == 1.0 else "4f",
              f"rectify {interp}: 4000x4800 jittered swath (f64 lon/lat, f32 var) -> "
                 f"{tgm.width}x{tgm.height} EPSG:4326 res {res:.6g}, 512^2 tiles "
                 "(K4 bbox + device tiling + K5 with K6 fused, end to end, coordinates "
                 "resident in HBM)",
              npx, ms, wall, 16 * S + 4 * S + 4 * npx,
              kern,
              dict(value=round(cpu_v, 2), unit="Mpixels/s", cores=cores, kind="port",
                   sample=f"the whole config: 4000x4800 swath -> {tgm.width}x{tgm.height}, "
                          f"C restatement of the numba kernels (bboxes, ij, var image; tiles "
                          f"on a {cores}-thread pool), best of 3 passes: {dt:.2f} s"),
              {"covered_px": covered, "kernels_us": kt,
               "unfused": {"k5_claim_resolve_ms": round(k5_ms, 4),
                           "k6_ms": round(lines[interp], 4), "pipeline_ms": round(sep_ms, 4)},
               "issue": issue})
    flags.raise_if_set("config 4" if div == 1.0 else "config 4f")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="1,2,3,4")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    args = ap.parse_args()
    for c in args.configs.split(","):
        {"1": config1, "2": config2, "2u": config2u, "3": config3, "3f": config3f,
         "4": config4, "4f": lambda a: config4(a, 2.0)}[c.strip()](args)


if __name__ == "__main__":
    main()

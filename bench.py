"""Benchmark: reproject bilinear EPSG:4326 -> EPSG:3857, 40960x40960 float32,
2048x2048 target tiles (BASELINE.json metric, configs[4]).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (driver, N > 1)

`python bench.py --gpus N` with N > 1 outside torchrun starts the N ranks
itself: the untouched parent (no GPU call made) runs `python -m
torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1
--master-port <free> bench.py <same arguments>` as a child and exits with its
status (launch_ranks); it refuses N above the visible GPU count.

One "step" = one pass of the hot path (xrs_reproject: the K1 gather, one
launch; its work items resolve their own axis entries) over the rank's share of ONE synthetic 40960^2 raster resident in
HBM.  Multi-GPU (configs[4]: one raster sharded over the GPUs):
the target rows are split at row granularity (``sharding.band_shard``), each
rank holds only the source rows its band reads and writes its own target
rows — independent partitions, no data-path collective, "scaling": "strong".
``--shard slices`` instead gives rank r its own whole raster (weak scaling).

`value` = target pixels of the whole job / max-over-ranks wall time.
Before the warm-up steps each rank measures the device-copy rate of its
source band (benchlib: a streaming float4 copy, the fastest shape measured on
MI355X, profiles/r03_region_copy.jsonl): `roofline.copy_GBs` /
`frac_of_copy`.  Those ~0.1 s of copies also bring the shader
clock from its idle level to the loaded one: the chip's DVFS needs ~30 ms of
load to ramp from ~1.6 to ~2.38 GHz and K1 follows the clock
(profiles/r03_ramp_probe.jsonl, r03_ramp_pmc_clock.csv); `clock_GHz` gives
the clock measured just before and just after the timed steps.
`roofline.achieved` = algorithmic bytes of all ranks (output + distinct
source pixels read, x4 B) / max-over-ranks kernel time (HIP events on the
launch stream); `peak` = N x 8 TB/s.  `traffic` = FETCH_SIZE + WRITE_SIZE per
launch from two rocprofv3 --pmc child passes of this workload before the
bench touches the GPU (N = 1): the L2's memory-side requests counted by size,
with three launches of known bytes beside it (scripts/pmc_traffic.py).
Rank 0 prints ONE JSON line.
"""

from __future__ import annotations

import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
METRIC = "Mpixels/s reproject bilinear 40960² f32; achieved HBM GB/s vs peak"

# config 5 geometry: source EPSG:4326 pixel centres, target EPSG:3857
SRC_X0, SRC_Y0 = -20.0, 70.96
TGT_MIN = (-2226000.0, 3504000.0)
GEN_ROWS = 1024          # the synthetic raster is generated in seeded 1024-row chunks


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
            for f in (np.floor, np.ceil):
                g = base + f(idx).astype(np.int64)
                g = g[(g >= 0) & (g < n)]
                mask[g] = True
    return int(rows.sum()) * int(cols.sum())


def synthetic_rows(j0: int, j1: int, width: int, device, seed: int = 20250905):
    """Rows [j0, j1) of the synthetic f32 raster: uniform [0, 1), generated in
    seeded GEN_ROWS-row chunks so that every rank's band is a slice of the
    SAME global raster."""
    import torch

    out = torch.empty((1, j1 - j0, width), device=device, dtype=torch.float32)
    gen = torch.Generator(device=device)
    for k in range(j0 // GEN_ROWS, (max(j1, j0 + 1) - 1) // GEN_ROWS + 1):
        c0, c1 = k * GEN_ROWS, (k + 1) * GEN_ROWS
        gen.manual_seed(seed + k)
        chunk = torch.rand((1, GEN_ROWS, width), generator=gen, device=device,
                           dtype=torch.float32)
        a, b = max(c0, j0), min(c1, j1)
        if b > a:
            out[:, a - j0:b - j0] = chunk[:, a - c0:b - c0]
    return out


def cpu_baseline(plan, tgm, seconds: float = 12.0, sweep=(1, 32, 128), sweep_seconds=3.0):
    """Oracle (numpy restatement of reproject.py:268-335 + the per-tile window
    copy of 499-530 + the per-pixel transform of 472-496) on host threads:
    one task per 2048^2 target tile on a thread pool (the dask threaded
    scheduler's shape), tiles taken from every tile row.  All cores of the
    affinity mask for `seconds`, plus a thread-count sweep (`sweep_seconds`
    each): numpy releases the GIL only inside its inner loops, so like
    dask's threaded scheduler the port scales far below linearly; `value` is
    the best rate of the sweep."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import gridmapping_ref as gref
    from oracle import reproject_ref

    cores = len(os.sched_getaffinity(0))
    ntx, nty = plan.num_tiles
    tiles = [(j, (7 * j + i) % ntx) for i in range(ntx) for j in range(nty)]
    xc, yc = tgm.x_coords.values, tgm.y_coords.values
    wy, wx = plan.win_height, plan.win_width
    pool_src = np.random.default_rng(1).random((1, wy, wx), dtype=np.float32)
    strips = 4   # rows of a tile in 4 strips (same per-pixel arithmetic, 1/4 the temporaries)

    def run_tile(jt):
        j, i = jt
        t = j * ntx + i
        r0, r1 = j * plan.tile_height, min(plan.dst_height, (j + 1) * plan.tile_height)
        c0, c1 = i * plan.tile_width, min(plan.dst_width, (i + 1) * plan.tile_width)
        win = np.array(pool_src)             # the reference's reorganised window copy
        x_coord = np.full((wx, 1, 1), plan.tile_x0[t], np.float32)
        y_coord = np.full((wy, 1, 1), plan.tile_y0[t], np.float32)
        step = -(-(r1 - r0) // strips)
        for s0 in range(r0, r1, step):
            xx, yy = np.meshgrid(xc[c0:c1], yc[s0:min(r1, s0 + step)])
            sxx, syy = gref.webmerc_inverse(xx, yy)
            reproject_ref.reproject_block(sxx, syy, win, x_coord, y_coord, plan.x_res,
                                          plan.y_res, "bilinear")
        return (r1 - r0) * (c1 - c0)

    def rate(threads, secs):
        px, k = 0, 0
        t0 = time.perf_counter()
        with ThreadPoolExecutor(max_workers=threads) as ex:
            while time.perf_counter() - t0 < secs:
                batch = [tiles[(k + q) % len(tiles)] for q in range(threads)]
                k += threads
                px += sum(ex.map(run_tile, batch))
        dt = time.perf_counter() - t0
        return px / dt / 1e6, px, dt

    rates = {}
    for n in sweep:
        if n < cores:
            rates[n] = round(rate(n, sweep_seconds)[0], 2)
    all_rate, px, dt = rate(cores, seconds)
    rates[cores] = round(all_rate, 2)
    best = max(rates, key=rates.get)
    return dict(value=rates[best], unit="Mpixels/s", cores=best, kind="port",
                threads_sweep={str(k): v for k, v in sorted(rates.items())},
                per_thread_Mpx_s=round(rates[best] / best, 3),
                sample=f"numpy oracle of the reference's per-tile path (bilinear, f32 in, f64 out "
                       f"as the reference, incl. per-pixel coordinate transform and window copy), "
                       f"one task per {plan.tile_width}x{plan.tile_height} target tile on a "
                       f"thread pool, tiles taken across all tile rows; {cores} threads "
                       f"(all cores of the affinity mask) for {dt:.1f} s "
                       f"({px // (plan.tile_width * plan.tile_height)} tiles) plus "
                       f"{sweep_seconds:.0f} s per point of the thread sweep; value = the best "
                       f"point ({best} threads): GIL-bound like dask's threaded scheduler "
                       f"(numpy releases the GIL only inside its inner loops)")


def measure_traffic(size: int, tile: int, out_dtype: str, timeout: int = 170):
    """HBM bytes per launch from two rocprofv3 --pmc child passes of
    scripts/pmc_traffic.py on this workload (separate passes within the TCC
    block's 4 counter slots, MI355X_MICROARCH.md §rocprofv3 PMC): read bytes
    from the size-resolved L2 -> memory requests (32 / 64 / 128 B), write
    bytes from the 32 / 64 B write requests — no correction factor; a float4
    copy, a 4-byte-lane copy and an identity K1 launch of known bytes run in
    the same process and are reported beside it (measured / known).  Must run
    before this process touches the GPU (the children are separate
    processes).  Returns the reduced dict or None (no rocprofv3, or a pass
    failed)."""
    prof = shutil.which("rocprofv3")
    if prof is None:
        return None
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import pmc_traffic

    d = tempfile.mkdtemp(prefix="xrs_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    env = dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp"))
    for name, counters in pmc_traffic.PASSES.items():
        cmd = ["timeout", "-s", "KILL", str(timeout), prof, "--pmc", *counters, "--kernel-trace",
               "--output-format", "csv", "-d", os.path.join(d, name), "-o", name, "--",
               sys.executable, os.path.join(ROOT, "scripts", "pmc_traffic.py"), "--size",
               str(size), "--tile", str(tile), "--out-dtype", out_dtype]
        r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                           text=True)
        if r.returncode != 0:
            print(f"bench: rocprofv3 pass {name} failed (rc {r.returncode}):\n"
                  f"{r.stdout[-2000:]}", file=sys.stderr)
            return None
    try:
        return pmc_traffic.reduce(d, size, out_dtype)
    except Exception as e:   # a missing / malformed counter file: report null traffic
        print(f"bench: PMC reduce failed: {e}", file=sys.stderr)
        return None
    finally:
        shutil.rmtree(d, ignore_errors=True)


def load_benchlib():
    """benchlib/libxrs_bench.so (measurement support; built by build())."""
    import ctypes

    lib = ctypes.CDLL(os.path.join(ROOT, "benchlib", "libxrs_bench.so"))
    lib.xrs_bench_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                   ctypes.c_int, ctypes.c_void_p]
    lib.xrs_bench_clock_probe.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_void_p]
    return lib


COPY_VARIANT = 2   # one float4 per thread, one 4 KiB block per 256 threads: 6.2 TB/s


def device_copy_rate(lib, src, stream, warm: int = 40, timed: int = 20) -> float:
    """GB/s (read + write) of a streaming copy of `src` into a scratch buffer of
    the same size, on `stream`; the first `warm` copies are untimed."""
    import torch

    nbytes = src.numel() * src.element_size()
    if nbytes == 0:
        return 0.0
    scratch = torch.empty_like(src)
    sh = int(stream.cuda_stream)

    def copy():
        if lib.xrs_bench_copy(src.data_ptr(), scratch.data_ptr(), nbytes, COPY_VARIANT, sh) != 0:
            raise RuntimeError("benchlib copy failed")

    for _ in range(warm):
        copy()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(timed):
        copy()
    e1.record(stream)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / timed
    del scratch
    return 2 * nbytes / (ms / 1e3) / 1e9


def clock_probe_launch(lib, stream, blocks: int = 1024, spin: int = 3000):
    """Queue the shader-clock probe on `stream` (no host wait: the GPU stays
    busy); clock_probe_read() takes its result later."""
    import torch

    buf = torch.zeros((blocks, 2), dtype=torch.int64, device=stream.device)
    if lib.xrs_bench_clock_probe(buf.data_ptr(), blocks, spin, int(stream.cuda_stream)) != 0:
        raise RuntimeError("benchlib clock probe failed")
    return buf


def clock_probe_read(buf) -> float:
    """Median over blocks of d(s_memtime) / d(s_memrealtime) x 100 MHz."""
    d = buf.cpu().numpy()
    return round(float(np.median(d[:, 0] / np.maximum(d[:, 1], 1))) * 0.1, 3)


def shader_clock_ghz(lib, stream, blocks: int = 1024, spin: int = 3000) -> float:
    buf = clock_probe_launch(lib, stream, blocks, spin)
    stream.synchronize()
    return clock_probe_read(buf)


KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"


def visible_gpu_count(nodes_dir: str = KFD_NODES, env=None) -> int:
    """GPUs this process may use, counted WITHOUT touching HIP: the KFD
    topology nodes with SIMDs (CPU nodes report simd_count 0), narrowed by
    ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES as the
    runtime narrows them.  torch.cuda.device_count() is not used: on ROCm it
    falls back to hipGetDeviceCount when amdsmi does not answer, which starts
    the HIP runtime in this parent.  Raises OSError when the topology cannot
    be read (the launcher then refuses instead of guessing)."""
    env = os.environ if env is None else env
    gpus = 0
    for name in sorted(os.listdir(nodes_dir)):
        props = os.path.join(nodes_dir, name, "properties")
        if not os.path.isfile(props):
            continue
        with open(props) as f:
            for line in f:
                key, _, val = line.partition(" ")
                if key == "simd_count" and int(val) > 0:
                    gpus += 1
                    break
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        sel = env.get(var)
        if sel is None:
            continue
        ids = [t for t in sel.split(",") if t.strip() != ""]
        # the runtime stops at the first invalid ordinal ("-1" hides every GPU)
        valid = 0
        for t in ids:
            t = t.strip()
            if t.lstrip("-").isdigit() and 0 <= int(t) < gpus:
                valid += 1
            elif not t.lstrip("-").isdigit():      # a UUID: counted as one device
                valid += 1
            else:
                break
        gpus = valid
    return gpus


def launch_ranks(n: int, argv: list[str]) -> int:
    """`--gpus N` (N > 1) from a plain `python bench.py` call: start the N
    ranks, one process per GPU, under torch.distributed.run as a CHILD of this
    parent, and return the child's exit status.  Rank 0 prints the JSON line;
    stdout and stderr pass through.  The parent makes no HIP call (never an
    exec after HIP init, and no runtime state to inherit): with the nccl
    (RCCL) backend it counts the visible GPUs from the KFD topology
    (visible_gpu_count) and refuses, status 2, when there are fewer than N or
    the topology cannot be read."""
    import socket

    backend = os.environ.get("XRS_BENCH_BACKEND", "nccl")
    cmd_tail = [os.path.abspath(__file__), *argv]
    if backend == "nccl" and "--dry-run" not in argv:
        try:
            have = visible_gpu_count()
        except OSError as e:
            have, why = 0, f" (KFD topology unreadable: {e})"
        else:
            why = ""
        if have < n:
            print(f"bench: --gpus {n} needs {n} visible GPUs, found {have}{why}; on an {n}-GPU "
                  f"node run: python -m torch.distributed.run --nnodes=1 --nproc-per-node {n} "
                  f"--master-addr 127.0.0.1 --master-port 29500 bench.py {' '.join(argv)}",
                  file=sys.stderr)
            return 2
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr", "127.0.0.1", f"--master-port={port}",
           *cmd_tail]
    env = dict(os.environ, XRS_BENCH_LAUNCHED="1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    # untimed warm-up: the kernel trace of a fresh process shows the first
    # ~15 launches 3-20 % slower than the steady state (profiles/r02_bench_kernel_trace.csv)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--size", type=int, default=40960)
    ap.add_argument("--tile", type=int, default=2048)
    ap.add_argument("--out-dtype", choices=["f32", "f64"], default="f32")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-traffic", action="store_true",
                    help="skip the two rocprofv3 --pmc passes (traffic: null)")
    ap.add_argument("--no-f64", action="store_true",
                    help="skip the secondary measurement with float64 output")
    ap.add_argument("--no-graph", action="store_true",
                    help="launch every step eagerly instead of replaying a captured hipGraph")
    ap.add_argument("--shard", choices=["bands", "slices"], default="bands",
                    help="bands: the ranks split the target rows of ONE raster, each holding "
                         "only the source rows its band reads (strong; configs[4]); "
                         "slices: rank r reprojects its own raster (weak)")
    ap.add_argument("--balance", choices=["rows", "bytes", "cost"], default="cost",
                    help="row-band split: equal target rows, equal algorithmic bytes, or "
                         "equal predicted K1 cost (sharding.band_splits; the default, weights "
                         "fitted in-sample to one-GPU rehearsals: max/mean 1.015 at 8 ranks in "
                         "profiles/r02_band_rehearsal.jsonl; N > 1 lines report every model's "
                         "prediction next to the measured per-rank times)")
    ap.add_argument("--dry-run", action="store_true",
                    help="host-only rehearsal of the rank logic (launcher, band split, gloo "
                         "collectives, JSON line with the ranks block): no GPU, no kernel; "
                         "value and roofline are null")
    args = ap.parse_args()

    from xcube_resampling_amd.sharding import band_shard, env_rank, max_over_ranks

    rank, world, local_rank = env_rank()
    if args.gpus > 1 and "RANK" not in os.environ:
        # a plain `python bench.py --gpus N`: start the N ranks (child processes)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    dry = args.dry_run
    if dry:
        args.no_traffic = args.no_cpu_baseline = args.no_f64 = args.no_graph = True
    # PMC passes first: child processes, before this process initialises HIP
    traffic = None
    if world == 1 and not args.no_traffic:
        traffic = measure_traffic(args.size, args.tile, args.out_dtype)
    src_gm, tgm, plan, lon, lat = workload(args.size, args.tile)   # host only
    # the CPU baseline runs before HIP is initialised (host threads only)
    cpu = None
    if world == 1 and rank == 0 and not args.no_cpu_baseline:
        cpu = cpu_baseline(plan, tgm, args.cpu_seconds)

    import torch
    import torch.distributed as dist

    from xcube_resampling_amd import kernels

    # one GPU per rank; XRS_BENCH_BACKEND=gloo with more ranks than GPUs is only
    # a rehearsal of the multi-rank logic on a smaller box (ranks share GPUs)
    backend = "gloo" if dry else os.environ.get("XRS_BENCH_BACKEND", "nccl")
    if dry:
        dev_index, device = None, torch.device("cpu")
    else:
        dev_index = local_rank % torch.cuda.device_count() if backend == "gloo" else local_rank
        torch.cuda.set_device(dev_index)
        device = torch.device("cuda", dev_index)
    # XRS_BENCH_DIST=1: the process group and every collective of the N > 1
    # path also at N = 1 (a one-GPU rehearsal of the RCCL calls the driver's
    # multi-GPU runs make)
    use_dist = world > 1 or os.environ.get("XRS_BENCH_DIST") == "1"
    if use_dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)

    out_np = np.float32 if args.out_dtype == "f32" else np.float64
    if args.shard == "bands":
        shard = band_shard(plan, world, rank, args.balance, np.dtype(out_np).itemsize)
        rows, (j0, j1) = shard.rows, shard.src_rows
        src = synthetic_rows(j0, j1, args.size, device)
    else:
        rows, (j0, j1) = (0, plan.dst_height), (0, plan.src_height)
        src = synthetic_rows(0, plan.src_height, args.size, device, seed=20250905 + 1000 * rank)
    flags = None if dry else kernels.ErrorFlags(device)
    benchlib = None if dry else load_benchlib()
    # the stream the kernels run on
    stream = None if dry else torch.cuda.current_stream(device)
    copy_rates = []

    def sync():
        if not dry:
            torch.cuda.synchronize()

    def make_step(out, dtype):
        def step():
            if dry:
                out.zero_()          # host stand-in: the rehearsal times no kernel
            elif rows[1] > rows[0]:
                kernels.reproject(src, plan, "bilinear", float("nan"), out_dtype=dtype, out=out,
                                  rows=rows, src_row0=j0, flags=flags, check=False)
        return step

    def barrier():
        if use_dist:
            if backend == "nccl":
                dist.barrier(device_ids=[dev_index])
            else:
                dist.barrier()

    def timed(step, steps, warmup):
        """(max-over-ranks wall ms/step, this rank's event ms/step)."""
        run = step
        if not args.no_graph:
            step()                       # tables uploaded, workspace allocated
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                step()
            run = g.replay
        barrier()   # the first collective sets the communicator up: not between warm-up and timing
        if not dry:
            ev0 = torch.cuda.Event(enable_timing=True)
            ev1 = torch.cuda.Event(enable_timing=True)
            # the same-run device-copy rate, measured back to back with the warm-up
            # steps: its ~0.1 s of streaming also takes the shader clock to its
            # loaded level (DVFS: ~30 ms of load from idle), as W steps alone may not
            copy_rates.append(device_copy_rate(benchlib, src, stream))
        else:
            copy_rates.append(0.0)
        for _ in range(warmup):
            run()
        # nothing on the host between the warm-up and the timed steps but the
        # barrier and the synchronize: an idle gap of a few ms lets the clock
        # drop, and the first timed launches ramp up again (kernel trace of
        # r03's first version: 17.6 ms of host work here, then 3.0 -> 2.5 ms)
        probe0 = None if dry else clock_probe_launch(benchlib, stream)   # read after timing
        sync()      # every rank's own queue drained ...
        barrier()   # ... before the ranks start together
        sync()
        t0 = time.perf_counter()
        if not dry:
            ev0.record(stream)
        for _ in range(steps):
            run()
        if not dry:
            ev1.record(stream)
        sync()
        t_own = time.perf_counter() - t0
        barrier()
        t1 = time.perf_counter()
        wall = max_over_ranks(t1 - t0, device) / steps * 1e3
        if dry:
            return wall, t_own / steps * 1e3, (None, None)
        clk0 = clock_probe_read(probe0)
        clk1 = shader_clock_ghz(benchlib, stream)
        return wall, ev0.elapsed_time(ev1) / steps, (clk0, clk1)

    out = torch.empty((1, rows[1] - rows[0], args.size), device=device,
                      dtype=torch.float32 if out_np == np.float32 else torch.float64)
    ms_per_step, kernel_ms, clocks = timed(make_step(out, out_np), args.steps, args.warmup)
    if flags is not None:
        flags.raise_if_set("bench reproject")

    copy_gbs = copy_rates[0]
    s_read = source_pixels_read(plan, rows) if rows[1] > rows[0] else 0
    out_bytes = (rows[1] - rows[0]) * args.size * np.dtype(out_np).itemsize
    my_bytes = out_bytes + 4 * s_read
    secondary = None
    if world == 1 and not args.no_f64 and out_np == np.float32:
        del out
        out64 = torch.empty((1, rows[1] - rows[0], args.size), device=device, dtype=torch.float64)
        ms64, k64, _ = timed(make_step(out64, np.float64), max(5, args.steps // 2),
                             max(2, args.warmup // 2))
        flags.raise_if_set("bench reproject f64")
        b64 = 8 * (rows[1] - rows[0]) * args.size + 4 * s_read
        secondary = {"out_dtype": "f64 (the reference's bilinear dtype)",
                     "ms_per_step": round(ms64, 4),
                     "value": round(args.size * args.size / (ms64 / 1e3) / 1e6, 1),
                     "kernel_ms": round(k64, 4), "algorithmic_bytes": int(b64),
                     "achieved_GBs": round(b64 / (k64 / 1e3) / 1e9, 1),
                     "frac": round(b64 / (k64 / 1e3) / 1e9 / HBM_PEAK_GBS, 4)}
        del out64

    rank_ms = None
    if use_dist:   # whole-job bytes, slowest rank's kernel time, every rank's time
        t = torch.tensor([float(my_bytes)], dtype=torch.float64,
                         device=device if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        alg_bytes = float(t.item())
        max_kernel_ms = max_over_ranks(kernel_ms, device)
        cdev = device if backend == "nccl" else "cpu"
        parts = [torch.zeros(2, dtype=torch.float64, device=cdev) for _ in range(world)]
        dist.all_gather(parts, torch.tensor([kernel_ms, copy_gbs], dtype=torch.float64,
                                            device=cdev))
        rank_ms = [round(float(p[0]), 4) for p in parts]
        copy_all = float(sum(float(p[1]) for p in parts))
    else:
        alg_bytes, max_kernel_ms = float(my_bytes), kernel_ms
        copy_all = copy_gbs
    n_rasters = world if args.shard == "slices" else 1
    value = n_rasters * args.size * args.size / (ms_per_step / 1e3) / 1e6
    peak = HBM_PEAK_GBS * world
    achieved = alg_bytes / (max_kernel_ms / 1e3) / 1e9

    if rank == 0:
        res = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "Mpixels/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.shard == "bands" else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded uniform [0,1) f32 raster, generated on device)",
            "config": {
                "workload": f"reproject EPSG:4326->EPSG:3857 bilinear {args.size}x{args.size} "
                            f"f32 source, {args.tile}x{args.tile} target tiles (configs[4]); "
                            + (f"one raster, target rows split over {world} GPU(s) "
                               f"(row granularity, balance={args.balance}), each holding only "
                               f"the source rows its band reads"
                               if args.shard == "bands" else
                               f"{world} raster(s) of an (N,{args.size},{args.size}) cube, "
                               f"1 per GPU"),
                "source_dtype": "f32",
                "out_dtype": args.out_dtype,
                "interp": "bilinear",
                "tiles": plan.num_tiles[0] * plan.num_tiles[1],
                "window": [plan.win_height, plan.win_width],
                "parallelism": f"{args.shard}{world}",
                "launch": "eager" if args.no_graph else "hipGraph replay (1 captured step)",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": peak,
                "unit": "GB/s",
                "frac": round(achieved / peak, 4),
                "traffic": traffic["hbm_bytes_per_launch"] if traffic else None,
                "kernel": "gather_separable_kernel<float,float,1>",
                "kernel_ms": round(max_kernel_ms, 4),
                "algorithmic_bytes": int(alg_bytes),
                "copy_GBs": round(copy_all, 1),
                "frac_of_copy": round(achieved / copy_all, 4) if copy_all > 0 else None,
                "copy": "same-run streaming float4 copy of each rank's source band (read + "
                        "write bytes / time; benchlib xrs_bench_copy), summed over ranks",
                "scope": "whole job: bytes of all ranks / slowest rank's kernel time; "
                         "peak = n_gpus x 8 TB/s",
            },
        }
        if dry:   # nothing above was measured on a GPU
            res["value"] = None
            res["roofline"] = None
            res["dry_run"] = ("host-only rehearsal (--dry-run): launcher, band split, gloo "
                              "collectives and the ranks block; no GPU, no kernel")
        res["clock_GHz"] = {"before_timed": clocks[0], "after_timed": clocks[1],
                            "note": "rank 0 shader clock (s_memtime / s_memrealtime probe) "
                                    "right outside the timed region"}
        if rank_ms is not None:
            from xcube_resampling_amd.sharding import band_splits, split_predictions
            res["ranks"] = {"kernel_ms": rank_ms,
                            "max_over_mean": round(max(rank_ms) / (sum(rank_ms) / world), 4)}
            if args.shard == "bands":
                cuts = band_splits(plan, world, args.balance, np.dtype(out_np).itemsize)
                res["ranks"]["cuts"] = cuts
                res["ranks"]["predicted"] = split_predictions(plan, cuts,
                                                              np.dtype(out_np).itemsize)
        if traffic:
            res["roofline"]["traffic_detail"] = {
                k: traffic[k] for k in ("read_bytes", "write_bytes", "calibration")}
            res["roofline"]["traffic_detail"]["read_over_algorithmic"] = round(
                traffic["read_bytes"] / (4 * s_read), 4) if s_read else None
            res["roofline"]["traffic_detail"]["requests"] = {
                k: traffic["launches"]["bench"][k] for k in ("rdreq", "rdreq_dram", "wrreq",
                                                             "wrreq_64B")}
        if secondary:
            res["f64_out"] = secondary
        if cpu is not None:
            res["cpu_baseline"] = cpu
        print(json.dumps(res), flush=True)
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

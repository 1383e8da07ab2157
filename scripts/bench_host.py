"""Host-resident end to end: a numpy (1, S, S) f32 raster in
host RAM -> numpy result, bilinear EPSG:4326 -> EPSG:3857 (config 5 geometry).

    python scripts/bench_host.py [--size 40960] [--reps 2]

  whole     : torch copy of the whole raster to HBM, one K1 launch, copy back
              (what a direct port of the reference's numpy path does)
  streamed  : streaming.reproject_host — through page-locked staging buffers, target
              bands of 2048 rows, H2D / K1 / D2H on three streams

One JSON line per mode: wall seconds (best of reps) and Mpixels/s, i.e. the
PCIe-inclusive rate.  bench.py's `value` stays the HBM-resident rate.
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=40960)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--band-rows", type=int, default=0)
    args = ap.parse_args()
    import torch

    import bench
    from xcube_resampling_amd import kernels, streaming

    dev = torch.device("cuda", 0)
    _, _, plan, _, _ = bench.workload(args.size, 2048)
    t0 = time.perf_counter()
    src = np.empty((1, args.size, args.size), np.float32)
    rng = np.random.default_rng(20250905)
    step = max(1, (64 << 20) // (4 * args.size))
    for r in range(0, args.size, step):
        src[0, r:r + step] = rng.random((min(step, args.size - r), args.size), dtype=np.float32)
    print(f"# source filled in {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    npx = args.size * args.size
    gb = src.nbytes / 1e9

    def line(mode, secs, extra):
        print(json.dumps({"mode": mode, "metric": "Mpixels/s reproject bilinear host->host "
                          "(PCIe-inclusive)", "value": round(npx / secs / 1e6, 1),
                          "unit": "Mpixels/s", "seconds": round(secs, 4),
                          "size": args.size, "source_GB": round(gb, 3), **extra}), flush=True)

    # whole-raster copies (pageable memory)
    whole = None
    times = []
    for _ in range(args.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d = torch.from_numpy(src).to(dev)
        o = kernels.reproject(d, plan, "bilinear", np.nan, out_dtype=np.float32)
        whole = o.cpu().numpy()
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
        del d, o
        print(f"# whole {times[-1]:.3f} s", file=sys.stderr, flush=True)
    torch.cuda.empty_cache()
    line("whole", min(times), {"reps": times})

    out = np.empty_like(whole)
    times = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        streaming.reproject_host(src, plan, "bilinear", np.nan, out_dtype=np.float32,
                                 band_rows=args.band_rows or None, out=out)
        times.append(time.perf_counter() - t0)
        print(f"# streamed {times[-1]:.3f} s", file=sys.stderr, flush=True)
    same = bool(np.array_equal(out, whole, equal_nan=True))
    line("streamed", min(times), {"reps": times, "bit_identical_to_whole": same,
                                  "band_rows": args.band_rows or plan.tile_height})
    if not same:
        sys.exit("streamed result differs from the whole-raster result")


if __name__ == "__main__":
    main()

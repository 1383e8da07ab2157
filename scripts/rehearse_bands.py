"""One-GPU rehearsal of bench.py's multi-GPU partition (config 5).

The N ranks of `bench.py --gpus N` are independent (no data-path collective):
rank r runs K1 on its row band of the one 40960^2 raster, holding only the
source rows that band reads.  Timing every rank's band here, one after the
other on one MI355X, gives each rank's kernel time — the slowest one sets the
job's time — without an 8-GPU node.

    python scripts/rehearse_bands.py [--worlds 1 2 4 8] [--balance rows bytes]

Prints one JSON line per (world, balance): per-rank ms (HIP events around
--reps back-to-back launches, median of 5), max/mean, and the strong-scaling projection
value = 40960^2 / max rank time.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=40960)
    ap.add_argument("--worlds", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--balance", nargs="+", default=["rows", "cost"])
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--warm", type=int, default=20)
    a = ap.parse_args()

    import torch

    import bench
    from xcube_resampling_amd import kernels
    from xcube_resampling_amd.sharding import band_shard

    dev = torch.device("cuda", 0)
    _, _, plan, _, _ = bench.workload(a.size, 2048)
    full = bench.synthetic_rows(0, a.size, a.size, dev)
    flags = kernels.ErrorFlags(dev)
    for world in a.worlds:
        for balance in a.balance:
            ranks = []
            for r in range(world):
                sh = band_shard(plan, world, r, balance)
                j0, j1 = sh.src_rows
                src = full[:, j0:j1].contiguous()     # the rank's own source band
                out = torch.empty((1, sh.row1 - sh.row0, a.size), device=dev,
                                  dtype=torch.float32)
                run = lambda: kernels.reproject(src, plan, "bilinear", np.nan,  # noqa: E731
                                                out_dtype=np.float32, out=out, rows=sh.rows,
                                                src_row0=j0, flags=flags, check=False)
                for _ in range(a.warm):   # steady state before timing (the first
                    run()                   # launches on a fresh band run slower)
                torch.cuda.synchronize()
                # back-to-back launches between two events (the host's launch
                # latency is hidden, as in the bench's graph replay); median of 5
                times = []
                for _ in range(5):
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(a.reps):
                        run()
                    e1.record()
                    e1.synchronize()
                    times.append(e0.elapsed_time(e1) / a.reps)
                flags.raise_if_set("rehearsal")
                ranks.append(dict(rank=r, rows=[sh.row0, sh.row1], src_rows=[j0, j1],
                                  ms=round(float(np.median(times)), 4)))
                del src, out
                torch.cuda.empty_cache()
            ms = np.array([x["ms"] for x in ranks])
            print(json.dumps(dict(world=world, balance=balance, max_ms=round(ms.max(), 4),
                                  mean_ms=round(ms.mean(), 4),
                                  max_over_mean=round(ms.max() / ms.mean(), 4),
                                  projected_mpx_s=round(a.size ** 2 / (ms.max() / 1e3) / 1e6, 1),
                                  ranks=ranks)), flush=True)


if __name__ == "__main__":
    main()

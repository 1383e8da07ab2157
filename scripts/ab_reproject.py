"""A/B timing of K1 gather variants in ONE process (interleaved rounds).

    python scripts/ab_reproject.py [--size 40960] [--rounds 5] [--variants 0,1]

Variants are selected through XRS_REPROJECT_VARIANT (read by libxrs at each
call); all variants produce bit-identical output (checked here).
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=40960)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--variants", default="0,1")
    ap.add_argument("--interp", default="bilinear")
    args = ap.parse_args()
    import torch

    import bench
    from xcube_resampling_amd import kernels

    # an arm is "V", "V@B" or "V@B/R": kernel variant V, B blocks per CU, R rows per item
    variants = args.variants.split(",")
    _, _, plan, _, _ = bench.workload(args.size, 2048)
    dev = torch.device("cuda", 0)
    src = torch.rand((1, args.size, args.size), device=dev, dtype=torch.float32)
    outs = {v: torch.empty((1, args.size, args.size), device=dev, dtype=torch.float32)
            for v in variants}
    out_dt = np.float32 if args.interp == "bilinear" else None
    times = {v: [] for v in variants}
    rng = np.random.default_rng(0)
    for rnd in range(args.rounds):
        for v in rng.permutation(variants):  # shuffled: no fixed first-in-round bias
            v = str(v)
            var, _, rest = v.partition("@")
            bpc, _, band = rest.partition("/")
            os.environ["XRS_REPROJECT_VARIANT"] = var
            for name, val in (("XRS_REPROJECT_BLOCKS_PER_CU", bpc), ("XRS_REPROJECT_BAND", band)):
                if val and val != "0":
                    os.environ[name] = val
                else:
                    os.environ.pop(name, None)
            kernels.reproject(src, plan, args.interp, np.nan, out_dtype=out_dt, out=outs[v])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                kernels.reproject(src, plan, args.interp, np.nan, out_dtype=out_dt, out=outs[v],
                                  check=False)
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / args.iters)
    ref = outs[variants[0]]
    for v in variants[1:]:
        same = torch.equal(torch.nan_to_num(outs[v], 12345.0), torch.nan_to_num(ref, 12345.0))
        print(f"variant {v} bit-identical to {variants[0]}: {same}")
    npx = args.size * args.size
    for v in variants:
        t = np.array(times[v])
        print(f"variant {v}: median {np.median(t):.3f} ms  min {t.min():.3f} ms  "
              f"({npx / np.median(t) / 1e3:.0f} Mpx/s)")


if __name__ == "__main__":
    main()

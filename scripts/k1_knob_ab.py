"""K1 work-shape arms through the test-only knobs (band height, grid cap in
blocks per CU = a persistent grid walking the band-major list in lockstep),
timed interleaved on one box against the product shape;
every arm's raster is compared with the product's bit for bit.
    python scripts/k1_knob_ab.py [--passes 2] [--steps 20] [--arms NAME,...]"""
from __future__ import annotations

import argparse

import numpy as np
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# (name, band rows, blocks per CU (0 = one-shot items))
ARMS = [("base", 0, 0), ("b8p4", 8, 4), ("b8p2", 8, 2), ("b16p4", 16, 4), ("b32p4", 32, 4),
        ("b4p4", 4, 4), ("b8", 8, 0), ("b16", 16, 0), ("b24", 24, 0), ("b40", 40, 0),
        ("b48", 48, 0), ("b64", 64, 0)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--passes", type=int, default=2)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--arms", default="")
    args = ap.parse_args()
    arms = [a for a in ARMS if not args.arms or a[0] in args.arms.split(",")]
    import bench
    import torch

    from xcube_resampling_amd import kernels
    from xcube_resampling_amd._native import testing_knob

    _, _, plan, _, _ = bench.workload(40960, 2048)
    dev = torch.device("cuda", 0)
    src = bench.synthetic_rows(0, plan.src_height, 40960, dev)
    flags = kernels.ErrorFlags(dev)
    out = torch.empty((1, 40960, 40960), device=dev, dtype=torch.float32)
    ref = None
    lib = bench.load_benchlib()
    stream = torch.cuda.current_stream(dev)
    for p in range(args.passes):
        for name, band, bpc in arms:
            with testing_knob("reproject_band", band), \
                    testing_knob("reproject_blocks_per_cu", bpc):
                step = lambda: kernels.reproject(src, plan, "bilinear", float("nan"),  # noqa
                                                 out_dtype=np.float32, out=out, flags=flags,
                                                 check=False)
                bench.device_copy_rate(lib, src[:, :4096], stream, warm=40, timed=2)
                for _ in range(10):
                    step()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(args.steps):
                    step()
                e1.record(stream)
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / args.steps
            if ref is None:
                ref = out.clone()
                same = True
            else:
                same = bool(torch.equal(out.view(torch.int32), ref.view(torch.int32)))
            flags.raise_if_set("k1 arm")
            print(json.dumps({"arm": name, "band": band or 32, "blocks_per_cu": bpc,
                              "pass": p + 1, "ms_per_launch": round(ms, 4),
                              "bit_equal_to_base": same}), flush=True)


if __name__ == "__main__":
    main()

"""K1 (config 5 bench workload) timed after a padding allocation of --pad-mb
MB, so the source and target rasters land at other device addresses; run per
library (XRS_LIBRARY) to see whether a work deal's rate depends on where the
rasters sit (the channel hash) rather than on the deal alone.
    XRS_LIBRARY=... python scripts/k1_pad_ab.py --pad-mb 0 [--steps 30]"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pad-mb", type=int, default=0)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--tag", default="")
    ap.add_argument("--out-dtype", choices=["f32", "f64"], default="f32")
    ap.add_argument("--no-xgen", action="store_true",
                    help="read the src_x table (coord_mode 0; libraries before round 5 "
                         "know no coord_mode 2)")
    args = ap.parse_args()
    import bench
    import torch

    from xcube_resampling_amd import kernels

    dev = torch.device("cuda", 0)
    pad = torch.empty(max(args.pad_mb, 1) << 20, dtype=torch.uint8, device=dev)
    _, _, plan, _, _ = bench.workload(40960, 2048)
    if args.no_xgen:
        import dataclasses
        plan = dataclasses.replace(plan, x_gen=None, _device_cache={})
    src = bench.synthetic_rows(0, plan.src_height, 40960, dev)
    flags = kernels.ErrorFlags(dev)
    f64 = args.out_dtype == "f64"
    out = torch.empty((1, 40960, 40960), device=dev, dtype=torch.float64 if f64 else torch.float32)
    stream = torch.cuda.current_stream(dev)

    def step():
        kernels.reproject(src, plan, "bilinear", float("nan"),
                          out_dtype=np.float64 if f64 else np.float32, out=out,
                          flags=flags, check=False)

    for _ in range(15):
        step()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(args.steps):
        step()
    e1.record(stream)
    torch.cuda.synchronize()
    # a checksum of the raster's bit patterns (arms must agree bit for bit)
    csum = 0
    for r in range(0, 40960, 4096):
        v = out[0, r:r + 4096].view(torch.int64 if f64 else torch.int32)
        csum = (csum + int((v & 0xFFFFFFF).sum(dtype=torch.int64)) * (r // 4096 + 1)) % (1 << 61) \
            if f64 else (csum + int(v.sum(dtype=torch.int64)) * (r // 4096 + 1)) % (1 << 61)
    flags.raise_if_set("k1 arm")
    print(json.dumps({"tag": args.tag, "out": args.out_dtype, "pad_mb": args.pad_mb, "src_ptr": hex(src.data_ptr()),
                      "out_ptr": hex(out.data_ptr()), "ms_per_launch": round(e0.elapsed_time(e1) / args.steps, 4),
                      "checksum": csum}))
    del pad


if __name__ == "__main__":
    main()

"""Config-2u kernels run a few times each (xrs_transform + K1c on the 2-D
tables, and the fused gather xrs_reproject_proj): the workload of
scripts/bench_configs.py config2u, for rocprofv3 counter passes.
    python scripts/time_2u.py [--reps N]"""
from __future__ import annotations

import argparse
import dataclasses
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--time", action="store_true",
                    help="time both paths (events) and print one JSON line")
    ap.add_argument("--tag", default="")
    args = ap.parse_args()
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
    src = torch.rand((1, size, size), device="cuda", dtype=torch.float32)
    out = torch.empty((1, size, size), device="cuda", dtype=torch.float64)
    flags = kernels.ErrorFlags(src.device)
    fplan = dataclasses.replace(plan, fuse_transform=True, _device_cache={})
    if args.time:
        import json

        def run(p, k):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for _ in range(3):
                kernels.reproject(src, p, "bilinear", float("nan"), out=out, flags=flags, check=False)
            e0.record()
            for _ in range(k):
                kernels.reproject(src, p, "bilinear", float("nan"), out=out, flags=flags, check=False)
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / k
        tables_ms = run(plan, 10)
        fused_ms = run(fplan, 10)
        flags.raise_if_set("time_2u")
        v = out.view(torch.int64)
        csum = int((v & 0xFFFFFFF).sum()) % (1 << 61)
        print(json.dumps({"tag": args.tag, "tables_ms": round(tables_ms, 4),
                          "fused_ms": round(fused_ms, 4), "checksum_fused": csum}), flush=True)
        return
    for _ in range(args.reps):
        plan._device_cache.clear()
        kernels.reproject(src, plan, "bilinear", float("nan"), out=out, flags=flags, check=False)
        kernels.reproject(src, fplan, "bilinear", float("nan"), out=out, flags=flags,
                          check=False)
    torch.cuda.synchronize()
    flags.raise_if_set("time_2u")
    print("time_2u done", flush=True)


if __name__ == "__main__":
    main()

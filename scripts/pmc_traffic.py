"""Workloads for PMC traffic measurement (run under rocprofv3 --pmc).

    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d D -o fetch -- \
        python scripts/pmc_traffic.py
    rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d D -o write -- \
        python scripts/pmc_traffic.py
    python scripts/pmc_traffic.py --reduce D   -> profiles/traffic_r01.json

Two launches per run, separated by a device sync:
  1. CALIBRATION: nearest reprojection EPSG:4326 -> EPSG:4326 onto the source's
     own grid (ix, iy exact integers): every source element is read exactly
     once with the same dword-gather access pattern as the bench kernel, so
     bytes read = 4*S and written = 4*N are known exactly.  gfx950's
     FETCH_SIZE under-reports wide streams (MI355X_MICROARCH.md §HBM); the
     calibration gives the correction factor for THIS access pattern.
  2. BENCH: the bench.py kernel (bilinear 4326 -> 3857, 40960^2, f32 out).
"""
import csv
import glob
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SIZE = 40960


def run():
    import torch

    import bench
    import xcube_resampling_amd as xrs
    from xcube_resampling_amd import kernels

    dev = torch.device("cuda", 0)
    src_gm, tgm, plan, lon, lat = bench.workload(SIZE, 2048)
    src = torch.rand((1, SIZE, SIZE), device=dev, dtype=torch.float32)
    # calibration: identity geometry (source grid as the target grid)
    ident = xrs.GridMapping.regular((SIZE, SIZE), (src_gm.x_min, src_gm.y_min), src_gm.xy_res,
                                    "EPSG:4326", tile_size=2048)
    cplan = xrs.plan_reproject(src_gm, ident, xrs.Transformer.from_crs(ident.crs, src_gm.crs,
                                                                       always_xy=True))
    out = torch.empty_like(src)
    kernels.reproject(src, cplan, "nearest", np.nan, out=out)
    torch.cuda.synchronize()
    assert torch.equal(out, src), "identity reprojection must copy the source"
    kernels.reproject(src, plan, "bilinear", np.nan, out_dtype=np.float32, out=out)
    torch.cuda.synchronize()


def reduce(d):
    rows = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "gather" not in r["Kernel_Name"]:
                continue
            rows.setdefault(r["Counter_Name"], []).append(
                (int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    out = {}
    for name, vals in rows.items():
        vals.sort()
        # per dispatch: sum over instances (counter rows per XCD/SE are summed)
        agg = {}
        for did, v in vals:
            agg[did] = agg.get(did, 0.0) + v
        out[name] = [agg[k] for k in sorted(agg)]
    fetch, write = out["FETCH_SIZE"], out["WRITE_SIZE"]
    S = N = SIZE * SIZE
    k_fetch = 4 * S / (fetch[0] * 1024)   # FETCH_SIZE is in KiB
    k_write = 4 * N / (write[0] * 1024)
    bench_read = fetch[1] * 1024 * k_fetch
    bench_write = write[1] * 1024 * k_write
    res = {
        "size": SIZE, "out_dtype": "f32", "kernel": "gather_separable_mlp_kernel<float,float,1,8,true,2> (non-temporal stores, one work item per block)",
        "hbm_bytes_per_launch": int(bench_read + bench_write),
        "read_bytes": int(bench_read), "write_bytes": int(bench_write),
        "raw_fetch_kib": fetch, "raw_write_kib": write,
        "calibration": {"fetch_factor": k_fetch, "write_factor": k_write,
                        "method": "identity nearest reprojection: 4*S bytes read, 4*N written"},
    }
    path = os.path.join(ROOT, "profiles", "traffic_r01.json")
    with open(path, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--reduce":
        reduce(sys.argv[2])
    else:
        run()

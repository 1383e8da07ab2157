"""Workload for PMC traffic measurement of K1 (run under rocprofv3 --pmc).

bench.py runs it twice as a child process before it touches the GPU itself:

    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d D/fetch -o fetch -- \
        python scripts/pmc_traffic.py --size 40960 --tile 2048 --out-dtype f32
    rocprofv3 --pmc WRITE_SIZE ... (same)

and reduces the two counter files with ``reduce(D, size, out_dtype)``.
By hand: ``python scripts/pmc_traffic.py --reduce D [--size S --out-dtype f32]``
writes profiles/traffic_<round>.json.

Two launches per run, separated by a device sync:
  1. CALIBRATION: nearest reprojection EPSG:4326 -> EPSG:4326 onto the source's
     own grid (ix, iy exact integers): every source element is read exactly
     once with the same dword-gather access pattern as the bench kernel, so
     bytes read = 4*S and written = 4*N are known exactly.  gfx950's
     FETCH_SIZE under-reports wide streams (MI355X_MICROARCH.md §HBM); the
     calibration gives the correction factor for THIS access pattern.
  2. BENCH: the bench.py kernel (bilinear 4326 -> 3857, f32 or f64 out).
"""
import argparse
import csv
import glob
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
KERNEL = "gather_separable_kernel"


def run(size: int, tile: int, out_dtype: str):
    import torch

    import bench
    import xcube_resampling_amd as xrs
    from xcube_resampling_amd import kernels

    dev = torch.device("cuda", 0)
    src_gm, tgm, plan, lon, lat = bench.workload(size, tile)
    src = bench.synthetic_rows(0, size, size, dev)
    # calibration: identity geometry (source grid as the target grid)
    ident = xrs.GridMapping.regular((size, size), (src_gm.x_min, src_gm.y_min), src_gm.xy_res,
                                    "EPSG:4326", tile_size=tile)
    cplan = xrs.plan_reproject(src_gm, ident, xrs.Transformer.from_crs(ident.crs, src_gm.crs,
                                                                       always_xy=True))
    out = torch.empty_like(src)
    kernels.reproject(src, cplan, "nearest", np.nan, out=out)
    torch.cuda.synchronize()
    assert torch.equal(out, src), "identity reprojection must copy the source"
    dt = np.float32 if out_dtype == "f32" else np.float64
    if dt == np.float64:
        del out
        out = torch.empty((1, size, size), device=dev, dtype=torch.float64)
    kernels.reproject(src, plan, "bilinear", np.nan, out_dtype=dt, out=out)
    torch.cuda.synchronize()


def _counters(d):
    rows = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if KERNEL not in r["Kernel_Name"]:
                    continue
                rows.setdefault(r["Counter_Name"], []).append(
                    (int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    out = {}
    for name, vals in rows.items():
        agg = {}   # per dispatch: sum over the instances (XCDs / SEs)
        for did, v in vals:
            agg[did] = agg.get(did, 0.0) + v
        out[name] = [agg[k] for k in sorted(agg)]
    return out


def reduce(d, size: int = 40960, out_dtype: str = "f32", write: bool = True, name=None):
    c = _counters(d)
    fetch, wr = c["FETCH_SIZE"], c["WRITE_SIZE"]
    if len(fetch) != 2 or len(wr) != 2:
        raise ValueError(f"expected 2 gather dispatches per pass, got {len(fetch)} / {len(wr)}")
    s = n = size * size
    k_fetch = 4 * s / (fetch[0] * 1024)   # FETCH_SIZE / WRITE_SIZE are in KiB
    k_write = 4 * n / (wr[0] * 1024)
    bench_read = fetch[1] * 1024 * k_fetch
    bench_write = wr[1] * 1024 * k_write
    res = {
        "size": size, "out_dtype": out_dtype, "kernel": KERNEL,
        "hbm_bytes_per_launch": int(bench_read + bench_write),
        "read_bytes": int(bench_read), "write_bytes": int(bench_write),
        "raw_fetch_kib": fetch, "raw_write_kib": wr,
        "calibration": {"fetch_factor": round(k_fetch, 4), "write_factor": round(k_write, 4),
                        "method": "identity nearest reprojection in the same process: "
                                  "4*S bytes read, 4*N written"},
    }
    if write:
        path = os.path.join(ROOT, "profiles", name or "traffic.json")
        with open(path, "w") as f:
            json.dump(res, f, indent=1)
    return res


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=40960)
    ap.add_argument("--tile", type=int, default=2048)
    ap.add_argument("--out-dtype", choices=["f32", "f64"], default="f32")
    ap.add_argument("--reduce", metavar="DIR")
    ap.add_argument("--name", default=None, help="output file name under profiles/")
    a = ap.parse_args()
    if a.reduce:
        print(json.dumps(reduce(a.reduce, a.size, a.out_dtype, name=a.name), indent=1))
    else:
        run(a.size, a.tile, a.out_dtype)

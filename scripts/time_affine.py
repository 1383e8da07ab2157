"""Config-1 K2 timed in isolation for A/B arms: the single 1024^2 chunk and
the dask shape (64 chunks of one geometry stacked on dim 0, one launch), K
launches replayed from a captured graph after a warm-up.  Slice 5 of the
stacked launch is checked against the single-chunk launch of the same slice
first (arms must agree bit for bit).  Prints one JSON line.
    XRS_LIBRARY=probe/ARM/pkg/lib/libxrs.so python scripts/time_affine.py --tag ARM"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="")
    ap.add_argument("--chunks", type=int, default=64)
    args = ap.parse_args()
    import torch

    import bench_configs as bc
    import xcube_resampling_amd as xrs
    import xcube_resampling_amd.affine as A
    from xcube_resampling_amd import kernels

    n = 1024
    res = 2.0 ** -10
    lon = 10 + (np.arange(n) + 0.5) * res
    lat = 51 - (np.arange(n) + 0.5) * res
    sgm = xrs.GridMapping.from_coords(xrs.DataArray(lon, "lon", name="lon"),
                                      xrs.DataArray(lat, "lat", name="lat"), "EPSG:4326")
    tgm = xrs.GridMapping.regular((n, n), (10.1, 50.05), 0.0009, "EPSG:4326")
    m = tgm.ij_transform_to(sgm)
    oc = (1, tgm.tile_height, tgm.tile_width)
    nb = args.chunks
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    srcb = torch.rand((nb, n, n), generator=g, device="cuda", dtype=torch.float32)
    planb = A.plan_affine(tuple(srcb.shape), np.dtype(np.float32), m, (nb, n, n), oc, 0,
                          "first", False, np.nan)
    plan1 = A.plan_affine((1, n, n), np.dtype(np.float32), m, (1, n, n), oc, 0, "first", False,
                          np.nan)
    outb = kernels.affine(srcb, planb)
    one = kernels.affine(srcb[5:6].contiguous(), plan1)
    assert torch.equal(outb[5:6].view(torch.int32), one.view(torch.int32)), "slice 5"
    src1 = srcb[:1].contiguous()
    out1 = torch.empty_like(one)
    ms1, _ = bc._timed(lambda: kernels.affine(src1, plan1, out1), 50, 5, graph=True)
    msb, _ = bc._timed(lambda: kernels.affine(srcb, planb, outb), 20, 5, graph=True)
    print(json.dumps({"tag": args.tag, "single_ms": round(ms1, 5), "batched_ms": round(msb, 5),
                      "batched_chunks": nb,
                      "batched_GBs_8B_per_px": round(nb * 8 * n * n / (msb / 1e3) / 1e9, 1)}),
          flush=True)


if __name__ == "__main__":
    main()

"""Config-4 rectify kernels timed in isolation (K4 + device tiles, K5 claim +
resolve, K6 nearest): the workload of scripts/bench_configs.py config4, for
rocprofv3 --kernel-trace --stats runs of kernel variants.  --fused samples the
variable inside K5's resolve pass (xrs_rectify_ij_var, no ij image written).
--res-div F divides the target resolution by F (F^2 more target pixels per
source quad: larger claim windows).
    python scripts/time_rectify.py [--reps N] [--fused] [--interp nearest|bilinear|triangular]
                                   [--res-div F] [--compact 0|1|2]"""

from __future__ import annotations

import argparse
import os
import sys

import numpy as np

# XRS_PYROOT: the package from another tree (an A/B arm of the host code)
sys.path.insert(0, os.environ.get("XRS_PYROOT") or
                os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--fused", action="store_true")
    ap.add_argument("--interp", default="nearest", choices=["nearest", "bilinear", "triangular"])
    ap.add_argument("--res-div", type=float, default=1.0)
    ap.add_argument("--compact", type=int, default=0,
                    help="claim walk: 0 per tile (product), 1 compacted, 2 per lane")
    args = ap.parse_args()
    import torch

    import xcube_resampling_amd as xrs
    from xcube_resampling_amd import _native, kernels
    from xcube_resampling_amd import rectify as R

    w, h = 4000, 4800
    rng = np.random.default_rng(20250905)
    i = np.arange(w)[None, :].astype(np.float64)
    j = np.arange(h)[:, None].astype(np.float64)
    lat = 60 - 0.0027 * j - 0.0004 * i + 1e-9 * (i - 2000) ** 2 \
        + rng.normal(0, 0.05 * 0.0027, (h, w))
    lon = 5 + 0.0045 * i + 0.0009 * j + rng.normal(0, 0.05 * 0.0045, (h, w))
    var = rng.random((1, h, w), dtype=np.float32)
    res = 0.0027 / args.res_div
    x0, y0 = float(np.floor(lon.min() / res) * res), float(np.floor(lat.min() / res) * res)
    tw, th = int(np.ceil((lon.max() - x0) / res)), int(np.ceil((lat.max() - y0) / res))
    tgm = xrs.GridMapping.regular((tw, th), (x0, y0), res, "EPSG:4326", tile_size=512)
    sgm = xrs.GridMapping.from_coords(xrs.DataArray(lon, ("y", "x"), name="lon"),
                                      xrs.DataArray(lat, ("y", "x"), name="lat"), "EPSG:4326")
    xy = (torch.from_numpy(lon).cuda(), torch.from_numpy(lat).cuda())
    src = torch.from_numpy(var).cuda()
    ntx = len(range(0, tgm.width, tgm.tile_width))
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    flags = kernels.ErrorFlags(src.device)   # checked once, after the timed loop
    if args.compact:
        _native.testing_knob("rectify_compact", args.compact).__enter__()
    for r in range(args.reps + 2):
        if r == 2:
            torch.cuda.synchronize()
            ev[0].record()
        t = R._device_tiles(sgm, tgm, xy)
        if args.fused:
            _, out = kernels.rectify_ij_var(xy[0], xy[1], t, tgm.height, tgm.width, tgm.x_res,
                                            -tgm.y_res, 1e-3, src, args.interp, float("nan"),
                                            keep_ij=False, flags=flags)
        else:
            ij = kernels.rectify_ij(xy[0], xy[1], t, ntx, tgm.height, tgm.width, tgm.x_res,
                                    -tgm.y_res, 1e-3, flags=flags)
            out = kernels.rectify_var(ij, src, args.interp, float("nan"), flags=flags)
    ev[1].record()
    torch.cuda.synchronize()
    flags.raise_if_set("time_rectify")
    bits = out.contiguous().view(torch.int32).to(torch.int64)   # output checksum (bits)
    csum = int((bits * (torch.arange(bits.numel(), device=bits.device).view(bits.shape) % 1009 + 1)).sum())
    print(f"{os.environ.get('XRS_LIBRARY', 'libxrs.so')}: {ev[0].elapsed_time(ev[1]) / args.reps:.3f} "
          f"ms per K4+K5+K6{' (fused)' if args.fused else ''} res/{args.res_div:g} walk {args.compact}, covered {int(torch.isfinite(out).sum())} px, "
          f"checksum {csum}", flush=True)


if __name__ == "__main__":
    main()

"""Host-resident end to end for the affine and rectify paths:
numpy in -> numpy out, as the reference's APIs take and return them
(affine.py:227-228, rectify.py:297-298).

    python scripts/bench_host_paths.py [--reps 3]

  affine  : 2 x 16384^2 f32, bilinear resample at a half-pixel offset
            (scale 1, offset 0.5) to 16384^2, 2048^2 output chunks
  rectify : config 4 (4000x4800 swath, 8266x5392 target) K6 bilinear over an
            f32 variable of 8 slices, the ij image resident in HBM
  whole     : page-locked DMA of the whole array, one launch, DMA back
  streamed  : streaming.affine_host / rectify_host — bands on three streams

One JSON line per (path, mode): best wall seconds of `reps` and the
PCIe-inclusive Mpixels/s; the streamed result is checked bit-identical.
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


def _line(path, mode, npx, secs, extra):
    print(json.dumps({"path": path, "mode": mode,
                      "metric": "target Mpixels/s host->host (PCIe-inclusive)",
                      "value": round(npx / secs / 1e6, 1), "unit": "Mpixels/s",
                      "seconds": round(secs, 4), **extra}), flush=True)


def _best(fn, reps):
    import torch

    times, out = [], None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    return min(times), times, out


def affine(reps):
    import xcube_resampling_amd.affine as A
    from xcube_resampling_amd import kernels, streaming

    n, nt = 16384, 2
    rng = np.random.default_rng(1)
    src = rng.random((nt, n, n), dtype=np.float32)
    m = ((1.0, 0.0, 0.5), (0.0, 1.0, 0.5))
    plan = A.plan_affine(src.shape, src.dtype, m, (nt, n, n), (1, 2048, 2048), 1, "first", False,
                         np.nan)

    def whole():
        d = streaming.host_to_device(src, "cuda:0")
        return streaming.device_to_host(kernels.affine(d, plan))

    tw, tws, ref = _best(whole, reps)
    out = np.empty_like(ref)
    ts, tss, got = _best(lambda: streaming.affine_host(src, plan, out=out), reps)
    npx = nt * n * n
    extra = {"workload": f"affine bilinear {nt}x{n}x{n} f32 (offset 0.5 px), 2048^2 chunks",
             "source_GB": round(src.nbytes / 1e9, 3)}
    _line("affine", "whole", npx, tw, dict(extra, reps=tws))
    _line("affine", "streamed", npx, ts, dict(extra, reps=tss,
                                              bit_identical=bool(np.array_equal(got, ref,
                                                                                equal_nan=True))))


def rectify(reps):
    import torch

    import xcube_resampling_amd as xrs
    from xcube_resampling_amd import kernels, streaming
    from xcube_resampling_amd import rectify as R

    w, h, nt = 4000, 4800, 8
    rng = np.random.default_rng(20250905)
    i = np.arange(w)[None, :].astype(np.float64)
    j = np.arange(h)[:, None].astype(np.float64)
    lat = 60 - 0.0027 * j - 0.0004 * i + 1e-9 * (i - 2000) ** 2 \
        + rng.normal(0, 0.05 * 0.0027, (h, w))
    lon = 5 + 0.0045 * i + 0.0009 * j + rng.normal(0, 0.05 * 0.0045, (h, w))
    res = 0.0027
    x0, y0 = float(np.floor(lon.min() / res) * res), float(np.floor(lat.min() / res) * res)
    tw_, th_ = int(np.ceil((lon.max() - x0) / res)), int(np.ceil((lat.max() - y0) / res))
    tgm = xrs.GridMapping.regular((tw_, th_), (x0, y0), res, "EPSG:4326", tile_size=512)
    sgm = xrs.GridMapping.from_coords(xrs.DataArray(lon, ("y", "x"), name="lon"),
                                      xrs.DataArray(lat, ("y", "x"), name="lat"), "EPSG:4326")
    ij = R._compute_target_source_ij(sgm, tgm, 1e-3)
    var = rng.random((nt, h, w), dtype=np.float32)

    def whole():
        d = streaming.host_to_device(var, "cuda:0")
        return streaming.device_to_host(kernels.rectify_var(ij, d, "bilinear", np.nan))

    tw, tws, ref = _best(whole, reps)
    out = np.empty_like(ref)
    ts, tss, got = _best(lambda: streaming.rectify_host(var, ij, "bilinear", np.nan, out=out),
                         reps)
    torch.cuda.synchronize()
    npx = nt * tgm.width * tgm.height
    extra = {"workload": f"rectify K6 bilinear, {nt} f32 slices of the config-4 swath "
                         f"({w}x{h} -> {tgm.width}x{tgm.height}), ij resident",
             "source_GB": round(var.nbytes / 1e9, 3), "result_GB": round(ref.nbytes / 1e9, 3)}
    _line("rectify", "whole", npx, tw, dict(extra, reps=tws))
    _line("rectify", "streamed", npx, ts, dict(extra, reps=tss,
                                               bit_identical=bool(np.array_equal(got, ref,
                                                                                 equal_nan=True))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--paths", default="affine,rectify")
    args = ap.parse_args()
    for p in args.paths.split(","):
        {"affine": affine, "rectify": rectify}[p](args.reps)


if __name__ == "__main__":
    main()

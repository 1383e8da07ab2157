"""Diagnose the fresh-process launch ramp of K1.

Runs the bench workload (config 5, 40960^2 bilinear f32 -> f32) in several
launch patterns and, right after every launch, the clock probe of
benchlib/xrs_bench.hip (shader clock = d s_memtime / d s_memrealtime x 100 MHz,
median over blocks).  If K1's duration follows the shader clock, the ramp is
the chip's clock management; if the clock is flat while K1 ramps, it is on the
memory side (or the product's).  One JSON line per pattern.

    python scripts/ramp_probe.py [--size 40960]   (needs benchlib/libxrs_bench.so:
                                                   make -C benchlib)
"""

from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=40960)
    ap.add_argument("--spin", type=int, default=3000)
    args = ap.parse_args()

    import torch

    import bench
    from xcube_resampling_amd import kernels

    probe = ctypes.CDLL(os.path.join(ROOT, "benchlib", "libxrs_bench.so"))
    probe.xrs_bench_clock_probe.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_void_p]
    probe.xrs_bench_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                     ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    _, _, plan, _, _ = bench.workload(args.size, 2048)
    src = bench.synthetic_rows(0, plan.src_height, args.size, dev)
    out = torch.empty((1, plan.dst_height, plan.dst_width), device=dev, dtype=torch.float32)
    scratch = torch.empty_like(src)
    flags = kernels.ErrorFlags(dev)
    stream = torch.cuda.current_stream(dev)
    sh = int(stream.cuda_stream)
    nblk = 2048
    stamps = torch.zeros((4096, nblk, 2), dtype=torch.int64, device=dev)
    slot = [0]

    def k1():
        kernels.reproject(src, plan, "bilinear", float("nan"), out_dtype=np.float32, out=out,
                          flags=flags, check=False)

    def copy():
        probe.xrs_bench_copy(src.data_ptr(), scratch.data_ptr(), src.numel() * 4, 0, sh)

    def clock():
        s = slot[0]
        slot[0] += 1
        probe.xrs_bench_clock_probe(stamps[s].data_ptr(), nblk, args.spin, sh)
        return s

    def run(name, fn, n, gap_s=0.0, idle_s=1.0, heater=0):
        torch.cuda.synchronize()
        time.sleep(idle_s)
        for _ in range(heater):
            copy()
        recs = []
        for _ in range(n):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            fn()
            e1.record(stream)
            s = clock()
            recs.append((e0, e1, s))
            if gap_s:
                torch.cuda.synchronize()
                time.sleep(gap_s)
        torch.cuda.synchronize()
        st = stamps.cpu().numpy()
        ms = [round(a.elapsed_time(b), 4) for a, b, _ in recs]
        ghz = []
        for _, _, s in recs:
            d = st[s]
            ghz.append(round(float(np.median(d[:, 0] / np.maximum(d[:, 1], 1))) * 0.1, 3))
        print(json.dumps({"pattern": name, "n": n, "gap_s": gap_s, "idle_s": idle_s,
                          "heater_copies": heater, "ms": ms, "clock_GHz": ghz}), flush=True)

    k1()
    torch.cuda.synchronize()
    flags.raise_if_set("ramp probe")
    run("k1_back_to_back_cold", k1, 60)
    run("k1_back_to_back_after_300ms_idle", k1, 30, idle_s=0.3)
    run("k1_isolated_20ms_gaps", k1, 20, gap_s=0.02)
    run("copy4_back_to_back_cold", copy, 60)
    run("k1_after_copy_heater_100", k1, 30, heater=100)
    run("k1_back_to_back_cold_again", k1, 60)


if __name__ == "__main__":
    main()

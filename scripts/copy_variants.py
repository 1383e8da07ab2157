"""Device-copy rate of the benchlib stream_copy variants and torch's D2D copy
(hipMemcpyAsync blit) on a buffer the size of config 5's source (6.7 GB), after
a warm-up that brings the shader clock to its loaded level (profiles/
r03_ramp_probe.jsonl).  Rate = (bytes read + bytes written) / time.  One JSON
line per variant and pass."""

from __future__ import annotations

import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import argparse

    import torch

    ap = argparse.ArgumentParser()
    ap.add_argument("--sections", default="copy,region,persistent")
    sections = ap.parse_args().sections.split(",")

    lib = ctypes.CDLL(os.path.join(ROOT, "benchlib", "libxrs_bench.so"))
    lib.xrs_bench_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                   ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    nbytes = 40960 * 40960 * 4
    a = torch.rand(nbytes // 4, device=dev)
    b = torch.empty_like(a)
    st = torch.cuda.current_stream(dev)
    sh = int(st.cuda_stream)
    names = {0: "stride nt", 1: "stride", 2: "u1", 3: "u4", 4: "u4 nt", 5: "u8", 6: "u8 nt",
             -1: "torch copy_ (hipMemcpy D2D)"}

    def run(v):
        if v < 0:
            b.copy_(a)
        elif lib.xrs_bench_copy(a.data_ptr(), b.data_ptr(), nbytes, v, sh) != 0:
            raise RuntimeError(f"variant {v} failed")

    for _ in range(100):
        run(2)
    for p in ((1, 2) if "copy" in sections else ()):
        for v in (0, 1, 2, 3, 4, 5, 6, -1):
            for _ in range(3):
                run(v)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            n = 20
            for _ in range(n):
                run(v)
            e1.record(st)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / n
            print(json.dumps({"variant": v, "name": names[v], "pass": p, "ms": round(ms, 4),
                              "GBs": round(2 * nbytes / ms / 1e6, 1)}), flush=True)
    assert torch.equal(a, b)

    # region copies in K1's work shape: (segw, band, rows in flight/2, nt, order)
    lib.xrs_bench_region_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p] + \
        [ctypes.c_int64] * 4 + [ctypes.c_int] * 3 + [ctypes.c_void_p]
    cases = [(512, 32, 4, 1, 1), (512, 32, 4, 0, 1), (512, 32, 4, 1, 0), (512, 8, 4, 1, 0),
             (1024, 8, 4, 1, 0), (2048, 8, 4, 1, 0), (2048, 32, 4, 1, 0), (4096, 4, 4, 1, 0),
             (40960, 1, 4, 1, 0), (1024, 1, 1, 0, 0), (1024, 1, 1, 1, 0), (2048, 2, 1, 1, 0)]
    if "bands" in sections:   # band shapes with K1's XCD deal (order 1)
        cases = [(512, 32, 4, 1, 1), (512, 64, 4, 1, 1), (512, 16, 4, 1, 1), (1024, 32, 4, 1, 1),
                 (1024, 16, 4, 1, 1), (1024, 8, 4, 1, 1), (2048, 16, 4, 1, 1), (2048, 8, 4, 1, 1),
                 (256, 64, 4, 1, 1), (256, 32, 4, 1, 1), (1024, 32, 8, 1, 1), (1024, 8, 2, 1, 1),
                 (1024, 8, 4, 1, 0), (1024, 16, 4, 1, 0), (512, 16, 2, 1, 1)]
    for p in ((1, 2) if "region" in sections or "bands" in sections else ()):
        for c in cases:
            def rc():
                if lib.xrs_bench_region_copy(a.data_ptr(), b.data_ptr(), 40960, 40960, *c, sh):
                    raise RuntimeError(f"region copy {c} failed")
            for _ in range(3):
                rc()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(20):
                rc()
            e1.record(st)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 20
            print(json.dumps({"region": dict(zip(("segw", "band", "rif", "nt", "order"), c)),
                              "pass": p, "ms": round(ms, 4),
                              "GBs": round(2 * nbytes / ms / 1e6, 1)}), flush=True)
    if "region" in sections or "bands" in sections:
        b.zero_()
        rc()
        torch.cuda.synchronize()
        assert torch.equal(a, b)

    # K1's shape with fewer blocks resident per CU (dynamic LDS as the limiter)
    lib.xrs_bench_region_copy_lds.argtypes = [ctypes.c_void_p, ctypes.c_void_p] + \
        [ctypes.c_int64] * 4 + [ctypes.c_int] * 4 + [ctypes.c_void_p]
    occ = [(c, bpc) for c in [(512, 32, 4, 1, 1), (1024, 8, 4, 1, 1), (1024, 32, 4, 1, 1)]
           for bpc in (1, 2, 3, 4, 6, 8)]
    for p in ((1, 2) if "occupancy" in sections else ()):
        for c, bpc in occ:
            lds = (160 * 1024) // bpc - 1024 if bpc < 8 else 0

            def oc():
                if lib.xrs_bench_region_copy_lds(a.data_ptr(), b.data_ptr(), 40960, 40960, *c,
                                                 lds, sh):
                    raise RuntimeError(f"region copy {c} failed")
            for _ in range(3):
                oc()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(20):
                oc()
            e1.record(st)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 20
            print(json.dumps({"occupancy": dict(zip(("segw", "band", "rif", "nt", "order"), c)),
                              "blocks_per_cu": bpc, "pass": p, "ms": round(ms, 4),
                              "GBs": round(2 * nbytes / ms / 1e6, 1)}), flush=True)

    # persistent row-walking copies: (float4 per thread per item, blocks, nt)
    lib.xrs_bench_persistent_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                              ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_int, ctypes.c_void_p]
    pcases = [(q, nb, nt) for q in (1, 2, 4) for nb in (1024, 2048, 4096, 8192) for nt in (0, 1)]
    for p in ((1,) if "persistent" in sections else ()):
        for c in pcases:
            def pc():
                if lib.xrs_bench_persistent_copy(a.data_ptr(), b.data_ptr(), 40960, 40960, *c, sh):
                    raise RuntimeError(f"persistent copy {c} failed")
            for _ in range(3):
                pc()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(20):
                pc()
            e1.record(st)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 20
            print(json.dumps({"persistent": dict(zip(("q", "blocks", "nt"), c)), "pass": p,
                              "ms": round(ms, 4), "GBs": round(2 * nbytes / ms / 1e6, 1)}),
                  flush=True)
        b.zero_()
        pc()
        torch.cuda.synchronize()
        assert torch.equal(a, b)


if __name__ == "__main__":
    main()

"""XCD-placement probe: does it matter which XCD moves which bytes?  Copies
a 6.7 GB buffer (config 5's source size) with benchlib xcd_copy for chunk
sizes 4 KB .. 64 KB and every rotation `shift` of the chunk -> XCD deal
(block b takes chunk (b/8)*8 + (b%8 + shift)%8).  One JSON line per case:
GB/s = (read + write bytes) / time, two interleaved passes."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    import torch

    lib = ctypes.CDLL(os.path.join(ROOT, "benchlib", "libxrs_bench.so"))
    lib.xrs_bench_xcd_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                       ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
    lib.xrs_bench_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                   ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    nbytes = 40960 * 40960 * 4
    a = torch.rand(nbytes // 4, device=dev)
    b = torch.empty_like(a)
    sh = int(torch.cuda.current_stream(dev).cuda_stream)
    for _ in range(100):
        lib.xrs_bench_copy(a.data_ptr(), b.data_ptr(), nbytes, 2, sh)
    chunks = [int(c) for c in (sys.argv[1].split(",") if len(sys.argv) > 1 else
                               ["4096", "8192", "16384", "65536"])]
    for p in (1, 2):
        for chunk in chunks:
            for shift in range(8):
                def run():
                    if lib.xrs_bench_xcd_copy(a.data_ptr(), b.data_ptr(), nbytes, chunk, shift, sh):
                        raise RuntimeError("xcd copy failed")
                for _ in range(3):
                    run()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    run()
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / 10
                print(json.dumps({"chunk": chunk, "shift": shift, "pass": p, "ms": round(ms, 4),
                                  "GBs": round(2 * nbytes / ms / 1e6, 1)}), flush=True)
    assert torch.equal(a, b)


if __name__ == "__main__":
    main()

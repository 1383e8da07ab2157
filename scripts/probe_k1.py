import sys, os, numpy as np, torch
sys.path.insert(0, os.getcwd())
import bench
from xcube_resampling_amd import kernels
size=40960
_, _, plan, _, _ = bench.workload(size, 2048)
src = torch.rand((1, size, size), device="cuda", dtype=torch.float32)
out = torch.empty_like(src)
def t(fn, it=5):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1)/it
for rnd in range(2):
    print("copy_", t(lambda: out.copy_(src)))
    print("bilinear", t(lambda: kernels.reproject(src, plan, "bilinear", np.nan, out_dtype=np.float32, out=out, check=False)))
    print("nearest", t(lambda: kernels.reproject(src, plan, "nearest", np.nan, out=out, check=False)))

"""Checksum of the bench workload's K1 raster (config 5, 40960^2 bilinear f32)
for the library XRS_LIBRARY names, so probe arms run in separate processes can
be compared with the product bit for bit.
    XRS_LIBRARY=... python scripts/k1_hash.py"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    import torch

    from xcube_resampling_amd import kernels

    _, _, plan, _, _ = bench.workload(40960, 2048)
    dev = torch.device("cuda", 0)
    src = bench.synthetic_rows(0, plan.src_height, 40960, dev)
    flags = kernels.ErrorFlags(dev)
    out = torch.empty((1, 40960, 40960), device=dev, dtype=torch.float32)
    kernels.reproject(src, plan, "bilinear", float("nan"), out_dtype=np.float32, out=out,
                      flags=flags, check=False)
    words = out.view(torch.int32).reshape(40960, 40960).to(torch.int64)
    # position-weighted sum of the raw words: any changed bit or moved pixel shows
    w = torch.arange(1, 40961, device=dev, dtype=torch.int64)
    h = int(((words * w).sum(dim=1) * w).sum().item())
    print(h)


if __name__ == "__main__":
    main()

"""Config-3 coarsen (16384^2 f32 -> 4096^2, 4x4 mean through the affine path)
timed in isolation for A/B arms of the K3i kernel: K launches replayed from a
captured graph after a warm-up; prints 'ms per launch'.  The corner block is
checked against the product's output first (arms must be bit-identical).
--frac shifts the target grid by 0.3 source pixels (a grid off the integral
layout: K3w since round 6, the generic K3 before); --generic forces the
generic K3 (test knob XRS_TESTING_AFFINE_GENERIC).
    XRS_LIBRARY=probe/ARM/pkg/lib/libxrs.so python scripts/time_coarsen.py [--frac]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main():
    import torch

    import bench_configs as bc
    import xcube_resampling_amd as xrs
    import xcube_resampling_amd.affine as A
    from xcube_resampling_amd import kernels

    n, k = 16384, 4
    res = 2.0 ** -10
    lon = (np.arange(n) + 0.5) * res
    lat = n * res - (np.arange(n) + 0.5) * res
    sgm = xrs.GridMapping.from_coords(xrs.DataArray(lon, "lon", name="lon"),
                                      xrs.DataArray(lat, "lat", name="lat"), "EPSG:4326")
    frac = "--frac" in sys.argv[1:]
    off = 0.3 * res if frac else 0.0
    if "--s35" in sys.argv[1:]:   # a 3.5x downscale: div 4, the div-x grid at scale 0.875
        frac = True
        tgm = xrs.GridMapping.regular((4681, 4681), (0.0, 0.0), res * 3.5, "EPSG:4326")
    else:
        tgm = xrs.GridMapping.regular((n // k, n // k), (off, off), res * k, "EPSG:4326")
    m = tgm.ij_transform_to(sgm)
    g = torch.Generator(device="cuda")
    g.manual_seed(20250905)
    src = torch.rand((1, n, n), generator=g, device="cuda", dtype=torch.float32)
    oc = (1, tgm.tile_height, tgm.tile_width)
    no = tgm.width
    plan = A.plan_affine(tuple(src.shape), np.dtype(np.float32), m, (1, no, no), oc, 1,
                         "mean", False, np.nan)
    knob = None
    if "--generic" in sys.argv[1:]:
        from xcube_resampling_amd._native import testing_knob
        knob = testing_knob("affine_generic", 1)
        knob.__enter__()
    out = kernels.affine(src, plan)
    ref = src[0].reshape(n // k, k, n // k, k).mean(dim=(1, 3))
    # interior pixels: the 4x4 mean (numpy pairwise order differs from torch's:
    # compare with a tolerance here; the GPU suite checks bit-exactness)
    if not frac:
        assert torch.allclose(out[0, :-1, :-1], ref[:-1, :-1], rtol=1e-6, atol=1e-6)
    ms, wall = bc._timed(lambda: kernels.affine(src, plan, out), 20, 5, graph=True)
    if knob is not None:
        knob.__exit__(None, None, None)
    tag = " s3.5" if "--s35" in sys.argv[1:] else (" frac" if frac else "")
    print(f"{os.environ.get('XRS_LIBRARY', 'product')}{tag}"
          f"{' generic' if knob is not None else ''}: "
          f"{ms:.4f} ms per launch "
          f"({(4 * n * n + 4 * no * no) / (ms / 1e3) / 1e9:.0f} GB/s)", flush=True)


if __name__ == "__main__":
    main()

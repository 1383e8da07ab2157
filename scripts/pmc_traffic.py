"""Workload for PMC traffic measurement of K1 (run under rocprofv3 --pmc).

bench.py runs it twice as a child process before it touches the GPU itself:

    rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum \\
        TCC_EA0_RDREQ_128B_sum --kernel-trace --output-format csv -d D/rd -o rd -- \\
        python scripts/pmc_traffic.py --size 40960 --tile 2048 --out-dtype f32
    rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_DRAM_sum ... (same)

and reduces the two counter files with ``reduce(D, size, out_dtype)``.
By hand: ``python scripts/pmc_traffic.py --reduce D [--size S --out-dtype f32]``.

Bytes are counted from the L2's memory-side requests BY SIZE: read bytes =
32 x RDREQ_32B + 64 x RDREQ_64B + 128 x RDREQ_128B, write bytes = 64 x
WRREQ_64B + 32 x (WRREQ - WRREQ_64B) (MI355X_MICROARCH.md §HBM: FETCH_SIZE
tallies 128-B requests at 64 B on gfx950; the size-resolved counters need no
such factor).  No correction is applied; instead three launches of KNOWN
byte counts run in the same process and are reported beside the bench
launch, each as measured / known:

  1. COPY16: benchlib float4 copy of the source raster (16-B lanes)
  2. COPY4 : benchlib 4-byte-lane copy of the same bytes (K1's tap width)
  3. IDENT : nearest reprojection EPSG:4326 -> EPSG:4326 onto the source's
             own grid — K1's own dword-gather pattern reading every source
             element exactly once (4*S read, 4*N written)
  4. BENCH : the bench.py kernel (bilinear 4326 -> 3857, f32 or f64 out)

RDREQ_DRAM (requests that reach DRAM rather than the die-level Infinity
Cache... as the counter counts them) is reported raw.
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
PASSES = {
    "rd": ["TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum",
           "TCC_EA0_RDREQ_128B_sum"],
    "wr": ["TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum", "TCC_EA0_RDREQ_DRAM_sum"],
}
LAUNCHES = ["copy16", "copy4", "ident", "bench"]
_MATCH = {"copy16": "copy_unrolled_kernel", "copy4": "copy_b32_kernel",
          "ident": KERNEL, "bench": KERNEL}


def run(size: int, tile: int, out_dtype: str):
    import torch

    import bench
    import xcube_resampling_amd as xrs
    from xcube_resampling_amd import kernels

    dev = torch.device("cuda", 0)
    src_gm, tgm, plan, lon, lat = bench.workload(size, tile)
    src = bench.synthetic_rows(0, size, size, dev)
    out = torch.empty_like(src)
    lib = bench.load_benchlib()
    sh = int(torch.cuda.current_stream(dev).cuda_stream)
    nbytes = src.numel() * 4
    for variant in (bench.COPY_VARIANT, 7):      # COPY16, COPY4
        if lib.xrs_bench_copy(src.data_ptr(), out.data_ptr(), nbytes, variant, sh) != 0:
            raise RuntimeError("benchlib copy failed")
        torch.cuda.synchronize()
        assert torch.equal(out, src)
    # IDENT: identity geometry (source grid as the target grid)
    ident = xrs.GridMapping.regular((size, size), (src_gm.x_min, src_gm.y_min), src_gm.xy_res,
                                    "EPSG:4326", tile_size=tile)
    cplan = xrs.plan_reproject(src_gm, ident, xrs.Transformer.from_crs(ident.crs, src_gm.crs,
                                                                       always_xy=True))
    out.zero_()
    torch.cuda.synchronize()
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
    """{launch: {counter: value summed over instances}} for the 4 launches, in
    dispatch order per kernel name."""
    rows = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.setdefault(r["Kernel_Name"], {}).setdefault(int(r["Dispatch_Id"]), {})
                per = rows[r["Kernel_Name"]][int(r["Dispatch_Id"])]
                per[r["Counter_Name"]] = per.get(r["Counter_Name"], 0.0) + \
                    float(r["Counter_Value"])
    out = {}
    for launch in LAUNCHES:
        disp = sorted((did, v) for name, ds in rows.items() if _MATCH[launch] in name
                      for did, v in ds.items())
        if launch == "copy16":
            disp = disp[:1]
        if launch in ("ident", "bench"):
            if len(disp) != 2:
                raise ValueError(f"expected 2 {KERNEL} dispatches, got {len(disp)}")
            disp = disp[:1] if launch == "ident" else disp[1:]
        if len(disp) != 1:
            raise ValueError(f"expected one {launch} dispatch, got {len(disp)}")
        out[launch] = disp[0][1]
    return out


def _bytes(c):
    rd = 32 * c["TCC_EA0_RDREQ_32B_sum"] + 64 * c["TCC_EA0_RDREQ_64B_sum"] + \
        128 * c["TCC_EA0_RDREQ_128B_sum"]
    n64 = c["TCC_EA0_WRREQ_64B_sum"]
    wr = 64 * n64 + 32 * (c["TCC_EA0_WRREQ_sum"] - n64)
    return rd, wr


def reduce(d, size: int = 40960, out_dtype: str = "f32", write: bool = False, name=None,
           bench_read_bytes: int | None = None):
    """Per launch: read / write bytes from the size-resolved request counters
    and, for the three calibration launches, measured / known.  d holds the
    'rd' and 'wr' pass directories (or one directory with both)."""
    c = {}
    for sub in PASSES:
        p = os.path.join(d, sub)
        for launch, vals in _counters(p if os.path.isdir(p) else d).items():
            c.setdefault(launch, {}).update(vals)
    n_src = size * size * 4
    out_b = size * size * (4 if out_dtype == "f32" else 8)
    known = {"copy16": (n_src, n_src), "copy4": (n_src, n_src), "ident": (n_src, n_src)}
    res = {"size": size, "out_dtype": out_dtype, "kernel": KERNEL, "launches": {}}
    for launch in LAUNCHES:
        rd, wr = _bytes(c[launch])
        e = {"read_bytes": int(rd), "write_bytes": int(wr),
             "rdreq": {k.split("_")[-2] if k.count("_") > 3 else "all": int(c[launch][k])
                       for k in PASSES["rd"]},
             "wrreq": int(c[launch]["TCC_EA0_WRREQ_sum"]),
             "wrreq_64B": int(c[launch]["TCC_EA0_WRREQ_64B_sum"]),
             "rdreq_dram": int(c[launch]["TCC_EA0_RDREQ_DRAM_sum"])}
        if launch in known:
            kr, kw = known[launch]
            e["read_over_known"] = round(rd / kr, 4)
            e["write_over_known"] = round(wr / kw, 4)
        res["launches"][launch] = e
    b = res["launches"]["bench"]
    res.update({
        "hbm_bytes_per_launch": b["read_bytes"] + b["write_bytes"],
        "read_bytes": b["read_bytes"], "write_bytes": b["write_bytes"],
        "write_over_algorithmic": round(b["write_bytes"] / out_b, 4),
        "calibration": {
            "method": "size-resolved L2->memory requests (32/64/128 B reads, 32/64 B writes), "
                      "no correction factor; launches of known bytes in the same process: "
                      + ", ".join(f"{k} read {res['launches'][k]['read_over_known']} / write "
                                  f"{res['launches'][k]['write_over_known']} of known"
                                  for k in known)},
    })
    if bench_read_bytes:
        res["read_over_algorithmic"] = round(b["read_bytes"] / bench_read_bytes, 4)
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
        print(json.dumps(reduce(a.reduce, a.size, a.out_dtype, write=bool(a.name), name=a.name),
                         indent=1))
    else:
        run(a.size, a.tile, a.out_dtype)

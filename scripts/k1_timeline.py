"""K1's item timeline (is the item prologue hidden?).
Runs the config-5 bench launch with the timeline probe arm (probe/k1tl: K1
with thread 0 of every item recording s_memrealtime at the item's start, at
the end of its prologue — column and row entries resolved, first taps about
to issue — and at its end, plus HW_ID / XCC_ID), then per CU sweeps the
items' intervals: the time some item of the CU is in its prologue while no
item of the CU streams taps ("exposed prologue"), the time the CU holds no
item, and the mean number of items resident.
    XRS_LIBRARY=probe/k1tl/pkg/lib/libxrs.so python scripts/k1_timeline.py OUT.json
    python scripts/k1_timeline.py --analyze OUT.npz        (no GPU: the saved timeline)"""
from __future__ import annotations

import ctypes
import json
import os
import sys
from collections import defaultdict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

TICK_US = 0.01   # s_memrealtime: 100 MHz


def sweep(iv):
    """iv: list of (t0, t1, t2) of one CU -> (span, exposed, idle, streaming, busy_area)."""
    ev = []
    for t0, t1, t2 in iv:
        ev += [(t0, 0, +1), (t1, 0, -1), (t1, 1, +1), (t2, 1, -1)]
    ev.sort()
    npro = nstr = 0
    last = ev[0][0]
    exposed = idle = streaming = area = 0
    for t, kind, d in ev:
        dt = t - last
        if dt > 0:
            if nstr > 0:
                streaming += dt
            elif npro > 0:
                exposed += dt
            else:
                idle += dt
            area += dt * (npro + nstr)
        last = t
        if kind == 0:
            npro += d
        else:
            nstr += d
    span = ev[-1][0] - ev[0][0]
    return span, exposed, idle, streaming, area


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else "k1_timeline.json"
    import bench
    import torch

    from xcube_resampling_amd import _native, kernels

    dev = torch.device("cuda", 0)
    _, _, plan, _, _ = bench.workload(40960, 2048)
    src = bench.synthetic_rows(0, plan.src_height, 40960, dev)
    flags = kernels.ErrorFlags(dev)
    out = torch.empty((1, 40960, 40960), device=dev, dtype=torch.float32)

    def step():
        kernels.reproject(src, plan, "bilinear", float("nan"), out_dtype=np.float32, out=out,
                          flags=flags, check=False)

    for _ in range(15):
        step()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    step()
    e1.record()
    torch.cuda.synchronize()
    flags.raise_if_set("k1 timeline")
    lib = _native.lib()
    n = (40960 // 32) * (40960 // 512)
    buf = np.zeros((n, 4), dtype=np.uint64)
    lib.xrs_probe_timeline.restype = ctypes.c_int
    lib.xrs_probe_timeline.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    assert lib.xrs_probe_timeline(buf.ctypes.data, n) == 0
    np.savez_compressed(os.path.splitext(out_path)[0] + ".npz", tl=buf)
    res = analyze(buf)
    res["kernel_ms_event"] = round(e0.elapsed_time(e1), 4)
    print(json.dumps(res))
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)


def residency(iv):
    """Time at each number of resident / streaming items of one CU, and the
    gaps from the last item end before an item's start to that start."""
    ev = []
    for a, b, c in iv:
        ev += [(a, 1, 0), (b, 0, 1), (c, -1, -1)]
    ev.sort()
    res = st = 0
    last = ev[0][0]
    hres, hst = defaultdict(int), defaultdict(int)
    for t, dr, ds in ev:
        dt = t - last
        if dt > 0:
            hres[res] += dt
            hst[st] += dt
        last = t
        res += dr
        st += ds
    ends = np.sort(np.array([c for _, _, c in iv]))
    gaps = []
    for a in sorted(a for a, _, _ in iv)[4:]:
        j = np.searchsorted(ends, a) - 1
        if j >= 0:
            gaps.append(a - ends[j])
    return hres, hst, gaps


def analyze(buf):
    ok = buf[:, 2] > 0
    t = buf[ok, :3].astype(np.int64)
    where = buf[ok, 3]
    t -= t[:, 0].min()
    xcc = (where >> 32) & 0xF
    cu = (where >> 8) & 0xFF   # cu_id, sh_id, se_id of HW_ID
    per = defaultdict(list)
    for k, (a, b, c) in zip(zip(xcc.tolist(), cu.tolist()), t.tolist()):
        per[k].append((a, b, c))
    tot = dict(span=0, exposed=0, idle=0, streaming=0, area=0)
    for iv in per.values():
        s, e, i, st, ar = sweep(iv)
        tot["span"] += s; tot["exposed"] += e; tot["idle"] += i
        tot["streaming"] += st; tot["area"] += ar
    pro = (t[:, 1] - t[:, 0]) * TICK_US
    item = (t[:, 2] - t[:, 0]) * TICK_US
    cu_end = np.array([max(c for _, _, c in iv) for iv in per.values()]) * TICK_US
    hres, hst, gaps = defaultdict(int), defaultdict(int), []
    for iv in per.values():
        a, b, g = residency(iv)
        for k, v in a.items():
            hres[k] += v
        for k, v in b.items():
            hst[k] += v
        gaps += g
    gaps = np.array(gaps) * TICK_US
    nres, nst = sum(hres.values()), sum(hst.values())
    res = {
        "items": int(ok.sum()), "cus": len(per),
        "span_us": round(float(t[:, 2].max()) * TICK_US, 1),
        "prologue_us_mean": round(float(pro.mean()), 3),
        "prologue_us_p50_p90": [round(float(np.percentile(pro, q)), 3) for q in (50, 90)],
        "item_us_mean": round(float(item.mean()), 3),
        "prologue_frac_of_item": round(float(pro.sum() / item.sum()), 4),
        "resident_items_mean": round(tot["area"] / tot["span"], 3),
        "exposed_prologue_frac": round(tot["exposed"] / tot["span"], 4),
        "idle_frac": round(tot["idle"] / tot["span"], 4),
        "streaming_frac": round(tot["streaming"] / tot["span"], 4),
        "cu_end_us_min_median_max": [round(float(np.min(cu_end)), 1),
                                     round(float(np.median(cu_end)), 1),
                                     round(float(np.max(cu_end)), 1)],
        "resident_items_time_frac": {k: round(v / nres, 4) for k, v in sorted(hres.items())},
        "streaming_items_time_frac": {k: round(v / nst, 4) for k, v in sorted(hst.items())},
        "gap_end_to_next_start_us_p10_p50_p90_mean": [
            round(float(np.percentile(gaps, q)), 2) for q in (10, 50, 90)] + [round(float(gaps.mean()), 2)],
    }
    return res


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--analyze":
        print(json.dumps(analyze(np.load(sys.argv[2])["tl"])))
    else:
        main()

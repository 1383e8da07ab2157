"""Per-kernel PMC counters, averaged per dispatch, for one counter pass over a
timing script (rocprofv3 --pmc as a child; at most 8 SQ / 4 TCC / 2 GRBM
counters per pass).
    python scripts/pmc_kernels.py --counters SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU \
        --kernels claim,resolve -- scripts/time_rectify.py --fused --reps 3"""
from __future__ import annotations

import argparse
import csv
import json
import os
import shutil
import subprocess
import sys
import tempfile
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--counters", required=True)
    ap.add_argument("--kernels", default="claim,resolve,ij_bboxes")
    ap.add_argument("--timeout", type=int, default=120)
    ap.add_argument("script", nargs=argparse.REMAINDER)
    args = ap.parse_args()
    script = [a for a in args.script if a != "--"]
    kernels = args.kernels.split(",")
    prof = shutil.which("rocprofv3")
    d = tempfile.mkdtemp(prefix="xrs_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    cmd = ["timeout", "-s", "KILL", str(args.timeout), prof, "--pmc",
           *args.counters.split(","), "--kernel-trace", "--output-format", "csv", "-d", d,
           "-o", "p", "--", sys.executable, os.path.join(ROOT, script[0]), *script[1:]]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        print(r.stdout[-3000:], file=sys.stderr)
        sys.exit(r.returncode)
    acc = defaultdict(float)
    disp = defaultdict(set)
    for root, _, files in os.walk(d):
        for f in files:
            if not f.endswith("counter_collection.csv"):
                continue
            for row in csv.DictReader(open(os.path.join(root, f))):
                k = next((n for n in kernels if n in row["Kernel_Name"]), None)
                if k is None:
                    continue
                acc[(k, row["Counter_Name"])] += float(row["Counter_Value"])
                disp[k].add(row["Dispatch_Id"])
    out = {}
    for k in kernels:
        n = max(len(disp[k]), 1)
        out[k] = {c: acc[(k, c)] / n for c in args.counters.split(",")}
        out[k]["dispatches"] = len(disp[k])
    print(json.dumps(out))


if __name__ == "__main__":
    main()

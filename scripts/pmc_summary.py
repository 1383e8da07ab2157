"""Per-dispatch averages of rocprofv3 --pmc counters for kernels whose name
matches a pattern:  python scripts/pmc_summary.py CSV [PATTERN ...]"""
import collections
import csv
import sys

pats = sys.argv[2:] or ["claim", "resolve"]
acc = collections.defaultdict(float)
ids = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    k = next((p for p in pats if p in r["Kernel_Name"]), None)
    if k is None:
        continue
    acc[(k, r["Counter_Name"])] += float(r["Counter_Value"])
    ids[k].add(r["Dispatch_Id"])
for (k, c), v in sorted(acc.items()):
    print(f"{k:10s} {c:22s} {v / len(ids[k]):.4g}")

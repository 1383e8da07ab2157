"""Print rocprofv3 kernel_stats.csv rows (readable names, average µs).
    python scripts/kstats.py STATS.csv [name-substring ...]"""
import csv
import sys

keys = sys.argv[2:]
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].replace("(anonymous namespace)::", "")
    if not keys or any(k in n for k in keys):
        print("   ", n[:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")

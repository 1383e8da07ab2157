"""Reduce rocprofv3 --pmc counter_collection CSVs: one line per dispatch of the
named kernels with every counter of every pass under DIR (recursive).
    python scripts/pmc_reduce.py DIR [kernel-substring ...]"""
import collections
import csv
import glob
import json
import os
import sys


def reduce(d, names=("gather_",)):
    out = collections.defaultdict(dict)
    for f in glob.glob(os.path.join(d, "**", "*_counter_collection.csv"), recursive=True):
        pas = os.path.basename(os.path.dirname(f))
        for r in csv.DictReader(open(f)):
            if not any(n in r["Kernel_Name"] for n in names):
                continue
            key = (pas, int(r["Dispatch_Id"]))
            e = out[key]
            e["kernel"] = r["Kernel_Name"].split("(")[0][-60:]
            e["ms"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            e["vgpr"] = int(r["VGPR_Count"])
            e[r["Counter_Name"]] = float(r["Counter_Value"])
    return out


if __name__ == "__main__":
    res = reduce(sys.argv[1], tuple(sys.argv[2:]) or ("gather_",))
    for k in sorted(res):
        print(json.dumps({"pass": k[0], "dispatch": k[1], **res[k]}))

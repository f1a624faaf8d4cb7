"""Per-kernel sums of rocprofv3 PMC counters (one line per kernel name).
usage: python tools/pmc_kernels.py <dir> [substring]"""
import collections
import csv
import glob
import os
import re
import sys

path = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if pat not in k:
            continue
        m = re.search(r"(\w+_kernel)<?([^>(]*)", k)
        name = (m.group(1) + "<" + m.group(2) + ">") if m else k[:60]
        agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[name].add(r.get("Dispatch_Id", ""))
    for name, c in sorted(agg.items()):
        print(f"{name:40s} n={len(disp[name]):3d} " + " ".join(f"{k}={v:.4g}" for k, v in sorted(c.items())))

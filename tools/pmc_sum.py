"""Sum rocprofv3 counter_collection CSVs per counter for kernels matching a pattern.
usage: python tools/pmc_sum.py <dir-or-csv> [kernel-substring]"""
import collections
import csv
import glob
import os
import sys

path = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
files = [path] if path.endswith(".csv") else glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)
for f in files:
    agg, n = collections.defaultdict(float), collections.Counter()
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            n[r["Counter_Name"]] += 1
    print(f, {k: "%.4g (%d)" % (v, n[k]) for k, v in sorted(agg.items())})

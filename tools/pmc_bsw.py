"""VALU lane-instructions per cell of the SW kernels, from rocprofv3 --pmc
SQ_INSTS_VALU runs of tools/bsw_bench.py (one per workload), written to
profiles/pmc_bsw.json for bench.py's SW roofline.

usage: python tools/pmc_bsw.py <c3_pmc_dir> <c3_bench.log> <fixed_pmc_dir> <fixed_bench.log> <tag>"""
import csv
import glob
import json
import os
import sys


def valu(d):
    tot, n = 0.0, set()
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "bsw_" in r["Kernel_Name"] and r["Counter_Name"] == "SQ_INSTS_VALU":
                tot += float(r["Counter_Value"])
                n.add(r.get("Dispatch_Id", ""))
    return tot


def cells(log, key):
    for line in open(log):
        if line.startswith("{"):
            return json.loads(line)[key]["cells"]
    raise SystemExit(f"no bench line in {log}")


def main():
    c3d, c3l, fxd, fxl, tag = sys.argv[1:6]
    out = {}
    for name, d, log in (("c3", c3d, c3l), ("fixed", fxd, fxl)):
        # bsw_bench.py --reps 1 runs the workload twice (warm-up + timed)
        v = valu(d) / 2
        c = cells(log, name)
        out[name] = {"valu_wave_instr": v, "cells": c, "valu_lane_instr_per_cell": round(64 * v / c, 3)}
    out["_note"] = ("SQ_INSTS_VALU (wave64 instructions) of every bsw_* kernel of one ksw_extend2 batch (keys, "
                    "bounds, pair / lane kernels), x64 lanes / evaluated cells; separate rocprofv3 --pmc runs")
    out["source"] = tag
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    json.dump(out, open(os.path.join(root, "profiles", "pmc_bsw.json"), "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

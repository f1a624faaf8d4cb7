"""SW counters per ksw_extend2 batch from the rocprofv3 --pmc passes of
tools/gpu_session.sh's `bswpmc` step (tools/bsw_bench.py, --reps 1 = one
warm-up + one timed batch, so totals are halved), written to
profiles/pmc_bsw.json for bench.py's SW roofline:
  * SQ issue counters of every bsw_* kernel for C3 and the fixed 151x251
    workload -> VALU lane-instructions per evaluated cell, stall fractions;
  * FETCH_SIZE / WRITE_SIZE of C3 -> HBM bytes per batch (against the
    algorithmic qlen + tlen + 24 bytes per task).

usage: python tools/pmc_bsw.py gpurun_out/<tag> <tag>"""
import csv
import re
import glob
import json
import os
import sys

BATCHES = 2.0  # bsw_bench.py --reps 1: warm-up + timed


def totals(d):
    tot = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "bsw_" in r["Kernel_Name"]:
                tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return {k: v / BATCHES for k, v in tot.items()}


def bench_line(log):
    for line in open(log):
        if line.startswith("{"):
            return json.loads(line)
    raise SystemExit(f"no bench line in {log}")


def main():
    src, tag = sys.argv[1:3]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = os.path.join(root, "profiles", "pmc_bsw.json")
    prev = json.load(open(path)) if os.path.exists(path) else {}  # sections this run did not profile are kept
    out = {}
    for name in ("c3", "fixed"):
        if not os.path.isdir(os.path.join(src, f"bswpmc_{name}")):
            if name in prev:
                out[name] = prev[name]
            continue
        sq = totals(os.path.join(src, f"bswpmc_{name}"))
        b = bench_line(os.path.join(src, f"bswpmc_{name}.log"))[name]
        d = {"cells": b["cells"], "tasks": b["tasks"], "counters_per_batch": sq,
             "valu_lane_instr_per_cell": round(64 * sq["SQ_INSTS_VALU"] / b["cells"], 3)}
        wc = sq.get("SQ_WAVE_CYCLES")
        for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY"):
            if wc and k in sq:
                d[k.lower() + "_frac_of_wave_cycles"] = round(sq[k] / wc, 4)
        out[name] = d
    fe = totals(os.path.join(src, "bswpmc_c3_fetch")).get("FETCH_SIZE") if "c3" in out else None
    wr = totals(os.path.join(src, "bswpmc_c3_write")).get("WRITE_SIZE")
    if fe is not None and wr is not None:
        out["c3"]["hbm_bytes_per_batch"] = int(round((2 * fe + wr) * 1024))  # 2 x FETCH_SIZE: gfx950 calibration
        out["c3"]["fetch_kib"], out["c3"]["write_kib"] = fe, wr
    gdir = os.path.join(src, "bswpmc_global")
    if not os.path.isdir(gdir) and "global" in prev:
        out["global"] = prev["global"]
    if os.path.isdir(gdir):  # ksw_global2: scores-only and scores + CIGAR runs, 2 each (warm-up + timed)
        tot = {}
        for f in glob.glob(os.path.join(gdir, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                n = r["Kernel_Name"]
                if "bsw_global" in n and r["Counter_Name"] == "SQ_INSTS_VALU":
                    k = "cigar" if re.search(r"<\d+, true", n) else "scores"  # bsw_global_lane_kernel<NB, CIG, U>
                    tot[k] = tot.get(k, 0.0) + float(r["Counter_Value"])
                elif "traceback" in n and r["Counter_Name"] == "SQ_INSTS_VALU":
                    tot["traceback"] = tot.get("traceback", 0.0) + float(r["Counter_Value"])
        g = bench_line(os.path.join(src, "bswpmc_global.log"))["global"]
        # each mode runs twice (warm-up + timed): scores-only DP, DP with direction rows + traceback
        out["global"] = {"band_cells": g["cells"], "tasks": g["tasks"],
                         "dp_valu_lane_instr_per_cell": round(64 * tot.get("scores", 0) / 2 / g["cells"], 3),
                         "dp_cigar_valu_lane_instr_per_cell": round(64 * tot.get("cigar", 0) / 2 / g["cells"], 3),
                         "traceback_valu_wave_instr": tot.get("traceback", 0) / 2}
        # the CIGAR pass as a whole: direction-row DP plus the traceback launch
        out["global"]["cigar_pass_valu_lane_instr_per_cell"] = round(
            64 * (tot.get("cigar", 0) + tot.get("traceback", 0)) / 2 / g["cells"], 3)
    adir = os.path.join(src, "bswpmc_align")
    if os.path.isdir(adir):  # ksw_align2: warm-up + timed batch
        tot = {}
        for f in glob.glob(os.path.join(adir, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if "bsw_align" in r["Kernel_Name"]:
                    tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        a = bench_line(os.path.join(src, "bswpmc_align.log"))["align"]
        q = {k: v / 2 for k, v in tot.items()}
        out["align"] = {"cells": a["cells"], "tasks": a["tasks"], "counters_per_batch": q,
                        "valu_lane_instr_per_cell": round(64 * q.get("SQ_INSTS_VALU", 0) / a["cells"], 3)}
        if q.get("SQ_WAVE_CYCLES"):
            out["align"]["sq_active_inst_any_frac_of_wave_cycles"] = round(q["SQ_ACTIVE_INST_ANY"] / q["SQ_WAVE_CYCLES"], 4)
    elif "align" in prev:
        out["align"] = prev["align"]
    out["_note"] = ("rocprofv3 --pmc of tools/bsw_bench.py --which <w> --reps 1 (separate passes: SQ issue/stall "
                    "counters, FETCH_SIZE, WRITE_SIZE), every bsw_* kernel of one ksw_extend2 batch (keys, bounds, "
                    "extension launch), halved for the warm-up batch; VALU per cell = SQ_INSTS_VALU x 64 / evaluated "
                    "cells; SQ_*_CYCLES / WAIT / ACTIVE in quad-cycles; fetch_kib / write_kib as rocprofv3 reports them, "
                    "hbm_bytes_per_batch = 2 x FETCH_SIZE + WRITE_SIZE (the gfx950 FETCH_SIZE calibration, "
                    "profiles/fetch_calibration.json)")
    out["source"] = tag if "c3" not in prev or os.path.isdir(os.path.join(src, "bswpmc_c3")) else prev.get("source")
    # per-section sources when a session collected only some sections
    if os.path.isdir(gdir) and not os.path.isdir(os.path.join(src, "bswpmc_c3")):
        out["global"]["source"] = tag
    if os.path.isdir(adir) and not os.path.isdir(os.path.join(src, "bswpmc_c3")):
        out["align"]["source"] = tag
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

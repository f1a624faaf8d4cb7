"""Sum rocprofv3 --pmc counters of the fp32 forward kernels per forward pass.
usage: python tools/pmc_sum_fwd.py DIR [passes] [cells_per_pass]"""
import csv
import glob
import sys

d = sys.argv[1]
passes = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
cells = float(sys.argv[3]) if len(sys.argv) > 3 else 22721383941.0
tot = {}
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "phmm3_kernel" in n or "phmm2_kernel" in n or "phmm_kernel<float, false, false>" in n:
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for k in sorted(tot):
    print(f"{k:28s} {tot[k] / passes:.4e}")
v = tot.get("SQ_INSTS_VALU")
if v:
    print("VALU lane-instr per cell", round(v / passes * 64 / cells, 3))
if "SQ_WAVE_CYCLES" in tot:
    wc = tot["SQ_WAVE_CYCLES"]
    for k in ("SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
        if k in tot:
            print(f"{k} / WAVE_CYCLES = {tot[k] / wc:.3f}")

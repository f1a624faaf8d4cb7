"""Per-pass SQ / HBM counters of the PairHMM fp32 forward kernels (column-
blocked phmm4_kernel and row-streamed phmm3_kernel) from a
tools/gpu_session.sh ... phmmpmc run (tools/phmm_bench.py --steps 1 --warmup 1:
two passes).  usage: python tools/pmc_cols.py gpurun_out/<tag> [passes] [cells]"""
import csv
import glob
import json
import os
import sys

src = sys.argv[1]
passes = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
cells = float(sys.argv[3]) if len(sys.argv) > 3 else 22721383941.0
tot = {}
for f in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if any(k in r["Kernel_Name"] for k in ("phmm4_kernel", "phmm3_kernel", "phmm2_kernel",
                                               "phmm_kernel<float, false, false")):
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
q = {k: v / passes for k, v in sorted(tot.items())}
wc, vi = q["SQ_WAVE_CYCLES"], q["SQ_INSTS_VALU"]
d = {"cells_per_pass": int(cells), "valu_lane_instr_per_cell": round(vi * 64 / cells, 3),
     "salu_instr_per_wave_instr_valu": round(q["SQ_INSTS_SALU"] / vi, 4),
     "lds_instr_per_wave_instr_valu": round(q["SQ_INSTS_LDS"] / vi, 4),
     "sq_active_inst_any_frac_of_wave_cycles": round(q["SQ_ACTIVE_INST_ANY"] / wc, 4),
     "sq_wait_inst_any_frac_of_wave_cycles": round(q["SQ_WAIT_INST_ANY"] / wc, 4),
     "sq_wait_any_frac_of_wave_cycles": round(q["SQ_WAIT_ANY"] / wc, 4)}
if "SQ_LDS_BANK_CONFLICT" in q:
    d["lds_bank_conflict_per_active_lds_cycle"] = round(q["SQ_LDS_BANK_CONFLICT"] / q["SQ_ACTIVE_INST_LDS"], 4)
if "FETCH_SIZE" in q:
    d["fetch_kib"] = q["FETCH_SIZE"]
if "WRITE_SIZE" in q:
    d["write_kib"] = q["WRITE_SIZE"]
print(json.dumps({"phmm_fwd_fp32": d, "counters_per_pass": q}, indent=1))

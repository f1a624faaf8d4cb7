"""Write profiles/pmc_phmm.json (+ the phmm_fwd_fp32 entry of
profiles/pmc_traffic.json) from a tools/pmc_phmm_r3.sh run: counters of the
fp32 forward kernels summed over their class launches, per forward pass
(tools/phmm_bench.py --steps 1 --warmup 1 = 2 passes), and the per-pass
summary copied to profiles/<round>/<tag>_pmc_phmm.txt.
usage: python tools/pmc_phmm_json.py gpurun_out/<tag> <round dir> <tag> [passes] [cells_per_pass]"""
import csv
import glob
import json
import os
import shutil
import sys

src, dst, tag = sys.argv[1:4]
passes = float(sys.argv[4]) if len(sys.argv) > 4 else 2.0
cells = float(sys.argv[5]) if len(sys.argv) > 5 else 22721383941.0
FWD = ("phmm4_kernel", "phmm3_kernel", "phmm2_kernel", "phmm_kernel<float, false, false>")
tot = {}
for f in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if any(k in r["Kernel_Name"] for k in FWD):
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
q = {k: v / passes for k, v in sorted(tot.items())}
wc = q["SQ_WAVE_CYCLES"]
vi = q["SQ_INSTS_VALU"]
d = {"cells_per_pass": int(cells),
     "valu_lane_instr_per_cell": round(vi * 64 / cells, 3),
     "salu_instr_per_wave_instr_valu": round(q["SQ_INSTS_SALU"] / vi, 4),
     "lds_instr_per_wave_instr_valu": round(q["SQ_INSTS_LDS"] / vi, 4),
     "sq_active_inst_any_frac_of_wave_cycles": round(q["SQ_ACTIVE_INST_ANY"] / wc, 4),
     "sq_wait_inst_any_frac_of_wave_cycles": round(q["SQ_WAIT_INST_ANY"] / wc, 4),
     "sq_wait_any_frac_of_wave_cycles": round(q["SQ_WAIT_ANY"] / wc, 4)}
if "SQ_LDS_BANK_CONFLICT" in q and "SQ_ACTIVE_INST_LDS" in q:
    d["lds_bank_conflict_per_active_lds_cycle"] = round(q["SQ_LDS_BANK_CONFLICT"] / q["SQ_ACTIVE_INST_LDS"], 4)
root = os.path.dirname(os.path.abspath(dst.rstrip("/"))) if os.path.basename(dst.rstrip("/")).startswith("r") else dst
json.dump({"phmm_fwd_fp32": d, "counters_per_pass": q,
           "_note": "rocprofv3 --pmc of tools/phmm_bench.py (C2, warmup + 1 timed pass; one counter group per run, "
                    "tools/pmc_phmm_r3.sh), counters of the fp32 forward kernels summed over their class launches and "
                    "divided by the passes; SQ_*_CYCLES / SQ_WAIT_* / SQ_ACTIVE_* are quad-cycles, SQ_INSTS_* wave64 "
                    "instructions; FETCH_SIZE / WRITE_SIZE in KiB as rocprofv3 reports them",
           "source": tag}, open(os.path.join(root, "pmc_phmm.json"), "w"), indent=1)
tp = os.path.join(root, "pmc_traffic.json")
t = json.load(open(tp)) if os.path.exists(tp) else {}
if "FETCH_SIZE" in q and "WRITE_SIZE" in q:
    t["phmm_fwd_fp32"] = int(round((q["FETCH_SIZE"] + q["WRITE_SIZE"]) * 1024))
    t["fetch_kib"], t["write_kib"], t["source"] = q["FETCH_SIZE"], q["WRITE_SIZE"], tag
    t.pop("phmm_fwd_fp32_source", None)
    t["_note"] = ("HBM bytes per fp32 forward pass (all hap-length class launches) on the default C2 workload = "
                  "(FETCH_SIZE + WRITE_SIZE) KiB * 1024 from separate rocprofv3 --pmc passes "
                  f"(gpurun_out/{tag}, summary in {os.path.relpath(dst, os.path.dirname(root))}/{tag}_pmc_phmm.txt), divided by the passes profiled.  "
                  "FETCH_SIZE as reported: bench.py prices HBM reads as 2 x FETCH_SIZE (the gfx950 calibration of "
                  "profiles/fetch_calibration.json, measured for 1, 4 and 16 B per-lane loads).")
    json.dump(t, open(tp, "w"), indent=1)
os.makedirs(dst, exist_ok=True)
if os.path.exists(os.path.join(src, "summary.txt")):
    shutil.copy(os.path.join(src, "summary.txt"), os.path.join(dst, f"{tag}_pmc_phmm.txt"))
else:  # the per-pass counters themselves
    with open(os.path.join(dst, f"{tag}_pmc_phmm.txt"), "w") as f:
        f.write(f"fp32 forward kernels {', '.join(FWD)}: counters per C2 pass ({passes:g} passes profiled)\n")
        for k, v in q.items():
            f.write(f"{k:28s} {v:18.1f}\n")
        f.write(json.dumps(d) + "\n")
print(json.dumps(d))

"""Summarise a gpu_session.sh profiling run into profiles/<round>/:
kernel stats, per-pass span of the fp32 PairHMM forward (its hap-length class
launches overlap on four streams, so per-launch durations add up to more
than the pass), HBM bytes per forward pass from the FETCH_SIZE / WRITE_SIZE
passes (-> profiles/pmc_traffic.json) and the SQ issue / stall counters per
forward pass (-> profiles/pmc_phmm.json), both read by bench.py.

usage: python tools/profile_summary.py gpurun_out/<tag> profiles/<round> <tag> [cells_per_pass]"""
import csv
import json
import os
import shutil
import sys

KERNELS = ("phmm3_kernel", "phmm2_kernel", "phmm_kernel<float, false, false>")  # fp32 forward: streamed, two-row, one-row
PASS_MARK = "phmm_keys_kernel"  # one schedule (keys kernel) per forward pass
C2_CELLS = 22721383941  # sum R*H of the default C2 workload (bench.py config.cells_per_gpu)


def is_fwd(name):
    return any(k in name for k in KERNELS)


def counters(path):
    """Counter totals of the forward-pass kernels, and the number of forward
    passes they span (= schedules run: one keys-kernel dispatch per pass)."""
    tot, marks = {}, set()
    for x in csv.DictReader(open(path)):
        if is_fwd(x["Kernel_Name"]):
            tot[x["Counter_Name"]] = tot.get(x["Counter_Name"], 0.0) + float(x["Counter_Value"])
        elif PASS_MARK in x["Kernel_Name"]:
            marks.add(x["Dispatch_Id"])
    return tot, max(1, len(marks))


def main():
    src, dst, tag = sys.argv[1:4]
    cells = int(sys.argv[4]) if len(sys.argv) > 4 else C2_CELLS
    os.makedirs(dst, exist_ok=True)
    summary = {"kernels": KERNELS}
    for f in ("bench.log", "benchq.log", "pytest_gpu.log"):
        if os.path.exists(os.path.join(src, f)):
            shutil.copy(os.path.join(src, f), os.path.join(dst, f"{tag}_{f}"))
    if os.path.exists(os.path.join(src, "prof", "run_kernel_trace.csv")):
        shutil.copy(os.path.join(src, "prof", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
        rows = list(csv.DictReader(open(os.path.join(src, "prof", "run_kernel_trace.csv"))))
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        # a pass = the forward launches between one schedule (keys kernel) and the next
        passes, cur = [], None
        for r in rows:
            if PASS_MARK in r["Kernel_Name"]:
                cur = []
                passes.append(cur)
            elif is_fwd(r["Kernel_Name"]) and cur is not None:
                cur.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
        passes = [p for p in passes if p]
        spans = [(max(e for _, e in p) - min(s for s, _ in p)) / 1e6 for p in passes]
        summary.update({"launches_per_pass": [len(p) for p in passes], "pass_span_ms": spans,
                        "pass_span_ms_warm_min": min(spans[1:] or spans or [0]),
                        "note": "span = last end - first start over the class launches of one forward pass; "
                                "compare with bench.py stages_ms.forward_fp32 (HIP events on the launch stream)"})
    pmc = {}
    for d in sorted(os.listdir(src)):
        p = os.path.join(src, d, "run_counter_collection.csv")
        if not (d.startswith("phmmpmc") or d.startswith("pmc_")) or not os.path.exists(p):
            continue
        shutil.copy(p, os.path.join(dst, f"{tag}_{d}.csv"))
        tot, npass = counters(p)
        for k, v in tot.items():
            pmc[k] = v / npass  # per forward pass
    summary["pmc_per_pass"] = pmc
    json.dump(summary, open(os.path.join(dst, f"{tag}_phmm_summary.json"), "w"), indent=1)
    root = os.path.dirname(dst.rstrip("/"))
    if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
        t = {"phmm_fwd_fp32": int(round((pmc["FETCH_SIZE"] + pmc["WRITE_SIZE"]) * 1024)),
             "_note": "HBM bytes per fp32 forward pass (all hap-length class launches) on the default C2 workload = "
                      "(FETCH_SIZE + WRITE_SIZE) KiB * 1024 from separate rocprofv3 --pmc passes "
                      f"(profiles/{os.path.basename(dst)}/{tag}_*.csv), divided by the passes profiled.  FETCH_SIZE "
                      "as reported: bench.py prices HBM reads as 2 x FETCH_SIZE (the gfx950 calibration of "
                      "profiles/fetch_calibration.json, measured for 1, 4 and 16 B per-lane loads).",
             "fetch_kib": pmc["FETCH_SIZE"], "write_kib": pmc["WRITE_SIZE"], "source": tag}
        json.dump(t, open(os.path.join(root, "pmc_traffic.json"), "w"), indent=1)
    if "SQ_INSTS_VALU" in pmc:
        q = {k: pmc[k] for k in sorted(pmc) if k.startswith("SQ_")}
        wc = pmc.get("SQ_WAVE_CYCLES")
        d = {"cells_per_pass": cells,
             "valu_lane_instr_per_cell": round(pmc["SQ_INSTS_VALU"] * 64 / cells, 3),
             "salu_instr_per_wave_instr_valu": round(pmc.get("SQ_INSTS_SALU", 0) / pmc["SQ_INSTS_VALU"], 4),
             "lds_instr_per_wave_instr_valu": round(pmc.get("SQ_INSTS_LDS", 0) / pmc["SQ_INSTS_VALU"], 4)}
        if wc:
            for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY"):
                if k in pmc:
                    d[k.lower() + "_frac_of_wave_cycles"] = round(pmc[k] / wc, 4)
        json.dump({"phmm_fwd_fp32": d, "counters_per_pass": q,
                   "_note": "rocprofv3 --pmc of tools/phmm_bench.py (C2, warmup + 1 timed pass), counters of the fp32 "
                            "forward kernels summed over their class launches and divided by the passes; "
                            "SQ_*_CYCLES / SQ_WAIT_* / SQ_ACTIVE_* are quad-cycles, SQ_INSTS_* wave64 instructions",
                   "source": tag}, open(os.path.join(root, "pmc_phmm.json"), "w"), indent=1)
    print(json.dumps(summary))


if __name__ == "__main__":
    main()

"""Summarise a gpu_session.sh profiling run into profiles/<round>/:
kernel stats, per-pass span of the fp32 PairHMM forward (its hap-length class
launches overlap on four streams, so per-launch durations add up to more
than the pass), and HBM bytes per forward pass from the FETCH_SIZE /
WRITE_SIZE passes (written to profiles/pmc_traffic.json for bench.py).

usage: python tools/profile_summary.py gpurun_out/<tag> profiles/<round> <tag>"""
import csv
import json
import os
import shutil
import sys

KERNEL = "phmm_kernel<float, false, false>"


def main():
    src, dst, tag = sys.argv[1:4]
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "prof", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
    for f in ("bench.log", "pytest_gpu.log"):
        if os.path.exists(os.path.join(src, f)):
            shutil.copy(os.path.join(src, f), os.path.join(dst, f"{tag}_{f}"))
    rows = list(csv.DictReader(open(os.path.join(src, "prof", "run_kernel_trace.csv"))))
    ph = sorted((r for r in rows if KERNEL in r["Kernel_Name"]), key=lambda r: int(r["Start_Timestamp"]))
    # a pass = the class launches that overlap in time
    passes, cur, end = [], [], -1
    for r in ph:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if cur and s > end:
            passes.append(cur)
            cur = []
        cur.append((s, e))
        end = max(end, e)
    if cur:
        passes.append(cur)
    spans = [(max(e for _, e in p) - min(s for s, _ in p)) / 1e6 for p in passes]
    summary = {"kernel": KERNEL, "launches_per_pass": [len(p) for p in passes], "pass_span_ms": spans,
               "note": "span = last end - first start over the overlapping class launches of one forward pass; "
                       "compare with bench.py stages_ms.forward_fp32 (HIP events on the launch stream)"}
    traffic = {}
    for f, cname in (("pmc_fetch", "FETCH_SIZE"), ("pmc_write", "WRITE_SIZE")):
        p = os.path.join(src, f, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        shutil.copy(p, os.path.join(dst, f"{tag}_{f}.csv"))
        r = [x for x in csv.DictReader(open(p)) if KERNEL in x["Kernel_Name"] and x["Counter_Name"] == cname]
        traffic[cname] = sum(float(x["Counter_Value"]) for x in r)  # KiB over one forward pass
        traffic[cname + "_launches"] = len(r)
    summary["pmc"] = traffic
    json.dump(summary, open(os.path.join(dst, f"{tag}_phmm_summary.json"), "w"), indent=1)
    if "FETCH_SIZE" in traffic and "WRITE_SIZE" in traffic:
        t = {"phmm_kernel<float,false,false>": int(round((traffic["FETCH_SIZE"] + traffic["WRITE_SIZE"]) * 1024)),
             "_note": "HBM bytes per fp32 forward pass (all hap-length class launches) on the default C2 workload = "
                      "(FETCH_SIZE + WRITE_SIZE) KiB * 1024 from separate rocprofv3 --pmc passes "
                      f"(profiles/{os.path.basename(dst)}/{tag}_pmc_*.csv).  FETCH_SIZE is uncorrected: the gfx950 1/2 "
                      "correction in MI355X_MICROARCH.md applies to 16-B/lane streaming loads; this kernel's reads "
                      "are 1-byte per-lane loads whose calibration is unmeasured.",
             "fetch_kib": traffic["FETCH_SIZE"], "write_kib": traffic["WRITE_SIZE"],
             "launches_per_pass": traffic["FETCH_SIZE_launches"], "source": f"{tag}"}
        json.dump(t, open(os.path.join(os.path.dirname(dst.rstrip("/")), "pmc_traffic.json"), "w"), indent=1)
    print(json.dumps(summary))


if __name__ == "__main__":
    main()

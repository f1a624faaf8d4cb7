"""Concurrency of the PairHMM passes of an `fcs-genome htc` run from a
rocprofv3 --kernel-trace CSV: how much of the time some forward kernel runs
is shared by kernels issued from two or more shard threads.
usage: python tools/htc_overlap.py <run_kernel_trace.csv>"""
import csv
import json
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
fwd = [r for r in rows if any(k in r["Kernel_Name"] for k in ("phmm3_kernel", "phmm2_kernel", "phmm_kernel<"))]
tid_key = "Thread_Id" if fwd and "Thread_Id" in fwd[0] else None
ev = []
for r in fwd:
    t = r.get(tid_key, "0") if tid_key else "0"
    ev.append((int(r["Start_Timestamp"]), 1, t))
    ev.append((int(r["End_Timestamp"]), -1, t))
ev.sort()
active = {}
busy = shared = 0
last = None
for ts, d, t in ev:
    if last is not None and active:
        dt = ts - last
        busy += dt
        if sum(1 for v in active.values() if v > 0) >= 2:
            shared += dt
    active[t] = active.get(t, 0) + d
    if active[t] == 0:
        del active[t]
    last = ts
threads = sorted({r.get(tid_key, "0") for r in fwd}) if tid_key else []
# every PairHMM-pass kernel (schedule, forward, fallback, rescue): their union
# (GPU busy with PairHMM work) against the sum of their durations
pk = [r for r in rows if any(k in r["Kernel_Name"] for k in ("phmm", "onesweep", "radix", "Sort", "sort"))]
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in pk)
union = 0
cur_s = cur_e = None
for a, b in iv:
    if cur_e is None or a > cur_e:
        if cur_e is not None:
            union += cur_e - cur_s
        cur_s, cur_e = a, b
    else:
        cur_e = max(cur_e, b)
if cur_e is not None:
    union += cur_e - cur_s
span = (max(b for _, b in iv) - min(a for a, _ in iv)) if iv else 0
print(json.dumps({"forward_kernels": len(fwd), "issuing_threads": len(threads),
                  "busy_ms": round(busy / 1e6, 3), "multi_thread_overlap_ms": round(shared / 1e6, 3),
                  "overlap_frac": round(shared / busy, 4) if busy else 0.0,
                  "pass_kernels": len(pk), "pass_kernels_sum_ms": round(sum(b - a for a, b in iv) / 1e6, 3),
                  "pass_kernels_union_ms": round(union / 1e6, 3), "first_to_last_ms": round(span / 1e6, 3)}))

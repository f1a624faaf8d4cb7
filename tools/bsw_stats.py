"""Work breakdown of the ksw_extend2 pair waves on C3 (diagnostic build only).

Needs a library built with -DFCS_BSW_STATS (tools/build_alt.sh stats
-DFCS_BSW_STATS) passed as FCSHIP_LIB.  Runs one C3 batch and prints, per
pair bucket (32/64/96/128/152 register columns): waves, rows, fast and masked
(edge) chunks, useful cells (bwa's evaluated cells), working / alive
task-rows and the summed row band-union width, and the derived efficiencies:
  slot_eff  = useful cells / (chunks x 8 columns x 128 tasks)
  edge_frac = masked chunks / all processed chunks
usage: FCSHIP_LIB=alt/stats.so python tools/bsw_stats.py [--reads N]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "falcon-genome_amd"))

import torch  # noqa: E402,F401  (first: one HIP runtime per process)

import bench  # noqa: E402

fcship = bench.load_fcship()
KEYS = ["waves", "rows", "fast_chunks", "masked_chunks", "useful_cells", "work_task_rows", "alive_task_rows",
        "union_width"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=500_000)
    ap.add_argument("--seed", type=int, default=20261015)
    args = ap.parse_args()
    lib = fcship.lib
    rd = lib.fcs_bsw_pair_stats_read
    rd.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    buf = (ctypes.c_ulonglong * 40)()
    t = fcship.synth_bsw(args.seed, args.reads, read_len=151, ref_len=10_000_000, w=100)
    rd(buf, 1)
    fcship.bsw_extend_batch(t)
    assert rd(buf, 1) == 0
    out = {}
    tot = dict.fromkeys(KEYS, 0)
    for bk, nc in enumerate([32, 64, 96, 128, 152]):
        d = {k: int(buf[8 * bk + i]) for i, k in enumerate(KEYS)}
        for k in KEYS:
            tot[k] += d[k]
        out[f"pair{nc}"] = d
    out["total"] = tot
    for d in out.values():
        ch = d["fast_chunks"] + d["masked_chunks"]
        d["slot_eff"] = round(d["useful_cells"] / max(1, ch * 8 * 128), 4)
        d["edge_frac"] = round(d["masked_chunks"] / max(1, ch), 4)
        d["cells_per_work_task_row"] = round(d["useful_cells"] / max(1, d["work_task_rows"]), 2)
        d["work_frac_of_wave_rows"] = round(d["work_task_rows"] / max(1, 128 * d["rows"]), 4)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

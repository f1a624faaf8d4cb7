"""Where the SW lane kernels spend their lanes: runs the bench workloads once on
a stats build (alt/stats.so, bsw_lane.hip compiled with -DFCS_BSW_STATS) and
prints per bucket: rows per wave, fast / masked chunk columns per row, and the
fraction of lane-columns that were useful band cells.
usage: FCSHIP_LIB=$PWD/alt/stats.so python tools/bsw_stats.py [--reads N]"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "falcon-genome_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
import fcship  # noqa: E402

NAMES = ["16", "32", "48", "64", "96", "128", "152", "96b8", "128b8", "152b8"]


def read(reset=True):
    a = (C.c_ulonglong * 128)()
    assert fcship.lib.fcs_bsw_stats_read(a, 1 if reset else 0) == 0
    return [list(a[8 * k: 8 * k + 8]) for k in range(16)]


PAIR_NAMES = ["p32", "p64", "p96", "p128", "p152"]


def read_pair(reset=True):
    a = (C.c_ulonglong * 40)()
    assert fcship.lib.fcs_bsw_pair_stats_read(a, 1 if reset else 0) == 0
    return [list(a[8 * k: 8 * k + 8]) for k in range(5)]


def report_pair(tag, st):
    out = {}
    for k, name in enumerate(PAIR_NAMES):
        waves, rows, fch, mch, useful, work, alive, width = st[k]
        if not waves:
            continue
        cols = 8 * (fch + mch)
        out[name] = {"waves": waves, "rows_per_wave": round(rows / waves, 1),
                     "fast_chunks_per_row": round(fch / rows, 2), "masked_chunks_per_row": round(mch / rows, 2),
                     "band_union_width": round(width / rows, 1),
                     "working_tasks_per_row": round(work / rows, 1), "alive_tasks_per_row": round(alive / rows, 1),
                     "useful_per_task_col": round(useful / (128 * cols), 3) if cols else 0,
                     "cells_per_working_task_row": round(useful / max(work, 1), 1), "cells": useful}
    print(tag, "pair", json.dumps(out, indent=1))


def report(tag, st):
    out = {}
    for k, name in enumerate(NAMES):
        waves, rows, fch, mch, fcol, mcol, useful, lrows = st[k]
        if not waves:
            continue
        cols = fcol + mcol
        out[name] = {"waves": waves, "rows_per_wave": round(rows / waves, 1),
                     "fast_cols_per_row": round(fcol / rows, 1), "masked_cols_per_row": round(mcol / rows, 1),
                     "lane_util_rows": round(lrows / (64 * rows), 3),
                     "useful_per_lane_col": round(useful / (64 * cols), 3) if cols else 0,
                     "useful_per_working_lane_row": round(useful / max(lrows, 1), 1),
                     "cells": useful}
    print(tag, json.dumps(out, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=250_000)
    ap.add_argument("--seed", type=int, default=20261015)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    fcship.lib.fcs_bsw_stats_read.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    fcship.lib.fcs_bsw_pair_stats_read.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    for which in ("c3", "fixed"):
        if which == "c3":
            t = fcship.synth_bsw(args.seed, args.reads, read_len=151, ref_len=10_000_000, w=100)
        else:
            t = fcship.synth_bsw(args.seed, 2 * args.reads, read_len=151, ref_len=10_000_000, w=100, mode=1,
                                 fixed_q=151, fixed_t=251)
        read()
        read_pair()
        args.reps = 1
        bench.bench_bsw(args, dev, t, reps=1)
        report(which, read())
        report_pair(which, read_pair())


if __name__ == "__main__":
    main()

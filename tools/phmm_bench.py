"""PairHMM-only timing (C2 shape) for A/B runs of alternative builds.
usage: python tools/phmm_bench.py [--pairs N] [--reps K] [--exact]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "falcon-genome_amd"))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--seed", type=int, default=20261015)
    args = ap.parse_args()
    bench.load_fcship()
    rk = bench.Ranks(False)
    ph = bench.bench_phmm(args, rk.dev, rk)
    print(json.dumps({"gcups": round(ph["cells"] * args.steps / ph["elapsed"] / 1e9, 1),
                      "fwd_ms": round(ph["fwd_ms"], 3), "kernel_gcups": round(ph["cells"] / ph["fwd_ms"] / 1e6, 1)}))


if __name__ == "__main__":
    main()

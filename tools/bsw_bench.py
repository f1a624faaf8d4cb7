"""SW-only timing for profiling runs: the two ksw_extend2 workloads of bench.py
(C3 seed extensions and the fixed 151x251 case), nothing else on the GPU.

usage: python tools/bsw_bench.py [--reads N] [--which c3|fixed|both]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "falcon-genome_amd"))

import torch  # noqa: E402  (first: one HIP runtime per process)

import bench  # noqa: E402

fcship = bench.load_fcship()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=500_000)
    ap.add_argument("--seed", type=int, default=20261015)
    ap.add_argument("--which", default="both", choices=["c3", "fixed", "both", "global", "align", "align16"])
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    out = {}
    if args.which in ("c3", "both"):
        t = fcship.synth_bsw(args.seed, args.reads, read_len=151, ref_len=10_000_000, w=100)
        r = bench.bench_bsw(args, dev, t, reps=args.reps)
        out["c3"] = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items() if not hasattr(v, "shape")}
    if args.which in ("fixed", "both"):
        t = fcship.synth_bsw(args.seed, 2 * args.reads, read_len=151, ref_len=10_000_000, w=100, mode=1,
                             fixed_q=151, fixed_t=251)
        r = bench.bench_bsw(args, dev, t, reps=args.reps)
        out["fixed"] = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items() if not hasattr(v, "shape")}
    if args.which == "global":  # bench.py's ksw_global2 workload, scores + CIGARs (reps + 1 runs each)
        t = fcship.synth_bsw(args.seed + 2, args.reads // 2, read_len=151, ref_len=10_000_000, w=16, mode=1,
                             fixed_q=151, fixed_t=151)
        out["global"] = bench.bench_bsw_global(args, dev, t, reps=args.reps)
    if args.which in ("align", "align16"):  # bench.py's ksw_align2 (mate rescue) workload, u8 or i16 tasks
        t = fcship.synth_bsw(args.seed + 3, args.reads // 4, read_len=151, ref_len=10_000_000, w=100, mode=1,
                             fixed_q=151, fixed_t=600)
        xt = 0x40000 | 0x80000 | (0x10000 if args.which == "align" else 0) | 19
        r = bench.bench_bsw_align(args, dev, t, xt, reps=args.reps)
        out[args.which] = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()
                           if not hasattr(v, "shape")}
    print(json.dumps(out))


if __name__ == "__main__":
    main()

#!/bin/bash
# A/B timings of the streamed PairHMM kernel: in-tree (auto K), forced K, and
# the alt/ builds (timing only).  usage: tools/ab_stream.sh TAG [K values...]
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-abs}; mkdir -p $O; shift
b() { timeout -k 10 300 python tools/phmm_bench.py 2>/dev/null | tail -1; }
echo "in-tree: $(b)" | tee -a $O/ab.log || exit 1
for k in "$@"; do echo "K=$k: $(FCSHIP_STREAM_K=$k b)" | tee -a $O/ab.log || exit 1; done
for f in alt/*.so; do echo "$f: $(FCSHIP_LIB=$PWD/$f b)" | tee -a $O/ab.log || exit 1; done
echo "in-tree again: $(b)" | tee -a $O/ab.log

#!/bin/bash
# Timing-only A/B (diagnostic builds whose results are wrong by design): the
# in-tree libfcship.so against every alt/*.so, interleaved three times.
# usage: tools/ab_time.sh phmm|bsw TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
WHICH=$1; O=gpurun_out/$2; mkdir -p "$O"
case $WHICH in
  phmm) BENCH="python tools/phmm_bench.py" ;;
  bsw) BENCH="python tools/bsw_bench.py" ;;
  *) echo "usage: $0 phmm|bsw TAG"; exit 2 ;;
esac
for pass in 1 2 3; do
  echo "in-tree: $(timeout -k 10 300 $BENCH 2>/dev/null | tail -1)" | tee -a "$O/ab.log" || exit 1
  for f in alt/*.so; do
    [ -e "$f" ] || continue
    echo "$f: $(FCSHIP_LIB=$PWD/$f timeout -k 10 300 $BENCH 2>/dev/null | tail -1)" | tee -a "$O/ab.log" || exit 1
  done
done

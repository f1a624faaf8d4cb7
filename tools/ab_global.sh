#!/bin/bash
# ksw_global2 A/B on the GPU box: bench.py's global workload (scores pass and
# CIGAR pass) with the in-tree libfcship.so against each alt/*.so given,
# interleaved three times, then the SW / seed-extension / host GPU tests of
# the in-tree build.   usage: tools/ab_global.sh TAG alt/X.so [...]
set -u
O=gpurun_out/$1; shift; mkdir -p $O
for i in 1 2 3; do
  echo "in-tree: $(timeout -k 10 300 python tools/bsw_bench.py --which global 2>/dev/null | tail -1)" | tee -a $O/ab.log || exit 1
  for f in "$@"; do
    echo "$f: $(FCSHIP_LIB=$PWD/$f timeout -k 10 300 python tools/bsw_bench.py --which global 2>/dev/null | tail -1)" | tee -a $O/ab.log || exit 1
  done
done
timeout -k 10 600 python -u -m pytest tests/test_bsw_gpu.py tests/test_seedext_gpu.py tests/test_host_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; exit $rc

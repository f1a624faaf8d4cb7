#!/bin/bash
# C2 PairHMM step with the bin schedule (default) against the rocPRIM radix
# schedule (FCS_PHMM_SCHEDULE=radix), interleaved three times.
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
for pass in 1 2 3; do
  echo "bins:  $(timeout -k 10 300 python tools/phmm_bench.py 2>/dev/null | tail -1)" || exit 1
  echo "radix: $(FCS_PHMM_SCHEDULE=radix timeout -k 10 300 python tools/phmm_bench.py 2>/dev/null | tail -1)" || exit 1
done

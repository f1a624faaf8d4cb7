#!/bin/bash
# A/B timing of kernel variants on the GPU box: the in-tree libfcship.so
# against every alt/*.so (built by tools/build_alt.sh), interleaved twice, then
# the GPU parity tests of each variant (FCSHIP_LIB) — a variant that fails
# parity is reported as such, whatever its time.
# usage: tools/ab.sh phmm|bsw TAG [alt/X.so ...]   (default: every alt/*.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
WHICH=$1; O=gpurun_out/$2; mkdir -p "$O"
shift 2
VARIANTS=("$@")
[ ${#VARIANTS[@]} -gt 0 ] || VARIANTS=(alt/*.so)
case $WHICH in
  phmm) BENCH="python tools/phmm_bench.py"; TESTS=tests/test_pairhmm_gpu.py ;;
  bsw) BENCH="python tools/bsw_bench.py"; TESTS="tests/test_bsw_gpu.py tests/test_seedext_gpu.py" ;;
  *) echo "usage: $0 phmm|bsw TAG"; exit 2 ;;
esac
for pass in 1 2; do
  echo "in-tree: $(timeout -k 10 300 $BENCH 2>/dev/null | tail -1)" | tee -a "$O/ab.log" || exit 1
  for f in "${VARIANTS[@]}"; do
    [ -e "$f" ] || continue
    echo "$f: $(FCSHIP_LIB=$PWD/$f timeout -k 10 300 $BENCH 2>/dev/null | tail -1)" | tee -a "$O/ab.log" || exit 1
  done
done
timeout -k 10 600 python -u -m pytest $TESTS -q -x -p no:cacheprovider --timeout 120 --timeout-method thread \
  > "$O/pytest_in_tree.log" 2>&1
rc=$?
echo "in-tree parity rc=$rc: $(tail -1 "$O/pytest_in_tree.log")" | tee -a "$O/ab.log"
[ $rc -le 1 ] || exit $rc
for f in "${VARIANTS[@]}"; do
  [ -e "$f" ] || continue
  FCSHIP_LIB=$PWD/$f timeout -k 10 600 python -u -m pytest $TESTS -q -x -p no:cacheprovider --timeout 120 \
    --timeout-method thread > "$O/pytest_$(basename "$f" .so).log" 2>&1
  rc=$?
  echo "$f parity rc=$rc: $(tail -1 "$O/pytest_$(basename "$f" .so).log")" | tee -a "$O/ab.log"
  [ $rc -le 1 ] || exit $rc
done

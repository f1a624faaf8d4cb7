# A/B of SW builds under alt/ against the in-tree one, then GPU SW parity of
# every alt build (FCSHIP_LIB) — an alternative kernel is only worth timing if exact.
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-aba}; mkdir -p $O
echo "in-tree: $(timeout -k 10 300 python tools/bsw_bench.py 2>/dev/null | tail -1)" | tee -a $O/ab.log || exit 1
for f in alt/*.so; do
  echo "$f: $(FCSHIP_LIB=$PWD/$f timeout -k 10 300 python tools/bsw_bench.py 2>/dev/null | tail -1)" | tee -a $O/ab.log || exit 1
done
echo "in-tree again: $(timeout -k 10 300 python tools/bsw_bench.py 2>/dev/null | tail -1)" | tee -a $O/ab.log || exit 1
for f in alt/*.so; do
  FCSHIP_LIB=$PWD/$f timeout -k 10 600 python -m pytest tests/test_bsw_gpu.py -q -x -p no:cacheprovider > $O/pytest_$(basename $f .so).log 2>&1; rc=$?
  echo "$f parity: $(tail -1 $O/pytest_$(basename $f .so).log)"
  [ $rc -eq 0 ] || exit $rc
done

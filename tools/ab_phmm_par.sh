# A/B of PairHMM builds under alt/ against the in-tree one, each alt build also
# run through the PairHMM GPU parity tests.  usage: tools/ab_phmm_par.sh TAG
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-abp}; mkdir -p $O
echo "base(in-tree): $(timeout -k 10 300 python tools/phmm_bench.py 2>/dev/null | tail -1)" | tee -a $O/ab.log || exit 1
for f in alt/*.so; do
  n=$(basename $f .so)
  FCSHIP_LIB=$PWD/$f timeout -k 10 300 python -m pytest tests/test_pairhmm_gpu.py -q -x -p no:cacheprovider > $O/pytest_$n.log 2>&1
  rc=$?
  echo "$f parity rc=$rc: $(tail -1 $O/pytest_$n.log)" | tee -a $O/ab.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  echo "$f: $(FCSHIP_LIB=$PWD/$f timeout -k 10 300 python tools/phmm_bench.py 2>/dev/null | tail -1)" | tee -a $O/ab.log || exit 1
done
echo "in-tree again: $(timeout -k 10 300 python tools/phmm_bench.py 2>/dev/null | tail -1)" | tee -a $O/ab.log

# A/B of SW builds under alt/ against the in-tree one; then GPU SW parity of the in-tree build.
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-abs}; mkdir -p $O
echo "in-tree: $(timeout -k 10 300 python tools/bsw_bench.py 2>/dev/null | tail -1)" | tee -a $O/ab.log || exit 1
for f in alt/*.so; do
  echo "$f: $(FCSHIP_LIB=$PWD/$f timeout -k 10 300 python tools/bsw_bench.py 2>/dev/null | tail -1)" | tee -a $O/ab.log || exit 1
done
echo "in-tree again: $(timeout -k 10 300 python tools/bsw_bench.py 2>/dev/null | tail -1)" | tee -a $O/ab.log || exit 1
timeout -k 10 600 python -m pytest tests/test_bsw_gpu.py -q -x -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; exit $rc

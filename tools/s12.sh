set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/s12; mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bsw_bench.py > $O/bsw.log 2>&1; rc=$?; tail -1 $O/bsw.log; exit $rc

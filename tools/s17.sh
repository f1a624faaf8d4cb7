set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/s17; mkdir -p $O
timeout -k 10 900 python -m pytest tests/test_host_gpu.py -q -x -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -40 $O/pytest.log; exit $rc

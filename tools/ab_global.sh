set -u
O=gpurun_out/r6g; mkdir -p $O
for i in 1 2 3; do
  echo "in-tree: $(timeout -k 10 300 python tools/bsw_bench.py --which global 2>/dev/null | tail -1)" | tee -a $O/ab.log || exit 1
  echo "alt/glane_bfe: $(FCSHIP_LIB=$PWD/alt/glane_bfe.so timeout -k 10 300 python tools/bsw_bench.py --which global 2>/dev/null | tail -1)" | tee -a $O/ab.log || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_bsw_gpu.py tests/test_seedext_gpu.py tests/test_host_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; exit $rc

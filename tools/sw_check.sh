# SW parity of the in-tree build, then the SW-only bench (C3 + fixed).
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-swc}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_bsw_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bsw_bench.py > $O/bench.log 2>&1; rc=$?
tail -1 $O/bench.log
[ $rc -eq 0 ] || exit $rc
# optional: per-kernel times of the C3 run
if [[ "${2:-}" == *prof* ]]; then
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/bsw_bench.py --which c3 --reps 2 > $O/prof.log 2>&1 || exit 1
  python3 - $O/prof/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'bsw' in r['Name']:
        print(r['Name'].split('(')[0][:60], r['Calls'], round(float(r['AverageNs'])/1e6, 3), 'ms avg')
PY
fi
if [[ "${2:-}" == *pmc* ]]; then
  export TMPDIR=/tmp
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS -d $O/pmc -o run --output-format csv -- python3 tools/bsw_bench.py --which c3 --reps 1 > $O/pmc.log 2>&1 || exit 1
  python3 tools/pmc_kernels.py $O/pmc bsw_
fi
if [[ "${2:-}" == *stall* ]]; then
  export TMPDIR=/tmp
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC -d $O/pmc2 -o run --output-format csv -- python3 tools/bsw_bench.py --which c3 --reps 1 > $O/pmc2.log 2>&1 || exit 1
  python3 tools/pmc_kernels.py $O/pmc2 bsw_
  timeout -k 10 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ -d $O/pmc3 -o run --output-format csv -- python3 tools/bsw_bench.py --which c3 --reps 1 > $O/pmc3.log 2>&1 || exit 1
  python3 tools/pmc_kernels.py $O/pmc3 bsw_
fi
if [[ "${2:-}" == *valu* ]]; then
  export TMPDIR=/tmp
  for w in c3 fixed; do
    timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU -d $O/valu_$w -o run --output-format csv -- python3 tools/bsw_bench.py --which $w --reps 1 > $O/valu_$w.log 2>&1 || exit 1
  done
fi
exit 0

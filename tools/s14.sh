set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/s14; mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/bsw_bench.py --reps 2 > $O/prof.log 2>&1; rc=$?
tail -1 $O/prof.log; exit $rc

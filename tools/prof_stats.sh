set -u
OUT=gpurun_out/$1; mkdir -p $OUT; export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-bsw > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1
rc=$?; echo rc=$rc; cd $GRAFT_REPO_ROOT
f=$(find $OUT/prof -name '*kernel_stats.csv' | head -1); echo $f; cut -d, -f1-8 $f | head -30

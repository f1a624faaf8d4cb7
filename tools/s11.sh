set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/s11; mkdir -p $O
bash tools/gpu_session.sh s11 tests benchq || exit 1
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || true
timeout -k 10 300 python tools/bsw_bench.py --which fixed --reads 250000 > $O/bsw_fixed.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVES -d $O/pmc_valu -o run --output-format csv -- python3 tools/bsw_bench.py --which fixed --reads 250000 --reps 1 > $O/pmc_valu.log 2>&1
echo rc=$?

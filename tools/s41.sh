# PairHMM LDS PMC of the in-tree build and of alt/*.so
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/s41; mkdir -p $O
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_BUSY_CU_CYCLES -d $O/in -o run --output-format csv -- python3 tools/phmm_bench.py --pairs 300000 --steps 1 --warmup 0 > $O/in.log 2>&1 || exit 1
for f in alt/*.so; do b=$(basename $f .so)
FCSHIP_LIB=$PWD/$f timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_BUSY_CU_CYCLES -d $O/$b -o run --output-format csv -- python3 tools/phmm_bench.py --pairs 300000 --steps 1 --warmup 0 > $O/$b.log 2>&1 || exit 1
done
echo done

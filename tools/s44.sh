# SW PMC (VALU/SALU instructions, busy cycles) for the in-tree build and alt/*.so
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/s44; mkdir -p $O
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES -d $O/in -o run --output-format csv -- python3 tools/bsw_bench.py --reads 250000 --reps 1 > $O/in.log 2>&1 || exit 1
for f in alt/*.so; do b=$(basename $f .so)
FCSHIP_LIB=$PWD/$f timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES -d $O/$b -o run --output-format csv -- python3 tools/bsw_bench.py --reads 250000 --reps 1 > $O/$b.log 2>&1 || exit 1
done
echo done

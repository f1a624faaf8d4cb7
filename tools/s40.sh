# PairHMM PMC: LDS vs VALU activity of the forward kernel
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/s40; mkdir -p $O
timeout -k 10 120 rocprofv3 -L > $O/list.txt 2>&1 || true
for c in SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VALU SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_VALU SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_ACTIVE_INST_SCA; do grep -q "$c" $O/list.txt && echo $c; done > $O/have.txt
cat $O/have.txt
P=$(head -4 $O/have.txt | tr '\n' ' ')
Q=$(sed -n 5,8p $O/have.txt | tr '\n' ' ')
R=$(sed -n 9,12p $O/have.txt | tr '\n' ' ')
timeout -k 10 300 rocprofv3 --pmc $P -d $O/p1 -o run --output-format csv -- python3 tools/phmm_bench.py --pairs 300000 --steps 1 --warmup 0 > $O/p1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc $Q -d $O/p2 -o run --output-format csv -- python3 tools/phmm_bench.py --pairs 300000 --steps 1 --warmup 0 > $O/p2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc $R SQ_WAVE_CYCLES -d $O/p3 -o run --output-format csv -- python3 tools/phmm_bench.py --pairs 300000 --steps 1 --warmup 0 > $O/p3.log 2>&1
echo rc=$?

#!/bin/bash
# PairHMM C2 forward pass under rocprofv3 PMC passes (one pass per run, each
# within the per-block slot limits: <= 8 SQ, <= 2 GRBM), then HBM bytes.
# usage: tools/pmc_phmm_r3.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1; mkdir -p "$OUT"; export TMPDIR=/tmp
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- \
    python3 tools/phmm_bench.py --steps 1 --warmup 1 > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
pass sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT
pass sq2 SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA \
  SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU
pass sq3 SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_INST_LEVEL_LDS SQ_LDS_IDX_ACTIVE SQ_THREAD_CYCLES_VALU \
  SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_FMA_F32
pass sq4 SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_LEVEL_VMEM \
  SQ_INST_CYCLES_VMEM_RD SQ_LEVEL_WAVES SQ_IFETCH
pass fetch FETCH_SIZE
pass write WRITE_SIZE
for d in sq1 sq2 sq3 sq4 fetch write; do python3 tools/pmc_kernels.py "$OUT/$d" phmm; done > "$OUT/summary.txt"
cat "$OUT/summary.txt"

#!/bin/bash
# One bounded GPU session on the gpurun box: parity tests, smoke, bench, and
# rocprofv3 kernel-trace / PMC passes.  Every GPU step has its own time limit
# and the script stops at the first failing step (no retries).
# usage: tools/gpu_session.sh TAG [info] [tests] [smoke] [bench] [prof] [pmc]
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))" | tee -a "$OUT/session.log"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/session.log"
  tail -3 "$OUT/$name.log" | tee -a "$OUT/session.log"
  if [ $rc -ne 0 ]; then echo "STOP after $name" | tee -a "$OUT/session.log"; exit $rc; fi
}
for step in "$@"; do
  case $step in
    info) run info 60 bash -c 'nproc; free -g; df -h /tmp /dev/shm "$0"; rocm-smi --showuse --showmemuse | head -20' "$ROOT" ;;
    tests) run pytest_gpu 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 900 python bench.py ;;
    benchq) run benchq 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e ;;
    prof) run prof 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
            python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-e2e ;;
    pmc) run pmc 900 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- \
            python3 "$ROOT/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-bsw --no-e2e &&
         run pmc2 900 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- \
            python3 "$ROOT/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-bsw --no-e2e ;;
    bswpmc)  # SW: SQ issue/stall counters for C3 and fixed, HBM bytes for C3 (separate passes)
      SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
      run bswpmc_c3 300 rocprofv3 --pmc $SQ -d "$OUT/bswpmc_c3" -o run --output-format csv -- \
            python3 "$ROOT/tools/bsw_bench.py" --which c3 --reps 1 &&
      run bswpmc_fixed 300 rocprofv3 --pmc $SQ -d "$OUT/bswpmc_fixed" -o run --output-format csv -- \
            python3 "$ROOT/tools/bsw_bench.py" --which fixed --reps 1 &&
      run bswpmc_c3_fetch 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/bswpmc_c3_fetch" -o run --output-format csv -- \
            python3 "$ROOT/tools/bsw_bench.py" --which c3 --reps 1 &&
      run bswpmc_c3_write 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/bswpmc_c3_write" -o run --output-format csv -- \
            python3 "$ROOT/tools/bsw_bench.py" --which c3 --reps 1 &&
      run bswpmc_global 300 rocprofv3 --pmc $SQ -d "$OUT/bswpmc_global" -o run --output-format csv -- \
            python3 "$ROOT/tools/bsw_bench.py" --which global --reps 1 &&
      run bswpmc_align 300 rocprofv3 --pmc $SQ -d "$OUT/bswpmc_align" -o run --output-format csv -- \
            python3 "$ROOT/tools/bsw_bench.py" --which align --reps 1 ;;
    globalpmc)  # ksw_global2 only (scores + CIGAR passes): SQ issue counters
      SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
      run bswpmc_global 300 rocprofv3 --pmc $SQ -d "$OUT/bswpmc_global" -o run --output-format csv -- \
            python3 "$ROOT/tools/bsw_bench.py" --which global --reps 1 ;;
    globalprof)  # ksw_global2 only: per-kernel durations (scores pass, direction-row DP, traceback)
      run globalprof 300 rocprofv3 --kernel-trace --stats -d "$OUT/globalprof" -o run --output-format csv -- \
            python3 "$ROOT/tools/bsw_bench.py" --which global ;;
    bgzfprof)  # BGZF inflate kernel: kernel trace + stats of the microbench (4,096 BAM-like members)
      run bgzfprof 300 rocprofv3 --kernel-trace --stats -d "$OUT/bgzfprof" -o run --output-format csv -- \
            python3 "$ROOT/tools/bgzf_bench.py" --reps 5 ;;
    bgzfpmc)  # BGZF inflate kernel: SQ counters (tools/pmc_bgzf.sh)
      run bgzfpmc 600 bash "$ROOT/tools/pmc_bgzf.sh" "$OUT/bgzfpmc" ;;
    e2eprobe)  # htc timeline at the bench's 31 Mbp (tools/e2e_probe.sh, htc only)
      run e2eprobe 900 env MBP=31 HTC_ONLY=1 bash "$ROOT/tools/e2e_probe.sh" ;;
    alignpmc)  # ksw_align2 only: SQ issue counters of one batch
      SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
      run bswpmc_align 300 rocprofv3 --pmc $SQ -d "$OUT/bswpmc_align" -o run --output-format csv -- \
            python3 "$ROOT/tools/bsw_bench.py" --which align --reps 1 ;;
    phmmpmc)  # PairHMM C2 forward pass: SQ issue/stall counters, then HBM bytes (separate passes)
      run phmmpmc_sq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
            SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d "$OUT/phmmpmc_sq" -o run --output-format csv -- \
            python3 "$ROOT/tools/phmm_bench.py" --steps 1 --warmup 1 &&
      run phmmpmc_sq2 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU \
            SQ_LDS_BANK_CONFLICT -d "$OUT/phmmpmc_sq2" -o run --output-format csv -- \
            python3 "$ROOT/tools/phmm_bench.py" --steps 1 --warmup 1 &&
      run phmmpmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/phmmpmc_fetch" -o run --output-format csv -- \
            python3 "$ROOT/tools/phmm_bench.py" --steps 1 --warmup 1 &&
      run phmmpmc_write 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/phmmpmc_write" -o run --output-format csv -- \
            python3 "$ROOT/tools/phmm_bench.py" --steps 1 --warmup 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== session done" | tee -a "$OUT/session.log"

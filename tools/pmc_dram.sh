#!/bin/bash
# L2 memory-side requests vs the DRAM-bound ones for the C3 ksw_extend2 batch
# and the C2 PairHMM pass.  FETCH_SIZE tallies every L2 miss, Infinity-Cache
# (MALL) hits included (MI355X_MICROARCH.md, HBM section); the *_DRAM request
# counters, when the box's rocprofv3 lists them, count only the requests that
# went on to HBM.  One counter block per pass, each pass under its own limit.
# usage: tools/pmc_dram.sh TAG
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$1
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1
grep -o 'TCC_[A-Z0-9_]*' "$OUT/avail.txt" | sort -u > "$OUT/tcc_counters.txt"
want=""
for c in TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_DRAM_sum; do
  base=${c%_sum}
  grep -qx "$base" "$OUT/tcc_counters.txt" && want="$want $c"
done
echo "counters:$want" | tee "$OUT/session.log"
[ -n "$want" ] || exit 0
# two passes of at most two TCC counters each (read pair, write pair)
rd=$(echo $want | tr ' ' '\n' | grep RDREQ | tr '\n' ' ')
wr=$(echo $want | tr ' ' '\n' | grep WRREQ | tr '\n' ' ')
for w in c3; do
  timeout -s KILL 120 rocprofv3 --pmc $rd -d "$OUT/bsw_rd" -o run --output-format csv -- \
    python3 "$ROOT/tools/bsw_bench.py" --which $w --reps 1 > "$OUT/bsw_rd.log" 2>&1 || exit $?
  if [ -n "$wr" ]; then
    timeout -s KILL 120 rocprofv3 --pmc $wr -d "$OUT/bsw_wr" -o run --output-format csv -- \
      python3 "$ROOT/tools/bsw_bench.py" --which $w --reps 1 > "$OUT/bsw_wr.log" 2>&1 || exit $?
  fi
done
timeout -s KILL 120 rocprofv3 --pmc $rd -d "$OUT/phmm_rd" -o run --output-format csv -- \
  python3 "$ROOT/tools/phmm_bench.py" --steps 1 --warmup 1 > "$OUT/phmm_rd.log" 2>&1 || exit $?
echo "done" | tee -a "$OUT/session.log"

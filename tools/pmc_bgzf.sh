#!/bin/bash
# SQ issue counters of the inflate kernel (tools/bgzf_bench.py, BAM-like and
# GVCF batches of 4096 members), one rocprofv3 pass per counter set.
OUT=${1:-gpurun_out/pmc_bgzf}
mkdir -p "$OUT"
for kind in bam gvcf; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES \
    SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d "$OUT/sq_$kind" -o run --output-format csv -- \
    python3 tools/bgzf_bench.py --kind $kind --reps 1 > "$OUT/sq_$kind.log" 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INST_CYCLES_SALU \
    SQ_ACTIVE_INST_LDS -d "$OUT/sq2_$kind" -o run --output-format csv -- \
    python3 tools/bgzf_bench.py --kind $kind --reps 1 > "$OUT/sq2_$kind.log" 2>&1 || exit 1
done
for f in $(find "$OUT" -name "*counter_collection.csv"); do
  echo "== $f"
  python3 - "$f" <<'PY'
import csv, sys, collections
tot = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if "bgzf_inflate" in r.get("Kernel_Name", ""):
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(tot.items()):
    print(f"  {k} {v:.4g}")
PY
done

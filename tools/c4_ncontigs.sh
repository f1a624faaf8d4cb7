#!/bin/bash
# The C4 job's host side vs its shard count: fcs-genome htc over a synthetic
# genome directory G (ref.fasta + sample.bam) on the CPU mock with placeholder
# likelihoods (FCS_MOCK_PHMM=1: no PairHMM work, every other stage as on the
# GPU path), T host threads = shard threads, gatk.ncontigs = each N given.
# Prints wall, the Haplotype Caller stage, the VCF tail and the shards' stage
# thread-seconds (longest shard too).
#   tools/c4_ncontigs.sh G T N1 [N2 ...]
set -u
G=$1; T=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
X=$ROOT/falcon-genome_amd/bin/fcs-genome
make -s -C "$ROOT/tests/cpu_mock" > /dev/null
W=$(mktemp -d /tmp/c4n.XXXX)
export LD_LIBRARY_PATH=$ROOT/tests/cpu_mock/build:${LD_LIBRARY_PATH:-} FCS_MOCK_PHMM=1 FCS_GPU_PHMM_COMBINE_MS=0
export FCS_TEMP_DIR=$W FCS_HOST_THREADS=$T FCS_GATK_NPROCS=$T FCS_GPU_DEVICES=0 FCS_TIMELINE=1
for N in "$@"; do
  rm -rf "$W/log"
  s=$(date +%s.%N)
  FCS_GATK_NCONTIGS=$N FCS_LOG_DIR=$W/log $X htc -f -r "$G/ref.fasta" -i "$G/sample.bam" -o "$W/out.g.vcf" 2> "$W/err" || { tail -5 "$W/err"; exit 1; }
  e=$(date +%s.%N)
  hc=$(grep -o "Haplotype Caller finishes in [0-9.]* seconds" "$W/err" | grep -o "[0-9.]*" | head -1)
  tail_s=$(grep -o "concat + bgzip + tabix finishes in [0-9.]* seconds" "$W/err" | grep -o "[0-9.]*" | head -1)
  echo "== ncontigs $N threads $T: wall $(awk -v a="$s" -v b="$e" "BEGIN{printf \"%.2f\", b - a}") s, Haplotype Caller stage ${hc} s, VCF tail ${tail_s:-?} s"
  grep -h "htc\] shard" "$W"/log/*.log | awk '{for(i=1;i<=NF;i++){ if($i=="reads,") r+=$(i-1); if($i=="decode"){d+=$(i+1)} if($i=="pileup"){p+=$(i+1)} if($i=="regions"&&$(i+2)=="s,"){g+=$(i+1)} if($i=="output"){o+=$(i+1)} if($i=="calls,"){t=$(i+1); sub(/^\(/,"",t)} } n++; if ($0 ~ / s \(PairHMM/) { match($0, /calls, [0-9.]+ s/); v=substr($0, RSTART+7, RLENGTH-9)+0; s+=v; if (v>mx) mx=v } } END{printf "   shards %d, shard thread-s %.1f (longest %.2f s): decode %.1f pileup %.1f regions %.1f output %.1f\n", n, s, mx, d, p, g, o}'
done
rm -rf "$W"

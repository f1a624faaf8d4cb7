#!/bin/bash
# align wall time on one GPU with 1, 2 and 4 device slots (the same device
# repeated in FCS_GPU_DEVICES): host stages of one chunk overlap another's GPU rounds.
# usage: tools/align_slots.sh TAG
set -eu
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1; mkdir -p "$OUT"; export TMPDIR=/tmp
W=$(mktemp -d /tmp/aslots.XXXX)
B=falcon-genome_amd/bin/fcs-genome
timeout -k 10 300 $B synth -o $W/a -c chr1:4000000 -x 30 --no-fastq --paired 350 --seed 1 > /dev/null 2>&1
timeout -k 10 300 $B index -r $W/a/ref.fasta --sa-intv 32 > /dev/null 2>&1
for devs in 0 0,0 0,0,0,0 0; do
  t0=$(date +%s.%N)
  FCS_GPU_DEVICES=$devs timeout -k 10 300 $B align -f -r $W/a/ref.fasta -1 $W/a/sample_1.fastq -2 $W/a/sample_2.fastq \
    -o $W/aln.bam > $OUT/align_$devs.log 2>&1
  t1=$(date +%s.%N)
  echo "slots $devs wall $(python3 -c "print(round($t1 - $t0, 2))") s: $(grep -o 'phases.*' $OUT/align_$devs.log | head -1)"
done | tee $OUT/slots.txt
rm -rf $W

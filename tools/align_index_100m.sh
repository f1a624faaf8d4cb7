#!/bin/bash
# VERDICT r2 #7 evidence: a 100 Mbp synthetic reference, its FMD index saved
# once (`fcs-genome index`, sampled SA at bwa's interval 32), then `align`
# mapping that index for 1M paired reads on the GPU.  usage: tools/align_index_100m.sh TAG
set -eu
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1; mkdir -p "$OUT"; export TMPDIR=/tmp
W=$(mktemp -d /tmp/r100.XXXX)
B=falcon-genome_amd/bin/fcs-genome
timeout -k 10 300 $B synth -o $W/d -c chr1:60000000,chr2:40000000 -x 1.5 --paired 350 --no-fastq --seed 3 > $OUT/synth.log 2>&1
( time timeout -k 10 600 $B index -r $W/d/ref.fasta --sa-intv 32 ) > $OUT/index.log 2>&1
ls -la $W/d/ref.fasta.fcsidx >> $OUT/index.log
for i in 1 2; do
  ( time timeout -k 10 600 $B align -f -r $W/d/ref.fasta -1 $W/d/sample_1.fastq -2 $W/d/sample_2.fastq -o $W/a.bam ) > $OUT/align_$i.log 2>&1
done
rm -rf $W
grep -h "fcs-genome align\|fcs-genome index\|real" $OUT/index.log $OUT/align_*.log

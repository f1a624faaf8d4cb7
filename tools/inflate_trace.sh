#!/bin/bash
# One htc run at 31 Mbp with GPU window inflate and the per-call phase trace.
W=$(mktemp -d /tmp/inftr.XXXX)
export FCS_TIMELINE=1 FCS_GPU_DEVICES=0 FCS_TEMP_DIR=$W FCS_GATK_NPROCS=${NPROCS:-16} FCS_LOG_DIR=$W/log
B=$GRAFT_REPO_ROOT/falcon-genome_amd/bin/fcs-genome
timeout 300 $B synth -o $W/d -c chr1:31000000 -x 30 --tumor --noisy-frac 0.01 --paired 350 > /dev/null || exit 1
for i in 1 2 3 4; do
  rm -rf $W/log
  FCS_GPU_BAM_INFLATE=true FCS_BGZF_TRACE=1 timeout 300 $B htc -f -r $W/d/ref.fasta -i $W/d/sample.bam -o $W/h.g.vcf 2> $W/htc.err || { tail -5 $W/htc.err; grep -rh "E::\|rror\|ail" $W/log | head -8; exit 1; }
  echo "== run $i"; grep -E "timeline\] exit" $W/htc.err; grep "fcs_bgzf_inflate" $W/htc.err | head -40
done
rm -rf $W

#!/bin/bash
# Where an htc run's wall goes after its last output: the same 31 Mbp htc with
# the GPU library (devices released beside the VCF tail, and not), and with the
# CPU mock (tests/cpu_mock, no GPU runtime), each timed by the shell and by the
# binary's own timeline.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
W=$(mktemp -d /tmp/exitp.XXXX)
export FCS_TIMELINE=1 FCS_GPU_DEVICES=0 FCS_LOG_DIR=$W/log FCS_TEMP_DIR=$W FCS_GATK_NPROCS=16
B=$R/falcon-genome_amd/bin/fcs-genome
timeout 300 $B synth -o $W/d -c chr1:${MBP:-31}000000 -x 30 --no-fastq > /dev/null 2>&1 || exit 1
for mode in gpu gpu-norelease mock gpu gpu-norelease mock; do
  rm -rf $W/log
  if [ $mode = mock ]; then
    { time LD_LIBRARY_PATH=$R/tests/cpu_mock/build FCS_MOCK_PHMM=gkl timeout 300 $B htc -f -r $W/d/ref.fasta -i $W/d/sample.bam -o $W/o.g.vcf 2> $W/err; } 2> $W/time || exit 1
  elif [ $mode = gpu-norelease ]; then
    { time FCS_GPU_RELEASE_EARLY=false timeout 300 $B htc -f -r $W/d/ref.fasta -i $W/d/sample.bam -o $W/o.g.vcf 2> $W/err; } 2> $W/time || exit 1
  else
    { time timeout 300 $B htc -f -r $W/d/ref.fasta -i $W/d/sample.bam -o $W/o.g.vcf 2> $W/err; } 2> $W/time || exit 1
  fi
  echo "$mode: $(grep -E 'exit' $W/err | tail -1) | $(grep real $W/time)"
done
rm -rf $W

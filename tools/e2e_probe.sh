#!/bin/bash
# Wall-time probe of the e2e commands on a GPU box (stage lines from stderr).
echo "cpu quota: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null); THP: $(cat /sys/kernel/mm/transparent_hugepage/enabled 2>/dev/null); nproc $(nproc)"
W=$(mktemp -d /tmp/e2e.XXXX)
export FCS_TIMELINE=1 FCS_GPU_DEVICES=0 FCS_LOG_DIR=$W/log FCS_TEMP_DIR=$W FCS_GATK_NPROCS=${NPROCS:-16}
MBP=${MBP:-4}
B=$GRAFT_REPO_ROOT/falcon-genome_amd/bin/fcs-genome
t() { local s=$(date +%s.%N); "$@"; local rc=$?; echo "  wall $(awk "BEGIN{print $(date +%s.%N) - $s}") s rc=$rc: $*" >&2; return $rc; }
t timeout 300 $B synth -o $W/d -c chr1:$((MBP * 1000000)) -x 30 --tumor --noisy-frac 0.01 --paired 350 > /dev/null || exit 1
for i in 1 2; do
  rm -rf $W/log
  { time timeout 300 $B htc -f -r $W/d/ref.fasta -i $W/d/sample.bam -o $W/h$i.g.vcf 2> $W/htc$i.err; } 2> $W/htc$i.time || { tail $W/htc$i.err; exit 1; }
  grep -E "finishes|Start|phase|timeline" $W/htc$i.err; grep -E "^(real|user|sys)" $W/htc$i.time
done
sed -e 's/^/  | /' $W/htc2.err | head -60
grep -h "htc\] shard" $W/log/*.log | head -4
grep -h "htc\] shard" $W/log/*.log | awk '{for(i=1;i<=NF;i++){if($i=="(decode"||$i=="decode"){d+=$(i+1)} if($i=="passes),"){p+=$(i-1)}}} END{print "decode thread-s", d, "decode passes", p, "shards", NR}'
ls -la $W/h2.g.vcf* >&2
[ -n "${HTC_ONLY:-}" ] && { rm -rf $W; exit 0; }
rm -rf $W/log
t timeout 300 $B mutect2 -r $W/d/ref.fasta -t $W/d/tumor.bam -n $W/d/sample.bam -o $W/m2.vcf 2> $W/m2.err
sed -e 's/^/  | /' $W/m2.err | head -60
grep -h "mutect2\] shard" $W/log/*.log | head -3
t timeout 300 $B htc -r $W/d/ref.fasta -i $W/d/sample.bam -o $W/hv.vcf -v 2> $W/htcv.err
grep -E "finishes" $W/htcv.err
grep -h "shard" $W/log/*.log 2>/dev/null | head -3
t timeout 300 $B align -r $W/d/ref.fasta -1 $W/d/sample_1.fastq -2 $W/d/sample_2.fastq -o $W/a.bam 2> $W/al.err
grep -E "finishes|fcs-genome align" $W/al.err
rm -rf $W

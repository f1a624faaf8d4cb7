#!/bin/bash
# htc at the bench's 31 Mbp with the window BAM blocks inflated on the GPU
# (FCS_GPU_BAM_INFLATE=true) and by the host's libdeflate (the default), twice
# each, alternating: wall, user CPU, the shards' decode thread-seconds, and
# that both write the same GVCF.
W=$(mktemp -d /tmp/infab.XXXX)
export FCS_TIMELINE=1 FCS_GPU_DEVICES=0 FCS_TEMP_DIR=$W FCS_GATK_NPROCS=${NPROCS:-16}
MBP=${MBP:-31}
B=$GRAFT_REPO_ROOT/falcon-genome_amd/bin/fcs-genome
timeout 300 $B synth -o $W/d -c chr1:$((MBP * 1000000)) -x 30 --tumor --noisy-frac 0.01 --paired 350 > /dev/null || exit 1
ls -la $W/d/sample.bam
for i in 1 2 3 4; do
  for mode in true false; do
    rm -rf $W/log
    export FCS_LOG_DIR=$W/log FCS_GPU_BAM_INFLATE=$mode
    { time timeout 300 $B htc -f -r $W/d/ref.fasta -i $W/d/sample.bam -o $W/h_$mode.g.vcf 2> $W/htc.err; } 2> $W/htc.time || { tail -3 $W/htc.err; grep -rh "E::\|rror\|what" $W/log | head -10; exit 1; }
    echo "== gpu_inflate=$mode run $i: $(grep -E '^(real|user)' $W/htc.time | tr '\n' ' ')"
    grep -E "timeline" $W/htc.err | tail -2
    grep -h "htc\] shard" $W/log/*.log | awk '{for(i=1;i<=NF;i++){if($i=="(decode"||$i=="decode"){d+=$(i+1)} if($i=="inflate"){g+=$(i+1); h+=$(i+4)}}} END{print "  decode thread-s", d, "shards", NR, "inflate chunks gpu", g, "host", h}'
  done
done
grep -h "htc\] shard" $W/log/*.log | head -2
cmp $W/h_true.g.vcf.gz $W/h_false.g.vcf.gz && echo "GVCF identical (gpu vs host inflate)"
rm -rf $W

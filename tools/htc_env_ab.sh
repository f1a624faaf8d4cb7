#!/bin/bash
# htc at 31 Mbp under two environments, alternating, three runs each:
#   tools/htc_env_ab.sh "A_ENV=1" "B_ENV=1"
# wall, stage thread-seconds of the shards, identical GVCFs.
A=$1; B=$2
W=$(mktemp -d /tmp/envab.XXXX)
export FCS_TIMELINE=1 FCS_GPU_DEVICES=0 FCS_TEMP_DIR=$W FCS_GATK_NPROCS=${NPROCS:-16}
X=$GRAFT_REPO_ROOT/falcon-genome_amd/bin/fcs-genome
timeout 300 $X synth -o $W/d -c chr1:31000000 -x 30 --tumor --noisy-frac 0.01 --paired 350 > /dev/null || exit 1
for i in 1 2 3; do
  for tag in A B; do
    [ $tag = A ] && E=$A || E=$B
    rm -rf $W/log
    { time env $E FCS_LOG_DIR=$W/log timeout 300 $X htc -f -r $W/d/ref.fasta -i $W/d/sample.bam -o $W/h_$tag.g.vcf 2> $W/err; } 2> $W/time || { tail -3 $W/err; exit 1; }
    echo "== $tag ($E) run $i: $(grep real $W/time) $(grep user $W/time) $(grep sys $W/time)"
    grep -h "timeline\] exit" $W/err | sed 's/^/  /' 
    grep -h "htc\] shard" $W/log/*.log | awk '{for(i=1;i<=NF;i++){if($i=="decode"){d+=$(i+1)} if($i=="(PairHMM"){p+=$(i+1)} if($i=="regions"&&$(i+1)~/^[0-9.]+$/&&$(i+2)=="s,"){r+=$(i+1)} if($i=="ran"){n+=$(i+1)}}} END{print "  decode", d, "phmm", p, "regions", r, "nested", n+0}'
  done
done
cmp $W/h_A.g.vcf.gz $W/h_B.g.vcf.gz && echo "GVCF identical"
rm -rf $W

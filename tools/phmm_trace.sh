#!/bin/bash
# htc at 31 Mbp with FCS_PHMM_TRACE=1, twice: per-call host phases of the
# PairHMM passes (lease wait, staging growth, fill, issue, sync wait), summed,
# plus the slowest calls.
W=$(mktemp -d /tmp/phtr.XXXX)
export FCS_TIMELINE=1 FCS_GPU_DEVICES=0 FCS_TEMP_DIR=$W FCS_GATK_NPROCS=${NPROCS:-16} FCS_PHMM_TRACE=1
X=$GRAFT_REPO_ROOT/falcon-genome_amd/bin/fcs-genome
timeout -k 5 60 $GRAFT_REPO_ROOT/tools/micro/init_probe || exit 1
timeout -k 5 60 $GRAFT_REPO_ROOT/tools/micro/init_probe || exit 1
timeout 300 $X synth -o $W/d -c chr1:31000000 -x 30 --tumor --noisy-frac 0.01 --paired 350 > /dev/null || exit 1
for i in 1 2 3; do
  rm -rf $W/log
  { time env FCS_LOG_DIR=$W/log timeout 300 $X htc -f -r $W/d/ref.fasta -i $W/d/sample.bam -o $W/h.g.vcf 2> $W/err; } 2> $W/time || { tail -3 $W/err; exit 1; }
  echo "== run $i: $(grep real $W/time)"
  grep -h "htc\] shard" $W/log/*.log | awk '{for(i=1;i<=NF;i++){if($i=="decode"){d+=$(i+1)} if($i=="(PairHMM"){p+=$(i+1)}}} END{print "  decode", d, "phmm", p}'
  grep -h fcs_phmm_trace $W/err $W/log/*.log 2>/dev/null | awk '{n++; for(i=2;i<=NF;i++){if($i~/^(lease|ensure|fill|issue|sync|device|total)$/) s[$i]+=$(i+1)} if($0~/grew/) g++} END{printf "  calls %d grew %d", n, g; for(k in s) printf " %s %.1f", k, s[k]; print " (ms)"}'
  if [ $i = 1 ]; then grep -h "timeline\]" $W/err | sed 's/^/    /'; grep -h fcs_phmm_trace $W/err | sort -k3 -g | sed 's/^/    /'; fi
  grep -h fcs_phmm_trace $W/err $W/log/*.log 2>/dev/null | awk '{print $NF, $0}' | sort -g -r | head -8 | cut -d' ' -f2- | sed 's/^/    /'
done
rm -rf $W

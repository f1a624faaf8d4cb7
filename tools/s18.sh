set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/s18; mkdir -p $O
D=/tmp/c4; rm -rf $D
B=falcon-genome_amd/bin/fcs-genome
( time timeout -k 10 300 $B synth -o $D -c chr1:2000000 -x 30 --tumor ) > $O/synth.log 2>&1 || exit 1
tail -5 $O/synth.log
cd /tmp
for np in 8 16 32; do
( time FCS_GATK_NPROCS=$np FCS_GPU_DEVICES=0 FCS_LOG_DIR=/tmp/log$np timeout -k 10 300 $GRAFT_REPO_ROOT/$B htc -r $D/ref.fasta -i $D/sample.bam -o /tmp/htc$np.vcf -f ) > $GRAFT_REPO_ROOT/$O/htc$np.log 2>&1 || exit 1
tail -4 $GRAFT_REPO_ROOT/$O/htc$np.log
grep -h "shard" /tmp/log$np/*.log | head -3
cat /tmp/log$np/*.log | grep -o "regions" | wc -l
done
( time FCS_GATK_NPROCS=16 FCS_GPU_DEVICES=0 timeout -k 10 300 $GRAFT_REPO_ROOT/$B mutect2 -r $D/ref.fasta -t $D/tumor.bam -n $D/sample.bam -o /tmp/m2.vcf -f ) > $GRAFT_REPO_ROOT/$O/m2.log 2>&1 || exit 1
tail -4 $GRAFT_REPO_ROOT/$O/m2.log
( time FCS_GPU_DEVICES=0 timeout -k 10 300 $GRAFT_REPO_ROOT/$B align -r $D/ref.fasta -1 $D/sample.fastq -o /tmp/aln.bam -f ) > $GRAFT_REPO_ROOT/$O/aln.log 2>&1 || exit 1
tail -6 $GRAFT_REPO_ROOT/$O/aln.log

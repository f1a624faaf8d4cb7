set -u
bash tools/ab.sh phmm r3d || exit $?
B=falcon-genome_amd/bin/fcs-genome; D=/tmp/m2d; O=gpurun_out/r3d
$B synth -o $D -c chr20:250000,chr21:100000 -x 30 --tumor --seed 11 --spike chr20:109380 --parts 6 > /dev/null || exit 5
FCS_TEMP_DIR=/tmp/m2t FCS_LOG_DIR=/tmp/m2l FCS_GATK_NCONTIGS=6 FCS_GATK_NPROCS=3 FCS_GPU_DEVICES=0 timeout -k 10 120 $B mutect2 -f -r $D/ref.fasta -t $D/tumor.bam -n $D/sample.bam -o $O/m2.vcf > $O/m2.log 2>&1
echo "mutect2 rc=$?"

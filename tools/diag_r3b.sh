#!/bin/bash
# r3b: full GPU suite (no -x) and one mutect2 run on the e2e test fixture's data
set -u
OUT=gpurun_out/r3b; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
B=falcon-genome_amd/bin/fcs-genome; D=/tmp/m2d
$B synth -o $D -c chr20:250000,chr21:100000 -x 30 --tumor --seed 11 --spike chr20:109380 --parts 6 > /dev/null || exit 5
FCS_TEMP_DIR=/tmp/m2t FCS_LOG_DIR=/tmp/m2l timeout -k 10 120 $B mutect2 -f -r $D/ref.fasta -t $D/tumor.bam -n $D/sample.bam -o $OUT/m2.vcf --dump-regions $OUT/m2dump > $OUT/m2.log 2>&1
echo "mutect2 rc=$?"
cp $D/truth.vcf $OUT/

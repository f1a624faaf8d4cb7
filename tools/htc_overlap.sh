#!/bin/bash
# rocprofv3 kernel trace of `fcs-genome htc` with 4 concurrent shard threads on
# one GPU, and the overlap of their PairHMM passes (tools/htc_overlap.py).
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-ovl}; mkdir -p $O
W=$(mktemp -d /tmp/ovl.XXXX)
export FCS_GPU_DEVICES=0 FCS_LOG_DIR=$W/log FCS_TEMP_DIR=$W FCS_GATK_NPROCS=${NPROCS:-4} TMPDIR=/tmp
B=$GRAFT_REPO_ROOT/falcon-genome_amd/bin/fcs-genome
MBP=${MBP:-4}  # genome size (Mbp); 31 = the C4 per-GPU share
timeout -k 10 300 $B synth -o $W/d -c chr1:$((MBP * 1000000)) -x 30 --no-fastq > /dev/null || exit 1
# the profiled process must exit by itself (it once hung at exit);
# the wall time of the whole rocprofv3 command is recorded next to the trace
t0=$(date +%s.%N)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
  $B htc -r $W/d/ref.fasta -i $W/d/sample.bam -o $W/h.g.vcf > $O/htc.log 2>&1
rc=$?
t1=$(date +%s.%N)
echo "rocprofv3 + htc rc=$rc wall $(python3 -c "print(round($t1 - $t0, 1))") s" | tee $O/exit.log
[ $rc -eq 0 ] || { tail $O/htc.log; exit 1; }
python3 $GRAFT_REPO_ROOT/tools/htc_overlap.py $O/prof/run_kernel_trace.csv | tee $O/overlap.json
cat $W/log/* 2>/dev/null | grep -h "shard" > $O/shards.log || true
rm -rf $W

#!/bin/bash
# CPU sanitizer runs of the host orchestrator (falcon-genome_amd/host) and the
# oracle.  Host only: GPU sanitizers are not
# available on the GPU pool, and libfcship.so (hipcc) is not rebuilt here.
#   ASAN, UBSAN: the whole CPU pytest suite against the SAN=<kind> builds
#     (FCS_SAN selects them in tests/host_lib.py and tests/oracle_lib.py; the
#     runtime is LD_PRELOADed with libstdc++ since python itself is not
#     instrumented); the fcs-genome CLI runs that the tests start use the
#     sanitized binary too.
#   TSAN: python + torch + the HIP runtime deadlock under TSAN's interposition,
#     so the threaded host code runs through tools/host_race.cpp and the
#     sanitized CLI (synth to a parts directory; synth interrupted by SIGINT).
# Usage: tools/sanitize.sh [log]   (default profiles/r2/sanitize.log)
set -uo pipefail
cd "$(dirname "$0")/.."
LOG=${1:-profiles/r2/sanitize.log}
mkdir -p "$(dirname "$LOG")"
STD=$(g++ -print-file-name=libstdc++.so.6)
W=$(mktemp -d /tmp/fcs_san.XXXXXX)
rc=0
{
  for SAN in address undefined thread; do
    make -C falcon-genome_amd/host SAN=$SAN -j8 >/dev/null && make -C oracle SAN=$SAN >/dev/null || { echo "build $SAN failed"; exit 1; }
  done
  echo "== ASAN ($(gcc --version | head -1)): CPU test suite"
  FCS_SAN=address LD_PRELOAD="$(gcc -print-file-name=libasan.so) $STD" \
    ASAN_OPTIONS=detect_leaks=0:alloc_dealloc_mismatch=0:log_path=$W/asan \
    timeout 900 python -m pytest tests -q -m "not gpu" -p no:cacheprovider 2>&1 | tail -2 || rc=1
  if ls $W/asan.* >/dev/null 2>&1; then cat $W/asan.*; rc=1; else echo "ASAN reports: none"; fi
  echo "== UBSAN: CPU test suite"
  FCS_SAN=undefined LD_PRELOAD="$(gcc -print-file-name=libubsan.so) $STD" \
    UBSAN_OPTIONS=print_stacktrace=1:log_path=$W/ubsan \
    timeout 900 python -m pytest tests -q -m "not gpu" -p no:cacheprovider 2>&1 | tail -2 || rc=1
  if ls $W/ubsan.* >/dev/null 2>&1; then cat $W/ubsan.*; rc=1; else echo "UBSAN reports: none"; fi
  echo "== TSAN: host_race driver + CLI"
  g++ -std=c++17 -O1 -g -fsanitize=thread tools/host_race.cpp -o $W/host_race \
    -Lfalcon-genome_amd/_san/thread -L falcon-genome_amd -lfcsgenome -lfcship \
    -Wl,-rpath,"$PWD/falcon-genome_amd/_san/thread:$PWD/falcon-genome_amd" || rc=1
  export TSAN_OPTIONS="log_path=$W/tsan:halt_on_error=0"
  mkdir -p $W/race && timeout 600 $W/host_race $W/race || rc=1
  SANBIN=falcon-genome_amd/_san/thread/bin/fcs-genome
  FCS_TEMP_DIR=$W/tmp1 FCS_LOG_DIR=$W/log timeout 600 $SANBIN synth -o $W/syn -c chr1:400000 -x 10 --parts 4 \
    >/dev/null 2>$W/synth.err && echo "synth --parts 4: ok" || { rc=1; tail -5 $W/synth.err; }
  FCS_TEMP_DIR=$W/tmp2 FCS_LOG_DIR=$W/log $SANBIN synth -o $W/syn2 -c chr1:40000000 -x 30 >/dev/null 2>$W/int.err &
  pid=$!; sleep 3; kill -INT $pid; wait $pid; st=$?
  [ $st -eq 130 ] && [ ! -e $W/tmp2 ] && echo "synth + SIGINT: exit 130, temp dir removed" || { rc=1; echo "SIGINT: exit $st"; }
  # htc with concurrent shards' PairHMM passes merged (host/caller.cpp
  # PassCombiner: shard threads, one leader per pass) against the CPU mock
  make -C tests/cpu_mock >/dev/null || rc=1
  LD_LIBRARY_PATH=$PWD/tests/cpu_mock/build FCS_GPU_DEVICES=0 FCS_MOCK_PHMM=gkl FCS_GATK_NCONTIGS=8 \
    FCS_GATK_NPROCS=4 FCS_GPU_PHMM_COMBINE_MS=500 FCS_TEMP_DIR=$W/tmp3 FCS_LOG_DIR=$W/log3 \
    timeout 600 $SANBIN htc -f -r $W/syn/ref.fasta -i $W/syn/sample.bam -o $W/m.vcf -v >/dev/null 2>$W/htc.err \
    && echo "htc with merged passes (8 shards, 4 threads): ok" || { rc=1; tail -5 $W/htc.err; }
  if ls $W/tsan.* >/dev/null 2>&1; then cat $W/tsan.*; rc=1; else echo "TSAN reports: none"; fi
  echo "sanitize rc=$rc"
} 2>&1 | tee "$LOG"
rm -rf "$W"
exit $rc

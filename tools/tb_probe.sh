#!/bin/bash
# Traceback-kernel probe: per-kernel durations of bench.py's global workload for
# the in-tree library and each alt/*.so given (FCSHIP_LIB), one rocprofv3
# kernel trace each.   usage: tools/tb_probe.sh TAG alt/X.so [...]
set -u
O=gpurun_out/$1; shift; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for f in in-tree "$@"; do
  n=$(basename $f .so)
  if [ $f = in-tree ]; then L=; else L=$PWD/$f; fi
  FCSHIP_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$n -o run --output-format csv -- python tools/bsw_bench.py --which global ${BSW_ARGS:-} > $O/$n.log 2>&1
  rc=$?
  echo "$n rc=$rc"
  case $rc in 124|137|134|139) exit $rc;; esac
done

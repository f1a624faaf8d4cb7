#!/bin/bash
# Build a variant of libfcship.so into alt/NAME.so for A/B runs on the GPU box
# (tools/ab_bsw.sh, tools/ab_phmm.sh, tools/bsw_stats.py).
# usage: tools/build_alt.sh NAME [extra hipcc flags...]
#   e.g. tools/build_alt.sh stats -DFCS_BSW_STATS
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
B=$ROOT/alt/build-$NAME
mkdir -p "$B" "$ROOT/alt"
cd "$ROOT/falcon-genome_amd"
FLAGS="-O3 -std=c++20 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-result $*"
objs=()
for s in csrc/*.hip csrc/*.cpp; do
  o=$B/$(basename "${s%.*}").o
  /opt/rocm/bin/hipcc $FLAGS -I../include -Icsrc -c -o "$o" "$s" &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,--no-undefined -o "$ROOT/alt/$NAME.so" "${objs[@]}"
echo "built alt/$NAME.so"

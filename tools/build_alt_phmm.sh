#!/bin/bash
# Build alt/NAME.so = the in-tree libfcship objects with phmm_kernels replaced by
# a variant source (for tools/ab_phmm.sh).  Run `make -C falcon-genome_amd` first.
# usage: tools/build_alt_phmm.sh NAME VARIANT.hip [extra hipcc flags...]
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; SRC=$(realpath "$2"); shift 2
mkdir -p "$ROOT/alt"
cd "$ROOT/falcon-genome_amd"
O=$ROOT/alt/phmm-$NAME.o
/opt/rocm/bin/hipcc -O3 -std=c++20 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-result "$@" \
  -I../include -Icsrc -c -o "$O" "$SRC"
objs=$(ls build/*.o | grep -v phmm_kernels)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,--no-undefined -o "$ROOT/alt/$NAME.so" "$O" $objs
echo "built alt/$NAME.so"

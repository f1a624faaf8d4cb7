#!/bin/bash
# Compile phmm_kernels.hip to gfx950 assembly and print, for the fp32 fast-path
# kernel, register use, spills and per-instruction counts inside the hot blocks.
# usage: tools/phmm_asm_stats.sh [source]   (default: the in-tree kernel)
set -e
SRC=${1:-$(dirname "$0")/../falcon-genome_amd/csrc/phmm_kernels.hip}
INC=$(dirname "$0")/../falcon-genome_amd
OUT=/tmp/phmm_stats.s
/opt/rocm/bin/hipcc -O3 -std=c++20 -fPIC --offload-arch=gfx950 -ffp-contract=off -I$INC/../include -I$INC/csrc \
  --cuda-device-only -S -o $OUT "$SRC" 2>/dev/null
K='_ZN3fcs11phmm_kernelIfLb0ELb0EE'
awk -v k="$K" 'index($0,k)==1 && /:/ {on=1} on {print} on && /s_endpgm/ {exit}' $OUT > /tmp/phmm_fast.s
grep -A40 "^    .name:.*phmm_kernelIfLb0ELb0" $OUT | grep -E "vgpr_count|spill_count|private_segment_fixed" | tr -s ' ' | tr '\n' ' '; echo
echo "total instr: $(grep -cE '^\s+[vsd][a-z_0-9]+ ' /tmp/phmm_fast.s)"
for op in v_mov_b32_e32 v_mov_b32_dpp v_cndmask_b32 v_cmp_ v_pk_fma_f32 v_fma_f32 v_fmac_f32 v_mul_f32 v_add_f32 v_and_b32 ds_read_b64 ds_read_u8 ds_write_b64 s_and_saveexec s_nop s_waitcnt; do
  printf "%-18s %6d\n" $op $(grep -c "^\s*$op" /tmp/phmm_fast.s || true)
done

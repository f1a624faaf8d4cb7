// VALU issue-rate microbenchmark for the PairHMM step's instruction mix on
// gfx950: cycles per wave-instruction per SIMD of one instruction kind, run by
// `waves` waves per SIMD (independent chains: eight accumulators per lane).
// Clock from s_memtime / s_memrealtime stamps of block 0 (diagnostic buffer
// only).  usage: valu_rate [waves_per_simd]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));           \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

constexpr int kIters = 4096;

#define BODY8(INSN) INSN(0) INSN(1) INSN(2) INSN(3) INSN(4) INSN(5) INSN(6) INSN(7)

typedef float f2 __attribute__((ext_vector_type(2)));

template <int K>
__global__ __launch_bounds__(256) void kern(float* out, unsigned long long* stamps, int iters) {
  float a[8];
  float b[8];
  f2 c[8], d[8];
  for (int i = 0; i < 8; ++i) {
    a[i] = threadIdx.x * 0.001f + i, b[i] = 1.0f + i * 1e-3f;
    c[i] = f2{a[i], b[i]};
    d[i] = f2{b[i], a[i] * 1e-3f};
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long m = 0x5555555555555555ull;
  if constexpr (K == 31) asm volatile("v_cmp_gt_f32 vcc, %0, %1" : : "v"(a[0]), "v"(b[1]) : "vcc");
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int rep = 0; rep < 2; ++rep) {
      if constexpr (K == 0) {  // v_fma_f32
#define I(j) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[j]) : "v"(b[j]), "v"(b[(j + 1) & 7]));
        BODY8(I)
#undef I
      } else if constexpr (K == 1) {  // v_pk_fma_f32 (two lanes' worth)
#define I(j) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(c[j]) : "v"(d[j]), "v"(d[(j + 1) & 7]));
        BODY8(I)
#undef I
      } else if constexpr (K == 2) {  // v_mov_b32_dpp row_shr:1
#define I(j) asm volatile("v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "=v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 3) {  // v_bfe_i32
#define I(j) asm volatile("v_bfe_i32 %0, %1, %2, 1" : "=v"(a[j]) : "v"(b[j]), "v"(b[(j + 3) & 7]));
        BODY8(I)
#undef I
      } else if constexpr (K == 4) {  // v_bitop3_b32
#define I(j) asm volatile("v_bitop3_b32 %0, %1, %2, %0 bitop3:0xe4" : "+v"(a[j]) : "v"(b[j]), "v"(b[(j + 1) & 7]));
        BODY8(I)
#undef I
      } else if constexpr (K == 5) {  // v_cndmask_b32_e64 with an SGPR-pair mask
#define I(j) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b[j]), "s"(m));
        BODY8(I)
#undef I
      } else if constexpr (K == 6) {  // v_mul_f32
#define I(j) asm volatile("v_mul_f32 %0, %1, %0" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 7) {  // v_add_u32
#define I(j) asm volatile("v_add_u32 %0, %1, %0" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 8) {  // v_pk_mul_f32
#define I(j) asm volatile("v_pk_mul_f32 %0, %1, %0" : "+v"(c[j]) : "v"(d[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 9) {  // v_cndmask_b32_dpp (VOP2 DPP, VCC)
#define I(j) asm volatile("v_cndmask_b32_dpp %0, %0, %1, vcc row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        BODY8(I)
#undef I
      } else if constexpr (K == 10) {  // v_perm_b32
#define I(j) asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(a[j]) : "v"(b[j]), "v"(b[(j + 1) & 7]));
        BODY8(I)
#undef I
      } else if constexpr (K == 11) {  // v_fmac_f32 (VOP2)
#define I(j) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a[j]) : "v"(b[j]), "v"(b[(j + 1) & 7]));
        BODY8(I)
#undef I
      } else if constexpr (K == 12) {
#define I(j) asm volatile("v_lshrrev_b32 %0, %1, %0" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 13) {
#define I(j) asm volatile("v_ashrrev_i32 %0, %1, %0" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 14) {
#define I(j) asm volatile("v_and_b32 %0, %1, %0" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 15) {  // VOPC compare -> VCC
#define I(j) asm volatile("v_cmp_eq_u32 vcc, %0, %1" : : "v"(a[j]), "v"(b[j]) : "vcc");
        BODY8(I)
#undef I
      } else if constexpr (K == 16) {  // VOP2 cndmask on VCC
#define I(j) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 17) {  // VOP2 DPP multiply
#define I(j) asm volatile("v_mul_f32_dpp %0, %1, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 18) {
#define I(j) asm volatile("v_add_f32_dpp %0, %1, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 19) {
#define I(j) asm volatile("v_mov_b32 %0, %1" : "=v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 20) {
#define I(j) asm volatile("v_bfe_u32 %0, %1, %2, 1" : "=v"(a[j]) : "v"(b[j]), "v"(b[(j + 3) & 7]));
        BODY8(I)
#undef I
      } else if constexpr (K == 21) {
#define I(j) asm volatile("v_cndmask_b32_e64 %0, %0, %1, vcc" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 23) {
#define I(j) asm volatile("v_bfi_b32 %0, %1, %2, %0" : "+v"(a[j]) : "v"(b[j]), "v"(b[(j + 1) & 7]));
        BODY8(I)
#undef I
      } else if constexpr (K == 24) {
#define I(j) asm volatile("v_fmac_f32_dpp %0, %1, %2 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(a[j]) : "v"(b[j]), "v"(b[(j + 1) & 7]));
        BODY8(I)
#undef I
      } else if constexpr (K == 25) {  // dpp move keeping `old` in lane 0 of each row
#define I(j) asm volatile("v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 26) {  // VOP2 DPP multiply, wave_shr:1
#define I(j) asm volatile("v_mul_f32_dpp %0, %1, %0 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 27) {  // v_pk_add_f32
#define I(j) asm volatile("v_pk_add_f32 %0, %1, %0" : "+v"(c[j]) : "v"(d[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 28) {  // v_sub_f32
#define I(j) asm volatile("v_sub_f32 %0, %1, %0" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 29) {  // v_mul_f32 VOP3 with abs/neg modifiers
#define I(j) asm volatile("v_mul_f32_e64 %0, |%1|, -%0" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 30) {  // one VOPC write of VCC, then eight VOP2 cndmask reads
        asm volatile("v_cmp_gt_f32 vcc, %0, %1" : : "v"(a[0]), "v"(b[1]) : "vcc");
#define I(j) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 31) {  // VOP2 cndmask, VCC written once before the loop
#define I(j) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 32) {  // one VOPC write, eight e64 cndmask reads of VCC
        asm volatile("v_cmp_gt_f32 vcc, %0, %1" : : "v"(a[0]), "v"(b[1]) : "vcc");
#define I(j) asm volatile("v_cndmask_b32_e64 %0, %0, %1, vcc" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 33) {
#define I(j) asm volatile("v_max_i32 %0, %1, %0" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 34) {
#define I(j) asm volatile("v_max3_i32 %0, %1, %2, %0" : "+v"(a[j]) : "v"(b[j]), "v"(b[(j + 1) & 7]));
        BODY8(I)
#undef I
      } else if constexpr (K == 35) {
#define I(j) asm volatile("v_pk_max_i16 %0, %1, %0" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 36) {
#define I(j) asm volatile("v_pk_add_u16 %0, %1, %0" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 37) {  // VOPC to an SGPR pair (e64)
#define I(j) asm volatile("v_cmp_gt_i32_e64 s[40:41], %0, %1" : : "v"(a[j]), "v"(b[j]) : "s40", "s41");
        BODY8(I)
#undef I
      } else if constexpr (K == 38) {
#define I(j) asm volatile("v_sub_u32 %0, %1, %0" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 39) {
#define I(j) asm volatile("v_max_f32 %0, %1, %0" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 40) {
#define I(j) asm volatile("v_pk_sub_u16 %0, %1, %0" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 41) {
#define I(j) asm volatile("v_pk_max_u16 %0, %1, %0" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 42) {  // 16-bit scalar VOP3 max (op_sel capable)
#define I(j) asm volatile("v_max_i16 %0, %1, %0" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 43) {
#define I(j) asm volatile("v_cmp_gt_i32 vcc, %0, %1" : : "v"(a[j]), "v"(b[j]) : "vcc");
        BODY8(I)
#undef I
      } else if constexpr (K == 44) {
#define I(j) asm volatile("v_med3_i32 %0, %1, %2, %0" : "+v"(a[j]) : "v"(b[j]), "v"(b[(j + 1) & 7]));
        BODY8(I)
#undef I
      } else if constexpr (K == 45) {  // one VOP2 cndmask (VCC) among seven v_fma_f32
        asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(a[0]) : "v"(b[0]));
#define I(j) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[j]) : "v"(b[j]), "v"(b[(j + 1) & 7]));
        I(1) I(2) I(3) I(4) I(5) I(6) I(7)
#undef I
      } else if constexpr (K == 46) {  // one VOP3 cndmask (VCC) among seven v_fma_f32
        asm volatile("v_cndmask_b32_e64 %0, %0, %1, vcc" : "+v"(a[0]) : "v"(b[0]));
#define I(j) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[j]) : "v"(b[j]), "v"(b[(j + 1) & 7]));
        I(1) I(2) I(3) I(4) I(5) I(6) I(7)
#undef I
      } else if constexpr (K == 47) {  // VOP2 v_addc_co_u32 (VCC carry in and out)
#define I(j) asm volatile("v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        BODY8(I)
#undef I
      } else if constexpr (K == 48) {  // VOP2 cndmask reading an SGPR-pair alias? (e32 with vcc, src0 SGPR)
#define I(j) asm volatile("v_cndmask_b32_e32 %0, 0, %0, vcc" : "+v"(a[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 50) {
#define I(j) asm volatile("v_add_u16 %0, %1, %0" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 51) {
#define I(j) asm volatile("v_sub_i16 %0, %1, %0 clamp" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 52) {
#define I(j) asm volatile("v_max3_i16 %0, %1, %2, %0" : "+v"(a[j]) : "v"(b[j]), "v"(b[(j + 1) & 7]));
        BODY8(I)
#undef I
      } else if constexpr (K == 53) {
#define I(j) asm volatile("v_add_u32_sdwa %0, %1, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 54) {
#define I(j) asm volatile("v_max_i32_sdwa %0, sext(%1), %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:DWORD" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 55) {
#define I(j) asm volatile("v_add3_u32 %0, %1, %2, %0" : "+v"(a[j]) : "v"(b[j]), "v"(b[(j + 1) & 7]));
        BODY8(I)
#undef I
      } else if constexpr (K == 56) {
#define I(j) asm volatile("v_max_i16_e64 %0, %1, %0" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 57) {
#define I(j) asm volatile("v_min_i32 %0, %1, %0" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 58) {
#define I(j) asm volatile("v_sub_u16 %0, %1, %0" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 59) {
#define I(j) asm volatile("v_max_u32 %0, %1, %0" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 60) {  // funnel shift: acc = (acc << 1) | (x >> 31)
#define I(j) asm volatile("v_alignbit_b32 %0, %0, %1, 31" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 61) {
#define I(j) asm volatile("v_lshl_or_b32 %0, %1, 4, %0" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 62) {
#define I(j) asm volatile("v_or3_b32 %0, %1, %2, %0" : "+v"(a[j]) : "v"(b[j]), "v"(b[(j + 1) & 7]));
        BODY8(I)
#undef I
      } else if constexpr (K == 63) {
#define I(j) asm volatile("v_and_or_b32 %0, %1, %2, %0" : "+v"(a[j]) : "v"(b[j]), "v"(b[(j + 1) & 7]));
        BODY8(I)
#undef I
      } else if constexpr (K == 64) {
#define I(j) asm volatile("v_lshl_add_u32 %0, %1, 2, %0" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 65) {
#define I(j) asm volatile("v_alignbyte_b32 %0, %0, %1, 3" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 66) {
#define I(j) asm volatile("v_min3_i32 %0, %1, %2, %0" : "+v"(a[j]) : "v"(b[j]), "v"(b[(j + 1) & 7]));
        BODY8(I)
#undef I
      } else if constexpr (K == 68) {  // byte -> float (VOP1)
#define I(j) asm volatile("v_cvt_f32_ubyte1 %0, %1" : "=v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 69) {  // prior as fma(m, e1 - e3, e3) on both halves
#define I(j) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(c[j]) : "v"(d[j]), "v"(d[(j + 1) & 7]));
        BODY8(I)
#undef I
      } else if constexpr (K == 70) {  // v_bfe_i32 mask + v_bitop3 select (the column kernel's prior, per half)
#define I(j) asm volatile("v_bfe_i32 %0, %1, 8, 1\n\tv_bitop3_b32 %0, %1, %2, %0 bitop3:0xe4" : "=&v"(a[j]) : "v"(b[j]), "v"(b[(j + 1) & 7]));
        BODY8(I)
#undef I
      } else if constexpr (K == 71) {  // v_cvt_f32_ubyte mask (the alternative, per half)
#define I(j) asm volatile("v_cvt_f32_ubyte2 %0, %1" : "=v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 72) {  // v_mov_b32_sdwa sext byte
#define I(j) asm volatile("v_mov_b32_sdwa %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1" : "=v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 73) {
#define I(j) asm volatile("v_lshrrev_b32 %0, 31, %1" : "=v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 74) {
#define I(j) asm volatile("v_pk_sub_u16 %0, %1, %0 clamp" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 75) {
#define I(j) asm volatile("v_pk_min_u16 %0, %1, %0" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 76) {
#define I(j) asm volatile("v_pk_mad_u16 %0, %1, %2, %0" : "+v"(a[j]) : "v"(b[j]), "v"(b[(j + 1) & 7]));
        BODY8(I)
#undef I
      } else if constexpr (K == 77) {
#define I(j) asm volatile("v_pk_mad_u16 %0, %1, %2, 0 op_sel_hi:[1,1,0] clamp" : "=v"(a[j]) : "v"(b[j]), "v"(b[(j + 1) & 7]));
        BODY8(I)
#undef I
      } else if constexpr (K == 78) {
#define I(j) asm volatile("v_pk_ashrrev_i16 %0, 15, %1 op_sel_hi:[0,1]" : "=v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 79) {
#define I(j) asm volatile("v_pk_lshlrev_b16 %0, 8, %1 op_sel_hi:[0,1]" : "=v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 80) {
#define I(j) asm volatile("v_sub_u16 %0, %1, %0 clamp" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      } else if constexpr (K == 67) {
#define I(j) asm volatile("v_sub_u32 %0, %1, %0\n\tv_alignbit_b32 %0, %0, %1, 31" : "+v"(a[j]) : "v"(b[j]));
        BODY8(I)
#undef I
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0;
  for (int i = 0; i < 8; ++i) s += a[i] + c[i].x + c[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    stamps[0] = t1 - t0;
    stamps[1] = r1 - r0;
  }
}

template <int K>
static void run(const char* name, int waves, float* out, unsigned long long* st, int ncu) {
  const int blocks = ncu * 4 * waves / 4;  // 256-thread blocks: 4 waves each
  auto k = kern<K>;
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, st, 64);  // warm
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, st, kIters);
  CHECK(hipEventRecord(e1));
  CHECK(hipDeviceSynchronize());
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long h[2];
  CHECK(hipMemcpy(h, st, sizeof h, hipMemcpyDeviceToHost));
  const double ghz = (double)h[0] / ((double)h[1] / 100e6) / 1e9;
  const double instr_per_simd = (double)blocks * 4 * kIters * 16 / (ncu * 4);
  std::printf("%-22s waves/SIMD %d  %.3f ms  clock %.2f GHz  cycles/instr/SIMD %.2f\n", name, waves, ms, ghz,
              ms * 1e-3 * ghz * 1e9 / instr_per_simd);
}

int main(int argc, char** argv) {
  const int waves = argc > 1 ? std::atoi(argv[1]) : 4;
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int ncu = p.multiProcessorCount;
  float* out;
  unsigned long long* st;
  CHECK(hipMalloc(&out, sizeof(float) * ncu * 4 * waves * 64 * 2));
  CHECK(hipMalloc(&st, 16));
  run<0>("v_fma_f32", waves, out, st, ncu);
  run<35>("v_pk_max_i16", waves, out, st, ncu);
  run<41>("v_pk_max_u16", waves, out, st, ncu);
  run<75>("v_pk_min_u16", waves, out, st, ncu);
  run<36>("v_pk_add_u16", waves, out, st, ncu);
  run<40>("v_pk_sub_u16", waves, out, st, ncu);
  run<74>("v_pk_sub_u16 clamp", waves, out, st, ncu);
  run<76>("v_pk_mad_u16", waves, out, st, ncu);
  run<77>("v_pk_mad_u16 clamp", waves, out, st, ncu);
  run<78>("v_pk_ashrrev_i16", waves, out, st, ncu);
  run<79>("v_pk_lshlrev_b16", waves, out, st, ncu);
  run<80>("v_sub_u16 clamp", waves, out, st, ncu);
  run<14>("v_and_b32", waves, out, st, ncu);
  run<68>("v_cvt_f32_ubyte1", waves, out, st, ncu);
  run<71>("v_cvt_f32_ubyte2", waves, out, st, ncu);
  run<69>("v_pk_fma_f32", waves, out, st, ncu);
  run<70>("bfe_i32 + bitop3 (2 instr)", waves, out, st, ncu);
  run<72>("v_mov_b32_sdwa sext byte", waves, out, st, ncu);
  run<73>("v_lshrrev_b32", waves, out, st, ncu);
  run<3>("v_bfe_i32", waves, out, st, ncu);
  run<4>("v_bitop3_b32", waves, out, st, ncu);
  run<60>("v_alignbit_b32", waves, out, st, ncu);
  run<61>("v_lshl_or_b32", waves, out, st, ncu);
  run<62>("v_or3_b32", waves, out, st, ncu);
  run<63>("v_and_or_b32", waves, out, st, ncu);
  run<64>("v_lshl_add_u32", waves, out, st, ncu);
  run<65>("v_alignbyte_b32", waves, out, st, ncu);
  run<66>("v_min3_i32", waves, out, st, ncu);
  run<67>("sub + alignbit (2 instr)", waves, out, st, ncu);
  run<42>("v_max_i16", waves, out, st, ncu);
  run<50>("v_add_u16", waves, out, st, ncu);
  run<58>("v_sub_u16", waves, out, st, ncu);
  run<51>("v_sub_i16 clamp", waves, out, st, ncu);
  run<52>("v_max3_i16", waves, out, st, ncu);
  run<56>("v_max_i16 e64", waves, out, st, ncu);
  run<53>("v_add_u32_sdwa byte", waves, out, st, ncu);
  run<54>("v_max_i32_sdwa sext word", waves, out, st, ncu);
  run<55>("v_add3_u32", waves, out, st, ncu);
  run<57>("v_min_i32", waves, out, st, ncu);
  run<59>("v_max_u32", waves, out, st, ncu);
  run<33>("v_max_i32", waves, out, st, ncu);
  return 0;
}

// FP32 VALU issue-rate probe for gfx950: v_fma_f32 vs v_pk_fma_f32 vs DPP
// moves, dependent and independent chains at 1..4 waves per SIMD.  Sizes the
// PairHMM step: does a packed FMA cost one issue slot or two?
// build: hipcc -O3 --offload-arch=gfx950 -o tools/fp_probe tools/fp_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

// OP 0: v_fma_f32 x2; 1: v_pk_fma_f32 x2 (on a 64-bit pair); 2: v_mov_b32_dpp row_shr:1 + v_fma_f32;
// 3: v_pk_mul_f32 + v_pk_fma_f32; 4: v_bfe_i32 + v_bfi_b32 (prior select)
template <int CHAINS, int OP>
__global__ __launch_bounds__(64) void probe(float* out, int iters, float b, float c) {
  float2 a[CHAINS];
#pragma unroll
  for (int k = 0; k < CHAINS; ++k) a[k] = make_float2(threadIdx.x + k, threadIdx.x - k);
  const float2 bb = make_float2(b, c), cc = make_float2(c, b);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 32; ++u) {
#pragma unroll
      for (int k = 0; k < CHAINS; ++k) {
        if constexpr (OP == 0)
          asm volatile("v_fma_f32 %0, %0, %1, %2\n\tv_fma_f32 %0, %0, %2, %1" : "+v"(a[k].x) : "v"(b), "v"(c));
        else if constexpr (OP == 1)
          asm volatile("v_pk_fma_f32 %0, %0, %1, %2\n\tv_pk_fma_f32 %0, %0, %2, %1" : "+v"(a[k]) : "v"(bb), "v"(cc));
        else if constexpr (OP == 2)
          asm volatile("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n\tv_fma_f32 %0, %0, %1, %2"
                       : "+v"(a[k].x) : "v"(b), "v"(c));
        else if constexpr (OP == 3)
          asm volatile("v_pk_mul_f32 %0, %0, %1\n\tv_pk_fma_f32 %0, %0, %2, %1" : "+v"(a[k]) : "v"(bb), "v"(cc));
        else
          asm volatile("v_bfe_i32 %0, %0, %1, 1\n\tv_bfi_b32 %0, %0, %1, %2"
                       : "+v"(a[k].x) : "v"(b), "v"(c));
      }
    }
  }
  float s = 0;
#pragma unroll
  for (int k = 0; k < CHAINS; ++k) s += a[k].x + a[k].y;
  out[blockIdx.x * 64 + threadIdx.x] = s;
}

template <int CHAINS, int OP>
void run(int waves_per_simd, float* out) {
  const int cus = 256, iters = 2000;
  const int blocks = cus * 4 * waves_per_simd;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((probe<CHAINS, OP>), dim3(blocks), dim3(64), 0, 0, out, 10, 1.f, 0.f);
  hipEventRecord(e0);
  hipLaunchKernelGGL((probe<CHAINS, OP>), dim3(blocks), dim3(64), 0, 0, out, iters, 1.f, 0.f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double instr = (double)blocks * iters * 32 * CHAINS * 2;  // wave64 instructions
  printf("op=%d chains=%d waves/simd=%d ms=%.3f cyc/instr/SIMD=%.2f\n", OP, CHAINS, waves_per_simd, ms,
         (ms * 1e-3 * 2.4e9) / (instr / (cus * 4)));
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

template <int OP>
void sweep(float* out) {
  for (int w : {1, 2, 4}) {
    run<1, OP>(w, out);
    run<4, OP>(w, out);
  }
}

int main() {
  float* out = nullptr;
  hipMalloc(&out, 256 * 4 * 8 * 64 * sizeof(float));
  sweep<0>(out);
  sweep<1>(out);
  sweep<2>(out);
  sweep<3>(out);
  sweep<4>(out);
  hipFree(out);
  return 0;
}

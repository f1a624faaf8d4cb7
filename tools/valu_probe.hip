// VALU issue-rate probe for gfx950: how many wave64 integer VALU instructions
// per second the chip retires for independent vs dependent chains at 1..8
// waves per SIMD.  Used to read SQ_INSTS_VALU and to size the SW kernels'
// per-cell instruction budget ("Banded SW").
// build: hipcc -O3 --offload-arch=gfx950 -o valu_probe tools/valu_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

// OP 0: v_add_u32 + v_max_i32; 1: v_pk_add_u16 + v_pk_max_i16 (packed int16);
// 2: v_lshl_or_b32 + v_perm_b32 (3-operand VOP3); 3: v_pk_sub_u16 clamp + v_pk_mad_u16
template <int CHAINS, int OP>
__global__ __launch_bounds__(64) void probe(int* out, int iters, int b, int c) {
  int a[CHAINS];
#pragma unroll
  for (int k = 0; k < CHAINS; ++k) a[k] = threadIdx.x + k;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 32; ++u) {
#pragma unroll
      for (int k = 0; k < CHAINS; ++k) {
        // one v_add_u32 + one v_max_i32 per chain step, kept by the data dependence
        if constexpr (OP == 0)
          asm volatile("v_add_u32 %0, %0, %1\n\tv_max_i32 %0, %0, %2" : "+v"(a[k]) : "v"(b), "v"(c));
        else if constexpr (OP == 1)
          asm volatile("v_pk_add_u16 %0, %0, %1\n\tv_pk_max_i16 %0, %0, %2" : "+v"(a[k]) : "v"(b), "v"(c));
        else if constexpr (OP == 2)
          asm volatile("v_lshl_or_b32 %0, %0, 3, %1\n\tv_perm_b32 %0, %0, %1, %2" : "+v"(a[k]) : "v"(b), "v"(c));
        else
          asm volatile("v_pk_sub_u16 %0, %0, %1 clamp\n\tv_pk_mad_u16 %0, %0, %1, %2" : "+v"(a[k]) : "v"(b), "v"(c));
      }
    }
  }
  int s = 0;
#pragma unroll
  for (int k = 0; k < CHAINS; ++k) s += a[k];
  out[blockIdx.x * 64 + threadIdx.x] = s;
}

template <int CHAINS, int OP = 0>
void run(int waves_per_simd, int* out) {
  const int cus = 256, iters = 2000;
  const int blocks = cus * 4 * waves_per_simd;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((probe<CHAINS, OP>), dim3(blocks), dim3(64), 0, 0, out, 10, 1, 0);
  hipEventRecord(e0);
  hipLaunchKernelGGL((probe<CHAINS, OP>), dim3(blocks), dim3(64), 0, 0, out, iters, 1, 0);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double instr = (double)blocks * iters * 32 * CHAINS * 2;  // wave64 instructions
  printf("op=%d chains=%d waves/simd=%d ms=%.3f wave-instr/s=%.3e lane-ops/s=%.3e cyc/instr/SIMD=%.2f\n", OP, CHAINS,
         waves_per_simd, ms, instr / (ms * 1e-3), 64 * instr / (ms * 1e-3),
         (ms * 1e-3 * 2.4e9) / (instr / (cus * 4)));
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

int main() {
  int* out = nullptr;
  hipMalloc(&out, 256 * 4 * 8 * 64 * sizeof(int));
  for (int w : {1, 2, 3, 4, 8}) {
    run<1>(w, out);
    run<4>(w, out);
  }
  for (int w : {2, 3, 4}) {
    run<4, 1>(w, out);
    run<4, 2>(w, out);
    run<4, 3>(w, out);
  }
  hipFree(out);
  return 0;
}

#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out) {
  unsigned a = 0xABCD0005u, b = 0x1234FFF0u, r0, r1, r2, r3, r4;
  asm volatile("v_max_i16 %0, %1, %2" : "=v"(r0) : "v"(a), "v"(b));
  asm volatile("v_max_i16_e64 %0, %1, %2" : "=v"(r1) : "v"(a), "v"(b));
  r2 = 0x77770000u;
  asm volatile("v_sub_u16_e64 %0, %1, %2" : "+v"(r2) : "v"(a), "v"(b));
  r3 = 0x55555555u;
  asm volatile("v_pk_max_i16 %0, %1, %2" : "=v"(r3) : "v"(a), "v"(b));
  asm volatile("v_sub_u16 %0, %1, %2" : "=v"(r4) : "v"(b), "v"(a));
  if (threadIdx.x == 0) { out[0] = r0; out[1] = r1; out[2] = r2; out[3] = r3; out[4] = r4; }
}
int main() {
  unsigned* d; hipMalloc(&d, 64); k<<<1, 64>>>(d); unsigned h[5]; hipMemcpy(h, d, 20, hipMemcpyDeviceToHost);
  printf("max_i16 e32 %08x\nmax_i16 e64 %08x\nsub_u16 e64 (dst was 77770000) %08x\npk_max_i16 %08x\nsub_u16 e32 %08x\n", h[0], h[1], h[2], h[3], h[4]);
  return 0;
}

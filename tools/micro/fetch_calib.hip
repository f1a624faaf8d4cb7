// FETCH_SIZE calibration for narrow per-lane loads (MI355X_MICROARCH.md: the
// counter is calibrated only for 16-B/lane streaming reads, where it reports
// half the bytes).  Each kernel reads a 1 GiB buffer exactly once, coalesced,
// with one load width: 1 B, 4 B or 16 B per lane.  Run under
//   rocprofv3 --pmc FETCH_SIZE -- tools/micro/fetch_calib
// and compare each dispatch's FETCH_SIZE (KiB) with the bytes printed here.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                   \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

template <class T>
__global__ void read_all(const T* __restrict__ p, size_t n, unsigned* __restrict__ out) {
  unsigned acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    if constexpr (sizeof(T) == 16) {
      const uint4 v = reinterpret_cast<const uint4*>(p)[i];
      acc += v.x ^ v.y ^ v.z ^ v.w;
    } else {
      acc += (unsigned)p[i];
    }
  }
  if (acc == 0x12345678u) out[0] = acc;  // keeps the loads; never true for the zeroed buffer
}

int main() {
  const size_t bytes = 1ull << 30;
  void* buf;
  unsigned* out;
  CHECK(hipMalloc(&buf, bytes));
  CHECK(hipMalloc(&out, 4));
  CHECK(hipMemset(buf, 0, bytes));
  CHECK(hipDeviceSynchronize());
  const int grid = 256 * 8 * 4;
  read_all<uint8_t><<<grid, 256>>>((const uint8_t*)buf, bytes, out);
  read_all<uint32_t><<<grid, 256>>>((const uint32_t*)buf, bytes / 4, out);
  read_all<uint4><<<grid, 256>>>((const uint4*)buf, bytes / 16, out);
  CHECK(hipDeviceSynchronize());
  std::printf("each dispatch read %zu bytes (%.1f KiB): 1 B, 4 B, 16 B per lane\n", bytes, bytes / 1024.0);
  return 0;
}

// Cost of bringing up the HIP runtime on one device, phase by phase (ms):
// first runtime call, stream, device and pinned allocations, first kernel.
//   hipcc --offload-arch=gfx950 -O2 -o tools/micro/init_probe tools/micro/init_probe.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void touch(int* p) { p[threadIdx.x] = threadIdx.x; }

int main() {
  using clk = std::chrono::steady_clock;
  auto t = clk::now();
  auto lap = [&](const char* what) {
    const auto n = clk::now();
    std::printf("%-16s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(n - t).count());
    t = n;
  };
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 1;
  lap("device count");
  if (hipSetDevice(0) != hipSuccess) return 1;
  lap("set device");
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
  lap("stream");
  int* d = nullptr;
  if (hipMalloc(&d, 64 << 20) != hipSuccess) return 1;
  lap("hipMalloc 64M");
  void* h = nullptr;
  if (hipHostMalloc(&h, 16 << 20, hipHostMallocDefault) != hipSuccess) return 1;
  lap("hipHostMalloc 16M");
  touch<<<1, 64, 0, s>>>(d);
  if (hipStreamSynchronize(s) != hipSuccess) return 1;
  lap("first kernel");
  touch<<<1, 64, 0, s>>>(d);
  if (hipStreamSynchronize(s) != hipSuccess) return 1;
  lap("second kernel");
  (void)hipFree(d);
  lap("hipFree");
  (void)hipHostFree(h);
  lap("hipHostFree");
  return 0;
}

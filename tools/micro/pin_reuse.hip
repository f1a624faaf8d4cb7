// Which buffer went wrong in the round-5 concurrent-inflate corruption?
// Experiments on the three ingredients of the pre-0d2f591 fcs_bgzf_inflate:
//
//   E1  H2D hipMemcpyAsync from PAGEABLE memory whose virtual range was
//       unmapped and mapped again (new physical pages, same address) between
//       copies -- what a window reader's freshly allocated chunk vectors did
//       (glibc serves 24 MiB vectors by mmap, and munmap/mmap hands the same
//       range back);
//   E2  the same for D2H into pageable memory;
//   E3  the stream-ordered pool (hipMallocAsync / hipFreeAsync) from 16
//       threads, one stream each, every allocation filled and checked by the
//       device with its owner's pattern;
//   E4  E1 from 16 threads at once, one stream each.
//
// Each trial's data carries a per-trial pattern; a stale copy shows up as
// words of an earlier trial.  Prints mismatching words per experiment.
//   hipcc --offload-arch=gfx950 -O2 -o tools/micro/pin_reuse tools/micro/pin_reuse.hip -lpthread
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(2);                                                           \
    }                                                                         \
  } while (0)

__host__ __device__ inline uint32_t pat(uint32_t tag, uint64_t i) { return (tag << 24) ^ (uint32_t)(i * 2654435761u); }

__global__ void fill(uint32_t* p, uint64_t n, uint32_t tag) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = pat(tag, i);
}

__global__ void check(const uint32_t* p, uint64_t n, uint32_t tag, unsigned* bad) {
  unsigned b = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    b += p[i] != pat(tag, i);
  if (b) atomicAdd(bad, b);
}

static uint64_t host_bad(const uint32_t* p, uint64_t n, uint32_t tag) {
  uint64_t b = 0;
  for (uint64_t i = 0; i < n; ++i) b += p[i] != pat(tag, i);
  return b;
}

static void* map(size_t bytes, void* at) {
  void* p = mmap(at, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | (at ? MAP_FIXED : 0), -1, 0);
  if (p == MAP_FAILED) std::exit(3);
  return p;
}

// E1 / E2 / E4 body: `trials` copies through one remapped pageable range.
static void remap_trials(bool h2d, size_t bytes, int trials, uint32_t tag0, std::atomic<uint64_t>& bad_words,
                         std::atomic<int>& bad_trials, std::atomic<int>& same_va) {
  const uint64_t n = bytes / 4;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  uint32_t* d;
  unsigned* dbad;
  CK(hipMalloc(&d, bytes));
  CK(hipMalloc(&dbad, 4));
  void* va = nullptr;
  for (int t = 0; t < trials; ++t) {
    const uint32_t tag = (tag0 + (uint32_t)t) & 0xff;
    auto* h = static_cast<uint32_t*>(map(bytes, va));
    if (va && h == va) same_va++;
    va = h;
    uint64_t b = 0;
    if (h2d) {
      for (uint64_t i = 0; i < n; ++i) h[i] = pat(tag, i);
      CK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s));
      CK(hipMemsetAsync(dbad, 0, 4, s));
      check<<<1024, 256, 0, s>>>(d, n, tag, dbad);
      unsigned hb = 0;
      CK(hipMemcpyAsync(&hb, dbad, 4, hipMemcpyDeviceToHost, s));
      CK(hipStreamSynchronize(s));
      b = hb;
    } else {
      std::memset(h, 0, bytes);
      fill<<<1024, 256, 0, s>>>(d, n, tag);
      CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s));
      CK(hipStreamSynchronize(s));
      b = host_bad(h, n, tag);
    }
    if (b) bad_words += b, bad_trials++;
    munmap(h, bytes);  // the next trial maps the same range again (MAP_FIXED)
  }
  CK(hipFree(d));
  CK(hipFree(dbad));
  CK(hipStreamDestroy(s));
}

// E3: one thread's stream-ordered pool allocations.
static void pool_trials(size_t bytes, int trials, uint32_t tid, unsigned* dbad) {
  const uint64_t n = bytes / 4;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int t = 0; t < trials; ++t) {
    const uint32_t tag = (tid * 31 + (uint32_t)t) & 0xff;
    uint32_t* x;
    CK(hipMallocAsync((void**)&x, bytes, s));
    fill<<<256, 256, 0, s>>>(x, n, tag);
    check<<<256, 256, 0, s>>>(x, n, tag, dbad + tid);
    CK(hipFreeAsync(x, s));
    if (t % 4 == 3) CK(hipStreamSynchronize(s));
  }
  CK(hipStreamSynchronize(s));
  CK(hipStreamDestroy(s));
}

int main(int argc, char** argv) {
  const int trials = argc > 1 ? std::atoi(argv[1]) : 40;
  CK(hipSetDevice(0));
  for (size_t mib : {1, 24}) {
    const size_t bytes = mib << 20;
    for (int h2d = 1; h2d >= 0; --h2d) {
      std::atomic<uint64_t> bw{0};
      std::atomic<int> bt{0}, sv{0};
      remap_trials(h2d, bytes, trials, 1, bw, bt, sv);
      std::printf("E%d %s pageable, remapped range, %2zu MiB, 1 thread : %3d of %d trials wrong (%llu words), "
                  "same address %d\n",
                  h2d ? 1 : 2, h2d ? "H2D from" : "D2H into", mib, bt.load(), trials, (unsigned long long)bw.load(),
                  sv.load());
    }
    {
      const int nt = 16;
      unsigned* dbad;
      CK(hipMalloc(&dbad, 4 * nt));
      CK(hipMemset(dbad, 0, 4 * nt));
      std::vector<std::thread> th;
      for (int k = 0; k < nt; ++k) th.emplace_back(pool_trials, bytes, trials * 4, (uint32_t)k, dbad);
      for (auto& t : th) t.join();
      unsigned hb[16];
      CK(hipMemcpy(hb, dbad, 4 * nt, hipMemcpyDeviceToHost));
      unsigned long long tot = 0;
      for (int k = 0; k < nt; ++k) tot += hb[k];
      std::printf("E3 stream-ordered pool, %2zu MiB, 16 threads x %d allocations: %llu wrong words\n", mib,
                  trials * 4, tot);
      CK(hipFree(dbad));
    }
    for (int h2d = 1; h2d >= 0; --h2d) {
      std::atomic<uint64_t> bw{0};
      std::atomic<int> bt{0}, sv{0};
      std::vector<std::thread> th;
      for (int k = 0; k < 16; ++k)
        th.emplace_back([&, k] { remap_trials(h2d, bytes, trials, 1 + 7 * k, bw, bt, sv); });
      for (auto& t : th) t.join();
      std::printf("E4 %s pageable, remapped ranges, %2zu MiB, 16 threads: %3d of %d trials wrong (%llu words)\n",
                  h2d ? "H2D from" : "D2H into", mib, bt.load(), 16 * trials, (unsigned long long)bw.load());
    }
  }
  return 0;
}

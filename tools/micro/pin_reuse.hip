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
//       device with its owner's pattern: (a) default pool attributes, (b) the
//       stream synchronised before each free, (c) opportunistic reuse and
//       internal dependencies switched off, (d) as (b) with every pool call
//       under one mutex, (e) one host thread over 16 streams, (f) control:
//       hipMalloc / hipFree from 16 threads;
//   E4  E1 from 16 threads at once, one stream each (fresh mappings).
//
// Each trial's data carries a per-trial pattern; a stale copy shows up as
// words of an earlier trial.  Prints mismatching words per experiment.
//   hipcc --offload-arch=gfx950 -O2 -rdynamic -o tools/micro/pin_reuse tools/micro/pin_reuse.hip -lpthread
#include <hip/hip_runtime.h>
#include <execinfo.h>
#include <signal.h>
#include <sys/mman.h>
#include <unistd.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
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

static volatile int g_exp = 0, g_trial = 0;
static void on_segv(int) {
  char b[96];
  const int n = std::snprintf(b, sizeof b, "SIGSEGV in experiment %d trial %d\n", g_exp, g_trial);
  (void)!write(2, b, (size_t)n);
  void* fr[32];
  backtrace_symbols_fd(fr, backtrace(fr, 32), 2);
  _exit(139);
}

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

static void* map(size_t bytes, void* at, bool fixed) {
  void* p = mmap(at, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | (at && fixed ? MAP_FIXED : 0), -1, 0);
  if (p == MAP_FAILED) std::exit(3);
  return p;
}

// E1 / E2 / E4 body: `trials` copies through one remapped pageable range.
// fixed: map the same range again with MAP_FIXED (one thread only: with
// several, a range one thread unmapped may already be another's).
static void remap_trials(bool h2d, size_t bytes, int trials, uint32_t tag0, std::atomic<uint64_t>& bad_words,
                         std::atomic<int>& bad_trials, std::atomic<int>& same_va, bool fixed) {
  const uint64_t n = bytes / 4;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  uint32_t* d;
  unsigned* dbad;
  CK(hipMalloc(&d, bytes));
  CK(hipMalloc(&dbad, 4));
  void* va = nullptr;
  for (int t = 0; t < trials; ++t) {
    g_trial = t;
    const uint32_t tag = (tag0 + (uint32_t)t) & 0xff;
    auto* h = static_cast<uint32_t*>(map(bytes, va, fixed));
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
    munmap(h, bytes);  // the next trial maps the range again (fixed), or whatever the kernel hands out
  }
  CK(hipFree(d));
  CK(hipFree(dbad));
  CK(hipStreamDestroy(s));
}

// E3: one thread's stream-ordered pool allocations.  sync_before_free: the
// stream is synchronised before each hipFreeAsync (the pre-0d2f591 inflate
// call's order: copies, kernel, copy back, event wait, then the free), so
// every allocation's work has finished before the pool gets it back.
static std::mutex g_pool_mu;
static bool g_pool_serialised = false;  // E3d: every hipMallocAsync / hipFreeAsync under one mutex
static bool g_plain_malloc = false;     // E3f (control): hipMalloc / hipFree instead of the pool

static void pool_trials(size_t bytes, int trials, uint32_t tid, unsigned* dbad, bool sync_before_free) {
  const uint64_t n = bytes / 4;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int t = 0; t < trials; ++t) {
    const uint32_t tag = 1 + (tid * 16 + (uint32_t)t % 16);  // distinct per thread
    uint32_t* x;
    {
      std::unique_lock<std::mutex> lk(g_pool_mu, std::defer_lock);
      if (g_pool_serialised) lk.lock();
      if (g_plain_malloc) CK(hipMalloc((void**)&x, bytes));
      else CK(hipMallocAsync((void**)&x, bytes, s));
    }
    fill<<<256, 256, 0, s>>>(x, n, tag);
    check<<<256, 256, 0, s>>>(x, n, tag, dbad + tid);
    if (sync_before_free) CK(hipStreamSynchronize(s));
    {
      std::unique_lock<std::mutex> lk(g_pool_mu, std::defer_lock);
      if (g_pool_serialised) lk.lock();
      if (g_plain_malloc) CK(hipFree(x));
      else CK(hipFreeAsync(x, s));
    }
    if (t % 4 == 3) CK(hipStreamSynchronize(s));
  }
  CK(hipStreamSynchronize(s));
  CK(hipStreamDestroy(s));
}

// E3e: one host thread, 16 streams in turn (no concurrent host calls at all).
static unsigned long long pool_one_thread(size_t bytes, int trials) {
  const uint64_t n = bytes / 4;
  const int ns = 16;
  hipStream_t s[ns];
  for (auto& x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
  unsigned* dbad;
  CK(hipMalloc(&dbad, 4));
  CK(hipMemset(dbad, 0, 4));
  for (int t = 0; t < trials * ns; ++t) {
    hipStream_t q = s[t % ns];
    const uint32_t tag = 1 + (uint32_t)(t % 250);
    uint32_t* x;
    CK(hipMallocAsync((void**)&x, bytes, q));
    fill<<<256, 256, 0, q>>>(x, n, tag);
    check<<<256, 256, 0, q>>>(x, n, tag, dbad);
    CK(hipFreeAsync(x, q));
  }
  CK(hipDeviceSynchronize());
  unsigned hb = 0;
  CK(hipMemcpy(&hb, dbad, 4, hipMemcpyDeviceToHost));
  CK(hipFree(dbad));
  for (auto& x : s) CK(hipStreamDestroy(x));
  return hb;
}

// E3 over 16 threads; returns the wrong words.
static unsigned long long pool_experiment(size_t bytes, int trials, bool sync_before_free) {
  const int nt = 16;
  unsigned* dbad;
  CK(hipMalloc(&dbad, 4 * nt));
  CK(hipMemset(dbad, 0, 4 * nt));
  std::vector<std::thread> th;
  for (int k = 0; k < nt; ++k) th.emplace_back(pool_trials, bytes, trials, (uint32_t)k, dbad, sync_before_free);
  for (auto& t : th) t.join();
  unsigned hb[16];
  CK(hipMemcpy(hb, dbad, 4 * nt, hipMemcpyDeviceToHost));
  unsigned long long tot = 0;
  for (int k = 0; k < nt; ++k) tot += hb[k];
  CK(hipFree(dbad));
  return tot;
}

int main(int argc, char** argv) {
  const int trials = argc > 1 ? std::atoi(argv[1]) : 40;
  std::setvbuf(stdout, nullptr, _IONBF, 0);
  signal(SIGSEGV, on_segv);
  CK(hipSetDevice(0));
  for (size_t mib : {1, 24}) {
    const size_t bytes = mib << 20;
    for (int h2d = 1; h2d >= 0; --h2d) {
      std::atomic<uint64_t> bw{0};
      std::atomic<int> bt{0}, sv{0};
      g_exp = (h2d ? 1 : 2) * 100 + (int)mib;
      remap_trials(h2d, bytes, trials, 1, bw, bt, sv, true);
      std::printf("E%d %s pageable, remapped range, %2zu MiB, 1 thread : %3d of %d trials wrong (%llu words), "
                  "same address %d\n",
                  h2d ? 1 : 2, h2d ? "H2D from" : "D2H into", mib, bt.load(), trials, (unsigned long long)bw.load(),
                  sv.load());
    }
    for (int variant = 0; variant < 4; ++variant) {
      g_pool_serialised = variant == 3;
      g_exp = 300 + 10 * variant + (int)mib;
      hipMemPool_t pool;
      CK(hipDeviceGetDefaultMemPool(&pool, 0));
      int on = variant == 2 ? 0 : 1;  // variant 2: no opportunistic reuse, no internal dependencies
      CK(hipMemPoolSetAttribute(pool, hipMemPoolReuseAllowOpportunistic, &on));
      CK(hipMemPoolSetAttribute(pool, hipMemPoolReuseAllowInternalDependencies, &on));
      const unsigned long long tot = pool_experiment(bytes, trials * 4, variant == 1 || variant == 3);
      std::printf("E3%c stream-ordered pool%s, %2zu MiB, 16 threads x %d allocations: %llu wrong words\n",
                  'a' + variant,
                  variant == 0   ? " (default attributes)"
                  : variant == 1 ? " (stream synchronised before each free)"
                  : variant == 2 ? " (opportunistic reuse and internal dependencies off)"
                                 : " (as b, every pool call under one process-wide mutex)",
                  mib, trials * 4, tot);
      on = 1;
      CK(hipMemPoolSetAttribute(pool, hipMemPoolReuseAllowOpportunistic, &on));
      CK(hipMemPoolSetAttribute(pool, hipMemPoolReuseAllowInternalDependencies, &on));
    }
    g_pool_serialised = false;
    g_exp = 350 + (int)mib;
    std::printf("E3e stream-ordered pool, one host thread, 16 streams in turn, %2zu MiB, %d allocations: %llu wrong "
                "words\n", mib, trials * 4 * 16, pool_one_thread(bytes, trials * 4));
    g_plain_malloc = true;
    g_exp = 360 + (int)mib;
    std::printf("E3f control: hipMalloc / hipFree, 16 threads, %2zu MiB, 16 x %d allocations: %llu wrong words\n", mib,
                trials * 4, pool_experiment(bytes, trials * 4, true));
    g_plain_malloc = false;
    for (int h2d = 1; h2d >= 0; --h2d) {
      std::atomic<uint64_t> bw{0};
      std::atomic<int> bt{0}, sv{0};
      std::vector<std::thread> th;
      g_exp = (h2d ? 400 : 500) + (int)mib;
      for (int k = 0; k < 16; ++k)
        th.emplace_back([&, k] { remap_trials(h2d, bytes, trials, 1 + 7 * k, bw, bt, sv, false); });
      for (auto& t : th) t.join();
      std::printf("E4 %s pageable, fresh mappings, %2zu MiB, 16 threads: %3d of %d trials wrong (%llu words)\n",
                  h2d ? "H2D from" : "D2H into", mib, bt.load(), 16 * trials, (unsigned long long)bw.load());
    }
  }
  return 0;
}

// Times the GPU bring-up steps a fresh fcs-genome process goes through before
// its first PairHMM call (HIP runtime init, context, tables, per-thread
// session), to see what the htc stage's first calls wait for.
// build: g++ -O2 -std=c++17 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude tools/init_probe.cpp \
//          -o tools/init_probe -Lfalcon-genome_amd -lfcship -L/opt/rocm/lib -lamdhip64 -lpthread \
//          -Wl,-rpath,'$ORIGIN/../falcon-genome_amd' -Wl,-rpath,/opt/rocm/lib
#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cstdio>
#include <thread>

#include "fcship.h"

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static int one_call(int n) {
  static uint8_t b[256], q[256], g[256], iq[256];
  for (int i = 0; i < 256; ++i) b[i] = "ACGT"[i & 3], q[i] = 30, g[i] = 10, iq[i] = 45;
  const fcs_phmm_read r{b, q, iq, iq, g, n};
  const fcs_phmm_hap h{b, n};
  double out = 0;
  fcs_phmm_opts o;
  fcs_phmm_opts_default(&o);
  return fcs_phmm_compute(&r, 1, &h, 1, &out, &o);
}

int main() {
  const double t0 = now_ms();
  int n = 0;
  (void)hipGetDeviceCount(&n);
  const double t1 = now_ms();
  (void)hipSetDevice(0);
  (void)hipFree(nullptr);
  const double t2 = now_ms();
  fcs_phmm_plan* plan = nullptr;
  int rc = fcs_phmm_plan_create(0, 16, &plan);
  const double t2b = now_ms();
  rc |= fcs_phmm_plan_destroy(plan);
  const double t2c = now_ms();
  rc |= one_call(1);
  const double t3 = now_ms();
  rc |= one_call(1);
  const double t4 = now_ms();
  double tt = 0;
  std::thread th([&] {
    const double a = now_ms();
    rc |= one_call(1);
    tt = now_ms() - a;
  });
  th.join();
  const double t5 = now_ms();
  double t16 = 0;
  {
    const double a = now_ms();
    std::thread ts[16];
    for (auto& t : ts) t = std::thread([&] { rc |= one_call(100); });
    for (auto& t : ts) t.join();
    t16 = now_ms() - a;
  }
  // the pieces of a session on a fresh thread
  double st_ms = 0, ev_ms = 0, hm_ms = 0, dm_ms = 0;
  std::thread tp([&] {
    double a = now_ms();
    hipStream_t s[4];
    for (auto& x : s) (void)hipStreamCreateWithFlags(&x, hipStreamNonBlocking);
    st_ms = now_ms() - a;
    a = now_ms();
    hipEvent_t e[7];
    for (auto& x : e) (void)hipEventCreateWithFlags(&x, hipEventDisableTiming);
    ev_ms = now_ms() - a;
    a = now_ms();
    void* h = nullptr;
    (void)hipHostMalloc(&h, 16 << 20, hipHostMallocDefault);
    hm_ms = now_ms() - a;
    a = now_ms();
    void* d = nullptr;
    (void)hipMalloc(&d, 16 << 20);
    dm_ms = now_ms() - a;
  });
  tp.join();
  std::printf("{\"four_streams_ms\": %.2f, \"seven_events_ms\": %.2f, \"host_malloc_16MB_ms\": %.2f, "
              "\"malloc_16MB_ms\": %.2f}\n", st_ms, ev_ms, hm_ms, dm_ms);
  std::printf("{\"plan_create_ms\": %.1f, \"plan_destroy_ms\": %.1f}\n", t2b - t2, t2c - t2b);
  std::printf("{\"devices\": %d, \"hip_init_ms\": %.1f, \"context_ms\": %.1f, \"first_call_ms\": %.1f, "
              "\"second_call_ms\": %.2f, \"new_thread_first_call_ms\": %.1f, \"thread_total_ms\": %.1f, "
              "\"sixteen_new_threads_ms\": %.1f, \"rc\": %d}\n",
              n, t1 - t0, t2 - t1, t3 - t2, t4 - t3, tt, t5 - t4, t16, rc);
  return rc != 0;
}

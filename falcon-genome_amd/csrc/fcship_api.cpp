// C-ABI of libfcship.so (include/fcship.h): argument checking, device state,
// host<->device marshaling and the multi-stage device pipelines.
//
// Error behaviour mirrors the reference's contract: a failing
// call returns a negative code and leaves a "[E::fcship] ..." message (the
// prefix LogUtils::findError scans task logs for,
// /root/reference/src/LogUtils.cpp:10-40) retrievable with fcs_last_error().
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#include "fcship_internal.h"

namespace fcs {

static thread_local std::string g_last_error;
static thread_local int64_t g_last_rescued = 0;
static thread_local double g_last_device_ms = 0, g_last_rescue_ms = 0;
void set_error(const std::string& msg) { g_last_error = msg; }
int fail(int code, const std::string& msg) {
  set_error(msg);
  return code;
}

namespace {

std::mutex g_dev_mu;
std::map<int, std::unique_ptr<DeviceTables>> g_tables;
int g_default_device = 0;

int check_device(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
    return fail(FCS_ERR_DEVICE, "[E::fcship] no HIP device available (libfcship requires an MI355X / gfx950)");
  if (device < 0 || device >= n) return fail(FCS_ERR_INVALID, "[E::fcship] device ordinal out of range");
  return FCS_OK;
}

struct ForkSet {
  hipStream_t side[kForkStreams - 1] = {};
  hipEvent_t fork = nullptr;
  hipEvent_t join[kForkStreams - 1] = {};
};

// Side streams and events of a launch stream on the current device, created
// on the stream's first fork and kept for the process (a stream costs about
// 3.5 ms to create on gfx950, so they are made once per launch stream, not
// per call or per thread).  A launch stream is used by one call at a time:
// a pooled session's stream by its lease holder, a caller's stream by the
// caller.
std::mutex g_fork_mu;
auto* g_fork_sets = new std::map<std::pair<int, hipStream_t>, ForkSet>();  // outlives static teardown

ForkSet* fork_set(hipStream_t s) {
  int device = 0;
  if (hipGetDevice(&device) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(g_fork_mu);
  auto* sets = g_fork_sets;
  auto it = sets->find({device, s});
  if (it != sets->end()) return &it->second;
  ForkSet f;
  if (hipEventCreateWithFlags(&f.fork, hipEventDisableTiming) != hipSuccess) return nullptr;
  for (int i = 0; i < kForkStreams - 1; ++i)
    if (hipStreamCreateWithFlags(&f.side[i], hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&f.join[i], hipEventDisableTiming) != hipSuccess)
      return nullptr;
  return &((*sets)[{device, s}] = f);
}

}  // namespace

int fork_streams(hipStream_t s, hipStream_t (&fs)[kForkStreams]) {
  ForkSet* f = fork_set(s);
  if (!f) return fail(FCS_ERR_DEVICE, "[E::fcship] cannot create side streams");
  FCS_HIP_CHECK(hipEventRecord(f->fork, s));
  fs[0] = s;
  for (int i = 0; i < kForkStreams - 1; ++i) {
    FCS_HIP_CHECK(hipStreamWaitEvent(f->side[i], f->fork, 0));
    fs[i + 1] = f->side[i];
  }
  return FCS_OK;
}

int join_streams(hipStream_t s, const hipStream_t (&fs)[kForkStreams]) {
  ForkSet* f = fork_set(s);
  if (!f) return fail(FCS_ERR_DEVICE, "[E::fcship] cannot create side streams");
  for (int i = 0; i < kForkStreams - 1; ++i) {
    FCS_HIP_CHECK(hipEventRecord(f->join[i], fs[i + 1]));
    FCS_HIP_CHECK(hipStreamWaitEvent(s, f->join[i], 0));
  }
  return FCS_OK;
}

namespace {

// Aligned sub-allocations of one staging buffer.
struct Layout {
  size_t total = 0;
  size_t add(size_t bytes) {
    const size_t o = total;
    total += (bytes + 255) & ~(size_t)255;
    return o;
  }
};

}  // namespace

// State of the synchronous host-pointer entry points on one device: a stream,
// a PairHMM plan and an SW plan grown to the largest batch seen, one device
// arena for the batch's inputs and outputs and one pinned host arena it is
// staged through (one H2D and one D2H copy per call).  After warm-up a call
// allocates nothing: no hipMalloc/hipFree (hipFree synchronises the whole
// device, so per-call frees serialised the Executor's concurrent shard
// threads on one GPU) and no null-stream operation.
//
// Sessions live in a per-device pool and a call leases one for its duration.
// Creating one costs four streams (its own and three fork side streams,
// about 14 ms together); with one session per calling thread, the htc stage's
// 16 shard threads spent 0.22 s creating 64 streams, serialised inside the
// runtime, before their first PairHMM call.  The pool holds at most
// FCS_SESSIONS_PER_DEVICE (default 4) sessions, which fcs_device_warmup
// creates ahead of time; a call finding all of them busy waits for one.
struct Session {
  int device = 0;
  hipStream_t s = nullptr;
  fcs_phmm_plan* phmm = nullptr;
  fcs_bsw_plan* bsw = nullptr;
  void* dev = nullptr;
  size_t dev_cap = 0;
  void* host = nullptr;
  size_t host_cap = 0;
  hipEvent_t ev[3] = {nullptr, nullptr, nullptr};  // PairHMM call: start, after forward, after rescue
  hipEvent_t done = nullptr;                        // inflate sessions: a blocking-sync event (no host spin)
  int ensure_dev(size_t bytes);
  int ensure_host(size_t bytes);
  int ensure_phmm(int64_t pairs);
  int ensure_bsw(int64_t tasks);
  template <typename T> T* d(size_t off) const { return reinterpret_cast<T*>(static_cast<char*>(dev) + off); }
  template <typename T> T* h(size_t off) const { return reinterpret_cast<T*>(static_cast<char*>(host) + off); }
};

namespace {

size_t grown(size_t need, size_t cap) { return std::max(need + need / 4, std::min<size_t>(2 * cap, need + (1u << 30))); }

// Pool kinds: the compute sessions (PairHMM / SW entry points) and the BGZF
// inflate sessions, a pool of their own so the htc shards' many small inflate
// calls (one per 4 MiB of compressed BAM) neither wait behind PairHMM passes
// nor pay for fork streams they never use.
enum SessionKind : int { kComputeSession = 0, kInflateSession = 1 };

int sessions_per_device(int kind = kComputeSession) {
  static const int n[2] = {[] {
                             const char* e = std::getenv("FCS_SESSIONS_PER_DEVICE");
                             const int v = e && *e ? std::atoi(e) : 4;
                             return std::max(1, std::min(v, 64));
                           }(),
                           [] {
                             const char* e = std::getenv("FCS_BGZF_SESSIONS_PER_DEVICE");
                             const int v = e && *e ? std::atoi(e) : 16;
                             return std::max(1, std::min(v, 64));
                           }()};
  return n[kind];
}

struct SessionPool {
  std::mutex mu;
  std::condition_variable cv;
  std::vector<Session*> all, idle;  // never freed: the pools outlive static teardown and the HIP runtime
  int creating = 0;
  bool releasing = false;  // fcs_device_release is resetting the device: leases are refused
};

SessionPool& session_pool(int device, int kind = kComputeSession) {
  static std::mutex mu;
  static auto* pools = new std::map<std::pair<int, int>, SessionPool*>();
  std::lock_guard<std::mutex> lk(mu);
  SessionPool*& p = (*pools)[{device, kind}];
  if (!p) p = new SessionPool();
  return *p;
}

// A new session on `device` (the current device), or null.
int64_t env_int(const char* name, int64_t dflt) {
  const char* e = std::getenv(name);
  return e && *e ? std::max<int64_t>(0, std::atoll(e)) : dflt;
}

Session* create_session(int device, int kind = kComputeSession) {
  auto* S = new Session();
  S->device = device;
  if (hipStreamCreateWithFlags(&S->s, hipStreamNonBlocking) != hipSuccess ||
      (kind == kComputeSession && !fork_set(S->s))) {
    delete S;  // a failed stream is not reused; nothing else was created
    return nullptr;
  }
  // FCS_SESSION_PRESIZE_MB (default 24, 0 = off): a compute session starts
  // with staging of that size and a PairHMM plan for FCS_SESSION_PRESIZE_PAIRS
  // (default 120000), so the first passes of a run (an htc shard's pass is
  // ~17 MB and ~90K pairs on the 30x panel) do not allocate pinned and device
  // memory while other threads' passes are in flight; sessions are created by
  // the warm-up, off the callers' path.  A failed presize only leaves the
  // session to grow on demand.
  static const size_t presize = (size_t)env_int("FCS_SESSION_PRESIZE_MB", 24) << 20;
  static const int64_t presize_pairs = env_int("FCS_SESSION_PRESIZE_PAIRS", 120000);
  if (kind == kComputeSession && presize > 0) {
    (void)(S->ensure_host(presize) || S->ensure_dev(presize) || (presize_pairs > 0 && S->ensure_phmm(presize_pairs)));
  }
  return S;
}

// Grows the pool of `device` (the current device) to n idle-or-busy sessions.
int prefill_sessions(int device, int n) {
  SessionPool& P = session_pool(device);
  n = std::min(n, sessions_per_device());
  for (;;) {
    {
      std::lock_guard<std::mutex> lk(P.mu);
      if (P.releasing) return fail(FCS_ERR_INVALID, "[E::fcship] the device is being released");
      if ((int)P.all.size() + P.creating >= n) return FCS_OK;
      ++P.creating;
    }
    Session* S = create_session(device);
    {
      std::lock_guard<std::mutex> lk(P.mu);
      --P.creating;
      if (S) P.all.push_back(S), P.idle.push_back(S);
    }
    P.cv.notify_one();
    if (!S) return fail(FCS_ERR_DEVICE, "[E::fcship] stream creation failed");
  }
}

// Synchronises a session's stream when it goes out of scope (before the
// lease returns the session to the pool): an error path must not hand the
// next holder a session whose H2D copy is still reading the pinned staging
// that holder is about to refill.
struct StreamDrain {
  hipStream_t s;
  ~StreamDrain() { (void)hipStreamSynchronize(s); }
};

// A session of `device` (the current device) held for one call.
class SessionLease {
 public:
  SessionLease() = default;
  SessionLease(const SessionLease&) = delete;
  SessionLease& operator=(const SessionLease&) = delete;
  ~SessionLease() { release(); }
  int acquire(int device, int kind = kComputeSession) {
    release();
    SessionPool& P = session_pool(device, kind);
    std::unique_lock<std::mutex> lk(P.mu);
    for (;;) {
      if (P.releasing) return fail(FCS_ERR_INVALID, "[E::fcship] the device is being released");
      if (!P.idle.empty()) {
        s_ = P.idle.back();
        P.idle.pop_back();
        pool_ = &P;
        return FCS_OK;
      }
      if ((int)P.all.size() + P.creating < sessions_per_device(kind)) break;
      P.cv.wait(lk);
    }
    ++P.creating;
    lk.unlock();
    Session* S = create_session(device, kind);
    lk.lock();
    --P.creating;
    if (!S) {
      P.cv.notify_one();
      return fail(FCS_ERR_DEVICE, "[E::fcship] stream creation failed");
    }
    P.all.push_back(S);
    s_ = S;
    pool_ = &P;
    return FCS_OK;
  }
  // An idle session whose arenas already hold `bytes` (host and device), or
  // false at once: no waiting, no session created, no arena grown.
  bool try_acquire(int device, int kind, size_t bytes) {
    release();
    SessionPool& P = session_pool(device, kind);
    std::lock_guard<std::mutex> lk(P.mu);
    if (P.releasing) return false;
    for (size_t i = 0; i < P.idle.size(); ++i) {
      Session* S = P.idle[i];
      if (S->host_cap >= bytes && S->dev_cap >= bytes) {
        P.idle.erase(P.idle.begin() + (long)i);
        s_ = S;
        pool_ = &P;
        return true;
      }
    }
    return false;
  }
  Session* operator->() const { return s_; }
  Session* get() const { return s_; }

 private:
  void release() {
    if (!s_) return;
    {
      std::lock_guard<std::mutex> lk(pool_->mu);
      pool_->idle.push_back(s_);
    }
    pool_->cv.notify_one();
    s_ = nullptr;
    pool_ = nullptr;
  }
  Session* s_ = nullptr;
  SessionPool* pool_ = nullptr;
};

BswParams to_params(const fcs_bsw_params* p) {
  BswParams q;
  std::memcpy(q.mat, p->mat, 25);
  q.o_del = p->o_del;
  q.e_del = p->e_del;
  q.o_ins = p->o_ins;
  q.e_ins = p->e_ins;
  q.end_bonus = p->end_bonus;
  q.zdrop = p->zdrop;
  int mx = 0;
  for (int i = 0; i < 25; ++i) mx = std::max<int>(mx, p->mat[i]);
  q.max_mat = mx;
  q.lane_ok = 1;
  for (int t = 0; t < 5; ++t) {
    uint32_t pk = 0;
    for (int c = 0; c < 5; ++c) {
      const int v = p->mat[t * 5 + c];
      if (v < -16 || v > 15) q.lane_ok = 0;
      pk |= ((uint32_t)v & 31u) << (5 * c);
    }
    q.matpack[t] = (int32_t)pk;
  }
  int mn4 = 0, mx4 = 0;
  for (int t = 0; t < 5; ++t)  // target rows A..N, query columns A..T (the pair kernel's tables)
    for (int c = 0; c < 4; ++c) mn4 = std::min<int>(mn4, p->mat[t * 5 + c]), mx4 = std::max<int>(mx4, p->mat[t * 5 + c]);
  q.pair_bias = -mn4;
  q.pair_cg = mx4 + q.pair_bias + 1;
  // the pair kernel's 16-bit z-drop arithmetic: |row distance| * e stays below 2^15
  q.pair_ok = (q.pair_cg <= 128 && p->e_del <= 16 && p->e_ins <= 16) ? 1 : 0;
  q.pair_k256 = 0x01000100;
  q.pair_one = 0x00010001;
  return q;
}

// Workspace for one SW schedule of up to cap tasks (plain hipMalloc: the
// library never uses the stream-ordered pool, see stream_workspace).
int ws_alloc(BswWorkspace& ws, int64_t cap) {
  ws.cap = cap;
  const size_t n = (size_t)std::max<int64_t>(cap, 1);
  size_t tmp = 0;
  FCS_HIP_CHECK(sort_pairs_u32(nullptr, tmp, nullptr, nullptr, nullptr, nullptr, (int)n, nullptr));
  ws.tmp_bytes = std::max<size_t>(tmp, 16);
  void** bufs[6] = {(void**)&ws.keys_in, (void**)&ws.keys_out, (void**)&ws.idx_in, (void**)&ws.idx_out,
                    (void**)&ws.bounds, &ws.tmp};
  const size_t sz[6] = {4 * n, 4 * n, 4 * n, 4 * n, (kBswWideBucket + 2) * sizeof(int64_t), ws.tmp_bytes};
  for (int i = 0; i < 6; ++i) FCS_HIP_CHECK(hipMalloc(bufs[i], sz[i]));
  return FCS_OK;
}

void ws_free(BswWorkspace& ws) {
  void* bufs[6] = {ws.keys_in, ws.keys_out, ws.idx_in, ws.idx_out, ws.bounds, ws.tmp};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  ws = BswWorkspace();
}

// The SW workspace of a caller's launch stream (fcs_bsw_extend_dev), kept per
// (device, stream) like the fork sets and grown with plain hipMalloc.  Round 5
// took it from the stream-ordered pool (hipMallocAsync / hipFreeAsync), as
// fcs_bgzf_inflate once took its scratch: on this runtime that pool hands
// memory still in use on one stream to an allocation on another.
// tools/micro/pin_reuse.hip (profiles/r6/r6b_pin_reuse.log) finds overlapping
// live allocations with 16 threads x 16 streams in every configuration tried
// (default attributes, the stream synchronised before each free, reuse
// attributes off, every pool call under one mutex) and from one thread over 16
// streams; hipMalloc / hipFree and pageable copies never.  That is the cause of
// the round-5 inflate corruption (member 0 of a call: the start of its input
// scratch, overwritten by another call).  The caller uses a stream for one call
// at a time, so one workspace per stream is enough.
std::map<std::pair<int, hipStream_t>, BswWorkspace>* g_stream_ws = new std::map<std::pair<int, hipStream_t>, BswWorkspace>();

int stream_workspace(int device, hipStream_t s, int64_t n, BswWorkspace** out) {
  std::lock_guard<std::mutex> lk(g_fork_mu);
  BswWorkspace& ws = (*g_stream_ws)[{device, s}];
  if (ws.cap < n || !ws.keys_in) {
    if (ws.keys_in) {
      FCS_HIP_CHECK(hipStreamSynchronize(s));  // the stream's last call may still read the old one
      ws_free(ws);
    }
    const int rc = ws_alloc(ws, std::max<int64_t>(n + n / 4, 4096));
    if (rc) {
      ws_free(ws);
      return rc;
    }
  }
  *out = &ws;
  return FCS_OK;
}

int check_params(const fcs_bsw_params* p) {
  if (!p) return fail(FCS_ERR_INVALID, "[E::fcship] null SW params");
  if (p->e_del <= 0 || p->e_ins <= 0 || p->o_del < 0 || p->o_ins < 0)
    return fail(FCS_ERR_INVALID, "[E::fcship] gap penalties must satisfy o >= 0, e > 0");
  return FCS_OK;
}

}  // namespace

// Stable LSD radix sort of (32-bit key, index) pairs.  rocPRIM's default picks
// a block sort + ~20 merge passes for n <= 2^20 (the C2 / C3 batch sizes:
// 0.16 ms of 7 us launches); a merge-sort limit of 0 forces its onesweep path
// (histogram + one pass per 8-bit digit) at every size.  Same order either way.
// The onesweep kernels' default tile (1024 threads x ~16 items) gives a 1M-key
// sort 62 workgroups on a 256-CU chip; 256 x 8 tiles give it ~490 but measured
// slower (C2 2.86 vs 2.93 TCUPS, C3 1.95 vs 2.05, profiles/r2/abt_*).
#ifndef FCS_SORT_BITS
#define FCS_SORT_BITS 0  // 0: rocPRIM's default onesweep config for the target
#endif
#ifndef FCS_SORT_BLOCK
#define FCS_SORT_BLOCK 1024
#endif
#ifndef FCS_SORT_ITEMS
#define FCS_SORT_ITEMS 8
#endif
#if FCS_SORT_BITS
using OnesweepConfig = rocprim::radix_sort_onesweep_config<rocprim::kernel_config<256, 12>,
                                                           rocprim::kernel_config<FCS_SORT_BLOCK, FCS_SORT_ITEMS>,
                                                           FCS_SORT_BITS, rocprim::block_radix_rank_algorithm::match>;
using SortConfig = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, OnesweepConfig, 0>;
#else
using SortConfig = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, rocprim::default_config, 0>;
#endif
hipError_t sort_pairs_u32(void* tmp, size_t& bytes, const uint32_t* kin, uint32_t* kout, const int32_t* vin,
                          int32_t* vout, int n, hipStream_t s, int end_bit) {
  return rocprim::radix_sort_pairs<SortConfig>(tmp, bytes, kin, kout, vin, vout, (size_t)n, 0, (unsigned)end_bit, s);
}

int get_device_tables(int device, DeviceTables** out) {
  std::lock_guard<std::mutex> lk(g_dev_mu);
  auto& slot = g_tables[device];
  if (!slot) slot.reset(new DeviceTables());
  DeviceTables& t = *slot;
  if (!t.ready) {
    FCS_SET_DEVICE((device));
    const size_t n = 3 * 128 + kMmEntries;
    std::vector<float> hf(n);
    std::vector<double> hd(n);
    build_phmm_tables_f(hf.data(), hf.data() + 128, hf.data() + 256, hf.data() + 384);
    build_phmm_tables_d(hd.data(), hd.data() + 128, hd.data() + 256, hd.data() + 384);
    FCS_HIP_CHECK(hipMalloc(&t.f_tabs, n * sizeof(float)));
    FCS_HIP_CHECK(hipMalloc(&t.d_tabs, n * sizeof(double)));
    FCS_HIP_CHECK(hipMemcpy(t.f_tabs, hf.data(), n * sizeof(float), hipMemcpyHostToDevice));
    FCS_HIP_CHECK(hipMemcpy(t.d_tabs, hd.data(), n * sizeof(double), hipMemcpyHostToDevice));
    t.tf = PhmmTables<float>{t.f_tabs, t.f_tabs + 128, t.f_tabs + 256, t.f_tabs + 384, ldexpf(1.f, 120),
                             log10f(ldexpf(1.f, 120))};
    t.td = PhmmTables<double>{t.d_tabs, t.d_tabs + 128, t.d_tabs + 256, t.d_tabs + 384, ldexp(1.0, 1020),
                              log10(ldexp(1.0, 1020))};
    t.ready = true;
  }
  *out = &t;
  return FCS_OK;
}

}  // namespace fcs

using namespace fcs;

// ------------------------------------------------------------------ plans
struct fcs_bsw_plan {
  int device = 0;
  BswWorkspace ws;
};

struct fcs_phmm_plan {
  int device = 0;
  int64_t max_pairs = 0;
  int32_t* idx_out = nullptr;  // the schedule: pair indices, launch class by class
  int32_t* rescue_list = nullptr;
  int32_t* fb_list = nullptr;                  // pairs the streamed kernel hands back (bytes outside ACGTN)
  unsigned long long* rescue_count = nullptr;  // [0] rescue count, [1] fallback count, then int64 class bounds
  unsigned long long* fb_count = nullptr;
  int64_t* bounds = nullptr;
  uint32_t* bin_hist = nullptr;    // the bin schedule's histogram (kept zero between schedules)
  uint32_t* bin_cursor = nullptr;  // and its running bin starts
  bool bin_zeroed = false;         // bin_hist zeroed on a schedule stream (then kept zero by the scan)
  int64_t scheduled = -1;  // n_pairs of the last schedule
  bool counters_zeroed = false;  // the last schedule's count kernel zeroed rescue_count[0..1]
};

namespace fcs {

int Session::ensure_dev(size_t bytes) {
  if (bytes <= dev_cap) return FCS_OK;
  FCS_HIP_CHECK(hipStreamSynchronize(s));
  if (dev) (void)hipFree(dev);
  dev = nullptr;
  dev_cap = 0;
  const size_t cap = grown(bytes, dev_cap);
  if (hipMalloc(&dev, cap) != hipSuccess) {
    dev = nullptr;
    return fail(FCS_ERR_NOMEM, "[E::fcship] hipMalloc of " + std::to_string(cap) + " bytes failed");
  }
  dev_cap = cap;
  return FCS_OK;
}

int Session::ensure_host(size_t bytes) {
  if (bytes <= host_cap) return FCS_OK;
  FCS_HIP_CHECK(hipStreamSynchronize(s));
  if (host) (void)hipHostFree(host);
  host = nullptr;
  host_cap = 0;
  const size_t cap = grown(bytes, host_cap);
  if (hipHostMalloc(&host, cap, hipHostMallocDefault) != hipSuccess) {
    host = nullptr;
    return fail(FCS_ERR_NOMEM, "[E::fcship] hipHostMalloc of " + std::to_string(cap) + " bytes failed");
  }
  host_cap = cap;
  return FCS_OK;
}

int Session::ensure_phmm(int64_t pairs) {
  if (phmm && phmm->max_pairs >= pairs) return FCS_OK;
  FCS_HIP_CHECK(hipStreamSynchronize(s));
  fcs_phmm_plan_destroy(phmm);
  phmm = nullptr;
  return fcs_phmm_plan_create(device, (int64_t)grown((size_t)pairs, 0), &phmm);
}

int Session::ensure_bsw(int64_t tasks) {
  if (bsw && bsw->ws.cap >= tasks) return FCS_OK;
  FCS_HIP_CHECK(hipStreamSynchronize(s));
  fcs_bsw_plan_destroy(bsw);
  bsw = nullptr;
  return fcs_bsw_plan_create(device, (int64_t)grown((size_t)tasks, 0), &bsw);
}

// FCSHIP_TEST_FAULT=drop_schedule: the PairHMM schedule publishes empty class
// ranges, as the round-1 null-stream memset race once did, so the forward
// pass computes nothing (tests/test_pairhmm_gpu.py checks it is reported).
static bool fault_drop_schedule() {
  static const bool on = [] {
    const char* e = std::getenv("FCSHIP_TEST_FAULT");
    return e && std::strcmp(e, "drop_schedule") == 0;
  }();
  return on;
}

}  // namespace fcs

static PhmmDevBatch to_dev(const fcs_phmm_batch* b) {
  PhmmDevBatch d;
  d.rb = b->read_bases;
  d.bq = b->read_bq;
  d.iq = b->read_iq;
  d.dq = b->read_dq;
  d.gq = b->read_gcp;
  d.read_off = b->read_off;
  d.read_len = b->read_len;
  d.hb = b->hap_bases;
  d.hap_off = b->hap_off;
  d.hap_len = b->hap_len;
  d.pair_read = b->pair_read;
  d.pair_hap = b->pair_hap;
  d.n_pairs = b->n_pairs;
  return d;
}

static int check_batch_shape(const fcs_phmm_batch* b) {
  if (!b) return fail(FCS_ERR_INVALID, "[E::fcship] null PairHMM batch");
  if (b->n_pairs < 0 || b->n_reads < 0 || b->n_haps < 0)
    return fail(FCS_ERR_INVALID, "[E::fcship] negative PairHMM batch size");
  if (b->n_pairs > 0x7FFFFFFF) return fail(FCS_ERR_UNSUPPORTED, "[E::fcship] more than 2^31-1 pairs per batch");
  if (b->n_pairs > 0 && (!b->read_bases || !b->read_bq || !b->read_iq || !b->read_dq || !b->read_gcp ||
                         !b->read_off || !b->read_len || !b->hap_bases || !b->hap_off || !b->hap_len ||
                         !b->pair_read || !b->pair_hap))
    return fail(FCS_ERR_INVALID, "[E::fcship] null pointer in PairHMM batch");
  if (b->max_hap_len < 0 || b->max_read_len < 0)
    return fail(FCS_ERR_INVALID, "[E::fcship] negative max length in PairHMM batch");
  return FCS_OK;
}

extern "C" {

const char* fcs_last_error(void) { return g_last_error.c_str(); }
const char* fcs_version(void) { return "fcship 0.1.0 (gfx950)"; }

int fcs_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int fcs_set_default_device(int32_t device) {
  int rc = check_device(device);
  if (rc) return rc;
  g_default_device = device;
  return FCS_OK;
}

void fcs_phmm_opts_default(fcs_phmm_opts* o) {
  if (!o) return;
  o->device = 0;
  o->use_fp64_rescue = 1;
  o->rescue_threshold = 1e-28f;
  o->exact_order = 0;
}

void fcs_bsw_params_default(fcs_bsw_params* p) {
  if (!p) return;
  // bwa_fill_scmat(a=1, b=4, -1): match a, mismatch -b, anything with N -1.
  for (int i = 0, k = 0; i < 4; ++i) {
    for (int j = 0; j < 4; ++j) p->mat[k++] = (int8_t)(i == j ? 1 : -4);
    p->mat[k++] = -1;
  }
  for (int j = 0; j < 5; ++j) p->mat[20 + j] = -1;
  p->o_del = 6;
  p->e_del = 1;
  p->o_ins = 6;
  p->e_ins = 1;
  p->end_bonus = 5;
  p->zdrop = 100;
}

int fcs_phmm_plan_create(int32_t device, int64_t max_pairs, fcs_phmm_plan** plan) {
  if (!plan || max_pairs < 0) return fail(FCS_ERR_INVALID, "[E::fcs_phmm_plan_create] bad arguments");
  int rc = check_device(device);
  if (rc) return rc;
  FCS_SET_DEVICE((device));
  DeviceTables* t = nullptr;
  rc = get_device_tables(device, &t);
  if (rc) return rc;
  std::unique_ptr<fcs_phmm_plan> p(new fcs_phmm_plan());
  p->device = device;
  p->max_pairs = max_pairs;
  const size_t n = (size_t)std::max<int64_t>(max_pairs, 1);
  FCS_HIP_CHECK(hipMalloc(&p->idx_out, n * 4));
  FCS_HIP_CHECK(hipMalloc(&p->rescue_list, n * 4));
  FCS_HIP_CHECK(hipMalloc(&p->fb_list, n * 4));
  FCS_HIP_CHECK(hipMalloc(&p->rescue_count, (2 + kPhmmLaunchClasses + 1) * sizeof(unsigned long long)));
  // Nothing is initialised here: every run writes the class bounds (the bounds
  // kernel stores all kPhmmClasses + 1 of them) and zeroes the rescue count on
  // the caller's stream.  (Round 1 zeroed them with a null-stream hipMemset,
  // which does not order against the non-blocking streams the plan runs on and
  // once landed after a schedule, so class launches computed nothing.)
  p->fb_count = p->rescue_count + 1;
  p->bounds = reinterpret_cast<int64_t*>(p->rescue_count + 2);
  constexpr size_t kBins = (size_t)1 << (kPhmmKeyBits - 4);
  FCS_HIP_CHECK(hipMalloc(&p->bin_hist, 2 * kBins * sizeof(uint32_t)));
  p->bin_cursor = p->bin_hist + kBins;
  *plan = p.release();  // (the bin histogram is zeroed on the first schedule's stream)
  return FCS_OK;
}

int fcs_phmm_plan_destroy(fcs_phmm_plan* p) {
  if (!p) return FCS_OK;
  ::fcs::DeviceScope dev_scope;
  (void)hipSetDevice(p->device);
  (void)hipFree(p->idx_out);
  (void)hipFree(p->rescue_list);
  (void)hipFree(p->fb_list);
  (void)hipFree(p->rescue_count);
  (void)hipFree(p->bin_hist);
  delete p;
  return FCS_OK;
}

int fcs_phmm_dev_schedule(fcs_phmm_plan* plan, const fcs_phmm_batch* b, void* stream) {
  if (!plan) return fail(FCS_ERR_INVALID, "[E::fcs_phmm_dev_schedule] null plan");
  int rc = check_batch_shape(b);
  if (rc) return rc;
  if (b->n_pairs > plan->max_pairs) return fail(FCS_ERR_INVALID, "[E::fcs_phmm_dev_schedule] batch exceeds plan");
  FCS_SET_DEVICE((plan->device));
  hipStream_t s = (hipStream_t)stream;
  const PhmmDevBatch d = to_dev(b);
  // The bin schedule: a counting sort on the key's top 12 bits in three
  // kernels (count, scan, scatter).  It replaced a 16-bit rocPRIM radix sort
  // (eight launches and look-back state fills, ≈ 0.15 ms of a 1M-pair C2 step;
  // A/B in profiles/r5/r5av_phmm_schedule_ab.log).  The histogram is zeroed
  // stream-ordered, once per plan (a synchronous hipMemset at plan creation
  // waited behind other shards' kernels on the device: htc PairHMM call time
  // 0.45 -> 2.2 thread-s in r5aw), and the scan kernel leaves it zero.  Any
  // failure before the scan ran may leave it dirty: the next schedule zeroes
  // it again.
  plan->scheduled = -1;
  if (!plan->bin_zeroed)
    FCS_HIP_CHECK(hipMemsetAsync(plan->bin_hist, 0, ((size_t)1 << (kPhmmKeyBits - 4)) * sizeof(uint32_t), s));
  plan->bin_zeroed = false;  // until the scan has been launched
  if ((rc = launch_phmm_bin_schedule(d, plan->idx_out, plan->bounds, plan->rescue_count, plan->bin_hist,
                                     plan->bin_cursor, s)))
    return rc;
  plan->bin_zeroed = true;
  plan->counters_zeroed = true;
  if (fault_drop_schedule()) FCS_HIP_CHECK(hipMemsetAsync(plan->bounds, 0, (kPhmmLaunchClasses + 1) * sizeof(int64_t), s));
  plan->scheduled = b->n_pairs;
  return FCS_OK;
}

int fcs_phmm_dev_forward(fcs_phmm_plan* plan, const fcs_phmm_batch* b, double* out, const fcs_phmm_opts* opts,
                         void* stream) {
  if (!plan || !opts) return fail(FCS_ERR_INVALID, "[E::fcs_phmm_dev_forward] null plan/opts");
  int rc = check_batch_shape(b);
  if (rc) return rc;
  if (plan->scheduled != b->n_pairs)
    return fail(FCS_ERR_INVALID, "[E::fcs_phmm_dev_forward] batch not scheduled (call fcs_phmm_dev_schedule)");
  if (b->n_pairs > 0 && !out) return fail(FCS_ERR_INVALID, "[E::fcs_phmm_dev_forward] null output");
  FCS_SET_DEVICE((plan->device));
  DeviceTables* t = nullptr;
  rc = get_device_tables(plan->device, &t);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  // rescue + fallback counts: zeroed by the schedule's keys kernel for the first
  // forward pass after it, by a memset for any further pass
  if (!plan->counters_zeroed)
    FCS_HIP_CHECK(hipMemsetAsync(plan->rescue_count, 0, 2 * sizeof(unsigned long long), s));
  plan->counters_zeroed = false;
  return launch_phmm_forward(to_dev(b), plan->idx_out, b->n_pairs, std::max(b->max_hap_len, 1), plan->bounds, *t,
                             opts->exact_order != 0, out, plan->rescue_list, plan->rescue_count,
                             opts->rescue_threshold, opts->use_fp64_rescue != 0, plan->fb_list, plan->fb_count, s);
}

int fcs_phmm_dev_rescue(fcs_phmm_plan* plan, const fcs_phmm_batch* b, double* out, const fcs_phmm_opts* opts,
                        void* stream) {
  if (!plan || !opts) return fail(FCS_ERR_INVALID, "[E::fcs_phmm_dev_rescue] null plan/opts");
  int rc = check_batch_shape(b);
  if (rc) return rc;
  if (!opts->use_fp64_rescue) return FCS_OK;
  FCS_SET_DEVICE((plan->device));
  DeviceTables* t = nullptr;
  rc = get_device_tables(plan->device, &t);
  if (rc) return rc;
  return launch_phmm_rescue(to_dev(b), plan->rescue_list, plan->rescue_count, b->n_pairs,
                            std::max(b->max_hap_len, 1), *t, opts->exact_order != 0, out, (hipStream_t)stream);
}

int fcs_phmm_dev_run(fcs_phmm_plan* plan, const fcs_phmm_batch* b, double* out, const fcs_phmm_opts* opts,
                     void* stream) {
  int rc = fcs_phmm_dev_schedule(plan, b, stream);
  if (rc) return rc;
  rc = fcs_phmm_dev_forward(plan, b, out, opts, stream);
  if (rc) return rc;
  return fcs_phmm_dev_rescue(plan, b, out, opts, stream);
}

int fcs_stream_release(int32_t device, void* stream) {
  int rc = check_device(device);
  if (rc) return rc;
  FCS_SET_DEVICE((device));
  ForkSet f;
  BswWorkspace ws;
  bool have_fork = false;
  {
    std::lock_guard<std::mutex> lk(g_fork_mu);
    auto wi = g_stream_ws->find({device, (hipStream_t)stream});
    if (wi != g_stream_ws->end()) {
      ws = wi->second;
      g_stream_ws->erase(wi);
    }
    auto it = g_fork_sets->find({device, (hipStream_t)stream});
    if (it != g_fork_sets->end()) {
      f = it->second;
      g_fork_sets->erase(it);
      have_fork = true;
    }
  }
  if (ws.keys_in) {
    (void)hipStreamSynchronize((hipStream_t)stream);
    ws_free(ws);
  }
  if (!have_fork) return FCS_OK;
  // tear down every side stream and event (best effort), then report the
  // first failure: an early return would leak the rest unreachably
  hipError_t first = hipSuccess;
  const char* what = nullptr;
  auto note = [&](hipError_t e, const char* w) {
    if (e != hipSuccess && first == hipSuccess) first = e, what = w;
  };
  for (int i = 0; i < kForkStreams - 1; ++i) {
    note(hipStreamSynchronize(f.side[i]), "hipStreamSynchronize");
    note(hipStreamDestroy(f.side[i]), "hipStreamDestroy");
    note(hipEventDestroy(f.join[i]), "hipEventDestroy");
  }
  note(hipEventDestroy(f.fork), "hipEventDestroy");
  if (first != hipSuccess)
    return fail(FCS_ERR_DEVICE, std::string("[E::fcs_stream_release] ") + what + ": " + hipGetErrorString(first));
  return FCS_OK;
}

int fcs_device_warmup(int32_t device, int32_t sessions) {
  int rc = check_device(device);
  if (rc) return rc;
  // a 1x1 PairHMM call: runtime, code objects, GKL tables and one session
  static const uint8_t b[1] = {'A'}, q[1] = {30}, g[1] = {10}, iq[1] = {45};
  const fcs_phmm_read r{b, q, iq, iq, g, 1};
  const fcs_phmm_hap h{b, 1};
  double out = 0;
  fcs_phmm_opts o;
  fcs_phmm_opts_default(&o);
  o.device = device;
  if ((rc = fcs_phmm_compute(&r, 1, &h, 1, &out, &o))) return rc;
  FCS_SET_DEVICE((device));
  return prefill_sessions(device, sessions <= 0 ? sessions_per_device() : sessions);
}

int fcs_phmm_last_device_ms(double* device_ms, double* rescue_ms) {
  if (!device_ms || !rescue_ms) return fail(FCS_ERR_INVALID, "[E::fcs_phmm_last_device_ms] null output");
  *device_ms = g_last_device_ms;
  *rescue_ms = g_last_rescue_ms;
  return FCS_OK;
}

int fcs_phmm_last_rescued(int64_t* count) {
  if (!count) return fail(FCS_ERR_INVALID, "[E::fcs_phmm_last_rescued] null count");
  *count = g_last_rescued;
  return FCS_OK;
}

int fcs_phmm_plan_rescue_count(fcs_phmm_plan* plan, void* stream, int64_t* count) {
  if (!plan || !count) return fail(FCS_ERR_INVALID, "[E::fcs_phmm_plan_rescue_count] bad arguments");
  FCS_SET_DEVICE((plan->device));
  unsigned long long v = 0;
  FCS_HIP_CHECK(hipMemcpyAsync(&v, plan->rescue_count, sizeof(v), hipMemcpyDeviceToHost, (hipStream_t)stream));
  FCS_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
  *count = (int64_t)v;
  return FCS_OK;
}

}  // extern "C"

namespace {

// Host side of one synchronous PairHMM pass: `fill` writes the batch's SoA
// arrays into the session's pinned staging at the offsets of `off` (order of
// PhmmStage), then one H2D copy, schedule + forward + rescue on the thread's
// stream into an output pre-filled with NaN, one D2H copy, and a check that
// every pair's result was written (a pair the schedule or a class launch
// skipped would otherwise go downstream as garbage).  Returns the results in
// pinned memory (valid while the caller holds the lease).
struct PhmmStage {
  int64_t n_reads = 0, n_haps = 0, n_pairs = 0, read_bytes = 0, hap_bytes = 0;
  int32_t max_read_len = 0, max_hap_len = 0;
};
enum { kRb, kBq, kIq, kDq, kGq, kRo, kRl, kHb, kHo, kHl, kPr, kPh, kNArr };

template <typename Fill>
int phmm_staged(const PhmmStage& g, const fcs_phmm_opts& opts, SessionLease& lease, Fill&& fill,
                const double** host_out) {
  int rc = check_device(opts.device);
  if (rc) return rc;
  FCS_SET_DEVICE((opts.device));
  // FCS_PHMM_TRACE=1: one stderr line per call with its host-side phases (ms)
  static const bool trace = std::getenv("FCS_PHMM_TRACE") != nullptr;
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  static const auto t_load = t0;  // the first call
  auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
  if ((rc = lease.acquire(opts.device))) return rc;
  const auto t_lease = clk::now();
  Session* S = lease.get();
  const size_t RB = (size_t)g.read_bytes, HB = (size_t)g.hap_bytes, nr = (size_t)g.n_reads, nh = (size_t)g.n_haps,
               np = (size_t)g.n_pairs;
  Layout L;
  size_t off[kNArr];
  for (int k = kRb; k <= kGq; ++k) off[k] = L.add(RB);
  off[kRo] = L.add(8 * nr);
  off[kRl] = L.add(4 * nr);
  off[kHb] = L.add(HB);
  off[kHo] = L.add(8 * nh);
  off[kHl] = L.add(4 * nh);
  off[kPr] = L.add(4 * np);
  off[kPh] = L.add(4 * np);
  const size_t in_bytes = L.total, out_off = L.add(8 * np);
  const bool grew = L.total > S->host_cap || L.total > S->dev_cap || !S->phmm || S->phmm->max_pairs < g.n_pairs;
  if ((rc = S->ensure_host(L.total)) || (rc = S->ensure_dev(L.total)) || (rc = S->ensure_phmm(g.n_pairs))) return rc;
  const auto t_ensure = clk::now();
  fill(S, off);
  const auto t_fill = clk::now();
  hipStream_t s = S->s;
  const StreamDrain drain{s};
  FCS_HIP_CHECK(hipMemcpyAsync(S->dev, S->host, in_bytes, hipMemcpyHostToDevice, s));
  fcs_phmm_batch d{};
  d.read_bases = S->d<uint8_t>(off[kRb]);
  d.read_bq = S->d<uint8_t>(off[kBq]);
  d.read_iq = S->d<uint8_t>(off[kIq]);
  d.read_dq = S->d<uint8_t>(off[kDq]);
  d.read_gcp = S->d<uint8_t>(off[kGq]);
  d.read_off = S->d<int64_t>(off[kRo]);
  d.read_len = S->d<int32_t>(off[kRl]);
  d.n_reads = g.n_reads;
  d.hap_bases = S->d<uint8_t>(off[kHb]);
  d.hap_off = S->d<int64_t>(off[kHo]);
  d.hap_len = S->d<int32_t>(off[kHl]);
  d.n_haps = g.n_haps;
  d.pair_read = S->d<int32_t>(off[kPr]);
  d.pair_hap = S->d<int32_t>(off[kPh]);
  d.n_pairs = g.n_pairs;
  d.read_bytes = g.read_bytes;
  d.hap_bytes = g.hap_bytes;
  d.max_read_len = g.max_read_len;
  d.max_hap_len = g.max_hap_len;
  double* dout = S->d<double>(out_off);
  FCS_HIP_CHECK(hipMemsetAsync(dout, 0xFF, 8 * np, s));  // all-ones = NaN: "not written"
  for (hipEvent_t& e : S->ev)
    if (!e) FCS_HIP_CHECK(hipEventCreate(&e));
  FCS_HIP_CHECK(hipEventRecord(S->ev[0], s));
  if ((rc = fcs_phmm_dev_schedule(S->phmm, &d, s)) || (rc = fcs_phmm_dev_forward(S->phmm, &d, dout, &opts, s)))
    return rc;
  FCS_HIP_CHECK(hipEventRecord(S->ev[1], s));
  if ((rc = fcs_phmm_dev_rescue(S->phmm, &d, dout, &opts, s))) return rc;
  FCS_HIP_CHECK(hipEventRecord(S->ev[2], s));
  double* hout = S->h<double>(out_off);
  FCS_HIP_CHECK(hipMemcpyAsync(hout, dout, 8 * np, hipMemcpyDeviceToHost, s));
  // into the input staging: its H2D copy is stream-ordered before this copy
  unsigned long long* hres = S->h<unsigned long long>(0);
  g_last_rescued = 0;
  if (opts.use_fp64_rescue)
    FCS_HIP_CHECK(hipMemcpyAsync(hres, S->phmm->rescue_count, sizeof(*hres), hipMemcpyDeviceToHost, s));
  const auto t_issue = clk::now();
  FCS_HIP_CHECK(hipStreamSynchronize(s));
  const auto t_sync = clk::now();
  if (opts.use_fp64_rescue) g_last_rescued = (int64_t)*hres;
  float ms_all = 0.f, ms_res = 0.f;
  FCS_HIP_CHECK(hipEventElapsedTime(&ms_all, S->ev[0], S->ev[2]));
  FCS_HIP_CHECK(hipEventElapsedTime(&ms_res, S->ev[1], S->ev[2]));
  g_last_device_ms = ms_all;
  g_last_rescue_ms = ms_res;
  if (trace)
    std::fprintf(stderr,
                 "[fcs_phmm_trace] at %.1f pairs %lld bytes %zu lease %.3f ensure %.3f%s fill %.3f issue %.3f sync %.3f "
                 "device %.3f total %.3f\n",
                 ms(t_load, t0), (long long)np, in_bytes, ms(t0, t_lease), ms(t_lease, t_ensure), grew ? " (grew)" : "",
                 ms(t_ensure, t_fill), ms(t_fill, t_issue), ms(t_issue, t_sync), (double)ms_all, ms(t0, t_sync));
  int64_t missing = 0;
  for (size_t k = 0; k < np; ++k) missing += std::isnan(hout[k]);
  if (missing)
    return fail(FCS_ERR_DEVICE, "[E::fcship] PairHMM: " + std::to_string(missing) + " of " + std::to_string(np) +
                                    " results were not written by the device pass");
  *host_out = hout;
  return FCS_OK;
}

}  // namespace

extern "C" {

int fcs_phmm_partition(const fcs_phmm_batch* b, int32_t n_slices, int64_t* cuts) {
  int rc = check_batch_shape(b);
  if (rc) return rc;
  if (n_slices <= 0 || !cuts) return fail(FCS_ERR_INVALID, "[E::fcs_phmm_partition] need n_slices > 0 and cuts");
  const int64_t n = b->n_pairs;
  std::vector<double> cum((size_t)n);
  double run = 0;
  for (int64_t p = 0; p < n; ++p) {
    const int32_t ri = b->pair_read[p], hi = b->pair_hap[p];
    if (ri < 0 || ri >= b->n_reads || hi < 0 || hi >= b->n_haps)
      return fail(FCS_ERR_INVALID, "[E::fcs_phmm_partition] pair index out of range");
    run += (double)b->read_len[ri] * (double)b->hap_len[hi];
    cum[p] = run;
  }
  // the cut where the running cost first reaches k/n of the total
  // (tests/sharding.py balanced_slices, its test oracle)
  cuts[0] = 0;
  for (int32_t k = 1; k < n_slices; ++k) {
    int64_t c;
    if (n == 0) c = 0;
    else if (run > 0) c = (int64_t)(std::lower_bound(cum.begin(), cum.end(), run * k / n_slices) - cum.begin()) + 1;
    else c = n * k / n_slices;
    cuts[k] = std::max(cuts[k - 1], std::min(c, n));
  }
  cuts[n_slices] = n;
  return FCS_OK;
}

int fcs_phmm_compute_pairs_multi(const fcs_phmm_batch* b, double* out_log10, const fcs_phmm_opts* opts_in,
                                 const int32_t* devices, int32_t n_devices) {
  if (n_devices <= 0 || !devices) return fail(FCS_ERR_INVALID, "[E::fcs_phmm_compute_pairs_multi] no devices");
  std::vector<int64_t> cuts((size_t)n_devices + 1);
  int rc = fcs_phmm_partition(b, n_devices, cuts.data());
  if (rc) return rc;
  if (b->n_pairs > 0 && !out_log10) return fail(FCS_ERR_INVALID, "[E::fcs_phmm_compute_pairs_multi] null output");
  fcs_phmm_opts opts;
  if (opts_in) opts = *opts_in;
  else fcs_phmm_opts_default(&opts);
  std::vector<int> rcs((size_t)n_devices, FCS_OK);
  std::vector<std::string> errs((size_t)n_devices);
  std::vector<int64_t> resc((size_t)n_devices, 0);
  std::vector<std::thread> th;
  for (int32_t k = 0; k < n_devices; ++k) {
    if (cuts[k + 1] == cuts[k]) continue;
    th.emplace_back([&, k] {
      fcs_phmm_batch sub = *b;
      sub.pair_read = b->pair_read + cuts[k];
      sub.pair_hap = b->pair_hap + cuts[k];
      sub.n_pairs = cuts[k + 1] - cuts[k];
      fcs_phmm_opts o = opts;
      o.device = devices[k];
      rcs[k] = fcs_phmm_compute_pairs(&sub, out_log10 + cuts[k], &o);
      if (rcs[k] != FCS_OK) errs[k] = fcs_last_error();
      int64_t r = 0;
      if (fcs_phmm_last_rescued(&r) == FCS_OK) resc[k] = r;
    });
  }
  for (auto& t : th) t.join();
  int64_t tot = 0;
  for (int32_t k = 0; k < n_devices; ++k) {
    if (rcs[k] != FCS_OK) return fail(rcs[k], errs[k]);
    tot += resc[k];
  }
  g_last_rescued = tot;
  return FCS_OK;
}

int fcs_phmm_compute_pairs(const fcs_phmm_batch* b, double* out_log10, const fcs_phmm_opts* opts_in) {
  int rc = check_batch_shape(b);
  if (rc) return rc;
  fcs_phmm_opts opts;
  if (opts_in) opts = *opts_in;
  else fcs_phmm_opts_default(&opts);
  if (b->n_pairs == 0) return FCS_OK;
  if (!out_log10) return fail(FCS_ERR_INVALID, "[E::fcs_phmm_compute_pairs] null output");
  // Validate indices and lengths on the host (the device path trusts its caller).
  PhmmStage g;
  g.n_reads = b->n_reads;
  g.n_haps = b->n_haps;
  g.n_pairs = b->n_pairs;
  g.read_bytes = b->read_bytes;
  g.hap_bytes = b->hap_bytes;
  for (int64_t p = 0; p < b->n_pairs; ++p) {
    const int32_t ri = b->pair_read[p], hi = b->pair_hap[p];
    if (ri < 0 || ri >= b->n_reads || hi < 0 || hi >= b->n_haps)
      return fail(FCS_ERR_INVALID, "[E::fcs_phmm_compute_pairs] pair index out of range");
  }
  for (int64_t r = 0; r < b->n_reads; ++r) {
    if (b->read_len[r] < 0 || b->read_off[r] < 0 || b->read_off[r] + b->read_len[r] > b->read_bytes)
      return fail(FCS_ERR_INVALID, "[E::fcs_phmm_compute_pairs] read extent outside read arrays");
    g.max_read_len = std::max(g.max_read_len, b->read_len[r]);
  }
  for (int64_t h = 0; h < b->n_haps; ++h) {
    if (b->hap_len[h] < 0 || b->hap_off[h] < 0 || b->hap_off[h] + b->hap_len[h] > b->hap_bytes)
      return fail(FCS_ERR_INVALID, "[E::fcs_phmm_compute_pairs] hap extent outside hap array");
    g.max_hap_len = std::max(g.max_hap_len, b->hap_len[h]);
  }
  const size_t RB = (size_t)b->read_bytes, HB = (size_t)b->hap_bytes, nr = (size_t)b->n_reads,
               nh = (size_t)b->n_haps, np = (size_t)b->n_pairs;
  const double* res = nullptr;
  SessionLease lease;  // holds the pinned results until they are copied out
  rc = phmm_staged(g, opts, lease, [&](Session* S, const size_t* off) {
    std::memcpy(S->h<void>(off[kRb]), b->read_bases, RB);
    std::memcpy(S->h<void>(off[kBq]), b->read_bq, RB);
    std::memcpy(S->h<void>(off[kIq]), b->read_iq, RB);
    std::memcpy(S->h<void>(off[kDq]), b->read_dq, RB);
    std::memcpy(S->h<void>(off[kGq]), b->read_gcp, RB);
    std::memcpy(S->h<void>(off[kRo]), b->read_off, 8 * nr);
    std::memcpy(S->h<void>(off[kRl]), b->read_len, 4 * nr);
    std::memcpy(S->h<void>(off[kHb]), b->hap_bases, HB);
    std::memcpy(S->h<void>(off[kHo]), b->hap_off, 8 * nh);
    std::memcpy(S->h<void>(off[kHl]), b->hap_len, 4 * nh);
    std::memcpy(S->h<void>(off[kPr]), b->pair_read, 4 * np);
    std::memcpy(S->h<void>(off[kPh]), b->pair_hap, 4 * np);
  }, &res);
  if (rc) return rc;
  std::memcpy(out_log10, res, 8 * np);
  return FCS_OK;
}

int fcs_phmm_compute(const fcs_phmm_read* reads, int32_t n_reads, const fcs_phmm_hap* haps, int32_t n_haps,
                     double* out_log10, const fcs_phmm_opts* opts) {
  if (n_reads < 0 || n_haps < 0 || (n_reads > 0 && !reads) || (n_haps > 0 && !haps))
    return fail(FCS_ERR_INVALID, "[E::fcs_phmm_compute] bad arguments");
  if ((int64_t)n_reads * n_haps == 0) return FCS_OK;
  if (!out_log10) return fail(FCS_ERR_INVALID, "[E::fcs_phmm_compute] null output");
  fcs_phmm_region r{reads, n_reads, haps, n_haps, out_log10};
  return fcs_phmm_compute_regions(&r, 1, opts);
}

// Many active regions in one device pass: the regions' reads and haplotypes
// are concatenated (straight into the pinned staging) into one SoA batch whose
// pair list is region-major and read-major within a region, so the flat
// result splits back into each region's read-major matrix by a running offset.
}  // extern "C"

namespace {
// Runs f(k0, k1) over contiguous region ranges: on the calling thread for a
// small batch, on up to 8 threads for a large one (a pass merged from many
// shards' batches, host/caller.cpp, stages ~100 MB through per-read memcpys;
// on one thread that serialised the shards waiting for it).
template <class F>
void for_region_ranges(int32_t n, int64_t bytes, F&& f) {
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const int nt = (int)std::min<int64_t>({8, (int64_t)hw, n, bytes / (4 << 20)});
  if (nt <= 1) {
    f(0, n);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(nt - 1);
  const int32_t chunk = (n + nt - 1) / nt;
  for (int t = 1; t < nt; ++t) {
    const int32_t a = t * chunk, b = std::min(n, a + chunk);
    if (a < b) th.emplace_back([&f, a, b] { f(a, b); });
  }
  f(0, std::min(n, chunk));
  for (auto& x : th) x.join();
}
}  // namespace

extern "C" {

int fcs_phmm_compute_regions(const fcs_phmm_region* regions, int32_t n_regions, const fcs_phmm_opts* opts_in) {
  if (n_regions < 0 || (n_regions > 0 && !regions))
    return fail(FCS_ERR_INVALID, "[E::fcs_phmm_compute_regions] bad arguments");
  PhmmStage g;
  // per-region starts in the packed batch (reads, haplotypes, pairs, read and
  // hap bytes): regions are staged independently, in parallel when large
  std::vector<int64_t> r_at(n_regions + 1), h_at(n_regions + 1), p_at(n_regions + 1), rb_at(n_regions + 1),
      hb_at(n_regions + 1);
  for (int32_t k = 0; k < n_regions; ++k) {
    const fcs_phmm_region& R = regions[k];
    r_at[k] = g.n_reads, h_at[k] = g.n_haps, p_at[k] = g.n_pairs, rb_at[k] = g.read_bytes, hb_at[k] = g.hap_bytes;
    if (R.n_reads < 0 || R.n_haps < 0 || (R.n_reads > 0 && !R.reads) || (R.n_haps > 0 && !R.haps))
      return fail(FCS_ERR_INVALID, "[E::fcs_phmm_compute_regions] malformed region");
    const int64_t pairs = (int64_t)R.n_reads * R.n_haps;
    if (pairs > 0 && !R.out_log10) return fail(FCS_ERR_INVALID, "[E::fcs_phmm_compute_regions] null region output");
    for (int32_t r = 0; r < R.n_reads; ++r) {
      const fcs_phmm_read& x = R.reads[r];
      if (x.len < 0 || (x.len > 0 && (!x.bases || !x.base_q || !x.ins_q || !x.del_q || !x.gcp)))
        return fail(FCS_ERR_INVALID, "[E::fcs_phmm_compute_regions] malformed read");
      g.read_bytes += x.len;
      g.max_read_len = std::max(g.max_read_len, x.len);
    }
    for (int32_t h = 0; h < R.n_haps; ++h) {
      if (R.haps[h].len < 0 || (R.haps[h].len > 0 && !R.haps[h].bases))
        return fail(FCS_ERR_INVALID, "[E::fcs_phmm_compute_regions] malformed haplotype");
      g.hap_bytes += R.haps[h].len;
      g.max_hap_len = std::max(g.max_hap_len, R.haps[h].len);
    }
    g.n_reads += R.n_reads;
    g.n_haps += R.n_haps;
    g.n_pairs += pairs;
  }
  if (g.n_pairs == 0) return FCS_OK;
  if (g.n_reads > INT32_MAX || g.n_haps > INT32_MAX || g.n_pairs > INT32_MAX)
    return fail(FCS_ERR_INVALID, "[E::fcs_phmm_compute_regions] more than 2^31 reads, haplotypes or pairs");
  fcs_phmm_opts opts;
  if (opts_in) opts = *opts_in;
  else fcs_phmm_opts_default(&opts);
  const double* res = nullptr;
  SessionLease lease;  // holds the pinned results until they are copied out
  const int rc = phmm_staged(g, opts, lease, [&](Session* S, const size_t* off) {
    uint8_t *rb = S->h<uint8_t>(off[kRb]), *bq = S->h<uint8_t>(off[kBq]), *iq = S->h<uint8_t>(off[kIq]),
            *dq = S->h<uint8_t>(off[kDq]), *gq = S->h<uint8_t>(off[kGq]), *hb = S->h<uint8_t>(off[kHb]);
    int64_t *roff = S->h<int64_t>(off[kRo]), *hoff = S->h<int64_t>(off[kHo]);
    int32_t *rlen = S->h<int32_t>(off[kRl]), *hlen = S->h<int32_t>(off[kHl]), *pr = S->h<int32_t>(off[kPr]),
            *ph = S->h<int32_t>(off[kPh]);
    for_region_ranges(n_regions, g.read_bytes + 8 * g.n_pairs, [&](int32_t k0, int32_t k1) {
      for (int32_t k = k0; k < k1; ++k) {
        const fcs_phmm_region& R = regions[k];
        int64_t ri = r_at[k], hi = h_at[k], pi = p_at[k], ro = rb_at[k], ho = hb_at[k];
        const int64_t r0 = ri, h0 = hi;
        for (int32_t r = 0; r < R.n_reads; ++r, ++ri) {
          const fcs_phmm_read& x = R.reads[r];
          roff[ri] = ro;
          rlen[ri] = x.len;
          if (x.len) {
            std::memcpy(rb + ro, x.bases, x.len);
            std::memcpy(bq + ro, x.base_q, x.len);
            std::memcpy(iq + ro, x.ins_q, x.len);
            std::memcpy(dq + ro, x.del_q, x.len);
            std::memcpy(gq + ro, x.gcp, x.len);
          }
          ro += x.len;
        }
        for (int32_t h = 0; h < R.n_haps; ++h, ++hi) {
          hoff[hi] = ho;
          hlen[hi] = R.haps[h].len;
          if (R.haps[h].len) std::memcpy(hb + ho, R.haps[h].bases, R.haps[h].len);
          ho += R.haps[h].len;
        }
        for (int32_t r = 0; r < R.n_reads; ++r)
          for (int32_t h = 0; h < R.n_haps; ++h, ++pi) {
            pr[pi] = (int32_t)(r0 + r);
            ph[pi] = (int32_t)(h0 + h);
          }
      }
    });
  }, &res);
  if (rc) return rc;
  for_region_ranges(n_regions, 8 * g.n_pairs, [&](int32_t k0, int32_t k1) {
    for (int32_t k = k0; k < k1; ++k) {
      const int64_t pairs = (int64_t)regions[k].n_reads * regions[k].n_haps;
      if (pairs) std::memcpy(regions[k].out_log10, res + p_at[k], 8 * (size_t)pairs);
    }
  });
  return FCS_OK;
}

// ------------------------------------------------------------------ banded SW
static BswDevBatch bsw_dev(const fcs_bsw_batch* b) {
  BswDevBatch d;
  d.qbuf = b->qbuf;
  d.qoff = b->qoff;
  d.qlen = b->qlen;
  d.tbuf = b->tbuf;
  d.toff = b->toff;
  d.tlen = b->tlen;
  d.h0 = b->h0;
  d.w = b->w;
  d.n = b->n;
  return d;
}

static int check_bsw_batch(const fcs_bsw_batch* b) {
  if (!b || b->n < 0) return fail(FCS_ERR_INVALID, "[E::fcship] bad SW batch");
  // byte buffers may be null when empty: a batch whose every target (or query)
  // is empty, e.g. left extensions of seeds that start at their window's edge
  // (bwa calls ksw_extend2 with tlen 0 there)
  if (b->n > 0 && ((!b->qbuf && b->qbytes > 0) || !b->qoff || !b->qlen || (!b->tbuf && b->tbytes > 0) || !b->toff ||
                   !b->tlen || !b->h0 || !b->w))
    return fail(FCS_ERR_INVALID, "[E::fcship] null pointer in SW batch");
  return FCS_OK;
}

int fcs_bsw_extend_dev(const fcs_bsw_batch* b, const fcs_bsw_params* params, int32_t* res, int64_t* cells,
                       int32_t device, void* stream) {
  int rc = check_bsw_batch(b);
  if (rc) return rc;
  if ((rc = check_params(params))) return rc;
  if (b->n > 0 && !res) return fail(FCS_ERR_INVALID, "[E::fcs_bsw_extend_dev] null result buffer");
  if ((rc = check_device(device))) return rc;
  if (b->n == 0) return FCS_OK;
  FCS_SET_DEVICE((device));
  hipStream_t s = (hipStream_t)stream;
  BswWorkspace* ws = nullptr;
  if ((rc = stream_workspace(device, s, b->n, &ws))) return rc;
  return launch_bsw_extend_sorted(bsw_dev(b), to_params(params), std::max(b->max_qlen, 0), std::max(b->max_tlen, 0),
                                  res, cells, *ws, s);
}

int fcs_bsw_plan_create(int32_t device, int64_t max_tasks, fcs_bsw_plan** plan) {
  if (!plan || max_tasks < 0) return fail(FCS_ERR_INVALID, "[E::fcs_bsw_plan_create] bad arguments");
  int rc = check_device(device);
  if (rc) return rc;
  FCS_SET_DEVICE((device));
  std::unique_ptr<fcs_bsw_plan> p(new fcs_bsw_plan());
  p->device = device;
  if ((rc = ws_alloc(p->ws, max_tasks))) {
    ws_free(p->ws);
    return rc;
  }
  *plan = p.release();
  return FCS_OK;
}

int fcs_bsw_plan_destroy(fcs_bsw_plan* plan) {
  if (!plan) return FCS_OK;
  ::fcs::DeviceScope dev_scope;
  (void)hipSetDevice(plan->device);
  ws_free(plan->ws);
  delete plan;
  return FCS_OK;
}

int fcs_bsw_extend_plan(fcs_bsw_plan* plan, const fcs_bsw_batch* b, const fcs_bsw_params* params, int32_t* res,
                        int64_t* cells, void* stream) {
  if (!plan) return fail(FCS_ERR_INVALID, "[E::fcs_bsw_extend_plan] null plan");
  int rc = check_bsw_batch(b);
  if (rc) return rc;
  if ((rc = check_params(params))) return rc;
  if (b->n > plan->ws.cap) return fail(FCS_ERR_INVALID, "[E::fcs_bsw_extend_plan] batch exceeds plan");
  if (b->n > 0 && !res) return fail(FCS_ERR_INVALID, "[E::fcs_bsw_extend_plan] null result buffer");
  if (b->n == 0) return FCS_OK;
  FCS_SET_DEVICE((plan->device));
  return launch_bsw_extend_sorted(bsw_dev(b), to_params(params), std::max(b->max_qlen, 0), std::max(b->max_tlen, 0),
                                  res, cells, plan->ws, (hipStream_t)stream);
}

int fcs_bsw_extend_batch(const fcs_bsw_batch* b, const fcs_bsw_params* params, int32_t* res, int64_t* cells,
                         int32_t device) {
  int rc = check_bsw_batch(b);
  if (rc) return rc;
  if ((rc = check_params(params))) return rc;
  if (b->n == 0) return FCS_OK;
  if (!res) return fail(FCS_ERR_INVALID, "[E::fcs_bsw_extend_batch] null result buffer");
  int32_t mq = 0, mt = 0;
  for (int64_t k = 0; k < b->n; ++k) {
    if (b->qlen[k] < 0 || b->tlen[k] < 0 || b->qoff[k] < 0 || b->toff[k] < 0 ||
        b->qoff[k] + b->qlen[k] > b->qbytes || b->toff[k] + b->tlen[k] > b->tbytes)
      return fail(FCS_ERR_INVALID, "[E::fcs_bsw_extend_batch] task extent outside buffers");
    if (b->h0[k] <= 0) return fail(FCS_ERR_INVALID, "[E::fcs_bsw_extend_batch] h0 must be > 0 (ksw_extend2 assert)");
    if (b->w[k] < 0) return fail(FCS_ERR_INVALID, "[E::fcs_bsw_extend_batch] negative band");
    mq = std::max(mq, b->qlen[k]);
    mt = std::max(mt, b->tlen[k]);
  }
  for (int64_t i = 0; i < b->qbytes; ++i)
    if (b->qbuf[i] > 4) return fail(FCS_ERR_INVALID, "[E::fcs_bsw_extend_batch] query base code > 4");
  for (int64_t i = 0; i < b->tbytes; ++i)
    if (b->tbuf[i] > 4) return fail(FCS_ERR_INVALID, "[E::fcs_bsw_extend_batch] target base code > 4");
  if ((rc = check_device(device))) return rc;
  FCS_SET_DEVICE((device));
  SessionLease lease;
  if ((rc = lease.acquire(device))) return rc;
  Session* S = lease.get();
  const size_t n = (size_t)b->n;
  Layout L;
  const size_t oq = L.add((size_t)b->qbytes), oqo = L.add(8 * n), oql = L.add(4 * n), ot = L.add((size_t)b->tbytes),
               oto = L.add(8 * n), otl = L.add(4 * n), oh0 = L.add(4 * n), ow = L.add(4 * n);
  const size_t in_bytes = L.total, ors = L.add(24 * n), ocl = L.add(8 * n);
  if ((rc = S->ensure_host(L.total)) || (rc = S->ensure_dev(L.total)) || (rc = S->ensure_bsw(b->n))) return rc;
  std::memcpy(S->h<void>(oq), b->qbuf, (size_t)b->qbytes);
  std::memcpy(S->h<void>(oqo), b->qoff, 8 * n);
  std::memcpy(S->h<void>(oql), b->qlen, 4 * n);
  std::memcpy(S->h<void>(ot), b->tbuf, (size_t)b->tbytes);
  std::memcpy(S->h<void>(oto), b->toff, 8 * n);
  std::memcpy(S->h<void>(otl), b->tlen, 4 * n);
  std::memcpy(S->h<void>(oh0), b->h0, 4 * n);
  std::memcpy(S->h<void>(ow), b->w, 4 * n);
  hipStream_t s = S->s;
  const StreamDrain drain{s};
  FCS_HIP_CHECK(hipMemcpyAsync(S->dev, S->host, in_bytes, hipMemcpyHostToDevice, s));
  BswDevBatch d;
  d.qbuf = S->d<uint8_t>(oq);
  d.qoff = S->d<int64_t>(oqo);
  d.qlen = S->d<int32_t>(oql);
  d.tbuf = S->d<uint8_t>(ot);
  d.toff = S->d<int64_t>(oto);
  d.tlen = S->d<int32_t>(otl);
  d.h0 = S->d<int32_t>(oh0);
  d.w = S->d<int32_t>(ow);
  d.n = b->n;
  if ((rc = launch_bsw_extend_sorted(d, to_params(params), mq, mt, S->d<int32_t>(ors), S->d<int64_t>(ocl),
                                     S->bsw->ws, s)))
    return rc;
  FCS_HIP_CHECK(hipMemcpyAsync(S->h<void>(ors), S->d<void>(ors), ocl + 8 * n - ors, hipMemcpyDeviceToHost, s));
  FCS_HIP_CHECK(hipStreamSynchronize(s));
  std::memcpy(res, S->h<void>(ors), 24 * n);
  if (cells) std::memcpy(cells, S->h<void>(ocl), 8 * n);
  return FCS_OK;
}

// Packs AoS tasks into an SoA host batch.
struct PackedTasks {
  std::vector<uint8_t> q, t;
  std::vector<int64_t> qoff, toff;
  std::vector<int32_t> qlen, tlen, h0, w;
  fcs_bsw_batch b{};
};

static int pack_tasks(const fcs_bsw_task* tasks, int32_t n, PackedTasks& pk) {
  pk.qoff.resize(n);
  pk.toff.resize(n);
  pk.qlen.resize(n);
  pk.tlen.resize(n);
  pk.h0.resize(n);
  pk.w.resize(n);
  for (int32_t k = 0; k < n; ++k) {
    const fcs_bsw_task& t = tasks[k];
    if (t.qlen < 0 || t.tlen < 0 || (t.qlen > 0 && !t.query) || (t.tlen > 0 && !t.target))
      return fail(FCS_ERR_INVALID, "[E::fcship] malformed SW task");
    pk.qoff[k] = (int64_t)pk.q.size();
    pk.toff[k] = (int64_t)pk.t.size();
    pk.q.insert(pk.q.end(), t.query, t.query + t.qlen);
    pk.t.insert(pk.t.end(), t.target, t.target + t.tlen);
    pk.qlen[k] = t.qlen;
    pk.tlen[k] = t.tlen;
    pk.h0[k] = t.h0;
    pk.w[k] = t.w;
  }
  pk.b.qbuf = pk.q.data();
  pk.b.qoff = pk.qoff.data();
  pk.b.qlen = pk.qlen.data();
  pk.b.tbuf = pk.t.data();
  pk.b.toff = pk.toff.data();
  pk.b.tlen = pk.tlen.data();
  pk.b.h0 = pk.h0.data();
  pk.b.w = pk.w.data();
  pk.b.n = n;
  pk.b.qbytes = (int64_t)pk.q.size();
  pk.b.tbytes = (int64_t)pk.t.size();
  return FCS_OK;
}

int fcs_bsw_extend_multi(const fcs_bsw_task* tasks, int32_t n, const fcs_bsw_params* params,
                         fcs_bsw_result* results, const int32_t* devices, int32_t n_devices) {
  if (n < 0 || (n > 0 && (!tasks || !results)) || n_devices <= 0 || !devices)
    return fail(FCS_ERR_INVALID, "[E::fcs_bsw_extend_multi] bad arguments");
  // §8e: contiguous slices of ~equal qlen * tlen, one device each, one host thread each
  std::vector<double> cum((size_t)n);
  double run = 0;
  for (int32_t i = 0; i < n; ++i) cum[i] = (run += (double)std::max(tasks[i].qlen, 0) * std::max(tasks[i].tlen, 0));
  std::vector<int32_t> cuts((size_t)n_devices + 1, 0);
  for (int32_t k = 1; k < n_devices; ++k) {
    int64_t c = run > 0 ? (int64_t)(std::lower_bound(cum.begin(), cum.end(), run * k / n_devices) - cum.begin()) + 1
                        : (int64_t)n * k / n_devices;
    cuts[k] = (int32_t)std::max<int64_t>(cuts[k - 1], std::min<int64_t>(c, n));
  }
  cuts[n_devices] = n;
  std::vector<int> rcs((size_t)n_devices, FCS_OK);
  std::vector<std::string> errs((size_t)n_devices);
  std::vector<std::thread> th;
  for (int32_t k = 0; k < n_devices; ++k) {
    if (cuts[k + 1] == cuts[k]) continue;
    th.emplace_back([&, k] {
      rcs[k] = fcs_bsw_extend(tasks + cuts[k], cuts[k + 1] - cuts[k], params, results + cuts[k], devices[k]);
      if (rcs[k] != FCS_OK) errs[k] = fcs_last_error();
    });
  }
  for (auto& t : th) t.join();
  for (int32_t k = 0; k < n_devices; ++k)
    if (rcs[k] != FCS_OK) return fail(rcs[k], errs[k]);
  return FCS_OK;
}

int fcs_bsw_extend(const fcs_bsw_task* tasks, int32_t n, const fcs_bsw_params* params, fcs_bsw_result* results,
                   int32_t device) {
  if (n < 0 || (n > 0 && (!tasks || !results))) return fail(FCS_ERR_INVALID, "[E::fcs_bsw_extend] bad arguments");
  if (n == 0) return FCS_OK;
  PackedTasks pk;
  int rc = pack_tasks(tasks, n, pk);
  if (rc) return rc;
  static_assert(sizeof(fcs_bsw_result) == 24, "result layout");
  return fcs_bsw_extend_batch(&pk.b, params, reinterpret_cast<int32_t*>(results), nullptr, device);
}

int fcs_bsw_global(const fcs_bsw_task* tasks, int32_t n, const fcs_bsw_params* params, int32_t* scores,
                   uint32_t* cigar_arena, const int64_t* cigar_off, const int32_t* cigar_cap, int32_t* n_cigar,
                   int32_t device) {
  if (n < 0 || (n > 0 && (!tasks || !scores))) return fail(FCS_ERR_INVALID, "[E::fcs_bsw_global] bad arguments");
  const bool want_cigar = cigar_arena != nullptr;
  if (want_cigar && (!cigar_off || !cigar_cap || !n_cigar))
    return fail(FCS_ERR_INVALID, "[E::fcs_bsw_global] CIGAR arena needs offsets, caps and counts");
  int rc = check_params(params);
  if (rc) return rc;
  if (n == 0) return FCS_OK;
  PackedTasks pk;
  if ((rc = pack_tasks(tasks, n, pk))) return rc;
  int32_t mq = 0, mt = 0;
  std::vector<int64_t> zoff(n);
  int64_t zt = 0, ct = 0;
  for (int32_t k = 0; k < n; ++k) {
    if (pk.w[k] < 0) return fail(FCS_ERR_INVALID, "[E::fcs_bsw_global] negative band");
    mq = std::max(mq, pk.qlen[k]);
    mt = std::max(mt, pk.tlen[k]);
    const int64_t ncol = std::min<int64_t>(pk.qlen[k], 2LL * pk.w[k] + 1);
    zoff[k] = zt;
    if (want_cigar) zt += ncol * pk.tlen[k];
    if (want_cigar) {
      if (cigar_cap[k] < 0 || cigar_off[k] < 0) return fail(FCS_ERR_INVALID, "[E::fcs_bsw_global] bad CIGAR extent");
      ct = std::max<int64_t>(ct, cigar_off[k] + cigar_cap[k]);
    }
  }
  for (int64_t i = 0; i < pk.b.qbytes; ++i)
    if (pk.q[i] > 4) return fail(FCS_ERR_INVALID, "[E::fcs_bsw_global] query base code > 4");
  for (int64_t i = 0; i < pk.b.tbytes; ++i)
    if (pk.t[i] > 4) return fail(FCS_ERR_INVALID, "[E::fcs_bsw_global] target base code > 4");
  if ((rc = check_device(device))) return rc;
  FCS_SET_DEVICE((device));
  SessionLease lease;
  if ((rc = lease.acquire(device))) return rc;
  Session* S = lease.get();
  const size_t nn = (size_t)n;
  // The direction matrix (and its offsets) only when CIGARs are wanted: a
  // scores-only batch needs none of it.
  Layout L;
  const size_t oq = L.add(pk.q.size()), oqo = L.add(8 * nn), oql = L.add(4 * nn), ot = L.add(pk.t.size()),
               oto = L.add(8 * nn), otl = L.add(4 * nn), oh0 = L.add(4 * nn), ow = L.add(4 * nn);
  const size_t ozo = want_cigar ? L.add(8 * nn) : 0, oco = want_cigar ? L.add(8 * nn) : 0,
               occ = want_cigar ? L.add(4 * nn) : 0;
  const size_t in_bytes = L.total, osc = L.add(4 * nn), onc = L.add(4 * nn), ocg = L.add(4 * (size_t)ct),
               ozb = want_cigar ? L.add((size_t)zt) : 0;
  if ((rc = S->ensure_host(in_bytes + 8 * nn + 4 * (size_t)ct + 1024)) || (rc = S->ensure_dev(L.total))) return rc;
  std::memcpy(S->h<void>(oq), pk.q.data(), pk.q.size());
  std::memcpy(S->h<void>(oqo), pk.qoff.data(), 8 * nn);
  std::memcpy(S->h<void>(oql), pk.qlen.data(), 4 * nn);
  std::memcpy(S->h<void>(ot), pk.t.data(), pk.t.size());
  std::memcpy(S->h<void>(oto), pk.toff.data(), 8 * nn);
  std::memcpy(S->h<void>(otl), pk.tlen.data(), 4 * nn);
  std::memcpy(S->h<void>(oh0), pk.h0.data(), 4 * nn);
  std::memcpy(S->h<void>(ow), pk.w.data(), 4 * nn);
  if (want_cigar) {
    std::memcpy(S->h<void>(ozo), zoff.data(), 8 * nn);
    std::memcpy(S->h<void>(oco), cigar_off, 8 * nn);
    std::memcpy(S->h<void>(occ), cigar_cap, 4 * nn);
  }
  hipStream_t s = S->s;
  const StreamDrain drain{s};
  FCS_HIP_CHECK(hipMemcpyAsync(S->dev, S->host, in_bytes, hipMemcpyHostToDevice, s));
  BswDevBatch d;
  d.qbuf = S->d<uint8_t>(oq);
  d.qoff = S->d<int64_t>(oqo);
  d.qlen = S->d<int32_t>(oql);
  d.tbuf = S->d<uint8_t>(ot);
  d.toff = S->d<int64_t>(oto);
  d.tlen = S->d<int32_t>(otl);
  d.h0 = S->d<int32_t>(oh0);
  d.w = S->d<int32_t>(ow);
  d.n = n;
  rc = launch_bsw_global(d, to_params(params), mq, mt, S->d<int32_t>(osc), want_cigar ? S->d<uint8_t>(ozb) : nullptr,
                         zt, want_cigar ? S->d<int64_t>(ozo) : nullptr, want_cigar ? S->d<uint32_t>(ocg) : nullptr,
                         want_cigar ? S->d<int64_t>(oco) : nullptr, want_cigar ? S->d<int32_t>(occ) : nullptr,
                         want_cigar ? S->d<int32_t>(onc) : nullptr, s);
  if (rc) return rc;
  // scores, counts and the CIGAR arena are contiguous in the layout
  const size_t back = want_cigar ? ocg + 4 * (size_t)ct - osc : 4 * nn;
  FCS_HIP_CHECK(hipMemcpyAsync(S->h<void>(in_bytes), S->d<void>(osc), back, hipMemcpyDeviceToHost, s));
  FCS_HIP_CHECK(hipStreamSynchronize(s));
  const char* hb = S->h<char>(in_bytes);
  std::memcpy(scores, hb, 4 * nn);
  if (want_cigar) {
    std::memcpy(n_cigar, hb + (onc - osc), 4 * nn);
    if (ct) std::memcpy(cigar_arena, hb + (ocg - osc), 4 * (size_t)ct);
    for (int32_t k = 0; k < n; ++k)
      if (n_cigar[k] > cigar_cap[k])
        return fail(FCS_ERR_INVALID, "[E::fcs_bsw_global] CIGAR longer than its arena slot");
  }
  return FCS_OK;
}

int fcs_bsw_global_dev(const fcs_bsw_batch* b, const fcs_bsw_params* params, int32_t* dev_scores, uint8_t* dev_zbuf,
                       int64_t zbytes, const int64_t* dev_zoff, uint32_t* dev_cigar, const int64_t* dev_cigar_off,
                       const int32_t* dev_cigar_cap, int32_t* dev_n_cigar, int32_t device, void* stream) {
  if (!b || b->n < 0 || (b->n > 0 && !dev_scores)) return fail(FCS_ERR_INVALID, "[E::fcs_bsw_global_dev] bad arguments");
  const bool want_cigar = dev_cigar != nullptr;
  if (want_cigar && (!dev_zbuf || !dev_zoff || !dev_cigar_off || !dev_cigar_cap || !dev_n_cigar))
    return fail(FCS_ERR_INVALID, "[E::fcs_bsw_global_dev] CIGARs need the direction matrix, offsets, caps and counts");
  int rc = check_params(params);
  if (rc) return rc;
  if (b->n == 0) return FCS_OK;
  if (b->n > 0x7FFFFFFF) return fail(FCS_ERR_UNSUPPORTED, "[E::fcs_bsw_global_dev] more than 2^31-1 tasks");
  if ((rc = check_device(device))) return rc;
  FCS_SET_DEVICE((device));
  BswDevBatch d;
  d.qbuf = b->qbuf;
  d.qoff = b->qoff;
  d.qlen = b->qlen;
  d.tbuf = b->tbuf;
  d.toff = b->toff;
  d.tlen = b->tlen;
  d.h0 = b->h0;
  d.w = b->w;
  d.n = b->n;
  return launch_bsw_global(d, to_params(params), std::max(b->max_qlen, 1), std::max(b->max_tlen, 1), dev_scores,
                           want_cigar ? dev_zbuf : nullptr, want_cigar ? zbytes : 0, want_cigar ? dev_zoff : nullptr,
                           dev_cigar, want_cigar ? dev_cigar_off : nullptr, want_cigar ? dev_cigar_cap : nullptr,
                           want_cigar ? dev_n_cigar : nullptr, (hipStream_t)stream);
}

int fcs_bsw_align(const fcs_bsw_task* tasks, int32_t n, const fcs_bsw_params* params, const int32_t* xtra,
                  fcs_kswr* out, int32_t device) {
  if (n < 0 || (n > 0 && (!tasks || !xtra || !out))) return fail(FCS_ERR_INVALID, "[E::fcs_bsw_align] bad arguments");
  int rc = check_params(params);
  if (rc) return rc;
  if (n == 0) return FCS_OK;
  PackedTasks pk;
  if ((rc = pack_tasks(tasks, n, pk))) return rc;
  int32_t mq = 0, mt = 0;
  for (int32_t k = 0; k < n; ++k) mq = std::max(mq, pk.qlen[k]), mt = std::max(mt, pk.tlen[k]);
  for (int64_t i = 0; i < pk.b.qbytes; ++i)
    if (pk.q[i] > 4) return fail(FCS_ERR_INVALID, "[E::fcs_bsw_align] query base code > 4");
  for (int64_t i = 0; i < pk.b.tbytes; ++i)
    if (pk.t[i] > 4) return fail(FCS_ERR_INVALID, "[E::fcs_bsw_align] target base code > 4");
  if ((rc = check_device(device))) return rc;
  FCS_SET_DEVICE((device));
  SessionLease lease;
  if ((rc = lease.acquire(device))) return rc;
  Session* S = lease.get();
  const size_t nn = (size_t)n;
  Layout L;
  const size_t oq = L.add(pk.q.size()), oqo = L.add(8 * nn), oql = L.add(4 * nn), ot = L.add(pk.t.size()),
               oto = L.add(8 * nn), otl = L.add(4 * nn), ox = L.add(4 * nn);
  const size_t in_bytes = L.total, oo = L.add(sizeof(fcs_kswr) * nn);
  if ((rc = S->ensure_host(L.total + 1024)) || (rc = S->ensure_dev(L.total))) return rc;
  std::memcpy(S->h<void>(oq), pk.q.data(), pk.q.size());
  std::memcpy(S->h<void>(oqo), pk.qoff.data(), 8 * nn);
  std::memcpy(S->h<void>(oql), pk.qlen.data(), 4 * nn);
  std::memcpy(S->h<void>(ot), pk.t.data(), pk.t.size());
  std::memcpy(S->h<void>(oto), pk.toff.data(), 8 * nn);
  std::memcpy(S->h<void>(otl), pk.tlen.data(), 4 * nn);
  std::memcpy(S->h<void>(ox), xtra, 4 * nn);
  hipStream_t s = S->s;
  const StreamDrain drain{s};
  FCS_HIP_CHECK(hipMemcpyAsync(S->dev, S->host, in_bytes, hipMemcpyHostToDevice, s));
  BswDevBatch d{};
  d.qbuf = S->d<uint8_t>(oq);
  d.qoff = S->d<int64_t>(oqo);
  d.qlen = S->d<int32_t>(oql);
  d.tbuf = S->d<uint8_t>(ot);
  d.toff = S->d<int64_t>(oto);
  d.tlen = S->d<int32_t>(otl);
  d.n = n;
  bool all_u8 = true;
  for (int32_t k = 0; k < n; ++k) all_u8 = all_u8 && (xtra[k] & FCS_KSW_XBYTE);
  if ((rc = launch_bsw_align(d, to_params(params), S->d<int32_t>(ox), mq, mt, S->d<int32_t>(oo), s, all_u8)))
    return rc;
  FCS_HIP_CHECK(hipMemcpyAsync(S->h<void>(oo), S->d<void>(oo), sizeof(fcs_kswr) * nn, hipMemcpyDeviceToHost, s));
  FCS_HIP_CHECK(hipStreamSynchronize(s));
  std::memcpy(out, S->h<void>(oo), sizeof(fcs_kswr) * nn);
  return FCS_OK;
}

int fcs_bsw_align_dev(const fcs_bsw_batch* b, const fcs_bsw_params* params, const int32_t* dev_xtra, fcs_kswr* dev_out,
                      int32_t device, void* stream) {
  if (!b || b->n < 0 || (b->n > 0 && (!dev_xtra || !dev_out)))
    return fail(FCS_ERR_INVALID, "[E::fcs_bsw_align_dev] bad arguments");
  int rc = check_params(params);
  if (rc) return rc;
  if (b->n == 0) return FCS_OK;
  if (b->n > 0x7FFFFFFF) return fail(FCS_ERR_UNSUPPORTED, "[E::fcs_bsw_align_dev] more than 2^31-1 tasks");
  if ((rc = check_device(device))) return rc;
  FCS_SET_DEVICE((device));
  BswDevBatch d{};
  d.qbuf = b->qbuf;
  d.qoff = b->qoff;
  d.qlen = b->qlen;
  d.tbuf = b->tbuf;
  d.toff = b->toff;
  d.tlen = b->tlen;
  d.h0 = b->h0;
  d.w = b->w;
  d.n = b->n;
  return launch_bsw_align(d, to_params(params), dev_xtra, std::max(b->max_qlen, 1), std::max(b->max_tlen, 1),
                          reinterpret_cast<int32_t*>(dev_out), (hipStream_t)stream, false);
}

fcs_kswr fcs_ksw_align2(int qlen, const uint8_t* query, int tlen, const uint8_t* target, int m, const int8_t* mat,
                        int o_del, int e_del, int o_ins, int e_ins, int xtra, void** qry) {
  fcs_kswr r{FCS_KSW_FAILED, -1, -1, -1, -1, -1, -1};
  if (m != 5) return (void)fail(FCS_ERR_UNSUPPORTED, "[E::fcs_ksw_align2] only m == 5 (bwa's alphabet) is supported"), r;
  if (!mat) return (void)fail(FCS_ERR_INVALID, "[E::fcs_ksw_align2] null matrix"), r;
  if (qry && *qry) return (void)fail(FCS_ERR_UNSUPPORTED, "[E::fcs_ksw_align2] cached query profiles unsupported"), r;
  fcs_bsw_params p;
  std::memcpy(p.mat, mat, 25);
  p.o_del = o_del;
  p.e_del = e_del;
  p.o_ins = o_ins;
  p.e_ins = e_ins;
  p.end_bonus = 0;
  p.zdrop = 0;
  fcs_bsw_task t{qlen, tlen, 0, 0, query, target};
  fcs_kswr out;
  if (fcs_bsw_align(&t, 1, &p, &xtra, &out, g_default_device)) return r;
  return out;
}

int fcs_ksw_extend2(int qlen, const uint8_t* query, int tlen, const uint8_t* target, int m, const int8_t* mat,
                    int o_del, int e_del, int o_ins, int e_ins, int w, int end_bonus, int zdrop, int h0, int* qle,
                    int* tle, int* gtle, int* gscore, int* max_off) {
  if (m != 5) return (void)fail(FCS_ERR_UNSUPPORTED, "[E::fcs_ksw_extend2] only m == 5 (bwa's alphabet) is supported"), FCS_KSW_FAILED;
  if (!mat) return (void)fail(FCS_ERR_INVALID, "[E::fcs_ksw_extend2] null matrix"), FCS_KSW_FAILED;
  fcs_bsw_params p;
  std::memcpy(p.mat, mat, 25);
  p.o_del = o_del;
  p.e_del = e_del;
  p.o_ins = o_ins;
  p.e_ins = e_ins;
  p.end_bonus = end_bonus;
  p.zdrop = zdrop;
  fcs_bsw_task t{qlen, tlen, h0, w, query, target};
  fcs_bsw_result r;
  int rc = fcs_bsw_extend(&t, 1, &p, &r, g_default_device);
  if (rc) return FCS_KSW_FAILED;
  if (qle) *qle = r.qle;
  if (tle) *tle = r.tle;
  if (gtle) *gtle = r.gtle;
  if (gscore) *gscore = r.gscore;
  if (max_off) *max_off = r.max_off;
  return r.score;
}

int fcs_ksw_global2(int qlen, const uint8_t* query, int tlen, const uint8_t* target, int m, const int8_t* mat,
                    int o_del, int e_del, int o_ins, int e_ins, int w, int* n_cigar, uint32_t** cigar) {
  if (m != 5) return (void)fail(FCS_ERR_UNSUPPORTED, "[E::fcs_ksw_global2] only m == 5 (bwa's alphabet) is supported"), FCS_KSW_FAILED;
  if (!mat) return (void)fail(FCS_ERR_INVALID, "[E::fcs_ksw_global2] null matrix"), FCS_KSW_FAILED;
  fcs_bsw_params p;
  std::memcpy(p.mat, mat, 25);
  p.o_del = o_del;
  p.e_del = e_del;
  p.o_ins = o_ins;
  p.e_ins = e_ins;
  p.end_bonus = 0;
  p.zdrop = 0;
  fcs_bsw_task t{qlen, tlen, 1, w, query, target};
  int32_t score = 0;
  const bool want = n_cigar && cigar;
  const int32_t cap = qlen + tlen + 2;
  std::vector<uint32_t> arena(want ? cap : 0);
  int64_t off = 0;
  int32_t nc = 0;
  int rc = fcs_bsw_global(&t, 1, &p, &score, want ? arena.data() : nullptr, want ? &off : nullptr,
                          want ? &cap : nullptr, want ? &nc : nullptr, g_default_device);
  if (rc) return FCS_KSW_FAILED;
  if (want) {
    *n_cigar = nc;
    *cigar = nc ? static_cast<uint32_t*>(std::malloc(sizeof(uint32_t) * nc)) : nullptr;
    if (nc && !*cigar) return (void)fail(FCS_ERR_NOMEM, "[E::fcs_ksw_global2] malloc failed"), FCS_KSW_FAILED;
    if (nc) std::memcpy(*cigar, arena.data(), sizeof(uint32_t) * nc);
  }
  return score;
}

int fcs_bgzf_index(const uint8_t* comp, int64_t comp_bytes, int64_t* coff, int64_t* uoff, int32_t cap,
                   int32_t* n_members, int64_t* comp_used) {
  if (!n_members || !comp_used || comp_bytes < 0 || cap < 0 || (comp_bytes > 0 && !comp) || !coff || !uoff)
    return fail(FCS_ERR_INVALID, "[E::fcs_bgzf_index] bad arguments");
  auto le16 = [&](int64_t at) { return (uint32_t)comp[at] | (uint32_t)comp[at + 1] << 8; };
  int64_t at = 0, u = 0;
  int32_t k = 0;
  while (k < cap && comp_bytes - at >= 18) {
    // gzip member with FEXTRA (RFC 1952) carrying the BGZF "BC" subfield
    if (comp[at] != 31 || comp[at + 1] != 139 || comp[at + 2] != 8 || !(comp[at + 3] & 4))
      return fail(FCS_ERR_INVALID, "[E::fcs_bgzf_index] no BGZF header at byte " + std::to_string(at));
    const int64_t xlen = le16(at + 10);
    if (comp_bytes - at < 12 + xlen) break;
    int64_t bsize = -1;
    for (int64_t x = at + 12; x + 4 <= at + 12 + xlen;) {
      const int64_t slen = le16(x + 2);
      if (comp[x] == 'B' && comp[x + 1] == 'C' && slen == 2 && x + 6 <= at + 12 + xlen) bsize = le16(x + 4);
      x += 4 + slen;
    }
    if (bsize < 0 || bsize + 1 < 12 + xlen + 8)
      return fail(FCS_ERR_INVALID, "[E::fcs_bgzf_index] no BGZF block size at byte " + std::to_string(at));
    const int64_t len = bsize + 1;
    if (comp_bytes - at < len) break;  // incomplete: left for the next call
    const int64_t isize = (int64_t)(le16(at + len - 4) | le16(at + len - 2) << 16);
    if (isize > 65536)
      return fail(FCS_ERR_INVALID, "[E::fcs_bgzf_index] member at byte " + std::to_string(at) + " inflates past 64 KiB");
    coff[k] = at;
    uoff[k] = u;
    at += len;
    u += isize;
    ++k;
  }
  coff[k] = at;
  uoff[k] = u;
  *n_members = k;
  *comp_used = at;
  return FCS_OK;
}

int fcs_bgzf_inflate_dev(const uint8_t* dev_comp, const int64_t* dev_coff, const int64_t* dev_uoff, int32_t n,
                         uint8_t* dev_out, int32_t* dev_status, int32_t device, void* stream) {
  if (n < 0 || (n > 0 && (!dev_comp || !dev_coff || !dev_uoff || !dev_out || !dev_status)))
    return fail(FCS_ERR_INVALID, "[E::fcs_bgzf_inflate_dev] bad arguments");
  if (n == 0) return FCS_OK;
  int rc = check_device(device);
  if (rc) return rc;
  FCS_SET_DEVICE((device));
  return launch_bgzf_inflate(dev_comp, dev_coff, dev_uoff, n, dev_out, dev_status, static_cast<hipStream_t>(stream));
}

namespace {

// fcs_bgzf_inflate / fcs_bgzf_inflate_try: `try_only` takes an idle inflate
// session whose arenas already fit the call, or returns FCS_BGZF_BUSY.
int bgzf_inflate_host(const uint8_t* comp, int64_t comp_bytes, uint8_t* out, int64_t out_cap, int64_t* comp_used,
                      int64_t* out_bytes, int32_t device, bool try_only) {
  if (!comp_used || !out_bytes || comp_bytes < 0 || (comp_bytes > 0 && !comp) || out_cap < 0 || (out_cap > 0 && !out))
    return fail(FCS_ERR_INVALID, "[E::fcs_bgzf_inflate] bad arguments");
  *comp_used = 0;
  *out_bytes = 0;
  // a member is at least 28 bytes (18 of header / trailer, 2 of DEFLATE); the
  // offset tables are this thread's, kept between calls (no fresh zeroed
  // pages per call)
  const int64_t most = std::min<int64_t>(comp_bytes / 20 + 1, 0x7FFFFFFE);
  static thread_local std::vector<int64_t> coff, uoff;
  if (coff.size() < (size_t)most + 1) {
    coff.resize((size_t)most + 1);
    uoff.resize((size_t)most + 1);
  }
  int32_t n = 0;
  int64_t used = 0;
  int rc = fcs_bgzf_index(comp, comp_bytes, coff.data(), uoff.data(), (int32_t)most, &n, &used);
  if (rc) return rc;
  const int64_t total = uoff[(size_t)n];
  if (total > out_cap)
    return fail(FCS_ERR_INVALID, "[E::fcs_bgzf_inflate] output needs " + std::to_string(total) + " bytes, capacity " +
                                     std::to_string(out_cap));
  *comp_used = used;
  if (n == 0) return FCS_OK;
  if ((rc = check_device(device))) return rc;
  FCS_SET_DEVICE((device));
  // FCS_BGZF_TRACE=1: one stderr line per call with its phases (ms)
  static const bool trace = std::getenv("FCS_BGZF_TRACE") != nullptr;
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  auto ms = [&](clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); };
  const size_t nn = (size_t)n;
  Layout L;
  const size_t oco = L.add(8 * (nn + 1)), ouo = L.add(8 * (nn + 1)), ocp = L.add((size_t)used + 16);
  const size_t in_bytes = L.total, ost = L.add(4 * nn), oout = L.add((size_t)total);
  SessionLease lease;
  if (try_only) {
    if (!lease.try_acquire(device, kInflateSession, L.total)) {
      *comp_used = 0;
      return FCS_BGZF_BUSY;
    }
  } else if ((rc = lease.acquire(device, kInflateSession))) {
    return rc;
  }
  Session* S = lease.get();
  // Through the session's pinned staging arena.  Copies straight from and to
  // the caller's pageable buffers with device scratch from the stream-ordered
  // pool were tried: with 16 shard threads calling at once, member 0 of a
  // call came out corrupt in about one htc run in four (r5ae, r5al, r5am),
  // never with the pinned arena.
  const double t_lease = ms(t0);
  if ((rc = S->ensure_host(L.total)) || (rc = S->ensure_dev(L.total))) return rc;
  const double t_alloc = ms(t0);
  std::memcpy(S->h<void>(oco), coff.data(), 8 * (nn + 1));
  std::memcpy(S->h<void>(ouo), uoff.data(), 8 * (nn + 1));
  std::memcpy(S->h<void>(ocp), comp, (size_t)used);
  const double t_in = ms(t0);
  hipStream_t s = S->s;
  const StreamDrain drain{s};
  FCS_HIP_CHECK(hipMemcpyAsync(S->dev, S->host, in_bytes, hipMemcpyHostToDevice, s));
  if ((rc = launch_bgzf_inflate(S->d<uint8_t>(ocp), S->d<int64_t>(oco), S->d<int64_t>(ouo), n, S->d<uint8_t>(oout),
                                S->d<int32_t>(ost), s)))
    return rc;
  FCS_HIP_CHECK(hipMemcpyAsync(S->h<void>(ost), S->d<void>(ost), L.total - ost, hipMemcpyDeviceToHost, s));
  // the calling shard thread sleeps until the copy lands: a spinning wait of
  // 16 shard threads costs more host time than the inflate saves
  if (!S->done) FCS_HIP_CHECK(hipEventCreateWithFlags(&S->done, hipEventBlockingSync | hipEventDisableTiming));
  FCS_HIP_CHECK(hipEventRecord(S->done, s));
  FCS_HIP_CHECK(hipEventSynchronize(S->done));
  const double t_gpu = ms(t0);
  const int32_t* st = S->h<int32_t>(ost);
  for (size_t k = 0; k < nn; ++k)
    if (st[k] != FCS_BGZF_OK) {
      static const char* what[4] = {"ok", "corrupt DEFLATE stream", "inflates past its ISIZE", "CRC-32 mismatch"};
      return fail(FCS_ERR_INVALID, "[E::fcs_bgzf_inflate] member " + std::to_string(k) + " at byte " +
                                       std::to_string(coff[k]) + ": " + what[st[k] & 3]);
    }
  std::memcpy(out, S->h<void>(oout), (size_t)total);
  *out_bytes = total;
  if (trace)
    std::fprintf(stderr, "[fcs_bgzf_inflate] %d members, %lld -> %lld bytes: lease %.2f alloc %.2f in %.2f gpu %.2f out %.2f ms\n",
                 n, (long long)used, (long long)total, t_lease, t_alloc - t_lease, t_in - t_alloc, t_gpu - t_in,
                 ms(t0) - t_gpu);
  return FCS_OK;
}

}  // namespace

int fcs_bgzf_inflate(const uint8_t* comp, int64_t comp_bytes, uint8_t* out, int64_t out_cap, int64_t* comp_used,
                     int64_t* out_bytes, int32_t device) {
  return bgzf_inflate_host(comp, comp_bytes, out, out_cap, comp_used, out_bytes, device, false);
}

int fcs_bgzf_inflate_try(const uint8_t* comp, int64_t comp_bytes, uint8_t* out, int64_t out_cap, int64_t* comp_used,
                         int64_t* out_bytes, int32_t device) {
  return bgzf_inflate_host(comp, comp_bytes, out, out_cap, comp_used, out_bytes, device, true);
}

int fcs_bgzf_warmup(int32_t device, int32_t sessions, int64_t arena_bytes) {
  if (sessions < 0 || arena_bytes < 0) return fail(FCS_ERR_INVALID, "[E::fcs_bgzf_warmup] bad arguments");
  int rc = check_device(device);
  if (rc) return rc;
  FCS_SET_DEVICE((device));
  sessions = std::min(sessions, sessions_per_device(kInflateSession));
  // lease them all at once (so each is a different session), size, return
  std::vector<std::unique_ptr<SessionLease>> held;
  for (int k = 0; k < sessions; ++k) {
    auto L = std::make_unique<SessionLease>();
    if ((rc = L->acquire(device, kInflateSession))) return rc;
    if ((rc = (*L)->ensure_host((size_t)arena_bytes)) || (rc = (*L)->ensure_dev((size_t)arena_bytes))) return rc;
    held.push_back(std::move(L));
  }
  return FCS_OK;
}

int fcs_device_release(int32_t device) {
  int rc = check_device(device);
  if (rc) return rc;
  SessionPool& C = session_pool(device, kComputeSession);
  SessionPool& I = session_pool(device, kInflateSession);
  {
    // one critical section from the idle check to the drop: a lease between
    // them would hold a session the reset destroys.  `releasing` then refuses
    // every lease (FCS_ERR_INVALID, or busy for a try) until the reset is done.
    std::scoped_lock lk(C.mu, I.mu);
    for (SessionPool* P : {&C, &I})
      if (P->releasing || P->creating || P->idle.size() != P->all.size())
        return fail(FCS_ERR_INVALID, "[E::fcs_device_release] a call on this device is still running");
    // the handles die with the reset below: the pools, fork sets and tables
    // are dropped (not destroyed one by one) and made again on the next call
    for (SessionPool* P : {&C, &I}) {
      P->all.clear();
      P->idle.clear();
      P->releasing = true;
    }
  }
  struct Reopen {  // leases are accepted again once the reset has returned (or failed)
    SessionPool *c, *i;
    ~Reopen() {
      std::scoped_lock lk(c->mu, i->mu);
      c->releasing = i->releasing = false;
    }
  } reopen{&C, &I};
  {
    std::lock_guard<std::mutex> lk(g_fork_mu);
    for (auto it = g_fork_sets->begin(); it != g_fork_sets->end();)
      it = it->first.first == device ? g_fork_sets->erase(it) : std::next(it);
    for (auto it = g_stream_ws->begin(); it != g_stream_ws->end();)
      it = it->first.first == device ? g_stream_ws->erase(it) : std::next(it);
  }
  {
    std::lock_guard<std::mutex> lk(g_dev_mu);
    auto it = g_tables.find(device);
    if (it != g_tables.end()) {
      (void)it->second.release();
      g_tables.erase(it);
    }
  }
  FCS_SET_DEVICE((device));
  FCS_HIP_CHECK(hipDeviceSynchronize());
  FCS_HIP_CHECK(hipDeviceReset());
  return FCS_OK;
}

int fcs_abi_symbol_count(void) { return 47; }

}  // extern "C"

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
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "fcship_internal.h"

namespace fcs {

static thread_local std::string g_last_error;
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

// One stream per (thread, device) for the synchronous host-pointer entry points.
hipStream_t thread_stream(int device) {
  static thread_local std::map<int, hipStream_t> streams;
  auto it = streams.find(device);
  if (it != streams.end()) return it->second;
  hipStream_t s = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return nullptr;
  streams[device] = s;
  return s;
}

struct ForkSet {
  hipStream_t side[kForkStreams - 1] = {};
  hipEvent_t fork = nullptr;
  hipEvent_t join[kForkStreams - 1] = {};
};

// Side streams and events of the calling thread on the current device.
ForkSet* fork_set() {
  int device = 0;
  if (hipGetDevice(&device) != hipSuccess) return nullptr;
  static thread_local std::map<int, ForkSet> sets;
  auto it = sets.find(device);
  if (it != sets.end()) return &it->second;
  ForkSet f;
  if (hipEventCreateWithFlags(&f.fork, hipEventDisableTiming) != hipSuccess) return nullptr;
  for (int i = 0; i < kForkStreams - 1; ++i)
    if (hipStreamCreateWithFlags(&f.side[i], hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&f.join[i], hipEventDisableTiming) != hipSuccess)
      return nullptr;
  return &(sets[device] = f);
}

}  // namespace

int fork_streams(hipStream_t s, hipStream_t (&fs)[kForkStreams]) {
  ForkSet* f = fork_set();
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
  ForkSet* f = fork_set();
  if (!f) return fail(FCS_ERR_DEVICE, "[E::fcship] cannot create side streams");
  for (int i = 0; i < kForkStreams - 1; ++i) {
    FCS_HIP_CHECK(hipEventRecord(f->join[i], fs[i + 1]));
    FCS_HIP_CHECK(hipStreamWaitEvent(s, f->join[i], 0));
  }
  return FCS_OK;
}

namespace {

// RAII device buffer for the synchronous paths.
struct DevBuf {
  void* p = nullptr;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  int alloc(size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (hipMalloc(&p, bytes) != hipSuccess) {
      p = nullptr;
      return fail(FCS_ERR_NOMEM, "[E::fcship] hipMalloc failed");
    }
    return FCS_OK;
  }
  template <typename T> T* as() const { return static_cast<T*>(p); }
};

int upload(DevBuf& d, const void* src, size_t bytes, hipStream_t s) {
  int rc = d.alloc(bytes);
  if (rc) return rc;
  if (bytes && src) FCS_HIP_CHECK(hipMemcpyAsync(d.p, src, bytes, hipMemcpyHostToDevice, s));
  return FCS_OK;
}

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

// Workspace for one SW schedule of up to cap tasks.  Stream-ordered
// allocation when `stream_alloc`, so the *_dev entry point stays asynchronous.
int ws_alloc(BswWorkspace& ws, int64_t cap, hipStream_t s, bool stream_alloc) {
  ws.cap = cap;
  const size_t n = (size_t)std::max<int64_t>(cap, 1);
  size_t tmp = 0;
  FCS_HIP_CHECK(sort_pairs_u32(nullptr, tmp, nullptr, nullptr, nullptr, nullptr, (int)n, s));
  ws.tmp_bytes = std::max<size_t>(tmp, 16);
  void** bufs[6] = {(void**)&ws.keys_in, (void**)&ws.keys_out, (void**)&ws.idx_in, (void**)&ws.idx_out,
                    (void**)&ws.bounds, &ws.tmp};
  const size_t sz[6] = {4 * n, 4 * n, 4 * n, 4 * n, (kBswWideBucket + 2) * sizeof(int64_t), ws.tmp_bytes};
  for (int i = 0; i < 6; ++i) {
    if (stream_alloc) FCS_HIP_CHECK(hipMallocAsync(bufs[i], sz[i], s));
    else FCS_HIP_CHECK(hipMalloc(bufs[i], sz[i]));
  }
  return FCS_OK;
}

void ws_free(BswWorkspace& ws, hipStream_t s, bool stream_alloc) {
  void* bufs[6] = {ws.keys_in, ws.keys_out, ws.idx_in, ws.idx_out, ws.bounds, ws.tmp};
  for (void* b : bufs)
    if (b) (void)(stream_alloc ? hipFreeAsync(b, s) : hipFree(b));
  ws = BswWorkspace();
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
using SortConfig = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                              rocprim::default_config, 0>;
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
    FCS_HIP_CHECK(hipSetDevice(device));
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
  uint32_t* keys_in = nullptr;
  uint32_t* keys_out = nullptr;
  int32_t* idx_in = nullptr;
  int32_t* idx_out = nullptr;
  void* sort_tmp = nullptr;
  size_t sort_tmp_bytes = 0;
  int32_t* rescue_list = nullptr;
  unsigned long long* rescue_count = nullptr;  // [0] rescue count, then int64 class bounds[7]
  int64_t* bounds = nullptr;
  int64_t scheduled = -1;  // n_pairs of the last schedule
};

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
  FCS_HIP_CHECK(hipSetDevice(device));
  DeviceTables* t = nullptr;
  rc = get_device_tables(device, &t);
  if (rc) return rc;
  std::unique_ptr<fcs_phmm_plan> p(new fcs_phmm_plan());
  p->device = device;
  p->max_pairs = max_pairs;
  const size_t n = (size_t)std::max<int64_t>(max_pairs, 1);
  FCS_HIP_CHECK(hipMalloc(&p->keys_in, n * 4));
  FCS_HIP_CHECK(hipMalloc(&p->keys_out, n * 4));
  FCS_HIP_CHECK(hipMalloc(&p->idx_in, n * 4));
  FCS_HIP_CHECK(hipMalloc(&p->idx_out, n * 4));
  FCS_HIP_CHECK(hipMalloc(&p->rescue_list, n * 4));
  FCS_HIP_CHECK(hipMalloc(&p->rescue_count, 8 * sizeof(unsigned long long)));
  // hipMemset runs on the null stream, which does not order against the
  // non-blocking streams the plan is used on: without the synchronize it could
  // land after a later schedule had written the class bounds next to the count
  // (zeroing them, so class launches computed nothing).  Waited for here; the
  // count and the bounds are rewritten stream-ordered on every run anyway.
  FCS_HIP_CHECK(hipMemset(p->rescue_count, 0, 8 * sizeof(unsigned long long)));
  FCS_HIP_CHECK(hipStreamSynchronize(nullptr));
  p->bounds = reinterpret_cast<int64_t*>(p->rescue_count + 1);
  size_t tmp = 0;
  FCS_HIP_CHECK(sort_pairs_u32(nullptr, tmp, p->keys_in, p->keys_out, p->idx_in, p->idx_out, (int)n, nullptr));
  p->sort_tmp_bytes = std::max<size_t>(tmp, 16);
  FCS_HIP_CHECK(hipMalloc(&p->sort_tmp, p->sort_tmp_bytes));
  *plan = p.release();
  return FCS_OK;
}

int fcs_phmm_plan_destroy(fcs_phmm_plan* p) {
  if (!p) return FCS_OK;
  (void)hipSetDevice(p->device);
  (void)hipFree(p->keys_in);
  (void)hipFree(p->keys_out);
  (void)hipFree(p->idx_in);
  (void)hipFree(p->idx_out);
  (void)hipFree(p->sort_tmp);
  (void)hipFree(p->rescue_list);
  (void)hipFree(p->rescue_count);
  delete p;
  return FCS_OK;
}

int fcs_phmm_dev_schedule(fcs_phmm_plan* plan, const fcs_phmm_batch* b, void* stream) {
  if (!plan) return fail(FCS_ERR_INVALID, "[E::fcs_phmm_dev_schedule] null plan");
  int rc = check_batch_shape(b);
  if (rc) return rc;
  if (b->n_pairs > plan->max_pairs) return fail(FCS_ERR_INVALID, "[E::fcs_phmm_dev_schedule] batch exceeds plan");
  FCS_HIP_CHECK(hipSetDevice(plan->device));
  hipStream_t s = (hipStream_t)stream;
  const PhmmDevBatch d = to_dev(b);
  rc = launch_phmm_keys(d, plan->keys_in, plan->idx_in, s);
  if (rc) return rc;
  if (b->n_pairs > 0) {
    size_t tmp = plan->sort_tmp_bytes;
    FCS_HIP_CHECK(sort_pairs_u32(plan->sort_tmp, tmp, plan->keys_in, plan->keys_out, plan->idx_in, plan->idx_out,
                                 (int)b->n_pairs, s, kPhmmKeyBits));
  }
  if ((rc = launch_phmm_bounds(plan->keys_out, b->n_pairs, plan->bounds, s))) return rc;
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
  FCS_HIP_CHECK(hipSetDevice(plan->device));
  DeviceTables* t = nullptr;
  rc = get_device_tables(plan->device, &t);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  FCS_HIP_CHECK(hipMemsetAsync(plan->rescue_count, 0, sizeof(unsigned long long), s));
  return launch_phmm_forward(to_dev(b), plan->idx_out, b->n_pairs, std::max(b->max_hap_len, 1), plan->bounds, *t,
                             opts->exact_order != 0, out, plan->rescue_list, plan->rescue_count,
                             opts->rescue_threshold, opts->use_fp64_rescue != 0, s);
}

int fcs_phmm_dev_rescue(fcs_phmm_plan* plan, const fcs_phmm_batch* b, double* out, const fcs_phmm_opts* opts,
                        void* stream) {
  if (!plan || !opts) return fail(FCS_ERR_INVALID, "[E::fcs_phmm_dev_rescue] null plan/opts");
  int rc = check_batch_shape(b);
  if (rc) return rc;
  if (!opts->use_fp64_rescue) return FCS_OK;
  FCS_HIP_CHECK(hipSetDevice(plan->device));
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

int fcs_phmm_plan_rescue_count(fcs_phmm_plan* plan, void* stream, int64_t* count) {
  if (!plan || !count) return fail(FCS_ERR_INVALID, "[E::fcs_phmm_plan_rescue_count] bad arguments");
  FCS_HIP_CHECK(hipSetDevice(plan->device));
  unsigned long long v = 0;
  FCS_HIP_CHECK(hipMemcpyAsync(&v, plan->rescue_count, sizeof(v), hipMemcpyDeviceToHost, (hipStream_t)stream));
  FCS_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
  *count = (int64_t)v;
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
  int32_t maxr = 0, maxh = 0;
  for (int64_t p = 0; p < b->n_pairs; ++p) {
    const int32_t ri = b->pair_read[p], hi = b->pair_hap[p];
    if (ri < 0 || ri >= b->n_reads || hi < 0 || hi >= b->n_haps)
      return fail(FCS_ERR_INVALID, "[E::fcs_phmm_compute_pairs] pair index out of range");
  }
  for (int64_t r = 0; r < b->n_reads; ++r) {
    if (b->read_len[r] < 0 || b->read_off[r] < 0 || b->read_off[r] + b->read_len[r] > b->read_bytes)
      return fail(FCS_ERR_INVALID, "[E::fcs_phmm_compute_pairs] read extent outside read arrays");
    maxr = std::max(maxr, b->read_len[r]);
  }
  for (int64_t h = 0; h < b->n_haps; ++h) {
    if (b->hap_len[h] < 0 || b->hap_off[h] < 0 || b->hap_off[h] + b->hap_len[h] > b->hap_bytes)
      return fail(FCS_ERR_INVALID, "[E::fcs_phmm_compute_pairs] hap extent outside hap array");
    maxh = std::max(maxh, b->hap_len[h]);
  }
  if ((rc = check_device(opts.device))) return rc;
  FCS_HIP_CHECK(hipSetDevice(opts.device));
  hipStream_t s = thread_stream(opts.device);
  if (!s) return fail(FCS_ERR_DEVICE, "[E::fcship] stream creation failed");
  DevBuf rb, bq, iq, dq, gq, ro, rl, hb, ho, hl, pr, ph, out;
  const size_t RB = (size_t)b->read_bytes, HB = (size_t)b->hap_bytes;
  if ((rc = upload(rb, b->read_bases, RB, s)) || (rc = upload(bq, b->read_bq, RB, s)) ||
      (rc = upload(iq, b->read_iq, RB, s)) || (rc = upload(dq, b->read_dq, RB, s)) ||
      (rc = upload(gq, b->read_gcp, RB, s)) || (rc = upload(ro, b->read_off, 8 * (size_t)b->n_reads, s)) ||
      (rc = upload(rl, b->read_len, 4 * (size_t)b->n_reads, s)) || (rc = upload(hb, b->hap_bases, HB, s)) ||
      (rc = upload(ho, b->hap_off, 8 * (size_t)b->n_haps, s)) ||
      (rc = upload(hl, b->hap_len, 4 * (size_t)b->n_haps, s)) ||
      (rc = upload(pr, b->pair_read, 4 * (size_t)b->n_pairs, s)) ||
      (rc = upload(ph, b->pair_hap, 4 * (size_t)b->n_pairs, s)) || (rc = out.alloc(8 * (size_t)b->n_pairs)))
    return rc;
  fcs_phmm_batch d = *b;
  d.read_bases = rb.as<uint8_t>();
  d.read_bq = bq.as<uint8_t>();
  d.read_iq = iq.as<uint8_t>();
  d.read_dq = dq.as<uint8_t>();
  d.read_gcp = gq.as<uint8_t>();
  d.read_off = ro.as<int64_t>();
  d.read_len = rl.as<int32_t>();
  d.hap_bases = hb.as<uint8_t>();
  d.hap_off = ho.as<int64_t>();
  d.hap_len = hl.as<int32_t>();
  d.pair_read = pr.as<int32_t>();
  d.pair_hap = ph.as<int32_t>();
  d.max_read_len = maxr;
  d.max_hap_len = maxh;
  fcs_phmm_plan* plan = nullptr;
  rc = fcs_phmm_plan_create(opts.device, b->n_pairs, &plan);
  if (rc) return rc;
  std::unique_ptr<fcs_phmm_plan, int (*)(fcs_phmm_plan*)> guard(plan, fcs_phmm_plan_destroy);
  rc = fcs_phmm_dev_run(plan, &d, out.as<double>(), &opts, s);
  if (rc) return rc;
  FCS_HIP_CHECK(hipMemcpyAsync(out_log10, out.p, 8 * (size_t)b->n_pairs, hipMemcpyDeviceToHost, s));
  FCS_HIP_CHECK(hipStreamSynchronize(s));
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
// are concatenated into one SoA batch whose pair list is region-major and
// read-major within a region, so the flat result splits back into each
// region's read-major matrix by a running offset.
int fcs_phmm_compute_regions(const fcs_phmm_region* regions, int32_t n_regions, const fcs_phmm_opts* opts) {
  if (n_regions < 0 || (n_regions > 0 && !regions))
    return fail(FCS_ERR_INVALID, "[E::fcs_phmm_compute_regions] bad arguments");
  int64_t nr = 0, nh = 0, np = 0, rt = 0, ht = 0;
  for (int32_t g = 0; g < n_regions; ++g) {
    const fcs_phmm_region& R = regions[g];
    if (R.n_reads < 0 || R.n_haps < 0 || (R.n_reads > 0 && !R.reads) || (R.n_haps > 0 && !R.haps))
      return fail(FCS_ERR_INVALID, "[E::fcs_phmm_compute_regions] malformed region");
    const int64_t pairs = (int64_t)R.n_reads * R.n_haps;
    if (pairs > 0 && !R.out_log10) return fail(FCS_ERR_INVALID, "[E::fcs_phmm_compute_regions] null region output");
    for (int32_t r = 0; r < R.n_reads; ++r) {
      const fcs_phmm_read& x = R.reads[r];
      if (x.len < 0 || (x.len > 0 && (!x.bases || !x.base_q || !x.ins_q || !x.del_q || !x.gcp)))
        return fail(FCS_ERR_INVALID, "[E::fcs_phmm_compute_regions] malformed read");
      rt += x.len;
    }
    for (int32_t h = 0; h < R.n_haps; ++h) {
      if (R.haps[h].len < 0 || (R.haps[h].len > 0 && !R.haps[h].bases))
        return fail(FCS_ERR_INVALID, "[E::fcs_phmm_compute_regions] malformed haplotype");
      ht += R.haps[h].len;
    }
    nr += R.n_reads;
    nh += R.n_haps;
    np += pairs;
  }
  if (np == 0) return FCS_OK;
  if (nr > INT32_MAX || nh > INT32_MAX)
    return fail(FCS_ERR_INVALID, "[E::fcs_phmm_compute_regions] more than 2^31 reads or haplotypes");
  std::vector<int64_t> roff(nr), hoff(nh);
  std::vector<int32_t> rlen(nr), hlen(nh), pr(np), ph(np);
  std::vector<uint8_t> rb(rt), bq(rt), iq(rt), dq(rt), gq(rt), hb(ht);
  int64_t ri = 0, hi = 0, pi = 0, ro = 0, ho = 0;
  for (int32_t g = 0; g < n_regions; ++g) {
    const fcs_phmm_region& R = regions[g];
    const int64_t r0 = ri, h0 = hi;
    for (int32_t r = 0; r < R.n_reads; ++r, ++ri) {
      const fcs_phmm_read& x = R.reads[r];
      roff[ri] = ro;
      rlen[ri] = x.len;
      if (x.len) {
        std::memcpy(&rb[ro], x.bases, x.len);
        std::memcpy(&bq[ro], x.base_q, x.len);
        std::memcpy(&iq[ro], x.ins_q, x.len);
        std::memcpy(&dq[ro], x.del_q, x.len);
        std::memcpy(&gq[ro], x.gcp, x.len);
      }
      ro += x.len;
    }
    for (int32_t h = 0; h < R.n_haps; ++h, ++hi) {
      hoff[hi] = ho;
      hlen[hi] = R.haps[h].len;
      if (R.haps[h].len) std::memcpy(&hb[ho], R.haps[h].bases, R.haps[h].len);
      ho += R.haps[h].len;
    }
    for (int32_t r = 0; r < R.n_reads; ++r)
      for (int32_t h = 0; h < R.n_haps; ++h, ++pi) {
        pr[pi] = (int32_t)(r0 + r);
        ph[pi] = (int32_t)(h0 + h);
      }
  }
  fcs_phmm_batch b{};
  b.read_bases = rb.data();
  b.read_bq = bq.data();
  b.read_iq = iq.data();
  b.read_dq = dq.data();
  b.read_gcp = gq.data();
  b.read_off = roff.data();
  b.read_len = rlen.data();
  b.n_reads = nr;
  b.hap_bases = hb.data();
  b.hap_off = hoff.data();
  b.hap_len = hlen.data();
  b.n_haps = nh;
  b.pair_read = pr.data();
  b.pair_hap = ph.data();
  b.n_pairs = np;
  b.read_bytes = rt;
  b.hap_bytes = ht;
  if (n_regions == 1) return fcs_phmm_compute_pairs(&b, regions[0].out_log10, opts);
  std::vector<double> flat(np);
  const int rc = fcs_phmm_compute_pairs(&b, flat.data(), opts);
  if (rc) return rc;
  int64_t off = 0;
  for (int32_t g = 0; g < n_regions; ++g) {
    const int64_t pairs = (int64_t)regions[g].n_reads * regions[g].n_haps;
    if (pairs) std::memcpy(regions[g].out_log10, flat.data() + off, 8 * (size_t)pairs);
    off += pairs;
  }
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
  if (b->n > 0 && (!b->qbuf || !b->qoff || !b->qlen || !b->tbuf || !b->toff || !b->tlen || !b->h0 || !b->w))
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
  FCS_HIP_CHECK(hipSetDevice(device));
  hipStream_t s = (hipStream_t)stream;
  BswWorkspace ws;
  if ((rc = ws_alloc(ws, b->n, s, true))) {
    ws_free(ws, s, true);
    return rc;
  }
  rc = launch_bsw_extend_sorted(bsw_dev(b), to_params(params), std::max(b->max_qlen, 0), std::max(b->max_tlen, 0),
                                res, cells, ws, s);
  ws_free(ws, s, true);
  return rc;
}

int fcs_bsw_plan_create(int32_t device, int64_t max_tasks, fcs_bsw_plan** plan) {
  if (!plan || max_tasks < 0) return fail(FCS_ERR_INVALID, "[E::fcs_bsw_plan_create] bad arguments");
  int rc = check_device(device);
  if (rc) return rc;
  FCS_HIP_CHECK(hipSetDevice(device));
  std::unique_ptr<fcs_bsw_plan> p(new fcs_bsw_plan());
  p->device = device;
  if ((rc = ws_alloc(p->ws, max_tasks, nullptr, false))) {
    ws_free(p->ws, nullptr, false);
    return rc;
  }
  *plan = p.release();
  return FCS_OK;
}

int fcs_bsw_plan_destroy(fcs_bsw_plan* plan) {
  if (!plan) return FCS_OK;
  (void)hipSetDevice(plan->device);
  ws_free(plan->ws, nullptr, false);
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
  FCS_HIP_CHECK(hipSetDevice(plan->device));
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
  FCS_HIP_CHECK(hipSetDevice(device));
  hipStream_t s = thread_stream(device);
  if (!s) return fail(FCS_ERR_DEVICE, "[E::fcship] stream creation failed");
  DevBuf qb, qo, ql, tb, to, tl, h0, w, rs, cl;
  const size_t n = (size_t)b->n;
  if ((rc = upload(qb, b->qbuf, (size_t)b->qbytes, s)) || (rc = upload(qo, b->qoff, 8 * n, s)) ||
      (rc = upload(ql, b->qlen, 4 * n, s)) || (rc = upload(tb, b->tbuf, (size_t)b->tbytes, s)) ||
      (rc = upload(to, b->toff, 8 * n, s)) || (rc = upload(tl, b->tlen, 4 * n, s)) ||
      (rc = upload(h0, b->h0, 4 * n, s)) || (rc = upload(w, b->w, 4 * n, s)) || (rc = rs.alloc(24 * n)) ||
      (rc = cl.alloc(8 * n)))
    return rc;
  fcs_bsw_batch d = *b;
  d.qbuf = qb.as<uint8_t>();
  d.qoff = qo.as<int64_t>();
  d.qlen = ql.as<int32_t>();
  d.tbuf = tb.as<uint8_t>();
  d.toff = to.as<int64_t>();
  d.tlen = tl.as<int32_t>();
  d.h0 = h0.as<int32_t>();
  d.w = w.as<int32_t>();
  d.max_qlen = mq;
  d.max_tlen = mt;
  rc = fcs_bsw_extend_dev(&d, params, rs.as<int32_t>(), cl.as<int64_t>(), device, s);
  if (rc) return rc;
  FCS_HIP_CHECK(hipMemcpyAsync(res, rs.p, 24 * n, hipMemcpyDeviceToHost, s));
  if (cells) FCS_HIP_CHECK(hipMemcpyAsync(cells, cl.p, 8 * n, hipMemcpyDeviceToHost, s));
  FCS_HIP_CHECK(hipStreamSynchronize(s));
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
    zt += ncol * pk.tlen[k];
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
  FCS_HIP_CHECK(hipSetDevice(device));
  hipStream_t s = thread_stream(device);
  if (!s) return fail(FCS_ERR_DEVICE, "[E::fcship] stream creation failed");
  DevBuf qb, qo, ql, tb, to, tl, h0, w, sc, zb, zo, cg, co, cc, nc;
  const size_t nn = (size_t)n;
  if ((rc = upload(qb, pk.q.data(), pk.q.size(), s)) || (rc = upload(qo, pk.qoff.data(), 8 * nn, s)) ||
      (rc = upload(ql, pk.qlen.data(), 4 * nn, s)) || (rc = upload(tb, pk.t.data(), pk.t.size(), s)) ||
      (rc = upload(to, pk.toff.data(), 8 * nn, s)) || (rc = upload(tl, pk.tlen.data(), 4 * nn, s)) ||
      (rc = upload(h0, pk.h0.data(), 4 * nn, s)) || (rc = upload(w, pk.w.data(), 4 * nn, s)) ||
      (rc = sc.alloc(4 * nn)) || (rc = zb.alloc((size_t)zt)) || (rc = upload(zo, zoff.data(), 8 * nn, s)))
    return rc;
  if (want_cigar) {
    if ((rc = cg.alloc(4 * (size_t)ct)) || (rc = upload(co, cigar_off, 8 * nn, s)) ||
        (rc = upload(cc, cigar_cap, 4 * nn, s)) || (rc = nc.alloc(4 * nn)))
      return rc;
  }
  BswDevBatch d;
  d.qbuf = qb.as<uint8_t>();
  d.qoff = qo.as<int64_t>();
  d.qlen = ql.as<int32_t>();
  d.tbuf = tb.as<uint8_t>();
  d.toff = to.as<int64_t>();
  d.tlen = tl.as<int32_t>();
  d.h0 = h0.as<int32_t>();
  d.w = w.as<int32_t>();
  d.n = n;
  rc = launch_bsw_global(d, to_params(params), mq, mt, sc.as<int32_t>(), want_cigar ? zb.as<uint8_t>() : nullptr,
                         zt, zo.as<int64_t>(), want_cigar ? cg.as<uint32_t>() : nullptr, co.as<int64_t>(),
                         cc.as<int32_t>(), nc.as<int32_t>(), s);
  if (rc) return rc;
  FCS_HIP_CHECK(hipMemcpyAsync(scores, sc.p, 4 * nn, hipMemcpyDeviceToHost, s));
  if (want_cigar) {
    FCS_HIP_CHECK(hipMemcpyAsync(n_cigar, nc.p, 4 * nn, hipMemcpyDeviceToHost, s));
    if (ct) FCS_HIP_CHECK(hipMemcpyAsync(cigar_arena, cg.p, 4 * (size_t)ct, hipMemcpyDeviceToHost, s));
  }
  FCS_HIP_CHECK(hipStreamSynchronize(s));
  if (want_cigar)
    for (int32_t k = 0; k < n; ++k)
      if (n_cigar[k] > cigar_cap[k])
        return fail(FCS_ERR_INVALID, "[E::fcs_bsw_global] CIGAR longer than its arena slot");
  return FCS_OK;
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

int fcs_abi_symbol_count(void) { return 30; }

}  // extern "C"

// Internal definitions shared by the gfx950 kernels and the C-ABI layer.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "fcship.h"

namespace fcs {

// ------------------------------------------------------------ error plumbing
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
#define FCS_HIP_CHECK(expr)                                                                  \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess)                                                                    \
      return ::fcs::fail(FCS_ERR_DEVICE, std::string("[E::fcship] ") + #expr + ": " +        \
                                             hipGetErrorString(_e));                         \
  } while (0)

// The caller's current device, restored when an entry point returns (every
// path): a host thread that drives another GPU is not switched by a call.
struct DeviceScope {
  int prev = -1;
  DeviceScope() {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  }
  ~DeviceScope() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  DeviceScope(const DeviceScope&) = delete;
  DeviceScope& operator=(const DeviceScope&) = delete;
};
#define FCS_SET_DEVICE(d)                 \
  ::fcs::DeviceScope _fcs_device_scope;   \
  FCS_HIP_CHECK(hipSetDevice(d))

// ------------------------------------------------------------ DPP cross-lane
// CDNA (gfx9) DPP controls.  row = 16 lanes.
enum : int {
  kDppRowShr1 = 0x111,
  kDppRowShr2 = 0x112,
  kDppRowShr4 = 0x114,
  kDppRowShr8 = 0x118,
  kDppRowRor1 = 0x121,
  kDppRowRor2 = 0x122,
  kDppRowRor4 = 0x124,
  kDppRowRor8 = 0x128,
  kDppWaveShr1 = 0x138,
  kDppRowBcast15 = 0x142,
  kDppRowBcast31 = 0x143,
};

// src taken from lane-1 within each 16-lane row; lane 0 of a row keeps `old`.
__device__ __forceinline__ int dpp_row_shr1_i(int old, int src) {
  return __builtin_amdgcn_update_dpp(old, src, kDppRowShr1, 0xF, 0xF, false);
}
__device__ __forceinline__ float dpp_row_shr1_f(float old, float src) {
  return __int_as_float(
      __builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(src), kDppRowShr1, 0xF, 0xF, false));
}
__device__ __forceinline__ double dpp_row_shr1_d(double old, double src) {
  const long long o = __double_as_longlong(old), s = __double_as_longlong(src);
  const int lo = __builtin_amdgcn_update_dpp((int)o, (int)s, kDppRowShr1, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(s >> 32), kDppRowShr1, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <typename T> __device__ __forceinline__ T dpp_row_shr1(T old, T src);
template <> __device__ __forceinline__ float dpp_row_shr1<float>(float old, float src) { return dpp_row_shr1_f(old, src); }
template <> __device__ __forceinline__ double dpp_row_shr1<double>(double old, double src) { return dpp_row_shr1_d(old, src); }

// Whole-wave shift by one lane: lane l gets src of lane l-1, lane 0 keeps `old`.
__device__ __forceinline__ int dpp_wave_shr1_i(int old, int src) {
  return __builtin_amdgcn_update_dpp(old, src, kDppWaveShr1, 0xF, 0xF, false);
}

// Inclusive max-scan over the 64 lanes of a wave (lane order), identity `neg`.
__device__ __forceinline__ int wave_incl_max(int v, int neg) {
  v = max(v, __builtin_amdgcn_update_dpp(neg, v, kDppRowShr1, 0xF, 0xF, false));
  v = max(v, __builtin_amdgcn_update_dpp(neg, v, kDppRowShr2, 0xF, 0xF, false));
  v = max(v, __builtin_amdgcn_update_dpp(neg, v, kDppRowShr4, 0xF, 0xF, false));
  v = max(v, __builtin_amdgcn_update_dpp(neg, v, kDppRowShr8, 0xF, 0xF, false));
  v = max(v, __builtin_amdgcn_update_dpp(neg, v, kDppRowBcast15, 0xA, 0xF, false));
  v = max(v, __builtin_amdgcn_update_dpp(neg, v, kDppRowBcast31, 0xC, 0xF, false));
  return v;
}

__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }

__device__ __forceinline__ int read_lane(int v, int lane) { return __builtin_amdgcn_readlane(v, lane); }
__device__ __forceinline__ int first_lane(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Max over the wave, result uniform.
__device__ __forceinline__ int wave_max(int v) {
  return read_lane(wave_incl_max(v, INT32_MIN), 63);
}

// ------------------------------------------------------------ ksw band limit
// bwa ksw_extend2's max_ins / max_del: (int)((double)(qlen * max_mat +
// end_bonus - o) / e + 1.), at least 1.  In integers: for e > 0 the truncation
// of n / e + 1 is (n + e) / e with C's truncating division (for |n| < 2^31 and
// e < 2^20 the double quotient never rounds across an integer), which keeps
// the f64 divide (and its register pairs) out of the SW kernels' wave setup.
__host__ __device__ __forceinline__ int bwa_max_gap(int qlen, int max_mat, int end_bonus, int o, int e) {
  if (e <= 0) return 0x7FFFFFFF;  // bwa divides by zero here; the cast of +inf saturates on gfx950: no limit
  const int n = qlen * max_mat + end_bonus - o;
  const int m = (n + e) / e;
  return m > 1 ? m : 1;
}

// ------------------------------------------------------------ PairHMM tables
// Host-computed (fcship_tables.cpp) GKL Context<T> tables, uploaded once per device.
template <typename T>
struct PhmmTables {
  const T* ph2pr;   // [128] 10^(-q/10)
  const T* dmatch;  // [128] 1 - ph2pr[q]          (prior on match)
  const T* dmis;    // [128] ph2pr[q] / 3          (prior on mismatch)
  const T* mm;      // [kMmEntries] matchToMatch(max,min) for quals 0..127
  T init_const;     // 2^120 (float) / 2^1020 (double)
  T log10_init;     // log10f(2^120) / log10(2^1020), host libm
};
constexpr int kMmEntries = (127 * 128) / 2 + 128;  // index (mx*(mx+1))/2 + mn, mx <= 127

// Raw device-side view of an fcs_phmm_batch.
struct PhmmDevBatch {
  const uint8_t *rb, *bq, *iq, *dq, *gq;
  const int64_t* read_off;
  const int32_t* read_len;
  const uint8_t* hb;
  const int64_t* hap_off;
  const int32_t* hap_len;
  const int32_t* pair_read;
  const int32_t* pair_hap;
  int64_t n_pairs;
};

// Per-device state shared by all calls (tables).
struct DeviceTables {
  bool ready = false;
  float* f_tabs = nullptr;   // ph2pr | dmatch | dmis | mm
  double* d_tabs = nullptr;
  PhmmTables<float> tf;
  PhmmTables<double> td;
};
int get_device_tables(int device, DeviceTables** out);

// Host table builder (fcship_tables.cpp).
void build_phmm_tables_f(float* ph2pr, float* dmatch, float* dmis, float* mm);
void build_phmm_tables_d(double* ph2pr, double* dmatch, double* dmis, double* mm);

// ------------------------------------------------------------ stream fork/join
// fs[0] = s itself; fs[1..] are per-(thread, device) side streams that wait
// for everything already queued on s.  join_streams makes s wait for them.
// Both are pure stream-ordered event operations (no host sync), so they also
// work inside a hipGraph stream capture.
constexpr int kForkStreams = 4;
int fork_streams(hipStream_t s, hipStream_t (&fs)[kForkStreams]);
int join_streams(hipStream_t s, const hipStream_t (&fs)[kForkStreams]);

// ------------------------------------------------------------ kernel launchers
// The bin schedule (counting sort on the key's top 12 bits): idx_out = the
// pairs in bin order, bounds = device int64[kPhmmLaunchClasses + 1] (the first
// position of each launch class, then n), counters[0..1] (the forward pass's
// rescue and fallback counts) zeroed; hist / cursor are
// uint32[1 << (kPhmmKeyBits - 4)], hist all zero on entry (left zero).
int launch_phmm_bin_schedule(const PhmmDevBatch& b, int32_t* idx_out, int64_t* bounds, unsigned long long* counters,
                             uint32_t* hist, uint32_t* cursor, hipStream_t s);
// fb_list / fb_count: pairs the streamed kernel hands back (haplotype bytes
// outside A/C/G/T/N), recomputed by the one-row kernel within this call.
int launch_phmm_forward(const PhmmDevBatch& b, const int32_t* order, int64_t count, int max_hap_len,
                        const int64_t* bounds, const DeviceTables& t, bool exact, double* out, int32_t* rescue_list,
                        unsigned long long* rescue_count, float thr, bool use_rescue, int32_t* fb_list,
                        unsigned long long* fb_count, hipStream_t s);
int launch_phmm_rescue(const PhmmDevBatch& b, const int32_t* list, const unsigned long long* count_dev,
                       int64_t max_count, int max_hap_len, const DeviceTables& t, bool exact, double* out,
                       hipStream_t s);

struct BswDevBatch {
  const uint8_t* qbuf;
  const int64_t* qoff;
  const int32_t* qlen;
  const uint8_t* tbuf;
  const int64_t* toff;
  const int32_t* tlen;
  const int32_t* h0;
  const int32_t* w;
  int64_t n;
};
struct BswParams {
  int8_t mat[25];
  int32_t o_del, e_del, o_ins, e_ins, end_bonus, zdrop;
  int32_t max_mat;
  int32_t matpack[5];  // row t: mat[t*5+q] as signed 5-bit fields at bit 5*q
  int32_t lane_ok;     // every mat entry fits a signed 5-bit field
  // two-tasks-per-lane kernel (bsw_pair.h): A/C/G/T scores biased to >= 0
  int32_t pair_ok;     // the biased A/C/G/T block fits a byte
  int32_t pair_bias;   // -min(0, min mat[t][q]), t < 5, q < 4
  int32_t pair_cg;     // max mat[t][q] (t < 5, q < 4) + pair_bias + 1
  int32_t pair_k256, pair_one;  // 0x01000100, 0x00010001: runtime constants (see bsw_pair.h pk_mad / pk_nz)
};
// SW schedule buckets: 0..9 lane-per-task kernels (bsw_lane.hip), 10..14
// two-tasks-per-lane kernels (bsw_pair.h), 15 = wave-per-task.
constexpr int kBswPairBucket0 = 10;
constexpr int kBswWideBucket = 15;
// Device scratch of one SW launch sequence (sort keys, schedule, bucket bounds).
struct BswWorkspace {
  int64_t cap = 0;
  uint32_t* keys_in = nullptr;
  uint32_t* keys_out = nullptr;
  int32_t* idx_in = nullptr;
  int32_t* idx_out = nullptr;
  int64_t* bounds = nullptr;  // [kBswWideBucket + 2]
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
};
// Stable radix sort of (key, index) pairs over key bits [0, end_bit).
hipError_t sort_pairs_u32(void* tmp, size_t& bytes, const uint32_t* kin, uint32_t* kout, const int32_t* vin,
                          int32_t* vout, int n, hipStream_t s, int end_bit = 32);
// SW schedule keys: bucket in bits [20, 24), below it the in-bucket order.
constexpr int kBswKeyBucketShift = 20;
constexpr int kBswKeyBits = 24;
// PairHMM schedule keys: launch class in bits [12, 16).  Launch classes
// 0 .. kLongClasses-1 run the row-streamed fp32 kernel (phmm_stream.h) on
// haplotypes longer than the column-blocked kernel takes, the next
// kColsLaunch the column-blocked kernel (phmm_cols.h), the last kPhmmClasses
// the grouped kernels (phmm2.h / phmm_kernel), each range longest first.
// PairHMM sort keys: 16 bits (two 8-bit radix passes; the in-class order keys
// hap length only: 24-bit keys that also ordered stream classes by read length
// measured slower).
constexpr int kPhmmKeyClassShift = 12;
constexpr int kPhmmKeyBits = 16;
constexpr int kStreamClasses = 4;
constexpr int kPhmmClasses = 6;
constexpr int kLongClasses = 2;  // phmm3 stream classes 3 and 2 (H <= 3700, <= 472)
constexpr int kColsLaunch = 8;   // phmm_cols.h classes (H <= 303, <= 271, .., <= 175)
constexpr int kPhmmLaunchClasses = kLongClasses + kColsLaunch + kPhmmClasses;
// Sorted schedule: one launch over the lane (0..9) and pair (kBswPairBucket0..+4)
// buckets, then the wave-per-task kernel over kBswWideBucket.
int launch_bsw_extend_sorted(const BswDevBatch& b, const BswParams& p, int max_qlen, int max_tlen, int32_t* res,
                             int64_t* cells, const BswWorkspace& ws, hipStream_t s);
// Wave-per-task kernel over sorted positions [bounds[kBswWideBucket], bounds[kBswWideBucket + 1]).
int launch_bsw_extend_wide(const BswDevBatch& b, const BswParams& p, int max_qlen, int max_tlen, int32_t* res,
                           int64_t* cells, const int32_t* order, const int64_t* bounds, hipStream_t s);
// all_u8: the caller knows every xtra has KSW_XBYTE (skips the 32-bit 16-lane launch)
int launch_bsw_align(const BswDevBatch& b, const BswParams& p, const int32_t* xtra, int max_qlen, int max_tlen,
                     int32_t* out, hipStream_t s, bool all_u8);
int launch_bsw_global(const BswDevBatch& b, const BswParams& p, int max_qlen, int max_tlen, int32_t* scores,
                      uint8_t* zbuf, int64_t zbytes, const int64_t* zoff, uint32_t* cigar, const int64_t* cigar_off,
                      const int32_t* cigar_cap, int32_t* n_cigar, hipStream_t s);
// One wave per BGZF member (bgzf_kernels.hip); coff / uoff have n + 1 entries.
int launch_bgzf_inflate(const uint8_t* comp, const int64_t* coff, const int64_t* uoff, int32_t n, uint8_t* out,
                        int32_t* status, hipStream_t s);

}  // namespace fcs

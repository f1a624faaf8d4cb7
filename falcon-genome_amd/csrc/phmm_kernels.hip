// PairHMM forward algorithm on gfx950 (CDNA4), fp32 pass + fp64 rescue.
//
// Algorithm: GATK/GKL PairHMM (GKL compute_full_prob,
// reached from /root/reference/src/workers/HTCWorker.cpp:51-85 and
// /root/reference/src/workers/Mutect2Worker.cpp:113-120).
//
// Mapping:
//   * one 64-lane wave processes FOUR independent (read, hap) pairs, one per
//     16-lane DPP row ("segment");
//   * inside a segment, lane l owns read row 16*s + l of stripe s and the
//     segment sweeps anti-diagonals: at step t lane l computes column t - l;
//   * the up-neighbour values (row r-1) arrive by DPP row_shr:1 from lane l-1;
//     lane 0 of the segment gets them from the segment's LDS boundary ring,
//     which lane 15 filled with the previous stripe's last row (and which holds
//     row 0 = {M=0, I=0, D=INITIAL_CONSTANT/H} plus the hap bases for stripe 0);
//     the DPP `old` operand delivers the LDS value to lane 0 for free;
//   * the diagonal values (r-1, c-1) are the previous step's up values and the
//     left values (r, c-1) are the lane's own previous outputs, so a cell costs
//     four DPP moves, one select for the emission prior and 8 FP ops;
//   * idle cells (c <= 0) compute exact zeros by construction, so no per-step
//     predicates are needed; the lane holding the last read row sums M and I
//     in column order like GKL's vector kernel.
// The file is compiled with -ffp-contract=off: the EXACT variant evaluates GKL's
// operation order bit-for-bit, the fast variant uses explicit fma().
#include <hip/hip_runtime.h>

#include "fcship_internal.h"

namespace fcs {

template <typename T> struct alignas(16) PhSlot;
template <> struct alignas(16) PhSlot<float> {
  float M, I, D;
  int hb;
};
template <> struct alignas(16) PhSlot<double> {
  double M, I, D;
  int hb;
  int pad;
};

__device__ __forceinline__ float fma_t(float a, float b, float c) { return fmaf(a, b, c); }
__device__ __forceinline__ double fma_t(double a, double b, double c) { return fma(a, b, c); }

// One stripe of one segment: steps 0..tend.  buf points at the segment's
// boundary ring, slot index = column + 16.
template <typename T, bool EXACT, bool SUM>
__device__ __forceinline__ void phmm_stripe(PhSlot<T>* __restrict__ buf, const int sl, const int tend, const T e1,
                                            const T e3, const T mm, const T gm, const T mx, const T xx, const T my,
                                            const T yy, const int rbase, const int lim, T& accM, T& accI) {
  T Mo = 0, Io = 0, Do = 0, Mp = 0, Ip = 0, Dp = 0;
  int ho = 0;
  PhSlot<T> nx = buf[16];
#pragma unroll 2
  for (int t = 0; t <= tend; ++t) {
    const PhSlot<T> cur = nx;
    nx = buf[t + 17];
    const T Mu = dpp_row_shr1<T>(cur.M, Mo);
    const T Iu = dpp_row_shr1<T>(cur.I, Io);
    const T Du = dpp_row_shr1<T>(cur.D, Do);
    const int hu = dpp_row_shr1_i(cur.hb, ho);
    const T prior = (hu == rbase || hu == 'N') ? e1 : e3;
    T Mn, In, Dn;
    if constexpr (EXACT) {
      Mn = ((Mp * mm + Ip * gm) + Dp * gm) * prior;
      In = Mu * mx + Iu * xx;
      Dn = Mo * my + Do * yy;
    } else {
      Mn = prior * fma_t(Mp, mm, fma_t(Ip, gm, Dp * gm));
      In = fma_t(Mu, mx, Iu * xx);
      Dn = fma_t(Mo, my, Do * yy);
    }
    if (sl == 15) {
      PhSlot<T> o;
      o.M = Mn;
      o.I = In;
      o.D = Dn;
      o.hb = hu;
      buf[t + 1] = o;
    }
    if constexpr (SUM) {
      if (t <= lim) {
        accM += Mn;
        accI += In;
      }
    }
    Mp = Mu;
    Ip = Iu;
    Dp = Du;
    Mo = Mn;
    Io = In;
    Do = Dn;
    ho = hu;
  }
}

template <typename T>
__device__ __forceinline__ void load_row(const PhmmDevBatch& b, const PhmmTables<T>& tab, bool valid, int64_t pos,
                                         T& e1, T& e3, T& mm, T& gm, T& mx, T& xx, T& my, T& yy, int& rbase) {
  e1 = e3 = mm = gm = mx = xx = my = yy = (T)0;
  rbase = -1;
  if (valid) {
    rbase = b.rb[pos];
    const int q = b.bq[pos] & 127, qi = b.iq[pos] & 127, qd = b.dq[pos] & 127, qc = b.gq[pos] & 127;
    e1 = tab.dmatch[q];
    e3 = (rbase == 'N') ? e1 : tab.dmis[q];
    const int hi = qi > qd ? qi : qd, lo = qi > qd ? qd : qi;
    mm = tab.mm[((hi * (hi + 1)) >> 1) + lo];
    gm = tab.dmatch[qc];
    mx = tab.ph2pr[qi];
    xx = tab.ph2pr[qc];
    my = tab.ph2pr[qd];
    yy = tab.ph2pr[qc];
  }
}

// FINAL_DOUBLE=false: fp32 pass (rescue queueing); true: fp64 pass.
template <typename T, bool EXACT, bool RESCUE_PASS>
__global__ __launch_bounds__(64) void phmm_kernel(const PhmmDevBatch b, const int32_t* __restrict__ order,
                                                  const unsigned long long* __restrict__ count_dev,
                                                  long long count_host, const int nslot, const PhmmTables<T> tab,
                                                  double* __restrict__ out, int32_t* __restrict__ rescue_list,
                                                  unsigned long long* __restrict__ rescue_count, const float thr,
                                                  const int use_rescue) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  PhSlot<T>* const slots = reinterpret_cast<PhSlot<T>*>(smem_raw);
  const int lane = threadIdx.x;
  const int seg = lane >> 4;
  const int sl = lane & 15;
  PhSlot<T>* const buf = slots + seg * nslot;
  const long long count = count_dev ? (long long)(*count_dev) : count_host;
  const long long ngroups = (count + 3) >> 2;

  for (long long g = blockIdx.x; g < ngroups; g += gridDim.x) {
    const long long idx = g * 4 + seg;
    const int p = (idx < count) ? order[idx] : -1;
    int R = 0, H = 0;
    int64_t ro = 0, ho = 0;
    if (p >= 0) {
      const int ri = b.pair_read[p], hi = b.pair_hap[p];
      R = b.read_len[ri];
      H = b.hap_len[hi];
      ro = b.read_off[ri];
      ho = b.hap_off[hi];
    }
    const bool active = (p >= 0) && R > 0 && H > 0;
    if (p >= 0 && !active && sl == 0) out[p] = -INFINITY;
    const int nstr = active ? (R + 15) >> 4 : 0;
    const int Hmax = wave_max(active ? H : 0);
    const int nstr_max = wave_max(nstr);
    if (nstr_max == 0) continue;

    // Boundary ring <- row 0: M = I = 0, D = INITIAL_CONSTANT / H for c in [0, H],
    // hap base of column c (1-based) in .hb.
    const T init = active ? tab.init_const / (T)H : (T)0;
    __syncthreads();
    for (int s = sl; s < nslot; s += 16) {
      const int c = s - 16;
      PhSlot<T> v{};
      v.M = 0;
      v.I = 0;
      v.D = (active && c >= 0 && c <= H) ? init : (T)0;
      v.hb = (active && c >= 1 && c <= H) ? (int)b.hb[ho + c - 1] : 0;
      buf[s] = v;
    }
    __syncthreads();

    // Row parameters of stripe 0; the next stripe's are loaded one stripe ahead.
    T e1, e3, mm, gm, mx, xx, my, yy;
    int rbase;
    load_row<T>(b, tab, active && sl < R, ro + sl, e1, e3, mm, gm, mx, xx, my, yy, rbase);
    T accM = 0, accI = 0;
    const int sum_stripe = active ? (R - 1) >> 4 : -1;
    const int sum_lane = active ? (R - 1) & 15 : -1;
    for (int st = 0; st < nstr_max; ++st) {
      const int nrow = (st + 1) * 16 + sl;
      T n_e1, n_e3, n_mm, n_gm, n_mx, n_xx, n_my, n_yy;
      int n_rbase;
      load_row<T>(b, tab, active && nrow < R, ro + nrow, n_e1, n_e3, n_mm, n_gm, n_mx, n_xx, n_my, n_yy, n_rbase);

      const bool seg_sums = (st == sum_stripe);
      const int any_sum = wave_max(seg_sums ? 1 : 0);
      if (any_sum) {
        // Do all live segments finish here?  Then stop at the last summing column.
        const int cont = wave_max((active && nstr > st + 1) ? 1 : 0);
        const int lim = (seg_sums && sl == sum_lane) ? sl + H : -1;
        const int tend = cont ? Hmax + 15 : wave_max(seg_sums ? sum_lane + H : 0);
        phmm_stripe<T, EXACT, true>(buf, sl, tend, e1, e3, mm, gm, mx, xx, my, yy, rbase, lim, accM, accI);
        if (seg_sums && sl == sum_lane) {
          const T sum = accM + accI;
          if constexpr (RESCUE_PASS) {
            out[p] = log10(sum) - (double)tab.log10_init;
          } else {
            if (use_rescue && sum < (T)thr) {
              const unsigned long long k = atomicAdd(rescue_count, 1ull);
              rescue_list[k] = p;
              out[p] = __builtin_nan("");
            } else {
              out[p] = (double)(log10f((float)sum) - (float)tab.log10_init);
            }
          }
        }
      } else {
        phmm_stripe<T, EXACT, false>(buf, sl, Hmax + 15, e1, e3, mm, gm, mx, xx, my, yy, rbase, -1, accM, accI);
      }
      e1 = n_e1;
      e3 = n_e3;
      mm = n_mm;
      gm = n_gm;
      mx = n_mx;
      xx = n_xx;
      my = n_my;
      yy = n_yy;
      rbase = n_rbase;
    }
  }
}

// Sort keys: descending (stripe count, hap length) -> ascending key order.
__global__ void phmm_keys_kernel(const PhmmDevBatch b, uint32_t* __restrict__ keys, int32_t* __restrict__ idx) {
  const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= b.n_pairs) return;
  const int R = b.read_len[b.pair_read[p]];
  const int H = b.hap_len[b.pair_hap[p]];
  const uint32_t ns = (uint32_t)min((R + 15) >> 4, 0xFFFF);
  const uint32_t hh = (uint32_t)min(max(H, 0), 0xFFFF);
  keys[p] = ((0xFFFFu - ns) << 16) | (0xFFFFu - hh);
  idx[p] = (int32_t)p;
}

static int nslot_for(int max_hap_len) {
  // >= Hmax + 33 slots; slot count = 4 (mod 16) so the four segment rings start
  // on different LDS bank groups (ds_read_b128 lane groups mix segments).
  int n = ((max_hap_len + 33 + 15) / 16) * 16 + 4;
  return n;
}

int launch_phmm_keys(const PhmmDevBatch& b, uint32_t* keys, int32_t* idx, hipStream_t s) {
  if (b.n_pairs <= 0) return FCS_OK;
  const int bs = 256;
  const long long nb = (b.n_pairs + bs - 1) / bs;
  hipLaunchKernelGGL(phmm_keys_kernel, dim3((unsigned)nb), dim3(bs), 0, s, b, keys, idx);
  FCS_HIP_CHECK(hipGetLastError());
  return FCS_OK;
}

template <typename T, bool EXACT, bool RESCUE>
static int launch_one(const PhmmDevBatch& b, const int32_t* order, const unsigned long long* count_dev,
                      long long count_host, long long max_groups, int max_hap_len, const PhmmTables<T>& tab,
                      double* out, int32_t* rescue_list, unsigned long long* rescue_count, float thr,
                      bool use_rescue, hipStream_t s) {
  const int nslot = nslot_for(max_hap_len);
  const size_t lds = (size_t)4 * nslot * sizeof(PhSlot<T>);
  if (lds > 160 * 1024)
    return fail(FCS_ERR_UNSUPPORTED, "[E::fcship] max_hap_len too large for the LDS boundary ring");
  auto kern = phmm_kernel<T, EXACT, RESCUE>;
  if (lds > 64 * 1024) FCS_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  long long grid = max_groups;
  const long long cap = 256LL * 64;  // grid-stride beyond this
  if (grid > cap) grid = cap;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(64), lds, s, b, order, count_dev, count_host, nslot, tab, out,
                     rescue_list, rescue_count, thr, use_rescue ? 1 : 0);
  FCS_HIP_CHECK(hipGetLastError());
  return FCS_OK;
}

int launch_phmm_forward(const PhmmDevBatch& b, const int32_t* order, int64_t count, int max_hap_len,
                        const DeviceTables& t, bool exact, double* out, int32_t* rescue_list,
                        unsigned long long* rescue_count, float thr, bool use_rescue, hipStream_t s) {
  if (count <= 0) return FCS_OK;
  const long long groups = (count + 3) / 4;
  if (exact)
    return launch_one<float, true, false>(b, order, nullptr, count, groups, max_hap_len, t.tf, out, rescue_list,
                                          rescue_count, thr, use_rescue, s);
  return launch_one<float, false, false>(b, order, nullptr, count, groups, max_hap_len, t.tf, out, rescue_list,
                                         rescue_count, thr, use_rescue, s);
}

int launch_phmm_rescue(const PhmmDevBatch& b, const int32_t* list, const unsigned long long* count_dev,
                       int64_t max_count, int max_hap_len, const DeviceTables& t, bool exact, double* out,
                       hipStream_t s) {
  if (max_count <= 0) return FCS_OK;
  // The rescued subset is usually tiny: a modest grid that strides over the
  // device-side count, so no host round trip is needed.
  long long groups = (max_count + 3) / 4;
  if (groups > 2048) groups = 2048;
  if (exact)
    return launch_one<double, true, true>(b, list, count_dev, 0, groups, max_hap_len, t.td, out, nullptr, nullptr,
                                          0.f, false, s);
  return launch_one<double, false, true>(b, list, count_dev, 0, groups, max_hap_len, t.td, out, nullptr, nullptr, 0.f,
                                         false, s);
}

}  // namespace fcs

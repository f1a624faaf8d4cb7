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
//   * up-neighbour values (row r-1, same column) arrive by DPP row_shr:1 from
//     lane l-1; lane 0 gets them through the DPP `old` operand from the
//     segment's LDS boundary ring, which lane 15 filled with the previous
//     stripe's last row (M, I: 8 bytes per column).  D of that row is not
//     stored: lane 0 re-derives it from the M stream with the same operation
//     lane 15 used, so it is bit-identical;
//   * diagonal values (r-1, c-1) are the previous step's up values and left
//     values (r, c-1) the lane's own previous outputs;
//   * the hap base of column t reaches lane 0 by DPP row_newbcast from a
//     register that holds 16 consecutive hap bytes (one LDS read per 16 steps),
//     and moves down the segment with the M/I/D values;
//   * idle cells (c <= 0) compute exact zeros by construction, so the step has
//     no predicates; the lane holding the read's last row sums M and I in
//     column order like GKL's vector kernel.
// Steps are unrolled in blocks of 16 (the DPP broadcast lane is an immediate),
// the ring is read four steps ahead and the next stripe's row parameters are
// gathered while the current stripe runs.
// Compiled with -ffp-contract=off: the EXACT variant keeps GKL's operation
// order bit-for-bit, the fast variant uses explicit fma().
#include <hip/hip_runtime.h>

#include <utility>

#include "fcship_internal.h"

namespace fcs {

template <typename T> struct alignas(2 * sizeof(T)) PhRing {
  T M, I;
};

__device__ __forceinline__ float fma_t(float a, float b, float c) { return fmaf(a, b, c); }
__device__ __forceinline__ double fma_t(double a, double b, double c) { return fma(a, b, c); }

// Lane S of each 16-lane row broadcast to its row (gfx90a+ DPP row_newbcast).
template <int S> __device__ __forceinline__ int row_bcast_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, 0x150 + S, 0xF, 0xF, false);
}
template <int S> __device__ __forceinline__ float row_bcast(float v) { return __int_as_float(row_bcast_i<S>(__float_as_int(v))); }
template <int S> __device__ __forceinline__ double row_bcast(double v) {
  const long long x = __double_as_longlong(v);
  const int lo = row_bcast_i<S>((int)x), hi = row_bcast_i<S>((int)(x >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

template <typename T>
struct RowP {
  T e1, e3, mm, gm, mx, xx, my, yy;
  int rbase;
};

template <typename T>
struct LaneState {
  T Mo, Io, Do;  // own outputs of the previous step: cell (r, c-1)
  T Mp, Ip, Dp;  // up values of the previous step:   cell (r-1, c-1)
  T Mq, Dq;      // boundary-row stream seen by lane 0: M, D of (r-1, c-1)
  int ho;        // hap base of the previous step's column
};

// One anti-diagonal step at t = t0 + S.
template <typename T, bool EXACT, bool SUM, int S>
__device__ __forceinline__ void phmm_step(LaneState<T>& L, PhRing<T> (&pf)[4], const int Q, const RowP<T>& p,
                                          const T myp, const T yyp, PhRing<T>* __restrict__ ring, const int t0,
                                          const bool top, const int lim, T& accM, T& accI) {
  const int t = t0 + S;
  const PhRing<T> cur = pf[S & 3];
  pf[S & 3] = ring[t + 20];  // column t + 4, four steps ahead
  T dq;
  if constexpr (EXACT) dq = L.Mq * myp + L.Dq * yyp;
  else dq = fma_t(L.Mq, myp, L.Dq * yyp);
  L.Mq = cur.M;
  L.Dq = dq;
  const int hb0 = row_bcast_i<S>(Q);
  const T Mu = dpp_row_shr1<T>(cur.M, L.Mo);
  const T Iu = dpp_row_shr1<T>(cur.I, L.Io);
  const T Du = dpp_row_shr1<T>(dq, L.Do);
  const int hu = dpp_row_shr1_i(hb0, L.ho);
  const T prior = (hu == p.rbase || hu == 'N') ? p.e1 : p.e3;
  T Mn, In, Dn;
  if constexpr (EXACT) {
    Mn = ((L.Mp * p.mm + L.Ip * p.gm) + L.Dp * p.gm) * prior;
    In = Mu * p.mx + Iu * p.xx;
    Dn = L.Mo * p.my + L.Do * p.yy;
  } else {
    Mn = prior * fma_t(L.Mp, p.mm, fma_t(L.Ip, p.gm, L.Dp * p.gm));
    In = fma_t(Mu, p.mx, Iu * p.xx);
    Dn = fma_t(L.Mo, p.my, L.Do * p.yy);
  }
  if (top) {
    PhRing<T> o;
    o.M = Mn;
    o.I = In;
    ring[t + 1] = o;  // column t - 15
  }
  if constexpr (SUM) {
    if (t <= lim) {
      accM += Mn;
      accI += In;
    }
  }
  L.Mp = Mu;
  L.Ip = Iu;
  L.Dp = Du;
  L.Mo = Mn;
  L.Io = In;
  L.Do = Dn;
  L.ho = hu;
}

template <typename T, bool EXACT, bool SUM>
__device__ __forceinline__ void phmm_block(LaneState<T>& L, PhRing<T> (&pf)[4], const int Q, const RowP<T>& p,
                                           const T myp, const T yyp, PhRing<T>* __restrict__ ring, const int t0,
                                           const bool top, const int lim, T& accM, T& accI) {
  [&]<int... S>(std::integer_sequence<int, S...>) {
    (phmm_step<T, EXACT, SUM, S>(L, pf, Q, p, myp, yyp, ring, t0, top, lim, accM, accI), ...);
  }(std::make_integer_sequence<int, 16>{});
}

struct RawRow {
  int rb, bq, iq, dq, gq;
};

__device__ __forceinline__ RawRow load_raw(const PhmmDevBatch& b, bool valid, int64_t pos) {
  RawRow r{-1, 0, 0, 0, 0};
  if (valid) {
    r.rb = b.rb[pos];
    r.bq = b.bq[pos];
    r.iq = b.iq[pos];
    r.dq = b.dq[pos];
    r.gq = b.gq[pos];
  }
  return r;
}

template <typename T>
__device__ __forceinline__ RowP<T> row_params(const PhmmTables<T>& tab, const RawRow& r) {
  RowP<T> p;
  if (r.rb < 0) {
    p.e1 = p.e3 = p.mm = p.gm = p.mx = p.xx = p.my = p.yy = (T)0;
    p.rbase = -1;
    return p;
  }
  const int q = r.bq & 127, qi = r.iq & 127, qd = r.dq & 127, qc = r.gq & 127;
  p.rbase = r.rb;
  p.e1 = tab.dmatch[q];
  p.e3 = (r.rb == 'N') ? p.e1 : tab.dmis[q];
  const int hi = qi > qd ? qi : qd, lo = qi > qd ? qd : qi;
  p.mm = tab.mm[((hi * (hi + 1)) >> 1) + lo];
  p.gm = tab.dmatch[qc];
  p.mx = tab.ph2pr[qi];
  p.xx = tab.ph2pr[qc];
  p.my = tab.ph2pr[qd];
  p.yy = tab.ph2pr[qc];
  return p;
}

// Runs one stripe: nblk blocks of 16 steps; the next stripe's parameters are
// gathered after the first block (their bytes were requested at stripe start).
template <typename T, bool EXACT, bool SUM>
__device__ __forceinline__ void phmm_stripe(LaneState<T>& L, const RowP<T>& p, const T myp, const T yyp,
                                            PhRing<T>* __restrict__ ring, const unsigned char* __restrict__ hapl,
                                            const int sl, const int nblk, const int lim, T& accM, T& accI,
                                            const PhmmTables<T>& tab, const RawRow& nraw, RowP<T>& np) {
  const bool top = sl == 15;
  PhRing<T> pf[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) pf[k] = ring[16 + k];
  int Q = hapl[sl];
  int Qn = hapl[16 + sl];
  phmm_block<T, EXACT, SUM>(L, pf, Q, p, myp, yyp, ring, 0, top, lim, accM, accI);
  np = row_params<T>(tab, nraw);
  for (int blk = 1; blk < nblk; ++blk) {
    Q = Qn;
    Qn = hapl[16 * (blk + 1) + sl];
    phmm_block<T, EXACT, SUM>(L, pf, Q, p, myp, yyp, ring, 16 * blk, top, lim, accM, accI);
  }
}

template <typename T, bool EXACT, bool RESCUE_PASS>
__global__ __launch_bounds__(64) void phmm_kernel(const PhmmDevBatch b, const int32_t* __restrict__ order,
                                                  const unsigned long long* __restrict__ count_dev,
                                                  long long count_host, const int nslot, const int nhap,
                                                  const PhmmTables<T> tab, double* __restrict__ out,
                                                  int32_t* __restrict__ rescue_list,
                                                  unsigned long long* __restrict__ rescue_count, const float thr,
                                                  const int use_rescue) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  const int lane = threadIdx.x;
  const int seg = lane >> 4;
  const int sl = lane & 15;
  PhRing<T>* const ring = reinterpret_cast<PhRing<T>*>(smem_raw) + seg * nslot;
  unsigned char* const hapl = smem_raw + (size_t)4 * nslot * sizeof(PhRing<T>) + seg * nhap;
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

    // Boundary ring <- row 0 (M = I = 0; its D = INITIAL_CONSTANT / H is
    // injected through lane 0's D stream) and the hap bytes by column.
    __syncthreads();
    for (int s = sl; s < nslot; s += 16) {
      PhRing<T> v;
      v.M = 0;
      v.I = 0;
      ring[s] = v;
    }
    for (int c = sl; c < nhap; c += 16)
      hapl[c] = (active && c >= 1 && c <= H) ? b.hb[ho + c - 1] : (unsigned char)0;
    __syncthreads();

    const T init = active ? tab.init_const / (T)H : (T)0;
    RowP<T> prm = row_params<T>(tab, load_raw(b, active && sl < R, ro + sl));
    T accM = 0, accI = 0;
    const int sum_stripe = active ? (R - 1) >> 4 : -1;
    const int sum_lane = active ? (R - 1) & 15 : -1;
    T myp = 0, yyp = 1;  // row 0: D(0, c) = init for every c
    for (int st = 0; st < nstr_max; ++st) {
      const int nrow = (st + 1) * 16 + sl;
      const RawRow nraw = load_raw(b, active && nrow < R, ro + nrow);
      RowP<T> nprm;
      LaneState<T> L;
      L.Mo = L.Io = L.Do = L.Mp = L.Ip = L.Dp = L.Mq = (T)0;
      L.Dq = (st == 0) ? init : (T)0;
      L.ho = 0;
      const bool seg_sums = (st == sum_stripe);
      const int any_sum = wave_max(seg_sums ? 1 : 0);
      if (any_sum) {
        // If no live segment continues past this stripe, stop after the last summed column.
        const int cont = wave_max((active && nstr > st + 1) ? 1 : 0);
        const int lim = (seg_sums && sl == sum_lane) ? sl + H : -1;
        const int tend = cont ? Hmax + 15 : wave_max(seg_sums ? sum_lane + H : 0);
        phmm_stripe<T, EXACT, true>(L, prm, myp, yyp, ring, hapl, sl, (tend + 16) >> 4, lim, accM, accI, tab, nraw,
                                    nprm);
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
        phmm_stripe<T, EXACT, false>(L, prm, myp, yyp, ring, hapl, sl, (Hmax + 31) >> 4, -1, accM, accI, tab, nraw,
                                     nprm);
      }
      // lane 0 of the next stripe derives D of this stripe's last row (lane 15)
      myp = row_bcast<15>(prm.my);
      yyp = row_bcast<15>(prm.yy);
      prm = nprm;
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

// Ring slots = column + 16 for columns -16 .. Hmax + 34 (block round-up plus
// the four-step read-ahead); hap bytes by column 0 .. 16 * (blocks + 1).
static int nslot_for(int max_hap_len) { return ((max_hap_len + 51 + 15) / 16) * 16; }
static int nhap_for(int max_hap_len) { return ((max_hap_len + 15 + 16) / 16 + 1) * 16; }

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
  const int nhap = nhap_for(max_hap_len);
  const size_t lds = (size_t)4 * nslot * sizeof(PhRing<T>) + (size_t)4 * nhap;
  if (lds > 160 * 1024)
    return fail(FCS_ERR_UNSUPPORTED, "[E::fcship] max_hap_len too large for the LDS boundary ring");
  auto kern = phmm_kernel<T, EXACT, RESCUE>;
  if (lds > 64 * 1024)
    FCS_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  long long grid = max_groups;
  const long long cap = 256LL * 64;  // grid-stride beyond this
  if (grid > cap) grid = cap;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(64), lds, s, b, order, count_dev, count_host, nslot, nhap, tab,
                     out, rescue_list, rescue_count, thr, use_rescue ? 1 : 0);
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

// PairHMM forward algorithm on gfx950 (CDNA4), fp32 pass + fp64 rescue.
//
// Algorithm: GATK/GKL PairHMM (GKL compute_full_prob,
// reached from /root/reference/src/workers/HTCWorker.cpp:51-85 and
// /root/reference/src/workers/Mutect2Worker.cpp:113-120).
//
// Mapping:
//   * one 64-lane wave processes FOUR independent (read, hap) pairs, one per
//     16-lane DPP row ("segment");
//   * inside a segment, lane l owns read row r = 16*s + l + 1 of stripe s and
//     the segment sweeps anti-diagonals: at step t lane l computes column
//     c = t - l;
//   * every lane also holds the transition parameters of row r + 1 and hands
//     the lane below two finished values per column: the diagonal sum
//     X(r, c) = (M*mm' + I*gm') + D*gm'  (GKL's order) and I(r+1, c).  The lane
//     below therefore computes M = prior * X and takes I as is, so a cell costs
//     two DPP row_shr:1 moves, one select for the emission prior and
//     1 + 2 + 3 + 2 FP ops (M, own D, X for below, I for below);
//   * lane 0 of a segment receives the same two values through the DPP `old`
//     operand from the segment's LDS boundary ring, which lane 15 filled during
//     the previous stripe (8 bytes per column); stripe 0 reads the ring
//     initialised with row 0 (X = (2^120/H)*gm_1, I = 0);
//   * each lane reads its hap base for column t - l from an LDS byte array
//     (LDS pipe, two steps ahead) instead of passing it between lanes;
//   * idle cells (c <= 0) compute exact zeros by construction, so a step has
//     no predicates; the lane holding the read's last row sums M and I in
//     column order like GKL's vector kernel.
// Steps are unrolled in blocks of 16, the ring is read two steps ahead and the
// next stripe's row parameters are gathered while the current stripe runs.
// Compiled with -ffp-contract=off: the EXACT variant keeps GKL's operation
// order bit-for-bit, the fast variant uses explicit fma().
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include <utility>

#include "fcship_internal.h"

namespace fcs {

// Ring / hap read-ahead in steps.  Two steps hide the LDS latency (one does
// not: -8%) and, as a shift register, let every ring read land in the register
// its DPP `old` operand needs: the four-deep rotation cost two v_mov per step
// and spilled 2 VGPRs; 2, 3 and 4 measured within 0.5% (gpurun_out/abp2).
constexpr int PFD = 2;
template <typename T> struct alignas(2 * sizeof(T)) PhRing {
  T X, I;
};

__device__ __forceinline__ float fma_t(float a, float b, float c) { return fmaf(a, b, c); }
__device__ __forceinline__ double fma_t(double a, double b, double c) { return fma(a, b, c); }

__device__ __forceinline__ unsigned char base_code(unsigned char b) {
  return b == 'A' ? 0 : b == 'C' ? 1 : b == 'G' ? 2 : b == 'T' ? 3 : b == 'N' ? 4 : 5;
}
__device__ __forceinline__ int base_mask(int rb) {
  const int c = base_code((unsigned char)rb);
  // N matches every hap code; a byte outside A/C/G/T/N equals no A/C/G/T hap
  // byte, so it matches only N (code 4) — bit-select groups have no code 5
  return c == 4 ? 0x7F : c == 5 ? 0x10 : (1 << c) | 0x10;
}
__device__ __forceinline__ float sel_bits(uint32_t m, float a, float b) {
  return __uint_as_float((__float_as_uint(a) & m) | (__float_as_uint(b) & ~m));
}
__device__ __forceinline__ double sel_bits(uint32_t m, double a, double b) {
  const unsigned long long mm = ((unsigned long long)m << 32) | m;
  return __longlong_as_double((long long)(((unsigned long long)__double_as_longlong(a) & mm) |
                                          ((unsigned long long)__double_as_longlong(b) & ~mm)));
}

// Hand-off to the next lane of a W-lane segment: row_shr:1 inside 16-lane DPP
// rows, wave_shr:1 over the whole wave (the fp64 rescue's one-pair waves);
// lane 0 of the segment keeps `old`.
template <typename T, int W>
__device__ __forceinline__ T dpp_shr1(T old, T src) {
  if constexpr (W == 16) {
    return dpp_row_shr1<T>(old, src);
  } else {
    static_assert(W == 64, "segments are 16 or 64 lanes");
    if constexpr (sizeof(T) == 4) {
      return __int_as_float(dpp_wave_shr1_i(__float_as_int(old), __float_as_int(src)));
    } else {
      const long long o = __double_as_longlong(old), v = __double_as_longlong(src);
      const int lo = dpp_wave_shr1_i((int)o, (int)v);
      const int hi = dpp_wave_shr1_i((int)(o >> 32), (int)(v >> 32));
      return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
    }
  }
}

// Last-row accumulation as a plain VALU add: left to the compiler, the two
// running sums get packed into v_pk_add_f32 with register moves around them.
__device__ __forceinline__ void acc_add(float& a, float x) { asm("v_add_f32 %0, %1, %2" : "=v"(a) : "v"(a), "v"(x)); }
__device__ __forceinline__ void acc_add(double& a, double x) {
  asm("v_add_f64 %0, %1, %2" : "=v"(a) : "v"(a), "v"(x));
}

template <typename T>
struct RowP {
  T e1, e3, my, yy;  // own row: emission priors, deletion transitions (my * gm of the row below unless EXACT)
  T mm, gm, mx, xx;  // row below: match/gap-to-match, insertion transitions
  int rbase;  // read base byte (byte-compare groups)
  int rmask;  // bit k set: hap code k (A,C,G,T,N = 0..4) matches this row's read base
};

template <typename T>
struct LaneState {
  T Mo, Do;  // own M, D at column c-1
  T Xp;      // X(r-1, c-1), received at the previous step
  T Xo, Io;  // what this lane sent at the previous step: X(r, c-1), I(r+1, c-1)
};

// One anti-diagonal step at t = t0 + S.
template <typename T, bool EXACT, bool SUM, bool BC, bool COND, int W, int S>
__device__ __forceinline__ void phmm_step(LaneState<T>& L, PhRing<T> (&pf)[PFD], int (&hq)[PFD],
                                          const unsigned char* __restrict__ hapl, const RowP<T>& p,
                                          PhRing<T>* __restrict__ ring, const int t0, const int sl, const bool top,
                                          const int lim, T& accM, T& accI) {
  const int t = t0 + S;
  const PhRing<T> cur = pf[0];
  const int hb = hq[0];
#pragma unroll
  for (int k = 0; k + 1 < PFD; ++k) {
    pf[k] = pf[k + 1];
    hq[k] = hq[k + 1];
  }
  pf[PFD - 1] = ring[t + W + PFD];  // lane-0 input for column t + PFD
  hq[PFD - 1] = hapl[t + W + PFD - sl];  // this lane's hap base for column t + PFD - l
  const T Xu = dpp_shr1<T, W>(cur.X, L.Xo);
  const T I = dpp_shr1<T, W>(cur.I, L.Io);
  T prior;
  if constexpr (BC) {  // group with bytes outside A/C/G/T/N: GKL's byte compare
    prior = (hb == p.rbase || hb == 'N') ? p.e1 : p.e3;
  } else {  // hap codes: one bit extract + one bit select, no compare/VCC
    prior = sel_bits((uint32_t)__builtin_amdgcn_sbfe(p.rmask, hb, 1), p.e1, p.e3);
  }
  const T M = L.Xp * prior;
  T D, Xn, In;
  if constexpr (EXACT) {
    D = L.Mo * p.my + L.Do * p.yy;
    Xn = (M * p.mm + I * p.gm) + D * p.gm;
    In = M * p.mx + I * p.xx;
  } else {
    D = fma_t(L.Mo, p.my, L.Do * p.yy);  // D' = gm * D (row_params)
    Xn = fma_t(M, p.mm, fma_t(I, p.gm, D));
    In = fma_t(M, p.mx, I * p.xx);
  }
  if (top) {
    PhRing<T> o;
    o.X = Xn;
    o.I = In;
    ring[t + 1] = o;  // column t - (W - 1)
  }
  if constexpr (SUM) {
    // The summing lane runs the last row with my = yy = 1, so its D is the
    // running sum of M over the columns to its left, in GKL's order; only I
    // needs an add.  Blocks wholly inside every summing lane's columns add
    // unconditionally (other lanes' sums are discarded); the tail block
    // compares and takes sum M = D + M at the last column.
    if constexpr (!COND) {
      acc_add(accI, I);
    } else {
      if (t <= lim) acc_add(accI, I);
      if (t == lim) accM = D + M;
    }
  }
  L.Xp = Xu;
  L.Xo = Xn;
  L.Io = In;
  L.Mo = M;
  L.Do = D;
}

template <typename T, bool EXACT, bool SUM, bool BC, bool COND, int W>
__device__ __forceinline__ void phmm_block(LaneState<T>& L, PhRing<T> (&pf)[PFD], int (&hq)[PFD],
                                           const unsigned char* __restrict__ hapl, const RowP<T>& p,
                                           PhRing<T>* __restrict__ ring, const int t0, const int sl, const bool top,
                                           const int lim, T& accM, T& accI) {
  [&]<int... S>(std::integer_sequence<int, S...>) {
    (phmm_step<T, EXACT, SUM, BC, COND, W, S>(L, pf, hq, hapl, p, ring, t0, sl, top, lim, accM, accI), ...);
  }(std::make_integer_sequence<int, 16>{});
}

struct RawRow {
  int rb, bq, dq, gq;   // own row
  int niq, ndq, ngq;    // row below
};

__device__ __forceinline__ RawRow load_raw(const PhmmDevBatch& b, int R, int64_t ro, int pos) {
  RawRow r{-1, 0, 0, 0, 0, 0, 0};
  if (pos < R) {
    const int64_t a = ro + pos;
    r.rb = b.rb[a];
    r.bq = b.bq[a];
    r.dq = b.dq[a];
    r.gq = b.gq[a];
    if (pos + 1 < R) {
      r.niq = b.iq[a + 1];
      r.ndq = b.dq[a + 1];
      r.ngq = b.gq[a + 1];
    }
  }
  return r;
}

// EXACT = false folds the row below's gap-to-match into the deletion
// recurrence: the lane carries D' = gm * D (my' = my * gm), so X = M*mm +
// I*gm + D*gm takes two FMAs instead of three.
template <typename T, bool EXACT>
__device__ __forceinline__ RowP<T> row_params(const PhmmTables<T>& tab, const RawRow& r) {
  RowP<T> p;
  p.e1 = p.e3 = p.my = p.yy = p.mm = p.gm = p.mx = p.xx = (T)0;
  p.rbase = -1;
  p.rmask = -1;
  if (r.rb < 0) return p;
  const int q = r.bq & 127, qd = r.dq & 127, qc = r.gq & 127;
  p.rbase = r.rb;
  p.rmask = base_mask(r.rb);
  p.e1 = tab.dmatch[q];
  p.e3 = (r.rb == 'N') ? p.e1 : tab.dmis[q];
  p.my = tab.ph2pr[qd];
  p.yy = tab.ph2pr[qc];
  const int ni = r.niq & 127, nd = r.ndq & 127, nc = r.ngq & 127;
  const int hi = ni > nd ? ni : nd, lo = ni > nd ? nd : ni;
  p.mm = tab.mm[((hi * (hi + 1)) >> 1) + lo];
  p.gm = tab.dmatch[nc];
  p.mx = tab.ph2pr[ni];
  p.xx = tab.ph2pr[nc];
  if constexpr (!EXACT) p.my = p.my * p.gm;
  return p;
}

// One stripe: nblk blocks of 16 steps; the next stripe's parameters are
// gathered after the first block (their bytes were requested at stripe start).
template <typename T, bool EXACT, bool SUM, bool BC, int W>
__device__ __forceinline__ void phmm_stripe(const RowP<T>& p, PhRing<T>* __restrict__ ring,
                                            const unsigned char* __restrict__ hapl, const int sl, const int nblk,
                                            const int lim, const int ulim, T& accM, T& accI,
                                            const PhmmTables<T>& tab, const RawRow& nraw, RowP<T>& np,
                                            const bool top) {
  LaneState<T> L;
  L.Mo = L.Do = L.Xp = L.Xo = L.Io = (T)0;
  PhRing<T> pf[PFD];
  int hq[PFD];
#pragma unroll
  for (int k = 0; k < PFD; ++k) {
    pf[k] = ring[W + k];
    hq[k] = hapl[W + k - sl];
  }
  // ulim: the smallest last-column step of the summing lanes (wave-uniform);
  // blocks that end before it need no compare
  if (!SUM || 15 < ulim)
    phmm_block<T, EXACT, SUM, BC, false, W>(L, pf, hq, hapl, p, ring, 0, sl, top, lim, accM, accI);
  else
    phmm_block<T, EXACT, SUM, BC, true, W>(L, pf, hq, hapl, p, ring, 0, sl, top, lim, accM, accI);
  np = row_params<T, EXACT>(tab, nraw);
  for (int blk = 1; blk < nblk; ++blk) {
    if (!SUM || 16 * blk + 15 < ulim)
      phmm_block<T, EXACT, SUM, BC, false, W>(L, pf, hq, hapl, p, ring, 16 * blk, sl, top, lim, accM, accI);
    else
      phmm_block<T, EXACT, SUM, BC, true, W>(L, pf, hq, hapl, p, ring, 16 * blk, sl, top, lim, accM, accI);
  }
}

// Per-segment ring stride in bytes.  nslot is a multiple of 16, so the four
// segments' rings start on the same LDS bank and their one-address reads /
// writes conflict 4-way (SQ_LDS_BANK_CONFLICT ~ 0.8 cycles per LDS op).  64
// bytes of padding remove 85% of the conflicts yet measured 1.3% slower on
// the C2 forward pass (profiles/r1: LDS is not the binding pipe), so none.
template <typename T>
__host__ __device__ constexpr int ring_stride(int nslot) {
  return nslot * (int)sizeof(PhRing<T>);
}

template <typename T, bool EXACT, bool RESCUE_PASS, int W = 16>
__global__ __launch_bounds__(64, (sizeof(T) == 4 && !EXACT) ? 4 : 1) void phmm_kernel(const PhmmDevBatch b, const int32_t* __restrict__ order,
                                                  const unsigned long long* __restrict__ count_dev,
                                                  long long count_host, const int64_t* __restrict__ bounds,
                                                  const int cls, const int nslot, const PhmmTables<T> tab,
                                                  double* __restrict__ out, int32_t* __restrict__ rescue_list,
                                                  unsigned long long* __restrict__ rescue_count, const float thr,
                                                  const int use_rescue, const int nseg) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  const int lane = threadIdx.x;
  const int seg = lane / W;
  const int sl = lane & (W - 1);
  // nseg = 4: four pairs per wave, one LDS ring each.  nseg = 1 (haplotypes too
  // long for four rings in 160 KB): one pair per wave, segments 1..3 idle on
  // segment 0's ring (they never write it: `top` and the setup are theirs only
  // when seg < nseg).
  const bool own_seg = seg < nseg;
  const int rseg = own_seg ? seg : 0;
  PhRing<T>* const ring = reinterpret_cast<PhRing<T>*>(smem_raw + rseg * ring_stride<T>(nslot));
  unsigned char* const hapl = smem_raw + (size_t)nseg * ring_stride<T>(nslot) + rseg * nslot;
  const bool top = own_seg && sl == W - 1;
  // forward pass: this launch's hap-length class of the sorted schedule; rescue: the device-side list count
  long long count = count_dev ? (long long)(*count_dev) : count_host;
  if (bounds) {
    order += bounds[cls];
    count = bounds[cls + 1] - bounds[cls];
  }
  const long long ngroups = (count + nseg - 1) / nseg;

  for (long long g = blockIdx.x; g < ngroups; g += gridDim.x) {
    const long long idx = g * nseg + seg;
    const int p = (own_seg && idx < count) ? order[idx] : -1;
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
    const int nstr = active ? (R + W - 1) / W : 0;
    const int Hmax = wave_max(active ? H : 0);
    const int nstr_max = wave_max(nstr);
    if (nstr_max == 0) continue;

    // Boundary ring <- row 0 as seen by row 1: X(0, c) = ((0*mm + 0*gm) + D(0,c)*gm_1)
    // = (2^120/H) * gm_1 for c in [0, H], I(1, c) = 0.  Hap bytes by column + 16.
    const T init = active ? tab.init_const / (T)H : (T)0;
    const T x0 = active ? init * tab.dmatch[b.gq[ro] & 127] : (T)0;
    __syncthreads();
    // Hap bytes go to LDS as codes A,C,G,T,N = 0..4 (6 = padding) for the
    // bit-select prior.  A hap byte outside A/C/G/T/N anywhere in the wave's
    // pairs switches the group to raw bytes and GKL's byte compare (read
    // bytes outside the set are exact on the code path: they match only N).
    // Eight slots per lane per batch: all eight byte loads are issued before
    // any is used, so a haplotype costs ~3 memory round trips, not one per slot.
    bool other = false;
    constexpr int kHB = 8;
    for (int s0 = sl; s0 < nslot; s0 += W * kHB) {
      unsigned char raw[kHB];
#pragma unroll
      for (int u = 0; u < kHB; ++u) {
        const int c = s0 + W * u - W;
        raw[u] = (active && c >= 1 && c <= H && c + W < nslot) ? b.hb[ho + c - 1] : (unsigned char)0;
      }
#pragma unroll
      for (int u = 0; u < kHB; ++u) {
        const int s = s0 + W * u, c = s - W;
        if (own_seg && s < nslot) {
          PhRing<T> v;
          v.X = (c >= 0 && c <= H) ? x0 : (T)0;
          v.I = 0;
          ring[s] = v;
          const bool in = active && c >= 1 && c <= H;
          const unsigned char code = in ? base_code(raw[u]) : (unsigned char)6;
          other |= code == 5;
          hapl[s] = code;
        }
      }
    }
    const bool bytecmp = __ballot(other) != 0ull;
    if (bytecmp && own_seg)
      for (int s = sl; s < nslot; s += W) {
        const int c = s - W;
        hapl[s] = (active && c >= 1 && c <= H) ? b.hb[ho + c - 1] : (unsigned char)0;
      }
    __syncthreads();

    RowP<T> prm = row_params<T, EXACT>(tab, load_raw(b, active ? R : 0, ro, sl));
    T accM = 0, accI = 0;
    const int sum_stripe = active ? (R - 1) / W : -1;
    const int sum_lane = active ? (R - 1) % W : -1;
    for (int st = 0; st < nstr_max; ++st) {
      const RawRow nraw = load_raw(b, active ? R : 0, ro, (st + 1) * W + sl);
      RowP<T> nprm;
      const bool seg_sums = (st == sum_stripe);
      const int any_sum = wave_max(seg_sums ? 1 : 0);
      if (any_sum) {
        // If no live segment continues past this stripe, stop after the last summed column.
        const int cont = wave_max((active && nstr > st + 1) ? 1 : 0);
        const int lim = (seg_sums && sl == sum_lane) ? sl + H : -1;
        const int ulim = -wave_max((seg_sums && sl == sum_lane) ? -(sl + H) : -0x7FFFFFFF);
        accM = accI = 0;  // a sum lives within its stripe; drop what unconditional blocks added before
        const int tend = cont ? Hmax + W - 1 : wave_max(seg_sums ? sum_lane + H : 0);
        RowP<T> sp = prm;  // the last row's D feeds only rows past R: reuse it as the M sum
        if (lim >= 0) sp.my = sp.yy = (T)1;
        if (bytecmp)
          phmm_stripe<T, EXACT, true, true, W>(sp, ring, hapl, sl, (tend + 16) >> 4, lim, ulim, accM, accI, tab, nraw, nprm, top);
        else
          phmm_stripe<T, EXACT, true, false, W>(sp, ring, hapl, sl, (tend + 16) >> 4, lim, ulim, accM, accI, tab, nraw, nprm, top);
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
        if (bytecmp)
          phmm_stripe<T, EXACT, false, true, W>(prm, ring, hapl, sl, (Hmax + W + 15) >> 4, -1, -1, accM, accI, tab, nraw, nprm, top);
        else
          phmm_stripe<T, EXACT, false, false, W>(prm, ring, hapl, sl, (Hmax + W + 15) >> 4, -1, -1, accM, accI, tab, nraw, nprm, top);
      }
      prm = nprm;
    }
  }
}

}  // namespace fcs

#include "phmm2.h"
#include "phmm_stream.h"
#include "phmm_cols.h"

namespace fcs {

// Slots (ring entries and hap bytes) = column + 16 for columns -16 .. Hmax + 34:
// stripes run to Hmax + 15 rounded up to a 16-step block, plus up to four steps of
// read-ahead.
static __host__ __device__ int nslot_for(int max_hap_len) { return ((max_hap_len + 51 + 15) / 16) * 16; }
// The same for W-lane segments: columns -W .. Hmax + 2W + 14 + PFD.
static __host__ __device__ int nslot_for_w(int max_hap_len, int W) {
  return ((max_hap_len + 2 * W + 19 + 15) / 16) * 16;
}

// Hap-length classes of the forward pass: class c < kPhmmClasses - 1 holds
// pairs with nslot_for(H) <= 224 + 32c (LDS 8.1 .. 12.7 KB per wave), the last
// class everything longer.  Each class is its own launch with LDS sized to the
// class, so short haplotypes run at 4 waves per SIMD instead of the 3 that the
// longest haplotype of the batch would allow.
static_assert(kPhmmLaunchClasses <= 16 && kPhmmKeyClassShift + 4 <= kPhmmKeyBits, "class fits the key");
__host__ __device__ inline int phmm_class(int H) {
  const int c = (nslot_for(H) - 224 + 31) / 32;
  return c < 0 ? 0 : c > kPhmmClasses - 1 ? kPhmmClasses - 1 : c;
}

// Schedule keys (16 bits; the bin schedule sorts on the top 12): a 4-bit launch class, then the
// in-class order, as ascending keys — each class is a contiguous range and the
// longest work comes first.  For kStreamMinR <= R <= kStreamMaxR: haplotypes
// longer than the column-blocked kernel's 303 columns take the row-streamed
// kernel's classes 3 and 2 (launch classes 0, 1), the others the column-
// blocked kernel's classes (launch classes kLongClasses .., widest first);
// everything else the grouped kernels' hap-length classes (longest first).
// In-class order: streamed and column-blocked, hap length descending;
// grouped, stripe count then hap length descending.  The clamps only change
// the order, never results.
__host__ __device__ inline int phmm_launch_class(int R, int H, int& stream_cls) {
  stream_cls = -1;
  if (R >= kStreamMinR && R <= kStreamMaxR && H >= 1) {
    static_assert(kColsMinR <= kStreamMinR, "column-blocked streams take every streamed read");
    const int cc = cols_class(H);
    stream_cls = cc >= 0 ? 0 : stream_class(H);
    if (cc >= 0) return kLongClasses + cc;
    if (stream_cls >= 2) return kStreamClasses - 1 - stream_cls;
    stream_cls = -1;
  }
  return kLongClasses + kColsLaunch + kPhmmClasses - 1 - phmm_class(max(H, 0));
}

__device__ __forceinline__ uint32_t phmm_key(const PhmmDevBatch& b, long long p) {
  const int R = b.read_len[b.pair_read[p]];
  const int H = b.hap_len[b.pair_hap[p]];
  int sc;
  const uint32_t cf = (uint32_t)phmm_launch_class(R, H, sc);
  const uint32_t hh = 0xFFFu - (uint32_t)min(max(H, 0), 0xFFF);
  // streamed: hap length (H <= 3700 fits 12 bits); grouped: stripe count (R < 33:
  // at most 3), then hap length in steps of 4
  uint32_t low;
  if (sc >= 0)
    low = hh;
  else
    low = ((3u - (uint32_t)min((max(R, 0) + 15) >> 4, 3)) << 10) | (0x3FFu - (uint32_t)min(max(H, 0) >> 2, 0x3FF));
  return (cf << kPhmmKeyClassShift) | low;
}

// ---- bin schedule: a counting sort on the key's top 12 bits (class, then the
// in-class order in steps of 16), three small kernels instead of the radix
// sort's eight launches and state fills.  Order inside a bin is arbitrary
// (results never depend on the order; the bins keep the longest work first
// to 16 haplotype bases).
constexpr int kPhmmBins = 1 << (kPhmmKeyBits - 4);
constexpr int kBinBlock = 1024, kBinItems = 4;
__device__ __forceinline__ int phmm_bin(const PhmmDevBatch& b, long long p) { return (int)(phmm_key(b, p) >> 4); }

__global__ __launch_bounds__(kBinBlock) void phmm_bin_count_kernel(const PhmmDevBatch b, uint32_t* __restrict__ hist,
                                                                    unsigned long long* __restrict__ counters) {
  __shared__ uint32_t h[kPhmmBins];
  for (int i = threadIdx.x; i < kPhmmBins; i += kBinBlock) h[i] = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    counters[0] = 0ull;
    counters[1] = 0ull;
  }
  __syncthreads();
  const long long base = (long long)blockIdx.x * (kBinBlock * kBinItems);
  for (int k = 0; k < kBinItems; ++k) {
    const long long p = base + (long long)k * kBinBlock + threadIdx.x;
    if (p < b.n_pairs) atomicAdd(&h[phmm_bin(b, p)], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kPhmmBins; i += kBinBlock)
    if (h[i]) atomicAdd(&hist[i], h[i]);
}

// One block: cursor = exclusive prefix of hist, bounds per launch class, hist
// zeroed again for the next schedule.
__global__ __launch_bounds__(kBinBlock) void phmm_bin_scan_kernel(uint32_t* __restrict__ hist,
                                                                   uint32_t* __restrict__ cursor, long long n,
                                                                   int64_t* __restrict__ bounds) {
  constexpr int kPer = kPhmmBins / kBinBlock;
  __shared__ uint32_t part[kBinBlock];
  const int t = threadIdx.x;
  uint32_t v[kPer], sum = 0;
  for (int j = 0; j < kPer; ++j) {
    v[j] = hist[t * kPer + j];
    sum += v[j];
  }
  part[t] = sum;
  __syncthreads();
  for (int off = 1; off < kBinBlock; off <<= 1) {  // inclusive scan of the per-thread sums
    const uint32_t x = t >= off ? part[t - off] : 0u;
    __syncthreads();
    part[t] += x;
    __syncthreads();
  }
  uint32_t run = part[t] - sum;
  for (int j = 0; j < kPer; ++j) {
    const int bin = t * kPer + j;
    cursor[bin] = run;
    if ((bin & 255) == 0 && (bin >> 8) < kPhmmLaunchClasses) bounds[bin >> 8] = run;
    run += v[j];
    hist[bin] = 0u;
  }
  if (t == 0) bounds[kPhmmLaunchClasses] = n;
}

__global__ __launch_bounds__(kBinBlock) void phmm_bin_scatter_kernel(const PhmmDevBatch b,
                                                                      uint32_t* __restrict__ cursor,
                                                                      int32_t* __restrict__ idx) {
  __shared__ uint32_t cnt[kPhmmBins], at[kPhmmBins];
  for (int i = threadIdx.x; i < kPhmmBins; i += kBinBlock) cnt[i] = 0;
  __syncthreads();
  const long long base = (long long)blockIdx.x * (kBinBlock * kBinItems);
  int bin[kBinItems];
  uint32_t rank[kBinItems];
  for (int k = 0; k < kBinItems; ++k) {
    const long long p = base + (long long)k * kBinBlock + threadIdx.x;
    bin[k] = p < b.n_pairs ? phmm_bin(b, p) : -1;
    rank[k] = bin[k] >= 0 ? atomicAdd(&cnt[bin[k]], 1u) : 0u;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kPhmmBins; i += kBinBlock)
    if (cnt[i]) at[i] = atomicAdd(&cursor[i], cnt[i]);  // this block's range of bin i
  __syncthreads();
  for (int k = 0; k < kBinItems; ++k)
    if (bin[k] >= 0) idx[at[bin[k]] + rank[k]] = (int32_t)(base + (long long)k * kBinBlock + threadIdx.x);
}

int launch_phmm_bin_schedule(const PhmmDevBatch& b, int32_t* idx_out, int64_t* bounds, unsigned long long* counters,
                             uint32_t* hist, uint32_t* cursor, hipStream_t s) {
  static_assert(kPhmmBins % kBinBlock == 0 && (kPhmmLaunchClasses << 8) <= kPhmmBins, "bins");
  const long long n = b.n_pairs > 0 ? b.n_pairs : 0;
  const unsigned nb = (unsigned)std::max<long long>((n + kBinBlock * kBinItems - 1) / (kBinBlock * kBinItems), 1);
  hipLaunchKernelGGL(phmm_bin_count_kernel, dim3(nb), dim3(kBinBlock), 0, s, b, hist, counters);
  FCS_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(phmm_bin_scan_kernel, dim3(1), dim3(kBinBlock), 0, s, hist, cursor, n, bounds);
  FCS_HIP_CHECK(hipGetLastError());
  if (n > 0) {
    hipLaunchKernelGGL(phmm_bin_scatter_kernel, dim3(nb), dim3(kBinBlock), 0, s, b, cursor, idx_out);
    FCS_HIP_CHECK(hipGetLastError());
  }
  return FCS_OK;
}

constexpr size_t kLdsBytes = 160 * 1024;

template <typename T, bool EXACT, bool RESCUE, int W = 16>
static int launch_one(const PhmmDevBatch& b, const int32_t* order, const unsigned long long* count_dev,
                      long long count_host, const int64_t* bounds, int cls, int nslot, long long max_groups,
                      const PhmmTables<T>& tab, double* out, int32_t* rescue_list, unsigned long long* rescue_count,
                      float thr, bool use_rescue, hipStream_t s) {
  // Four rings per wave when they fit the 160 KB of LDS, else one (long
  // haplotypes: fp32 up to ~4.5 kb at four, ~18 kb at one; fp64 ~2.3 / ~9.5 kb).
  // 64-lane segments: one pair (one ring) per wave.
  int nseg = 64 / W;
  size_t lds = (size_t)nseg * (ring_stride<T>(nslot) + nslot);
  if (lds > kLdsBytes && nseg > 1) {
    nseg = 1;
    lds = (size_t)ring_stride<T>(nslot) + nslot;
    max_groups *= 4;
  }
  if (lds > kLdsBytes)
    return fail(FCS_ERR_UNSUPPORTED, "[E::fcship] haplotype too long for the LDS boundary ring (max_hap_len " +
                                         std::to_string(nslot - 67) + ")");
  auto kern = phmm_kernel<T, EXACT, RESCUE, W>;
  if (lds > 64 * 1024)
    FCS_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  long long grid = max_groups;
  // One four-pair group per workgroup up to 64K groups per class launch (grid-
  // stride beyond): the dispatcher then hands groups out in the schedule's
  // longest-first order and the tail is one group deep.  A 16K cap (each
  // workgroup striding over ~3 groups) measured 4% slower on C2
  // (gpurun_out/p5); the surplus workgroups of a class exit at once.
  const long long cap = 65536;
  if (grid > cap) grid = cap;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(64), lds, s, b, order, count_dev, count_host, bounds, cls, nslot,
                     tab, out, rescue_list, rescue_count, thr, use_rescue ? 1 : 0, nseg);
  FCS_HIP_CHECK(hipGetLastError());
  return FCS_OK;
}

// Pairs per segment stream of the streamed kernel: as many as keep >= ~24K
// waves in flight for the batch (8 x 3 waves x 256 CUs x 4 SIMDs), at most
// kStreamMaxK (a stream's quantisation loss is < 1/2 stripe in K pairs).
// FCSHIP_STREAM_K=k (tests) forces k pairs per stream on any batch size.
static int stream_pairs_per_segment(int64_t n) {
  static const int forced = [] {
    const char* e = std::getenv("FCSHIP_STREAM_K");
    return e ? std::atoi(e) : 0;
  }();
  if (forced > 0) return std::min(forced, kStreamMaxK);
  const int64_t k = n / (4 * 24576);
  return (int)std::max<int64_t>(1, std::min<int64_t>(kStreamMaxK, k));
}

// Pairs per half-stream of the column-blocked kernel: as many as keep >= ~24K
// waves in flight for the batch (8 half-streams per wave), at most 8.
// FCSHIP_STREAM_K=k (tests) forces k here too.
static int cols_pairs_per_half(int64_t n) {
  static const int forced = [] {
    const char* e = std::getenv("FCSHIP_STREAM_K");
    return e ? std::atoi(e) : 0;
  }();
  if (forced > 0) return std::min(forced, 8);
  const int64_t k = n / (8 * 24576);
  return (int)std::max<int64_t>(1, std::min<int64_t>(8, k));
}

int launch_phmm_forward(const PhmmDevBatch& b, const int32_t* order, int64_t count, int max_hap_len,
                        const int64_t* bounds, const DeviceTables& t, bool exact, double* out, int32_t* rescue_list,
                        unsigned long long* rescue_count, float thr, bool use_rescue, int32_t* fb_list,
                        unsigned long long* fb_count, hipStream_t s) {
  if (count <= 0) return FCS_OK;
  const long long groups = (count + 3) / 4;
  const int ns_max = nslot_for(max_hap_len);
  const int c_max = phmm_class(max_hap_len);
  // One launch per launch class (ranges from the device-side bounds), forked
  // over streams so a class's tail overlaps the next class; classes above the
  // batch's longest haplotype are empty and not launched.
  hipStream_t fs[kForkStreams];
  if (const int rc = fork_streams(s, fs); rc != FCS_OK) return rc;
  int fork = 0;
  // Haplotypes longer than the column-blocked kernel takes: row-streamed
  // classes 3 and 2 (launch classes 0, 1: H in (472, 3700], (303, 472]).
  for (int j = 0; j < kLongClasses; ++j) {
    const int sc = kStreamClasses - 1 - j;
    const int lo = j == 0 ? stream_class_hmax(sc - 1) : cols_hmax(0);
    if (max_hap_len <= lo) continue;
    const int hmax = std::min(stream_class_hmax(sc), max_hap_len);
    hipStream_t st = fs[fork++ % kForkStreams];
    if (exact) {  // GKL operation order: the one-row kernel over the same range
      const int rc = launch_one<float, true, false>(b, order, nullptr, count, bounds, j, nslot_for(hmax), groups, t.tf,
                                                   out, rescue_list, rescue_count, thr, use_rescue, st);
      if (rc != FCS_OK) return rc;
      continue;
    }
    const size_t lds = (size_t)stream_lds(hmax);
    if (lds > kLdsBytes) return fail(FCS_ERR_UNSUPPORTED, "[E::fcship] streamed PairHMM class exceeds LDS");
    const int K = stream_pairs_per_segment(count);
    const int w = stream_class_waves(sc);
    // the range's last pairs run one per segment: about two rounds of the
    // chip's wave slots (256 CUs x 4 SIMDs x w), so the launch ends on short waves
    const int tail = 2 * 4 * 1024 * w;
    const unsigned grid = (unsigned)std::min<long long>(
        std::max<long long>((count + 4 * K - 1) / (4 * K) + (tail + 3) / 4, 1), 65536);
    auto launch = [&](auto kern) -> int {
      if (lds > 64 * 1024)
        FCS_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      hipLaunchKernelGGL(kern, dim3(grid), dim3(64), lds, st, b, order, bounds, j, K, tail, stream_nslot(hmax),
                         stream_hstride(hmax), t.tf, out, rescue_list, rescue_count, thr, use_rescue ? 1 : 0, fb_list,
                         fb_count);
      FCS_HIP_CHECK(hipGetLastError());
      return FCS_OK;
    };
    const int rc = w >= 3 ? launch(phmm3_kernel<3>) : w == 2 ? launch(phmm3_kernel<2>) : launch(phmm3_kernel<1>);
    if (rc != FCS_OK) return rc;
  }
  // The column-blocked kernel (phmm_cols.h): every other streamed pair, by
  // columns per lane (launch classes kLongClasses .., widest first).
  for (int c = 0; c < kColsLaunch; ++c) {
    const int lo = c + 1 < kColsLaunch ? cols_hmax(c + 1) : 0;
    if (max_hap_len <= lo) continue;
    const int j = kLongClasses + c;
    hipStream_t st = fs[fork++ % kForkStreams];
    if (exact) {
      const int rc = launch_one<float, true, false>(b, order, nullptr, count, bounds, j,
                                                   nslot_for(std::min(cols_hmax(c), max_hap_len)), groups, t.tf, out,
                                                   rescue_list, rescue_count, thr, use_rescue, st);
      if (rc != FCS_OK) return rc;
      continue;
    }
    const int K = cols_pairs_per_half(count);
    // the range's last pairs run one per half-stream: about one round of the
    // chip's wave slots (256 CUs x 4 SIMDs x 3 waves x 8 half-streams)
    const int tail = 1024 * 3 * 8;
    const unsigned grid = (unsigned)std::min<long long>(
        std::max<long long>((count + 8 * K - 1) / (8 * K) + (tail + 7) / 8, 1), 65536);
    auto launch = [&](auto kern) -> int {
      hipLaunchKernelGGL(kern, dim3(grid), dim3(64), (size_t)kColsLds, st, b, order, bounds, j, K, tail, t.tf, out,
                         rescue_list, rescue_count, thr, use_rescue ? 1 : 0, fb_list, fb_count);
      FCS_HIP_CHECK(hipGetLastError());
      return FCS_OK;
    };
    static_assert(cols_C(0) == 19 && cols_C(1) == 17 && cols_C(7) == 11 && kColsClasses == 8, "launch table below");
    int rc;
    switch (cols_C(c)) {
      case 19: rc = launch(phmm4_kernel<19>); break;
      case 17: rc = launch(phmm4_kernel<17>); break;
      case 16: rc = launch(phmm4_kernel<16>); break;
      case 15: rc = launch(phmm4_kernel<15>); break;
      case 14: rc = launch(phmm4_kernel<14>); break;
      case 13: rc = launch(phmm4_kernel<13>); break;
      case 12: rc = launch(phmm4_kernel<12>); break;
      default: rc = launch(phmm4_kernel<11>); break;
    }
    if (rc != FCS_OK) return rc;
  }
  // Grouped classes (reads shorter than kStreamMinR or longer than kStreamMaxR; empty in most batches):
  // kept off fs[0], which carries the longest-haplotype stream class, so an
  // empty grouped launch does not extend the pass after it; and launched with
  // at most kGroupedGrid workgroups striding over the class (about 2.7 rounds of
  // the chip's wave slots at 3 waves/SIMD), since the host does not know the
  // class sizes and each of 64K empty workgroups still takes a dispatch, a wave
  // slot and its LDS while it reads the bounds.
  constexpr long long kGroupedGrid = 8192;
  int gfork = 0;
  for (int j = kPhmmClasses - 1 - c_max; j < kPhmmClasses; ++j) {
    const int c = kPhmmClasses - 1 - j;
    const int lc = kLongClasses + kColsLaunch + j;  // launch class of grouped class c
    const int ns = (c == kPhmmClasses - 1) ? ns_max : std::min(224 + 32 * c, ns_max);
    hipStream_t st = fs[1 + gfork++ % (kForkStreams - 1)];
    // the two-rows-per-lane kernel (phmm2.h) for the FMA-order pass when its
    // four rings fit (ring slots >= H + 65, hap bytes + 16)
    const int ns2 = ns + 16;
    const size_t lds2 = (size_t)phmm2_lds(ns2);
    if (!exact && lds2 <= kLdsBytes) {
      if (lds2 > 64 * 1024)
        FCS_HIP_CHECK(
            hipFuncSetAttribute((const void*)phmm2_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds2));
      const unsigned grid = (unsigned)std::min<long long>(std::max<long long>(groups, 1), kGroupedGrid);
      hipLaunchKernelGGL(phmm2_kernel, dim3(grid), dim3(64), lds2, st, b, order, bounds, lc, ns2, t.tf, out,
                         rescue_list, rescue_count, thr, use_rescue ? 1 : 0);
      FCS_HIP_CHECK(hipGetLastError());
      continue;
    }
    const int rc = exact ? launch_one<float, true, false>(b, order, nullptr, count, bounds, lc, ns, groups, t.tf, out,
                                                           rescue_list, rescue_count, thr, use_rescue, st)
                         : launch_one<float, false, false>(b, order, nullptr, count, bounds, lc, ns, groups, t.tf, out,
                                                            rescue_list, rescue_count, thr, use_rescue, st);
    if (rc != FCS_OK) return rc;
  }
  if (const int rc = join_streams(s, fs); rc != FCS_OK) return rc;
  if (exact) return FCS_OK;
  // Pairs the streamed kernel handed back (device-side list): the one-row
  // kernel with GKL's byte compare, appending to the same rescue list.
  return launch_one<float, false, false>(b, fb_list, fb_count, 0, nullptr, 0, ns_max,
                                         std::min<long long>(groups, 2048), t.tf, out, rescue_list, rescue_count, thr,
                                         use_rescue, s);
}

int launch_phmm_rescue(const PhmmDevBatch& b, const int32_t* list, const unsigned long long* count_dev,
                       int64_t max_count, int max_hap_len, const DeviceTables& t, bool exact, double* out,
                       hipStream_t s) {
  if (max_count <= 0) return FCS_OK;
  // The rescued subset is usually tiny (tens to hundreds of pairs per call), so
  // its time is one pair's latency: 64-lane segments, one pair per wave, run
  // 64-row stripes — a third of the 16-row stripes' sequential steps at 150-base
  // reads.  A modest grid strides over the device-side count (no host round
  // trip).  Haplotypes too long for a 64-lane ring take the 16-lane kernel.
  const int ns64 = nslot_for_w(max_hap_len, 64);
  if ((size_t)ring_stride<double>(ns64) + ns64 <= kLdsBytes) {
    const long long g64 = std::min<long long>(max_count, 4096);
    if (exact)
      return launch_one<double, true, true, 64>(b, list, count_dev, 0, nullptr, 0, ns64, g64, t.td, out, nullptr,
                                                nullptr, 0.f, false, s);
    return launch_one<double, false, true, 64>(b, list, count_dev, 0, nullptr, 0, ns64, g64, t.td, out, nullptr,
                                               nullptr, 0.f, false, s);
  }
  long long groups = (max_count + 3) / 4;
  if (groups > 2048) groups = 2048;
  if (exact)
    return launch_one<double, true, true>(b, list, count_dev, 0, nullptr, 0, nslot_for(max_hap_len), groups, t.td, out,
                                          nullptr, nullptr, 0.f, false, s);
  return launch_one<double, false, true>(b, list, count_dev, 0, nullptr, 0, nslot_for(max_hap_len), groups, t.td, out,
                                         nullptr, nullptr, 0.f, false, s);
}

}  // namespace fcs

// bwa ksw_align2 (local Smith-Waterman with the second-best score and the
// alignment start) on gfx950: the kernel of bwa mem's mate rescue
// (bwamem_pair.c mem_matesw), which the reference runs inside `bwa-flow mem`
// (/root/reference/src/workers/BWAWorker.cpp:134-166).  Restated algorithm:
// oracle/ksw_align_oracle.c, bit-exact target.
//
// bwa's ksw_u8 / ksw_i16 are Farrar striped SSE2 kernels and their results
// depend on the striping: with p lanes (16 u8 / 8 i16) and slen = ceil(qlen /
// p) segments, query position x sits in lane x / slen, and
//   * the first pass runs F only down a lane's own segments (blocks of slen
//     consecutive positions), so E(i + 1, x) opens from that first-pass H1;
//   * the lazy-F loop then carries F across the blocks; it only raises H
//     (never E), and bwa's column maximum is taken from H1.
// Here a group of W lanes (a 16-lane DPP row, four tasks per wave, for
// qlen <= 160; the whole 64-lane wave for longer queries) runs one task; lane
// l of the group owns the NK consecutive positions x = l NK + k, padded to
// slen * p as bwa's profile is (padding scores 0), so the max-plus scans are a
// running max along the lane's registers plus one group scan of lane totals.
// Per target base (one column):
//   M  = sat(Hprev(x - 1) + s)            (u8: biased, saturating; i16: saturating)
//   M' = max(M, E)
//   F1 = max(0, max over x' < x in x's block of M'(x') - oe_ins - (x - 1 - x') e_ins)
//   H1 = max(M', F1),  E <- max(E - e_del, H1 - oe_del) (floored at 0)
//   F  = the same over every x' < x,  H = max(H1, F)
// (F opened from an F-raised H is dominated, so both F's are max-plus scans of
// M'; a block-id term in the scan value keeps the first one inside its block).
// Column maxima, bwa's b[] list (LDS), te / qe / score2 / te2, and the
// KSW_XSTART second pass over the reversed query and target prefixes run in
// the same group.  With W = 16 the four tasks of a wave run their columns in
// lock-step (the wave loops to its longest target; a group past its own end or
// early exit computes masked columns).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>

#include "bsw_scan.h"
#include "fcship_internal.h"

namespace fcs {

constexpr int kKswXByte = 0x10000, kKswXStop = 0x20000, kKswXSubo = 0x40000, kKswXStart = 0x80000;
constexpr int kBlockBig = 1 << 20;  // > the range of one block's scan values; block ids < 16
constexpr int kAlignSegQ = 160;                // longest query of the 16-lane groups (NK = 10 slots)
constexpr long long kAlignGridCap = 1 << 20;  // workgroups per launch (they stride beyond)

// Group-level primitives: W = 16 (a DPP row) or 64 (the wave).
template <int W>
__device__ __forceinline__ int grp_lane() {
  return W == 64 ? lane_id() : (lane_id() & 15);
}
// Inclusive max scan inside the group (lanes without a source see `neg`).
template <int W>
__device__ __forceinline__ int grp_incl_max(int v, int neg) {
  if constexpr (W == 64) {
    return wave_incl_max(v, neg);
  } else {
    v = max(v, __builtin_amdgcn_update_dpp(neg, v, kDppRowShr1, 0xF, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(neg, v, kDppRowShr2, 0xF, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(neg, v, kDppRowShr4, 0xF, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(neg, v, kDppRowShr8, 0xF, 0xF, false));
    return v;
  }
}
// The group's last lane's value, in every lane of the group.
template <int W>
__device__ __forceinline__ int grp_last(int v) {
  if constexpr (W == 64) {
    return read_lane(v, 63);
  } else {
    // ds_swizzle bit mode inside 32-lane halves: lane -> (lane & 0x10) | 0x0F
    return __builtin_amdgcn_ds_swizzle(v, 0x10 | (0x0F << 5));
  }
}
// The group's maximum in every lane: W = 16, a butterfly of row rotations
// (no LDS round trip on the column loop's critical path).
template <int W>
__device__ __forceinline__ int grp_max(int v) {
  if constexpr (W == 64) {
    return grp_last<W>(grp_incl_max<W>(v, INT32_MIN));
  } else {
    // (every lane has a source, so old = 0 with bound_ctrl is never used; that
    // form folds into v_max_i32_dpp)
    v = max(v, __builtin_amdgcn_update_dpp(0, v, kDppRowRor8, 0xF, 0xF, true));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, kDppRowRor4, 0xF, 0xF, true));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, kDppRowRor2, 0xF, 0xF, true));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, kDppRowRor1, 0xF, 0xF, true));
    return v;
  }
}
// Lane l <- lane l - 1 of the group's value; the group's lane 0 <- `first`.
template <int W>
__device__ __forceinline__ int grp_shr1(int first, int v) {
  if constexpr (W == 64) return dpp_wave_shr1_i(first, v);
  else return __builtin_amdgcn_update_dpp(first, v, kDppRowShr1, 0xF, 0xF, false);
}
// Exclusive prefix max over the group's positions x = lane * NS + k (each
// lane holds NS consecutive positions), seeded with kScanNeg: a running max
// along the lane's own slots, and one group scan of the lanes' totals.
template <int W, int NS>
__device__ __forceinline__ void grp_excl_scan(const int (&u)[NS], int (&ex)[NS]) {
  int run[NS];
  run[0] = u[0];
#pragma unroll
  for (int k = 1; k < NS; ++k) run[k] = max(run[k - 1], u[k]);
  const int cin = grp_shr1<W>(kScanNeg, grp_incl_max<W>(run[NS - 1], kScanNeg));  // lanes below
  ex[0] = cin;
#pragma unroll
  for (int k = 1; k < NS; ++k) ex[k] = max(cin, run[k - 1]);
}

struct AlignRun {
  int score, te, qe, score2, te2;
};

// One ksw_u8 / ksw_i16 run of query q[x] (x < qlen, read through q_at) against
// target t[j] (j < tlen, LDS, read through t_at) in this lane's group.  minsc /
// endsc as bwa's.  live: the group runs this task (group-uniform).  Every lane
// of the wave calls it (the column loop is wave-uniform); blist is the
// group's b[] area.
template <int W, int NK, class QAt, class TAt>
__device__ AlignRun align_run(const BswParams& p, bool live, int qlen, QAt q_at, int tlen, TAt t_at, bool u8,
                              int shift, int max_mat, int minsc, int endsc, uint32_t* __restrict__ blist) {
  const int gl = grp_lane<W>();
  const int pl = u8 ? 16 : 8;
  const int slen = (qlen + pl - 1) / pl;
  const int nlen = live ? slen * pl : 0;
  const int oe_del = p.o_del + p.e_del, oe_ins = p.o_ins + p.e_ins, e_del = p.e_del, e_ins = p.e_ins;
  // Per slot: the biased profile bytes (mat[a][q] + shift, a = 0..3 in plo;
  // a = 4 (N) in byte k % 4 of phi[k / 4]: v_perm picks the score by the
  // target code), and the scan
  // offsets c1 = x e_ins - oe_ins + block * kBlockBig, c2 = x e_ins - oe_ins
  // (u = M' + c turns both max-plus scans into plain max scans).
  constexpr int NP = (NK + 3) / 4;
  int Hp[NK], E[NK], Hm[NK], plo[NK], phi[NP], c1[NK], c2[NK];
#pragma unroll
  for (int k = 0; k < NP; ++k) phi[k] = 0;
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int x = gl * NK + k;
    const int qb = (live && x < qlen) ? q_at(x) : -1;  // padding: score 0 against every base
    auto sc = [&](int a) { return ((qb < 0 ? 0 : (int)p.mat[a * 5 + qb]) + shift) & 0xFF; };
    plo[k] = sc(0) | (sc(1) << 8) | (sc(2) << 16) | (sc(3) << 24);
    phi[k / 4] |= sc(4) << (8 * (k % 4));
    c2[k] = x * e_ins - oe_ins;
    c1[k] = c2[k] + (slen > 0 ? x / slen : 0) * kBlockBig;
    Hp[k] = E[k] = Hm[k] = 0;
  }
  // M = sat(H + s): u8 max(min(H + s', 255) - shift, 0), i16 clamp to 16 bits;
  // with s' = s + shift both are one med3 of H + s' - shift
  const int mlo = u8 ? 0 : -32768, mhi = u8 ? 255 - shift : 32767;
  // group-uniform state: best score / column, b[]'s size and last entry; Hm:
  // the H column of the best score (bwa's Hmax, for qe).  (A packed
  // max-and-position key per cell instead of the copy saves the 10 VGPRs that
  // give 3 waves per SIMD, and measured 12% slower: profiles/r4/r4k_*.)
  int gmax = 0, te = -1, n_b = 0, last_i = -2, last_v = 0;
  bool run = live && tlen > 0;
  const int ncol = W == 64 ? tlen : wave_max(run ? tlen : 0);
  for (int i = 0; i < ncol; ++i) {
    if (__ballot(run) == 0ull) break;
    const bool act = run && i < tlen;
    const int tb = act ? t_at(i) : 4;
    // byte 0 selects the score (plo byte tb, or phi byte 4 + k % 4 for N), the rest 0
    uint32_t sel[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) sel[r] = 0x0C0C0C00u | (uint32_t)(tb + (tb == 4 ? r : 0));
    int Mp[NK], u1[NK], u2[NK];
    // H(i - 1, x - 1): the previous slot of this lane, for slot 0 the last slot
    // of the lane below (position -1: 0)
    const int hd0 = grp_shr1<W>(0, Hp[NK - 1]);
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int hd = k == 0 ? hd0 : Hp[k - 1];
      const int sb = (int)__builtin_amdgcn_perm((uint32_t)phi[k / 4], (uint32_t)plo[k], sel[k % 4]);
      const int m = max(min(max(hd + sb - shift, mlo), mhi), E[k]);
      Mp[k] = m;
      u1[k] = m + c1[k];
      u2[k] = m + c2[k];
    }
    int ex1[NK], ex2[NK];
    grp_excl_scan<W, NK>(u1, ex1);
    grp_excl_scan<W, NK>(u2, ex2);
    // Positions past nlen (the group's last lanes) compute values that feed
    // only later positions; they are kept out of the column maximum.  A block's
    // first position sees only earlier blocks in ex1, whose smaller block term
    // makes f1 negative, and position 0 sees kScanNeg: no tests needed.
    int imax = 0, Hn[NK];
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int x = gl * NK + k;
      const int h1 = max(Mp[k], ex1[k] - c1[k] - p.o_ins);  // max(M', F1): F1 >= 0 is implied by M' >= 0
      E[k] = max(max(E[k] - e_del, h1 - oe_del), 0);
      Hn[k] = max(h1, ex2[k] - c2[k] - p.o_ins);
      Hp[k] = Hn[k];
      imax = max(imax, x < nlen ? h1 : 0);
    }
    imax = grp_max<W>(imax);
    if (act && imax >= minsc) {  // bwa's b[]: append, or raise the last entry when it holds the previous column
      if (n_b == 0 || last_i + 1 != i) {
        if (gl == 0) blist[n_b] = (uint32_t)imax << 16 | (uint32_t)i;
        ++n_b;
        last_i = i, last_v = imax;
      } else if (last_v < imax) {
        if (gl == 0) blist[n_b - 1] = (uint32_t)imax << 16 | (uint32_t)i;
        last_i = i, last_v = imax;
      }
    }
    if (act && imax > gmax) {
      gmax = imax;
      te = i;
#pragma unroll
      for (int k = 0; k < NK; ++k) Hm[k] = Hn[k];
      if ((u8 && gmax + shift >= 255) || gmax >= endsc) run = false;
    }
    if (!(i + 1 < tlen)) run = false;
  }
  AlignRun r{u8 ? (gmax + shift < 255 ? gmax : 255) : gmax, te, -1, -1, -1};
  // the b[] stores of lane 0 before other lanes of its group read them (one
  // wave per workgroup: LDS ops complete in order; this orders the compiler)
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  const bool tail = live && (!u8 || r.score != 255);
  int mx = -1;
#pragma unroll
  for (int k = 0; k < NK; ++k)
    if (gl * NK + k < nlen) mx = max(mx, Hm[k]);
  mx = grp_max<W>(mx);
  int qx = 0x7FFFFFFF;  // the smallest position holding the column maximum (bwa's memory-order scan)
#pragma unroll
  for (int k = 0; k < NK; ++k)
    if (gl * NK + k < nlen && Hm[k] == mx) qx = min(qx, gl * NK + k);
  const int qe_min = -grp_max<W>(-qx);
  const int qe_best = nlen > 0 ? qe_min : -1;  // an empty query: bwa's scan finds nothing
  const int w = max_mat > 0 ? (r.score + max_mat - 1) / max_mat : 0;
  const int low = te - w, high = te + w;
  int best = -1, bte = -1;
  const int nbl = tail ? n_b : 0;
  const int nbmax = W == 64 ? nbl : wave_max(nbl);
  for (int j0 = 0; j0 < nbmax; j0 += W) {  // the first entry (column order) of the largest score outside the window
    const int j = j0 + gl;
    if (j < nbl) {
      const uint32_t e = blist[j];
      const int c = (int)(e & 0xFFFF), v = (int)(e >> 16);
      if ((c < low || c > high) && v > best) best = v, bte = c;
    }
  }
  const int vmax = grp_max<W>(best);
  const int te2 = -grp_max<W>(-(bte >= 0 && best == vmax ? bte : 0x7FFFFFFF));
  if (tail) {
    r.qe = qe_best;
    if (vmax > -1) r.score2 = vmax, r.te2 = te2;
  }
  return r;
}

// ---------------------------------------------------------------- packed
// bwa's ksw_u8 tasks (XBYTE: every H, E, M' in [0, 255]) and ksw_i16 tasks in
// 16-lane groups, on pairs of positions in packed 16-bit halves: lane l's ten
// positions x = 10 l + k sit in five registers, lo half k = j, hi half
// k = j + 5, so one VOP3P instruction does two cells.  The scan values are
// biased to stay non-negative (c2 = x e_ins + 1, c1 = c2 + block * big with
// big = Mmax + 2 + 159 e_ins > the spread of one block's values, Mmax the
// largest H / E / M'), so 0 is the scan's empty value and the signed
// differences ex - c fit in 16 bits while blocks * big + o_ins < 32768
// (align_packed_ok; 16 blocks for u8, 8 for i16).  u8: Mmax = 255.  i16: a
// local score never exceeds qlen * max_mat (each query base adds at most
// max_mat), so Mmax = 160 max_mat for the queries of the 16-lane groups, far
// below bwa's 16-bit saturation, which therefore never acts.  Same recurrence,
// same results as align_run<16, 10> (tests/test_bsw_gpu.py).
typedef uint16_t au16x2 __attribute__((ext_vector_type(2)));
typedef int16_t ai16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ au16x2 AV(uint32_t x) { return __builtin_bit_cast(au16x2, x); }
__device__ __forceinline__ ai16x2 AS(uint32_t x) { return __builtin_bit_cast(ai16x2, x); }
__device__ __forceinline__ uint32_t AU(au16x2 x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ uint32_t AI(ai16x2 x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ uint32_t ap_maxu(uint32_t a, uint32_t b) {
  return AU(__builtin_elementwise_max(AV(a), AV(b)));
}
__device__ __forceinline__ uint32_t ap_minu(uint32_t a, uint32_t b) {
  return AU(__builtin_elementwise_min(AV(a), AV(b)));
}
__device__ __forceinline__ uint32_t ap_maxi(uint32_t a, uint32_t b) {
  return AI(__builtin_elementwise_max(AS(a), AS(b)));
}
__device__ __forceinline__ uint32_t ap_add(uint32_t a, uint32_t b) { return AU(AV(a) + AV(b)); }
__device__ __forceinline__ uint32_t ap_sub(uint32_t a, uint32_t b) { return AU(AV(a) - AV(b)); }
__device__ __forceinline__ uint32_t ap_subs(uint32_t a, uint32_t b) {
  return AU(__builtin_elementwise_sub_sat(AV(a), AV(b)));
}

// Mmax: 255 (u8) or kAlignSegQ * max_mat (i16); blocks: 16 (u8) or 8 (i16)
__host__ __device__ inline int align_packed_big(int mmax, int e_ins) { return mmax + 2 + 159 * e_ins; }
__host__ __device__ inline int align_i16_mmax(int max_mat) { return kAlignSegQ * (max_mat > 0 ? max_mat : 0); }
__host__ __device__ inline bool align_packed_ok(int mmax, int blocks, int o_ins, int e_ins) {
  return o_ins >= 0 && e_ins >= 0 && e_ins <= 200 && mmax <= 8192 &&
         blocks * align_packed_big(mmax, e_ins) + o_ins + 1 < 32768;
}

template <class QAt, class TAt>
__device__ AlignRun align_run_pk(const BswParams& p, bool live, int qlen, QAt q_at, int tlen, TAt t_at, bool u8,
                                 int shift, int max_mat, int minsc, int endsc, uint32_t* __restrict__ blist) {
  constexpr int W = 16, NK = 10, NP = 5;
  const int gl = grp_lane<W>();
  const int pl = u8 ? 16 : 8;
  const int slen = (qlen + pl - 1) / pl;
  const int nlen = live ? slen * pl : 0;
  const int big = align_packed_big(u8 ? 255 : align_i16_mmax(max_mat), p.e_ins);
  const int mtop = u8 ? 255 - shift : 0x7FFF;  // u8: bwa's saturation at 255 (biased); i16: never reached
  // c1 / c2: the scan offsets; o1 / o2 = c + o_ins (f = ex - c - o_ins).
  // Positions past nlen (the group's last lanes, when slen < 10) feed only
  // later such positions; mh = 0 there (M = 0), no block term in c1 (so every
  // scan value stays below 2^15) and o1 = o2 = 0x7FFF (both F's <= 0) keep
  // their H and E at 0, so they drop out of the column maximum without a mask.
  uint32_t H[NP], E[NP], Hm[NP], plo[NK], phi[NP], c1[NP], c2[NP], o1[NP], o2[NP], mh[NP];
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    uint32_t n2 = 0, a1 = 0, a2 = 0, b1 = 0, b2 = 0, m2 = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = j + 5 * h, x = gl * NK + k;
      const int qb = (live && x < qlen) ? q_at(x) : -1;  // padding: score 0 against every base
      auto sc = [&](int a) { return (uint32_t)(((qb < 0 ? 0 : (int)p.mat[a * 5 + qb]) + shift) & 0xFF); };
      plo[k] = sc(0) | (sc(1) << 8) | (sc(2) << 16) | (sc(3) << 24);
      const bool in = x < nlen;
      const int cc2 = x * p.e_ins + 1;
      const int cc1 = in ? cc2 + (x / slen) * big : cc2;  // block ids < pl inside nlen only
      n2 |= sc(4) << (16 * h);
      a1 |= (uint32_t)cc1 << (16 * h);
      a2 |= (uint32_t)cc2 << (16 * h);
      b1 |= (uint32_t)(in ? cc1 + p.o_ins : 0x7FFF) << (16 * h);
      b2 |= (uint32_t)(in ? cc2 + p.o_ins : 0x7FFF) << (16 * h);
      m2 |= (uint32_t)(in ? mtop : 0) << (16 * h);
    }
    phi[j] = n2, c1[j] = a1, c2[j] = a2, o1[j] = b1, o2[j] = b2, mh[j] = m2;
    H[j] = E[j] = Hm[j] = 0;
  }
  const uint32_t SH = (uint32_t)shift * 0x10001u;
  const uint32_t ED = (uint32_t)p.e_del * 0x10001u, OED = (uint32_t)(p.o_del + p.e_del) * 0x10001u;
  int gmax = 0, te = -1, n_b = 0, last_i = -2, last_v = 0;
  bool run = live && tlen > 0;
  const int ncol = wave_max(run ? tlen : 0);
  for (int i = 0; i < ncol; ++i) {
    if (__ballot(run) == 0ull) break;
    const bool act = run && i < tlen;
    const int tb = act ? t_at(i) : 0;
    // lo half: byte tb of plo[j]; hi half: byte tb of plo[j + 5]; zero-extended
    const uint32_t sel = 0x0C000C00u | (uint32_t)tb | ((uint32_t)(tb + 4) << 16);
    uint32_t sb[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) sb[j] = __builtin_amdgcn_perm(plo[j + 5], plo[j], sel);
    if (__ballot(tb == 4) != 0ull) {  // an N in some group's target column: the per-position N scores
      const bool isn = tb == 4;
#pragma unroll
      for (int j = 0; j < NP; ++j) sb[j] = isn ? phi[j] : sb[j];
    }
    // H(i - 1, x - 1): lo of pair 0 is the lane below's position 9 (hi of its
    // pair 4; group lane 0: position -1, 0), hi of pair 0 this lane's position 4
    const uint32_t hb = (uint32_t)grp_shr1<W>(0, (int)H[NP - 1]);
    const uint32_t hd0 = __builtin_amdgcn_perm(H[NP - 1], hb, 0x05040302u);
    uint32_t Mp[NP], r1[NP], r2[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      const uint32_t hd = j == 0 ? hd0 : H[j - 1];
      const uint32_t m = ap_maxu(ap_minu(ap_subs(ap_add(hd, sb[j]), SH), mh[j]), E[j]);
      Mp[j] = m;
      const uint32_t u1 = ap_add(m, c1[j]), u2 = ap_add(m, c2[j]);
      r1[j] = j == 0 ? u1 : ap_maxu(r1[j - 1], u1);
      r2[j] = j == 0 ? u2 : ap_maxu(r2[j - 1], u2);
    }
    // lane totals (lo: positions 0..4, hi: 5..9), group scan, carries per half
    const int lo1 = (int)(r1[NP - 1] & 0xFFFF), lo2 = (int)(r2[NP - 1] & 0xFFFF);
    const int t1 = max(lo1, (int)(r1[NP - 1] >> 16)), t2 = max(lo2, (int)(r2[NP - 1] >> 16));
    const int ci1 = grp_shr1<W>(0, grp_incl_max<W>(t1, 0)), ci2 = grp_shr1<W>(0, grp_incl_max<W>(t2, 0));
    const uint32_t C1 = (uint32_t)ci1 | ((uint32_t)max(ci1, lo1) << 16);
    const uint32_t C2 = (uint32_t)ci2 | ((uint32_t)max(ci2, lo2) << 16);
    uint32_t imp = 0, Hn[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      const uint32_t ex1 = j == 0 ? C1 : ap_maxu(C1, r1[j - 1]);
      const uint32_t ex2 = j == 0 ? C2 : ap_maxu(C2, r2[j - 1]);
      const uint32_t h1 = ap_maxi(Mp[j], ap_sub(ex1, o1[j]));  // signed: ex1 - c1 - o_ins may be negative
      E[j] = ap_maxu(ap_subs(E[j], ED), ap_subs(h1, OED));
      Hn[j] = ap_maxi(h1, ap_sub(ex2, o2[j]));
      H[j] = Hn[j];
      imp = ap_maxu(imp, h1);
    }
    const int imax = grp_max<W>(max((int)(imp & 0xFFFF), (int)(imp >> 16)));
    if (act && imax >= minsc) {
      if (n_b == 0 || last_i + 1 != i) {
        if (gl == 0) blist[n_b] = (uint32_t)imax << 16 | (uint32_t)i;
        ++n_b;
        last_i = i, last_v = imax;
      } else if (last_v < imax) {
        if (gl == 0) blist[n_b - 1] = (uint32_t)imax << 16 | (uint32_t)i;
        last_i = i, last_v = imax;
      }
    }
    if (act && imax > gmax) {
      gmax = imax;
      te = i;
#pragma unroll
      for (int j = 0; j < NP; ++j) Hm[j] = Hn[j];
      if ((u8 && gmax + shift >= 255) || gmax >= endsc) run = false;
    }
    if (!(i + 1 < tlen)) run = false;
  }
  AlignRun r{!u8 || gmax + shift < 255 ? gmax : 255, te, -1, -1, -1};
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  const bool tail = live && (!u8 || r.score != 255);
  int mx = -1, qx = 0x7FFFFFFF;
#pragma unroll
  for (int j = 0; j < NP; ++j)
#pragma unroll
    for (int h = 0; h < 2; ++h)
      if (gl * NK + j + 5 * h < nlen) mx = max(mx, (int)((Hm[j] >> (16 * h)) & 0xFFFF));
  mx = grp_max<W>(mx);
#pragma unroll
  for (int j = 0; j < NP; ++j)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int x = gl * NK + j + 5 * h;
      if (x < nlen && (int)((Hm[j] >> (16 * h)) & 0xFFFF) == mx) qx = min(qx, x);
    }
  const int qe_min = -grp_max<W>(-qx);
  const int qe_best = nlen > 0 ? qe_min : -1;
  const int w = max_mat > 0 ? (r.score + max_mat - 1) / max_mat : 0;
  const int low = te - w, high = te + w;
  int best = -1, bte = -1;
  const int nbl = tail ? n_b : 0;
  const int nbmax = wave_max(nbl);
  for (int j0 = 0; j0 < nbmax; j0 += W) {
    const int j = j0 + gl;
    if (j < nbl) {
      const uint32_t e = blist[j];
      const int c = (int)(e & 0xFFFF), v = (int)(e >> 16);
      if ((c < low || c > high) && v > best) best = v, bte = c;
    }
  }
  const int vmax = grp_max<W>(best);
  const int te2 = -grp_max<W>(-(bte >= 0 && best == vmax ? bte : 0x7FFFFFFF));
  if (tail) {
    r.qe = qe_best;
    if (vmax > -1) r.score2 = vmax, r.te2 = te2;
  }
  return r;
}

// Groups of W lanes run tasks: W = 64, one task per workgroup iteration; W =
// 16, four consecutive tasks.  The 16-lane launch takes the queries up to
// seg_q, the 64-lane launch the longer ones.  LDS per group: b[] (2 B per
// target base) and the target.  pk: 0 every task of the launch, 1 (the PK
// kernel) the waves whose 16-lane tasks are all u8, 2 the other waves; both
// launches see the same per-wave test.  (When the gap costs and matrix keep
// the i16 tasks' scan values in 16 bits, the PK kernel takes every 16-lane
// task with pk = 0 and the 32-bit 16-lane launch is not made.)
template <int W, int NK, bool PK>
__global__ __launch_bounds__(64) void bsw_align_kernel(const BswDevBatch b, const BswParams p,
                                                       const int32_t* __restrict__ xtra, int32_t* __restrict__ out,
                                                       int max_tlen, int seg_q, int pk) {
  extern __shared__ __align__(16) unsigned char smem[];
  constexpr int G = 64 / W;  // groups per wave
  const int grp = lane_id() / W, gl = grp_lane<W>();
  const size_t bcap = ((size_t)max_tlen + 1) / 2;  // b[] appends are >= 2 columns apart
  uint32_t* const blist = reinterpret_cast<uint32_t*>(smem) + (size_t)grp * bcap;
  uint8_t* const tl = smem + 4 * (size_t)G * bcap + (size_t)grp * max_tlen;
  // bwa's shift (u8 bias) and max_mat from the 5 x 5 matrix, as ksw_qinit
  int mn = 127, mxm = 0;
  for (int a = 0; a < 25; ++a) mn = min(mn, (int)p.mat[a]), mxm = max(mxm, (int)p.mat[a]);
  const int shift = (256 - (int)(uint8_t)(int8_t)mn) & 0xFF;
  const long long ngroups = (b.n + G - 1) / G;
  for (long long g = blockIdx.x; g < ngroups; g += gridDim.x) {
    const long long task = g * G + grp;
    int qlen = 0, tlen = 0, xt = 0;
    if (task < b.n) qlen = b.qlen[task], tlen = b.tlen[task], xt = xtra[task];
    bool mine = task < b.n && (W == 64 ? qlen > seg_q : qlen <= seg_q);
    if (pk != 0) {
      const bool u8w = __ballot(mine && !(xt & kKswXByte)) == 0ull;
      mine = mine && u8w == (pk == 1);
    }
    const uint8_t* __restrict__ q = b.qbuf + (mine ? b.qoff[task] : 0);
    const uint8_t* __restrict__ tg = b.tbuf + (mine ? b.toff[task] : 0);
    if (mine)
      for (int i = gl; i < tlen; i += W) tl[i] = tg[i];
    __syncthreads();
    const bool u8 = (xt & kKswXByte) != 0;
    const int minsc = (xt & kKswXSubo) ? xt & 0xffff : 0x10000;
    const int endsc = (xt & kKswXStop) ? xt & 0xffff : 0x10000;
    auto qf = [&](int x) { return (int)q[x]; };
    auto tf = [&](int j) { return (int)tl[j]; };
    AlignRun r;
    if constexpr (PK) r = align_run_pk(p, mine, qlen, qf, tlen, tf, u8, shift, mxm, minsc, endsc, blist);
    else r = align_run<W, NK>(p, mine, qlen, qf, tlen, tf, u8, shift, mxm, minsc, endsc, blist);
    __syncthreads();  // the first pass's b[] reads before the second pass (which appends nothing)
    // bwa: reverse query[0, qe] and target[0, te] in place (the rest of the
    // target unchanged, full tlen), stop at the first score, no b[] list
    const bool second = mine && (xt & kKswXStart) && !((xt & kKswXSubo) && r.score < (xt & 0xffff));
    const int qe = r.qe, te = r.te;
    auto qr = [&](int x) { return (int)q[qe - x]; };
    auto tr = [&](int j) { return (int)tl[j <= te ? te - j : j]; };
    AlignRun rr;
    if constexpr (PK) rr = align_run_pk(p, second, qe + 1, qr, tlen, tr, u8, shift, mxm, 0x10000, r.score, blist);
    else rr = align_run<W, NK>(p, second, qe + 1, qr, tlen, tr, u8, shift, mxm, 0x10000, r.score, blist);
    int tb = -1, qb = -1;
    if (second && rr.score == r.score) tb = r.te - rr.te, qb = r.qe - rr.qe;
    if (mine && gl == 0) {
      int32_t* o = out + 7 * task;
      o[0] = r.score, o[1] = r.te, o[2] = r.qe, o[3] = r.score2, o[4] = r.te2, o[5] = tb, o[6] = qb;
    }
    __syncthreads();  // the next tasks rewrite the targets and the b[] lists
  }
}

int launch_bsw_align(const BswDevBatch& b, const BswParams& p, const int32_t* xtra, int max_qlen, int max_tlen,
                     int32_t* out, hipStream_t s, bool all_u8) {
  if (b.n <= 0) return FCS_OK;
  static_assert(3 * FCS_ALIGN_MAX_TLEN + 18 <= 160 * 1024, "FCS_ALIGN_MAX_TLEN must fit one wave's LDS");
  if (max_qlen > FCS_ALIGN_MAX_QLEN) return fail(FCS_ERR_UNSUPPORTED, "[E::fcship] ksw_align2: qlen > 1024 unsupported");
  {  // the profile holds mat + shift as bytes (shift = -min, as bwa's u8 bias)
    int mn = 127, mx = -128;
    for (int a = 0; a < 25; ++a) mn = std::min(mn, (int)p.mat[a]), mx = std::max(mx, (int)p.mat[a]);
    const int shift = (256 - (int)(uint8_t)(int8_t)mn) & 0xFF;
    if (mx + shift > 255)
      return fail(FCS_ERR_UNSUPPORTED, "[E::fcship] ksw_align2: a scoring matrix without a negative entry is unsupported");
  }
  const int mt = std::max(max_tlen, 1);
  // LDS per group: b[] + target = 3 B per target base (b[] entries: score << 16
  // | column, 4 B; an append needs the last entry's column != i - 1, so at most
  // ceil(tlen / 2) entries; scores <= 32767 and columns < 65536 fit 16 bits
  // each).  Queries <= kAlignSegQ
  // run four tasks per wave in 16-lane groups (NK = 10: slen * p <= 160) while
  // four groups' areas fit the CU's 160 KB; longer queries, and every query
  // when the target windows are longer (mate rescue with wide insert-size
  // distributions), run one task per wave.
  constexpr size_t kLdsMax = 160 * 1024;
  const size_t per_group = 4 * (((size_t)mt + 1) / 2) + (size_t)mt;
  const size_t lds16 = 4 * per_group + 16, lds64 = per_group + 16;
  if (lds64 > kLdsMax)
    return fail(FCS_ERR_UNSUPPORTED, "[E::fcship] ksw_align2: target longer than " +
                                         std::to_string((kLdsMax - 18) / 3) + " bases unsupported");
  const bool seg = lds16 <= kLdsMax;
  const int seg_q = seg ? kAlignSegQ : -1;
  auto go = [&](const void* kern, unsigned grid, size_t lds, auto launch) -> int {
    if (lds > 64 * 1024)
      FCS_HIP_CHECK(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    launch(grid, lds);
    FCS_HIP_CHECK(hipGetLastError());
    return FCS_OK;
  };
  int rc = FCS_OK;
  // 16-lane tasks: the packed kernel takes the waves of u8 tasks (when the gap
  // costs keep its 16-bit scan values in range) and, when the i16 tasks' range
  // fits as well, every wave; otherwise the 32-bit kernel takes the rest
  // (skipped when the caller knows every task is u8)
  int max_mat = 0;
  for (int a = 0; a < 25; ++a) max_mat = std::max(max_mat, (int)p.mat[a]);
  const bool packed = seg && align_packed_ok(255, 16, p.o_ins, p.e_ins);
  const bool packed16 = packed && align_packed_ok(align_i16_mmax(max_mat), 8, p.o_ins, p.e_ins);
  // one workgroup per four tasks (per task for W = 64): the dispatcher
  // balances the uneven task lengths and early exits
  const unsigned grid16 = (unsigned)std::min<long long>((b.n + 3) / 4, kAlignGridCap);
  if (packed)
    rc = go((const void*)bsw_align_kernel<16, 10, true>, grid16, lds16, [&](unsigned grid, size_t lds) {
      hipLaunchKernelGGL((bsw_align_kernel<16, 10, true>), dim3(grid), dim3(64), lds, s, b, p, xtra, out, mt, seg_q,
                         packed16 ? 0 : 1);
    });
  if (rc == FCS_OK && seg && !(packed && (all_u8 || packed16)))
    rc = go((const void*)bsw_align_kernel<16, 10, false>, grid16, lds16, [&](unsigned grid, size_t lds) {
      hipLaunchKernelGGL((bsw_align_kernel<16, 10, false>), dim3(grid), dim3(64), lds, s, b, p, xtra, out, mt, seg_q,
                         packed ? 2 : 0);
    });
  if (rc == FCS_OK && max_qlen > seg_q) {
    const unsigned grid = (unsigned)std::min<long long>(b.n, kAlignGridCap);
    // slots of 64 positions for slen * p (p = 16 u8 / 8 i16: at most qlen + 15)
    if (max_qlen + 15 <= 256)
      rc = go((const void*)bsw_align_kernel<64, 4, false>, grid, lds64, [&](unsigned g, size_t lds) {
        hipLaunchKernelGGL((bsw_align_kernel<64, 4, false>), dim3(g), dim3(64), lds, s, b, p, xtra, out, mt, seg_q, 0);
      });
    else
      rc = go((const void*)bsw_align_kernel<64, 17, false>, grid, lds64, [&](unsigned g, size_t lds) {
        hipLaunchKernelGGL((bsw_align_kernel<64, 17, false>), dim3(g), dim3(64), lds, s, b, p, xtra, out, mt, seg_q,
                           0);
      });
  }
  return rc;
}

}  // namespace fcs

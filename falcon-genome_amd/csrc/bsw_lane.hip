// ksw_extend2 with one task per LANE (gfx950), for the bwa-typical envelope:
// qlen <= 151, every score fits in int16, mat entries in [-16, 15].
//
// Algorithm: bwa ksw.c ksw_extend2, reached from
// /root/reference/src/workers/BWAWorker.cpp:134-166.
//
// Mapping (DESIGN.md §Banded SW, "lane kernel"): the wave takes 64 tasks of
// similar (qlen, tlen) from the device-sorted schedule; each lane runs bwa's
// row loop verbatim for its own task.  bwa's eh[] lives in registers as
// packed int16 pairs (h | e << 16), indexed by compile-time column numbers in
// a fully unrolled column loop, so the band bookkeeping (including the stale
// eh[] entries that bwa re-reads when the band grows) is reproduced exactly.
// Per cell: 2 ops for the profile score (5-bit fields selected by the query
// code), then bwa's max/add chain; no cross-lane traffic at all.  A kCW-column
// chunk is skipped when it lies outside the band of every live lane (one
// wave-wide min/max per row), and lanes whose task ended idle under EXEC.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <utility>

#include "fcship_internal.h"

namespace fcs {

__device__ __forceinline__ int wave_min_i(int v) { return -wave_max(-v); }

#ifdef FCS_BSW_STATS
// Diagnostic build only (tools/bsw_stats.py): per-bucket counters of waves,
// rows, fast / masked chunks and columns, useful lane-cells, working lane-rows.
__device__ unsigned long long g_bsw_stats[16][8];
__shared__ unsigned long long s_bsw_stats[8];
#define BSW_STAT(k, v) \
  do {                  \
    if (threadIdx.x == 0) s_bsw_stats[k] += (v); \
  } while (0)
#else
#define BSW_STAT(k, v) \
  do {                  \
  } while (0)
#endif

// Columns per chunk: the unit of the per-row band skip and of the
// fast (inside every lane's band) vs masked (some lane's band edge) choice.
constexpr int kCW = 8;

// Query profile by byte permute: the row's score table is two registers
// (s0 bytes = mat[tb][A, C, G, T], s1 byte 0 = mat[tb][N]) and every group of
// four columns has a selector dword in LDS (byte k = 4 + q for q in A..T, 0
// for N), so one v_perm_b32 yields the four columns' scores as signed bytes,
// which the h + s add reads in place (SDWA byte select).
template <int NC> constexpr int QG = NC / 4;  // selector dwords per lane

// nz | (x != 0) << sh as v_min_u32 + v_lshl_or_b32 (the compiler's own
// cmp/cndmask/or form costs one more VALU op per cell).
template <int SH>
__device__ __forceinline__ uint32_t or_nz_bit(uint32_t nz, uint32_t x) {
  uint32_t t, r;
  asm("v_min_u32 %0, %1, 1" : "=v"(t) : "v"(x));
  asm("v_lshl_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(t), "i"(SH), "v"(nz));
  return r;
}

// bwa's `M = M ? M + q[j] : 0` as min(hp + s, 32 hp): identical whenever hp > 0
// (s <= 15 < 31 hp), and <= 0 when hp == 0, where every consumer (max with
// e, f >= 0; max(M - oe, 0)) treats it exactly like 0.  No VCC select, so no
// VALU-writes-VCC hazard nops either.
__device__ __forceinline__ int diag_m(int hp, int s) { return min(hp + s, hp << 5); }

// Registers holding bwa's eh[] for NC columns: one per column (h | e << 16),
// or, when every score of the task fits a byte (B8), one per column pair
// (h0 | e0 << 8 | h1 << 16 | e1 << 24) — half the register file, so the
// 152-column kernel runs 3 waves per SIMD instead of 2.
template <int NC, bool B8> constexpr int EhN = B8 ? NC / 2 : NC;

// Words of the per-row "eh[j] != 0" bitmap (bit j for column j).
template <int NC> constexpr int NZW = (NC + 31) / 32;

template <int NC>
struct LaneRow {
  int beg, end, h1, f;
  uint32_t key;  // max over the row of (h << 16 | j): row max and its arg-max, ties to the larger j
  uint32_t kpend;  // key candidate of the even column of a pair, folded with the odd one by one v_max3
  uint32_t xst;    // byte-packed layout: the even column's new 16-bit entry, stored with the odd one
  uint32_t s0, s1;  // this row's score table (see QG)
  uint32_t sc;      // scores of the current four columns, one signed byte each
  uint32_t qn[kCW / 4], qx[kCW / 4];  // selectors of this chunk / the next (prefetched)
  uint32_t nz[NZW<NC>];
};

// m ? a : b per bit (v_bfi_b32); m is all-ones or zero here.  Inline asm so
// the compiler does not turn it back into compare + v_cndmask.
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
  return r;
}

// Row key update in pairs of columns: even J parks its candidate, odd J folds
// both with one v_max3 (chunks hold an even number of columns).
template <int J, int NC>
__device__ __forceinline__ void fold_key(LaneRow<NC>& r, uint32_t k) {
  if constexpr (J % 2 == 0) r.kpend = k;
  else r.key = max(max(r.key, r.kpend), k);
}

// New entry of column J: direct, or (B8) parked for the even column and
// stored with the odd one as one register (chunks hold whole pairs).
template <int J, int NC, bool B8>
__device__ __forceinline__ void eh_store(uint32_t (&eh)[(EhN<NC, B8>)], LaneRow<NC>& r, uint32_t v) {
  if constexpr (!B8) eh[J] = v;
  else if constexpr (J % 2 == 0) r.xst = v;
  else eh[J / 2] = r.xst | (v << 16);
}

// bwa's inner-loop body for column J.  MASKED = false: every working lane has
// J inside [beg, end).  MASKED = true (a chunk crossing some lane's band
// edge): the body runs unconditionally and bit J of `bm` (low half: J in
// [beg, end); high half: J in [beg, end]) selects what it may change, with
// sign-extended 1-bit masks and bit-selects instead of branches: eh[J] only
// for J in [beg, end] (at J == end bwa stores {h1, 0}), h1 / f / the row key
// only for J in [beg, end).  Lanes not working this row compute garbage they
// never read again.
template <int J, int NC, bool SYM, bool MASKED, bool B8>
__device__ __forceinline__ void lane_cell(uint32_t (&eh)[(EhN<NC, B8>)], const uint32_t* __restrict__ qs, LaneRow<NC>& r,
                                          const uint32_t bm, const int e_del, const int oe_del, const int e_ins,
                                          const int oe_ins) {
  constexpr int ES = B8 ? 8 : 16;  // bit offset of e inside a column entry
  uint32_t x;                      // this column's entry (h | e << ES)
  int hp, e;
  if constexpr (B8) {
    constexpr int sh = 16 * (J % 2);
    const uint32_t w = eh[J / 2];
    hp = (int)((w >> sh) & 0xFFu);
    e = (int)((w >> (sh + 8)) & 0xFFu);
    x = (w >> sh) & 0xFFFFu;
  } else {
    x = eh[J];
    hp = (int)(x & 0xFFFFu);
    e = (int)(x >> 16);
  }
  if constexpr (J % 4 == 0) r.sc = __builtin_amdgcn_perm(r.s0, r.s1, r.qn[(J % kCW) / 4]);
  const int s = (int)(int8_t)(uint8_t)(r.sc >> (8 * (J % 4)));
  const int M = diag_m(hp, s);
  const int h = max(max(M, e), r.f);
  int en, fn;
  if constexpr (SYM) {  // o_del == o_ins and e_del == e_ins (bwa defaults)
    const int mo = M - oe_del;
    en = max(max(e - e_del, mo), 0);
    fn = max(max(r.f - e_del, mo), 0);
  } else {
    en = max(max(e - e_del, M - oe_del), 0);
    fn = max(max(r.f - e_ins, M - oe_ins), 0);
  }
  if constexpr (!MASKED) {
    fold_key<J>(r, ((uint32_t)h << 16) | (uint32_t)J);
    r.f = fn;
    const uint32_t xn = (uint32_t)r.h1 | ((uint32_t)en << ES);
    eh_store<J, NC, B8>(eh, r, xn);
    r.h1 = h;
    r.nz[J / 32] = or_nz_bit<J % 32>(r.nz[J / 32], xn);
  } else {
    const uint32_t ms = (uint32_t)__builtin_amdgcn_sbfe(bm, J % kCW, 1);        // J in [beg, end)
    const uint32_t mx = (uint32_t)__builtin_amdgcn_sbfe(bm, kCW + J % kCW, 1);  // J in [beg, end]
    // a masked-off h contributes (0 << 16 | J): below any positive row max,
    // and a zero row max ends the task before its arg-max is used
    fold_key<J>(r, (((uint32_t)h & ms) << 16) | (uint32_t)J);
    r.f = (int)bfi(ms, (uint32_t)fn, (uint32_t)r.f);
    const uint32_t xn = (uint32_t)r.h1 | (((uint32_t)en & ms) << ES);
    const uint32_t xo = bfi(mx, xn, x);
    eh_store<J, NC, B8>(eh, r, xo);
    r.h1 = (int)bfi(ms, (uint32_t)h, (uint32_t)r.h1);
    r.nz[J / 32] = or_nz_bit<J % 32>(r.nz[J / 32], xo);  // bits outside [beg, end] are masked after the row
  }
}

// Bits [lo, hi) of a kCW-column chunk starting at column c0, clamped.
__device__ __forceinline__ uint32_t chunk_bits(int lo, int hi, int c0) {
  const int a = min(max(lo - c0, 0), kCW), b = min(max(hi - c0, 0), kCW);
  return ((1u << b) - 1u) & ~((1u << a) - 1u);
}

// Passes the chunk's inputs through an empty asm on each path.  Without it
// the compiler hoists the two paths' common head (every column's score and
// unpacking) above the fast/masked branch, keeping a chunk of temporaries
// live at once: spills in the 152-column kernels.
__device__ __forceinline__ void opaque(uint32_t& x) { asm volatile("" : "+v"(x)); }

template <int C, int L, int NC, bool B8>
__device__ __forceinline__ void opaque_chunk(uint32_t (&eh)[(EhN<NC, B8>)], LaneRow<NC>& r) {
  constexpr int j0 = kCW * C, j1 = kCW * C + L - 1;
  constexpr int e0 = B8 ? j0 / 2 : j0, e1 = B8 ? j1 / 2 : j1;
  [&]<int... K>(std::integer_sequence<int, K...>) {
    (opaque(eh[e0 + K]), ...);
  }(std::make_integer_sequence<int, e1 - e0 + 1>{});
  opaque(r.s0);
  opaque(r.s1);
}

template <int C, int NC, bool SYM, bool B8>
__device__ __forceinline__ void lane_chunk(uint32_t (&eh)[(EhN<NC, B8>)], const uint32_t* __restrict__ qs, LaneRow<NC>& r,
                                           const int cmin, const int cmax, const int bmax,
                                           const int emin, const int e_del,
                                           const int oe_del, const int e_ins, const int oe_ins) {
  constexpr int L = (NC - kCW * C) < kCW ? (NC - kCW * C) : kCW;  // last chunk may be partial
  static_assert(L % 2 == 0, "fold_key pairs columns within a chunk");
  if (kCW * C <= cmax && kCW * C + L - 1 >= cmin) {
    // selectors of the next chunk: in flight while this one computes
    if constexpr (kCW * (C + 1) < NC) {
#pragma unroll
      for (int k = 0; k < kCW / 4; ++k) r.qx[k] = qs[64 * ((kCW / 4) * (C + 1) + k)];
    }
    // Fast path when the whole chunk lies strictly inside the band of every
    // live lane (no per-column band test, no eh[end] write in this chunk):
    // a scalar test against the wave's largest beg and smallest end.
    if (bmax <= kCW * C && kCW * C + L - 1 < emin) {
      // Lanes not working this row run the body too: a lane that is done
      // never reads its state again, and an empty row ends its task (its
      // row-start h1 is kept aside).  No EXEC branch, so no join copies.
      BSW_STAT(2, 1);
      BSW_STAT(4, L);
      opaque_chunk<C, L, NC, B8>(eh, r);
      [&]<int... S>(std::integer_sequence<int, S...>) {
        (lane_cell<kCW * C + S, NC, SYM, false, B8>(eh, qs, r, 0u, e_del, oe_del, e_ins, oe_ins), ...);
      }(std::make_integer_sequence<int, L>{});
    } else {
      BSW_STAT(3, 1);
      BSW_STAT(5, L);
      opaque_chunk<C, L, NC, B8>(eh, r);
      const uint32_t bm = chunk_bits(r.beg, r.end, kCW * C) | (chunk_bits(r.beg, r.end + 1, kCW * C) << kCW);
      [&]<int... S>(std::integer_sequence<int, S...>) {
        (lane_cell<kCW * C + S, NC, SYM, true, B8>(eh, qs, r, bm, e_del, oe_del, e_ins, oe_ins), ...);
      }(std::make_integer_sequence<int, L>{});
    }
#pragma unroll
    for (int k = 0; k < kCW / 4; ++k) r.qn[k] = r.qx[k];
  }
}

// 64 consecutive tasks of the sorted schedule, starting at `base`.
template <int NC, bool SYM, bool B8>
__device__ __forceinline__ void lane_wave(const BswDevBatch& b, const BswParams& p, const int32_t* __restrict__ order,
                                          const long long base, const long long hi, int32_t* __restrict__ res,
                                          int64_t* __restrict__ cells_out, uint32_t* __restrict__ qsel,
                                          const uint32_t* __restrict__ mtab) {
  const int lane = threadIdx.x;
  const long long k = base + lane;
  const bool has = k < hi;
  const long long task = has ? order[k] : 0;
  int qlen = 0, tlen = 0, h0 = 1, w = 0;
  const uint8_t* __restrict__ q = b.qbuf;
  const uint8_t* __restrict__ tg = b.tbuf;
  if (has) {
    qlen = b.qlen[task];
    tlen = b.tlen[task];
    h0 = b.h0[task];
    w = b.w[task];
    q = b.qbuf + b.qoff[task];
    tg = b.tbuf + b.toff[task];
  }
  const int e_del = p.e_del, e_ins = p.e_ins, oe_del = p.o_del + p.e_del, oe_ins = p.o_ins + p.e_ins;

  // this lane's query selectors (columns past qlen score as N)
  uint32_t* __restrict__ qs = qsel + lane;
#pragma unroll
  for (int g = 0; g < QG<NC>; ++g) {
    uint32_t v = 0;
#pragma unroll
    for (int z = 0; z < 4; ++z) {
      const int j = 4 * g + z;
      const uint32_t qb = (j < qlen) ? (uint32_t)q[j] : 4u;
      v |= (qb < 4u ? 4u + qb : 0u) << (8 * z);
    }
    qs[64 * g] = v;
  }
  uint32_t eh[(EhN<NC, B8>)];
  const int h1v = h0 > oe_ins ? h0 - oe_ins : 0;
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    int hv = 0;
    if (j == 0) hv = h0;
    else if (j == 1) hv = (j <= qlen) ? h1v : 0;
    else hv = (j <= qlen) ? max(h1v - (j - 1) * e_ins, 0) : 0;
    if constexpr (B8) {
      if (j % 2 == 0) eh[j / 2] = (uint32_t)hv;
      else eh[j / 2] |= (uint32_t)hv << 16;
    } else {
      eh[j] = (uint32_t)hv;
    }
  }
  {
    const int max_ins = bwa_max_gap(qlen, p.max_mat, p.end_bonus, p.o_ins, e_ins);
    w = w < max_ins ? w : max_ins;
    const int max_del = bwa_max_gap(qlen, p.max_mat, p.end_bonus, p.o_del, e_del);
    w = w < max_del ? w : max_del;
  }

  int mx = h0, max_i = -1, max_j = -1, max_ie = -1, gscore = -1, max_off = 0;
  int ncell = 0;  // <= qlen * tlen < 2^31 in this envelope
  bool done = !has;
  LaneRow<NC> r;
  r.beg = 0;
  r.end = qlen;
  int tcur = (tlen > 0) ? tg[0] : 0;
  int tnext = (tlen > 1) ? tg[1] : 0;
  for (int i = 0;; ++i) {
    const bool alive = !done && i < tlen;
    if (__ballot(alive) == 0ull) break;
    const int tb = tcur;
    tcur = tnext;
    tnext = (alive && i + 2 < tlen) ? tg[i + 2] : 0;
    if (alive) {
      if (r.beg < i - w) r.beg = i - w;
      if (r.end > i + w + 1) r.end = i + w + 1;
      if (r.end > qlen) r.end = qlen;
      r.h1 = 0;
      if (r.beg == 0) {
        r.h1 = h0 - (p.o_del + e_del * (i + 1));
        if (r.h1 < 0) r.h1 = 0;
      }
    }
    const bool empty = alive && r.beg >= r.end;
    const bool work = alive && !empty;
    const int h1_row = r.h1;
    BSW_STAT(1, 1);
    BSW_STAT(7, __popcll(__ballot(work)));
    const int cmin = wave_min_i(work ? r.beg : (1 << 20));
    const int cmax = wave_max(work ? r.end : -1);
    const int bmax = wave_max(work ? r.beg : -1);
    const int emin = wave_min_i(work ? r.end : (1 << 20));
    {
      const uint2 t2 = reinterpret_cast<const uint2*>(mtab)[min((unsigned)tb, 4u)];
      r.s0 = t2.x;
      r.s1 = t2.y;
    }
    {
      // selectors of the row's first chunk (the wave's leftmost band column)
      const int c0 = min(max(cmin, 0), NC - 1) / kCW;
#pragma unroll
      for (int k = 0; k < kCW / 4; ++k) r.qn[k] = qs[64 * ((kCW / 4) * c0 + k)];
    }
    r.f = 0;
    r.key = 0;
#pragma unroll
    for (int k = 0; k < NZW<NC>; ++k) r.nz[k] = 0;
    [&]<int... C>(std::integer_sequence<int, C...>) {
      (lane_chunk<C, NC, SYM, B8>(eh, qs, r, cmin, cmax, bmax, emin, e_del, oe_del, e_ins, oe_ins), ...);
    }(std::make_integer_sequence<int, (NC + kCW - 1) / kCW>{});
    if (empty) {
      // bwa stores eh[end] = {h1, 0} and stops (beg >= end ends the row loop
      // for good), so only the to-end score of this row matters
      if (r.beg == qlen) {
        max_ie = gscore > h1_row ? max_ie : i;
        gscore = gscore > h1_row ? gscore : h1_row;
      }
      done = true;
    }
    if (work) {
      ncell += r.end - r.beg;
      if (r.end == qlen) {
        max_ie = gscore > r.h1 ? max_ie : i;
        gscore = gscore > r.h1 ? gscore : r.h1;
      }
      const int m = (int)(r.key >> 16), mj = (int)(r.key & 0xFFFFu);
      if (m == 0) {
        done = true;
      } else if (m > mx) {
        mx = m, max_i = i, max_j = mj;
        const int d = mj > i ? mj - i : i - mj;
        max_off = max_off > d ? max_off : d;
      } else if (p.zdrop > 0) {
        if (i - max_i > mj - max_j) {
          if (mx - m - ((i - max_i) - (mj - max_j)) * e_del > p.zdrop) done = true;
        } else {
          if (mx - m - ((mj - max_j) - (i - max_i)) * e_ins > p.zdrop) done = true;
        }
      }
      if (!done) {
        // bwa's trims: first non-zero eh in [beg, end) (else end), last non-zero
        // in [beg', end]; bits are kept for [beg, end] only, the entries bwa wrote this row
        int first = -1, last = -1;
#pragma unroll
        for (int k = 0; k < NZW<NC>; ++k) {
          // keep bits of [beg, end] only (masked chunks also set bits for untouched entries)
          const int a = min(max(r.beg - 32 * k, 0), 32), z = min(max(r.end + 1 - 32 * k, 0), 32);
          const uint32_t keep = (z >= 32 ? ~0u : ((1u << z) - 1u)) & (a >= 32 ? 0u : ~((1u << a) - 1u));
          const uint32_t wbits = r.nz[k] & keep;
          if (first < 0 && wbits) first = 32 * k + __builtin_ctz(wbits);
          if (wbits) last = 32 * k + 31 - __builtin_clz(wbits);
        }
        r.beg = (first >= 0) ? first : r.end;
        r.end = (last >= 0) ? min(last + 2, qlen) : min(r.beg + 1, qlen);
      }
    }
  }
#ifdef FCS_BSW_STATS
  {
    int tot = ncell;
    for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o);
    BSW_STAT(6, tot);
    BSW_STAT(0, 1);
  }
#endif
  if (has) {
    int32_t* o = res + 6 * task;
    o[0] = mx;
    o[1] = max_j + 1;
    o[2] = max_i + 1;
    o[3] = max_ie + 1;
    o[4] = gscore;
    o[5] = max_off;
    if (cells_out) cells_out[task] = ncell;
  }
}

}  // namespace fcs

#include "bsw_pair.h"

namespace fcs {

// Wave classes of the single extension launch, in dispatch order: workgroup w
// takes the w-th wave of the concatenation of these buckets' sorted ranges
// (64 tasks per lane wave, 128 per pair wave).  Widest columns first, and at
// equal width the one-task-per-lane waves (the longest per wave) before the
// pair waves, so the dispatcher packs longest-first (LPT) and short waves fill
// the tail.  Empty buckets contribute no waves; the grid is an upper bound
// (n / 64 + one per class), and the surplus workgroups come last and exit at
// once, in the tail.  One launch instead of one per bucket: concurrent
// near-empty bucket launches on side streams slowed the pair waves of a bwa
// batch by 1-5%.
constexpr int kExtClasses = 15;
__constant__ const int8_t kExtOrder[kExtClasses] = {
    9, 6, kBswPairBucket0 + 4,      // 152 columns: byte lane, lane, pair
    8, 5, kBswPairBucket0 + 3,      // 128
    7, 4, kBswPairBucket0 + 2,      // 96
    kBswPairBucket0 + 1, 3, 2,      // 64, 64, 48
    kBswPairBucket0, 1, 0};         // 32, 32, 16

template <bool SYM>
__global__ __launch_bounds__(64, 2) void bsw_ext_kernel(const BswDevBatch b, const BswParams p,
                                                       const int32_t* __restrict__ order,
                                                       const int64_t* __restrict__ bounds, int32_t* __restrict__ res,
                                                       int64_t* __restrict__ cells_out) {
  // pair waves: [chunk][lane] selector uint4s + 5 table dwords; lane waves:
  // [group][lane] selector dwords + 5 uint2 tables (the same bytes)
  constexpr int kSel = PCH<152> * 64;
  static_assert(QG<152> * 64 * 4 <= kSel * 16, "lane selectors fit the pair selector area");
  __shared__ uint4 smem[kSel + 3];
  long long t = blockIdx.x;
  int bucket = -1;
  long long lo = 0, hi = 0;
  for (int s = 0; s < kExtClasses; ++s) {
    const int c = kExtOrder[s];
    const int per = c >= kBswPairBucket0 ? 128 : 64;
    const long long blo = bounds[c], bhi = bounds[c + 1];
    const long long nw = (bhi - blo + per - 1) / per;
    if (t < nw) {
      bucket = c, lo = blo + per * t, hi = bhi;
      break;
    }
    t -= nw;
  }
  if (bucket < 0) return;
  const bool pair = bucket >= kBswPairBucket0;
  if (threadIdx.x < 5) {
    const int tb = threadIdx.x;
    if (pair) {
      uint32_t v = 0;
      for (int c = 0; c < 4; ++c) v |= (uint32_t)(uint8_t)(p.mat[tb * 5 + c] + p.pair_bias) << (8 * c);
      reinterpret_cast<uint32_t*>(smem + kSel)[tb] = v;
    } else {
      uint32_t s0 = 0;
      for (int c = 0; c < 4; ++c) s0 |= (uint32_t)(uint8_t)p.mat[tb * 5 + c] << (8 * c);
      reinterpret_cast<uint2*>(smem + kSel)[tb] = make_uint2(s0, (uint32_t)(uint8_t)p.mat[tb * 5 + 4]);
    }
  }
#ifdef FCS_BSW_STATS
  if (threadIdx.x < 8) s_bsw_stats[threadIdx.x] = 0, s_pair_stats[threadIdx.x] = 0;
#endif
  __syncthreads();
  uint32_t* const qsel = reinterpret_cast<uint32_t*>(smem);
  const uint32_t* const tab = reinterpret_cast<const uint32_t*>(smem + kSel);
  switch (bucket) {
    case kBswPairBucket0 + 4: pair_wave<152, SYM>(b, p, order, lo, hi, res, cells_out, smem, tab); break;
    case kBswPairBucket0 + 3: pair_wave<128, SYM>(b, p, order, lo, hi, res, cells_out, smem, tab); break;
    case kBswPairBucket0 + 2: pair_wave<96, SYM>(b, p, order, lo, hi, res, cells_out, smem, tab); break;
    case kBswPairBucket0 + 1: pair_wave<64, SYM>(b, p, order, lo, hi, res, cells_out, smem, tab); break;
    case kBswPairBucket0: pair_wave<32, SYM>(b, p, order, lo, hi, res, cells_out, smem, tab); break;
    case 9: lane_wave<152, SYM, true>(b, p, order, lo, hi, res, cells_out, qsel, tab); break;
    case 8: lane_wave<128, SYM, true>(b, p, order, lo, hi, res, cells_out, qsel, tab); break;
    case 7: lane_wave<96, SYM, true>(b, p, order, lo, hi, res, cells_out, qsel, tab); break;
    case 5: lane_wave<128, SYM, false>(b, p, order, lo, hi, res, cells_out, qsel, tab); break;
    case 4: lane_wave<96, SYM, false>(b, p, order, lo, hi, res, cells_out, qsel, tab); break;
    case 3: lane_wave<64, SYM, false>(b, p, order, lo, hi, res, cells_out, qsel, tab); break;
    case 2: lane_wave<48, SYM, false>(b, p, order, lo, hi, res, cells_out, qsel, tab); break;
    case 1: lane_wave<32, SYM, false>(b, p, order, lo, hi, res, cells_out, qsel, tab); break;
    default: lane_wave<16, SYM, false>(b, p, order, lo, hi, res, cells_out, qsel, tab); break;
  }
#ifdef FCS_BSW_STATS
  __syncthreads();
  if (threadIdx.x < 8) {
    if (pair) atomicAdd(&g_pair_stats[bucket - kBswPairBucket0][threadIdx.x], s_pair_stats[threadIdx.x]);
    else atomicAdd(&g_bsw_stats[bucket][threadIdx.x], s_bsw_stats[threadIdx.x]);
  }
#endif
}

#ifdef FCS_BSW_STATS
extern "C" int fcs_bsw_stats_read(unsigned long long* out, int reset) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bsw_stats), sizeof(g_bsw_stats)) != hipSuccess) return -1;
  if (reset) {
    static const unsigned long long z[16][8] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_bsw_stats), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

// Bucket of a task: 0..6 = 16-bit lane kernels with 16/32/48/64/96/128/152
// register columns (152 = bwa reads up to 151 bp); 7..9 = byte-packed lane
// kernels with 96/128/152 columns for tasks whose scores all fit a byte (the
// register saving buys a third wave per SIMD there; at <= 64 columns the
// 16-bit layout already runs 3-4 waves and is cheaper per cell);
// kBswPairBucket0..+4 = two-tasks-per-lane kernels (bsw_pair.h) with
// 32/64/96/128/152 columns for tasks whose biased scores fit a byte and whose
// query holds no N (`acgt`), with tlen < 1024 (the pair kernel's 16-bit row
// bookkeeping); kBswWideBucket = wave-per-task kernel
// (long queries, scores beyond int16, matrices beyond 5 bits).
__device__ __forceinline__ int bsw_bucket(int qlen, int tlen, int h0, bool acgt, const BswParams& p) {
  const long long bound = (long long)h0 + (long long)qlen * p.max_mat;  // no cell can score more
  const int need = qlen + 1;
  if (p.pair_ok && acgt && h0 > 0 && need <= 152 && tlen < 1024 && bound + p.pair_cg - 1 <= 255)
    return kBswPairBucket0 + (need <= 32 ? 0 : need <= 64 ? 1 : need <= 96 ? 2 : need <= 128 ? 3 : 4);
  if (!p.lane_ok || h0 <= 0 || bound >= 32000) return kBswWideBucket;
  if (need <= 16) return 0;
  if (need <= 32) return 1;
  if (need <= 48) return 2;
  if (need <= 64) return 3;
  const int c = need <= 96 ? 4 : need <= 128 ? 5 : need <= 152 ? 6 : -1;
  if (c < 0) return kBswWideBucket;
  if (bound < 256) return c + 3;
  // 16-bit entries for 152 columns do not fit the extension kernel's 256
  // VGPRs (the lane wave spilled 16 of them, in the row loop): such tasks
  // (qlen > 127 with a query N or scores >= 256 — rare under bwa) take the
  // wave-per-task kernel instead
  return c == 6 ? kBswWideBucket : c;
}

// No base outside A/C/G/T (code >= 4) among the n query bytes at s: aligned
// 16-byte loads (the caller's buffers come from hipMalloc, so an aligned block
// holding one of the task's bytes lies inside the allocation), edge bytes masked.
__device__ __forceinline__ bool bsw_query_acgt(const uint8_t* s, int n) {
  if (n <= 0) return true;
  const uintptr_t b = (uintptr_t)s, e = b + (uintptr_t)n, a0 = b & ~(uintptr_t)15;
  uint32_t any = 0;
  for (uintptr_t blk = a0; blk < e; blk += 16) {
    const uint4 v = *reinterpret_cast<const uint4*>(blk);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uintptr_t d = blk + 4 * q;
      uint32_t keep = 0xFFFFFFFFu;
      if (d < b) keep = b - d >= 4 ? 0u : ~0u << (8 * (b - d));
      if (d + 4 > e) keep &= d >= e ? 0u : ~0u >> (8 * (d + 4 - e));
      any |= w[q] & keep;
    }
  }
  return (any & 0xFCFCFCFCu) == 0;
}

__global__ void bsw_keys_kernel(const BswDevBatch b, const BswParams p, uint32_t* __restrict__ keys,
                                int32_t* __restrict__ idx) {
  const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= b.n) return;
  const int qlen = b.qlen[k], tlen = b.tlen[k], h0 = b.h0[k];
  // the pair kernels score target N rows from their table but take queries
  // without N only (a query N would need a fifth score per column)
  const bool acgt = p.pair_ok && qlen < 152 && bsw_query_acgt(b.qbuf + b.qoff[k], qlen);
  const uint32_t bk = (uint32_t)bsw_bucket(qlen, tlen, h0, acgt, p);
  // Rows a task is expected to run: an extension that keeps matching peaks
  // near row qlen with score ~h0 + qlen*max_mat and then decays by e_del per
  // row until the row max hits 0 (bwa's m == 0 exit), capped by tlen.  Tasks
  // of a wave sorted by this run about as long as each other, so fewer lanes
  // idle behind the wave's longest task.
  const long long est = min((long long)tlen, (long long)qlen +
                                                 ((long long)h0 + (long long)qlen * p.max_mat) / max(p.e_del, 1) + 1);
  // longest first inside a bucket (the sort is ascending): the last waves of a
  // launch are the short ones, so the launch's tail is short.  24-bit key (three
  // 8-bit radix passes): bucket | qlen / 4 | h0 | rows beyond qlen / 4, each
  // descending.  h0 right after the (coarse) query length groups tasks whose
  // band of nonzero cells grows alike (its width follows the running score),
  // so a wave's band union wastes fewer lane-columns: C3 +4% over ordering by
  // exact qlen then rows (gpurun_out/k1, k2).  The clamps only touch
  // wave-per-task tasks; the order never changes results.
  {
    const uint32_t q = 63u - (uint32_t)(min(max(qlen, 0), 255) >> 2);
    const uint32_t h = 255u - (uint32_t)min(max(h0, 0), 255);
    const uint32_t e = 63u - (uint32_t)(min(max(est - (long long)qlen, 0LL), 255LL) >> 2);
    keys[k] = (bk << kBswKeyBucketShift) | (q << 14) | (h << 6) | e;
  }
  idx[k] = (int32_t)k;
}

// bounds[c] = first sorted position whose bucket >= c, c = 0..kBswWideBucket + 1.
__global__ void bsw_bounds_kernel(const uint32_t* __restrict__ keys, long long n, int64_t* __restrict__ bounds) {
  const long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (k > n) return;
  const int cur = (k < n) ? (int)(keys[k] >> kBswKeyBucketShift) : kBswWideBucket + 1;
  const int prev = (k > 0) ? (int)(keys[k - 1] >> kBswKeyBucketShift) : -1;
  for (int c = prev + 1; c <= cur; ++c) bounds[c] = k;
}

int launch_bsw_extend_sorted(const BswDevBatch& b, const BswParams& p, int max_qlen, int max_tlen, int32_t* res,
                             int64_t* cells, const BswWorkspace& ws, hipStream_t s) {
  if (b.n <= 0) return FCS_OK;
  if (b.n > ws.cap) return fail(FCS_ERR_INVALID, "[E::fcship] SW batch larger than its plan");
  const int bs = 256;
  hipLaunchKernelGGL(bsw_keys_kernel, dim3((unsigned)((b.n + bs - 1) / bs)), dim3(bs), 0, s, b, p, ws.keys_in, ws.idx_in);
  FCS_HIP_CHECK(hipGetLastError());
  size_t tmp = ws.tmp_bytes;
  FCS_HIP_CHECK(sort_pairs_u32(ws.tmp, tmp, ws.keys_in, ws.keys_out, ws.idx_in, ws.idx_out, (int)b.n, s, kBswKeyBits));
  hipLaunchKernelGGL(bsw_bounds_kernel, dim3((unsigned)((b.n + 1 + bs - 1) / bs)), dim3(bs), 0, s, ws.keys_out,
                     (long long)b.n, ws.bounds);
  FCS_HIP_CHECK(hipGetLastError());
  // one launch for every pair and lane bucket (an upper bound of their waves)
  const unsigned grid = (unsigned)((b.n + 63) / 64 + kExtClasses);
  if (p.o_del == p.o_ins && p.e_del == p.e_ins)
    hipLaunchKernelGGL(bsw_ext_kernel<true>, dim3(grid), dim3(64), 0, s, b, p, ws.idx_out, ws.bounds, res, cells);
  else
    hipLaunchKernelGGL(bsw_ext_kernel<false>, dim3(grid), dim3(64), 0, s, b, p, ws.idx_out, ws.bounds, res, cells);
  FCS_HIP_CHECK(hipGetLastError());
  // wave-per-task kernel over the sorted tail (empty in bwa batches: its grid
  // of exits runs after the extension launch, not beside it)
  return launch_bsw_extend_wide(b, p, max_qlen, max_tlen, res, cells, ws.idx_out, ws.bounds, s);
}

}  // namespace fcs

// ksw_extend2 with TWO tasks per lane in packed 16-bit arithmetic (gfx950
// VOP3P), for the bwa-typical envelope: qlen <= 151, every score of the task
// below 256 after the score bias, no N in the query, h0 > 0.
//
// Algorithm: bwa ksw.c ksw_extend2, reached from
// /root/reference/src/workers/BWAWorker.cpp:134-166.  Same row loop, band
// bookkeeping, z-drop and trims as the one-task lane kernel (bsw_lane.hip);
// what changes is the data layout of a cell, so that every VALU op of the
// cell body works on two tasks at once (task A = low 16 bits, B = high).
//
// Layout:
//  * bwa's eh[j] of both tasks in ONE register: bytes [eA, hA, eB, hB].
//  * Values are carried in the "x256" domain: a 16-bit half holds v << 8.
//    Unpacking is one AND (h) and one packed shift (e); repacking the new
//    entry {h1, e'} of both tasks is one v_perm_b32.
//  * Scores: one v_perm_b32 per two columns turns the per-lane selector
//    dword [qA_j, qA_j+1, 4+qB_j, 4+qB_j+1] and the row's two 4-byte score
//    tables (mat[t][0..3] + bias, t = this row's target base of A / B, N
//    included) into
//    the four biased scores; v_pk_mad_u16 (x256, which also drops the other
//    column's byte) or AND+add puts them in the x256 domain on top of h.
//  * bwa's `M = M ? M + q : 0` is min(h + s', gate) - bias with
//    gate = sat(C * h) (0 iff h == 0, above any h + s' otherwise), all
//    saturating packed ops; every later max / saturating subtract is exactly
//    bwa's max(., 0) arithmetic.
//  * Row max and arg-max: packed max of (h << 8 | j); ties go to the larger j
//    as in bwa.  Trims: at row end, scans of the stored entries chunk by
//    chunk from the band's edges (first / last non-zero entry per task half;
//    chunk_nz / last_col), usually one chunk each since the band moves about
//    a column per row.
//
// Band edges without per-cell predicates:
//  * left: every eh[] entry left of a task's `beg` is kept at zero (bwa's
//    trims only skip zero entries; the one entry a band cut (i - w) leaves
//    behind per row is zeroed in the row it leaves the band).  Zero inputs
//    make zero outputs, so the chain (h1, f) enters `beg` as zero exactly as
//    bwa restarts it; only chunks holding a cut column mask their inputs.
//  * right: chunks reaching some task's `end` run with per-half masks: no
//    e' at j == end (bwa stores {h1, 0}), entries beyond `end` keep their
//    stale values (bwa re-reads them when the band grows), and h1 at `end` is
//    captured for the to-end score.
// Device code only: included by bsw_lane.hip, whose single extension launch
// (bsw_ext_kernel) runs pair waves and lane waves side by side.
#pragma once
#include <hip/hip_runtime.h>

#include <utility>

#include "fcship_internal.h"

namespace fcs {

#ifdef FCS_BSW_STATS
// Diagnostic build only (tools/bsw_stats.py): per pair bucket, counters of
// waves, rows, fast / masked chunks, useful cells, working and alive task-rows,
// and the row band union width.
__device__ unsigned long long g_pair_stats[5][8];
__shared__ unsigned long long s_pair_stats[8];
#define PAIR_STAT(k, v) \
  do {                  \
    if (threadIdx.x == 0) s_pair_stats[k] += (v); \
  } while (0)
extern "C" int fcs_bsw_pair_stats_read(unsigned long long* out, int reset) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pair_stats), sizeof(g_pair_stats)) != hipSuccess) return -1;
  if (reset) {
    static const unsigned long long z[5][8] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_pair_stats), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#else
#define PAIR_STAT(k, v) \
  do {                  \
  } while (0)
#endif

namespace {

// ---------------------------------------------------------------- packed ops
// Clang vector builtins (not inline asm) wherever a pattern exists, so the
// hazard recognizer sees real instructions and inserts no defensive s_nop.
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
typedef int16_t i16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 V(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ uint32_t U(u16x2 x) { return __builtin_bit_cast(uint32_t, x); }

__device__ __forceinline__ uint32_t pk_max(uint32_t a, uint32_t b) { return U(__builtin_elementwise_max(V(a), V(b))); }
__device__ __forceinline__ uint32_t pk_min(uint32_t a, uint32_t b) { return U(__builtin_elementwise_min(V(a), V(b))); }
// max(a - s, 0) per half (v_pk_sub_u16 clamp)
__device__ __forceinline__ uint32_t pk_subs(uint32_t a, uint32_t s) {
  return U(__builtin_elementwise_sub_sat(V(a), V(s)));
}
__device__ __forceinline__ uint32_t pk_add(uint32_t a, uint32_t b) { return U(V(a) + V(b)); }
// a * s + c per half (mod 2^16): v_pk_mad_u16 (s must not be a compile-time
// power of two, or the compiler splits it into a shift and an add)
__device__ __forceinline__ uint32_t pk_mad(uint32_t a, uint32_t s, uint32_t c) { return U(V(a) * V(s) + V(c)); }
// min(a * s, 65535) per half: no builtin for a saturating multiply-add
__device__ __forceinline__ uint32_t pk_gate(uint32_t a, uint32_t s) {
  uint32_t r;
  asm("v_pk_mad_u16 %0, %1, %2, 0 op_sel_hi:[1,1,0] clamp" : "=v"(r) : "v"(a), "s"(s));
  return r;
}
__device__ __forceinline__ uint32_t pk_shl8(uint32_t a) { return U(V(a) << (u16x2)(8)); }
// (a != 0) per half as 0 / 1, with `one` a runtime 0x00010001 (a literal 1
// turns min(a, 1) into compare + select)
__device__ __forceinline__ uint32_t pk_nz(uint32_t a, uint32_t one) { return pk_min(a, one); }
// all-ones per half where (signed) a < b.  The shift is inline asm: as a
// builtin, LLVM turns the sign extraction back into compares + selects.
__device__ __forceinline__ uint32_t pk_lt(uint32_t a, uint32_t b) {
  const uint32_t d = __builtin_bit_cast(uint32_t, __builtin_bit_cast(i16x2, a) - __builtin_bit_cast(i16x2, b));
  uint32_t r;
  asm("v_pk_ashrrev_i16 %0, 15, %1 op_sel_hi:[0,1]" : "=v"(r) : "v"(d));
  return r;
}
// In-place updates of eh[] entries (tied operands): every path through a
// chunk leaves an entry in its own register, so chunk joins need no copies.
__device__ __forceinline__ void and_in_place(uint32_t& x, uint32_t m) { asm("v_and_b32 %0, %0, %1" : "+v"(x) : "v"(m)); }
// A copy in a register of its own (the entry's register stays with eh[]).
__device__ __forceinline__ uint32_t vcopy(uint32_t x) {
  uint32_t r;
  asm("v_mov_b32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}
// x = m ? x : k per bit
__device__ __forceinline__ void bfi_in_place(uint32_t& x, uint32_t m, uint32_t k) {
  asm("v_bfi_b32 %0, %1, %0, %2" : "+v"(x) : "v"(m), "v"(k));
}
// Returns x through a volatile asm: values derived from the result cannot be
// computed before the enclosing conditional block, so the edge passes stay
// behind their branch instead of being speculated into every chunk.
__device__ __forceinline__ uint32_t launder(uint32_t x) {
  asm volatile("" : "+v"(x));
  return x;
}
__device__ __forceinline__ uint32_t pbfi(uint32_t m, uint32_t a, uint32_t b) { return (m & a) | (~m & b); }
// m ? a : b per bit in one full-rate v_bitop3_b32 (as phmm's sel_v): compiler
// selects on a compare come out as VOP2 v_cndmask_b32 reading VCC, ~20 cycles
// each on gfx950
__device__ __forceinline__ uint32_t bsel(uint32_t m, uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xe4" : "=v"(r) : "v"(a), "v"(b), "v"(m));
  return r;
}
// v_ffbl_b32 / v_ffbh_u32 (lowest set bit / leading zeros) OR a word offset:
// both return ~0u for a zero word, so an empty word yields ~0u and a v_min_u32
// chain finds the first / last set bit.  As builtins (ctz with a -1 default)
// the compiler turns that min chain into compare + VOP2 select pairs.
__device__ __forceinline__ uint32_t ffbl_or(uint32_t w, uint32_t off) {
  uint32_t r;
  asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(w));
  return r | off;
}
__device__ __forceinline__ uint32_t ffbh_or(uint32_t w, uint32_t off) {
  uint32_t r;
  asm("v_ffbh_u32 %0, %1" : "=v"(r) : "v"(w));
  return r | off;
}

__device__ __forceinline__ uint32_t pack2(int a, int b) { return ((uint32_t)a & 0xFFFFu) | ((uint32_t)b << 16); }

// ---------------------------------------------------------------- layout
constexpr int kPW = 8;  // columns per chunk (skip / fast / masked unit)
template <int NC> constexpr int PCH = (NC + kPW - 1) / kPW;  // chunks

// Wave-uniform constants of the cell body (x256 domain, both halves).
struct PairK {
  uint32_t k256;       // 0x0100 | 0x0100 << 16
  uint32_t one;        // 0x0001 | 0x0001 << 16
  uint32_t cg;         // gate multiplier C = max biased score + 1
  uint32_t bias;       // score bias << 8
  uint32_t oed, ed, oei, ei;  // (o + e) << 8 and e << 8 of deletions / insertions
};

template <int NC>
struct PairRow {
  uint32_t F, H1, KEY, CAP;
  uint32_t tabA, tabB;       // biased score tables of this row's target bases
  uint32_t BEGM1, END;       // per half: beg - 1, end
  uint32_t O;                // scores of the current column pair
  uint4 sel[2];              // selector dwords, double-buffered by chunk parity
};

// bwa's inner-loop body for column J of both tasks, the same code for every
// chunk.  Edge chunks wrap it in pair_chunk's pre-pass (inputs outside
// [beg, end) zeroed) and post-pass (entries beyond end restored).
template <int J, int NC, bool SYM>
__device__ __forceinline__ void pair_cell(uint32_t (&eh)[NC], PairRow<NC>& r, const PairK& k) {
  constexpr uint32_t JJ = (uint32_t)J | ((uint32_t)J << 16);
  const uint32_t w = eh[J];
  const uint32_t HP = w & 0xFF00FF00u;
  const uint32_t E = pk_shl8(w);
  uint32_t t;
  if constexpr (J % 2 == 0) {
    constexpr int g = (J % kPW) / 2;
    const uint4& cs = r.sel[(J / kPW) & 1];
    const uint32_t sl = g == 0 ? cs.x : g == 1 ? cs.y : g == 2 ? cs.z : cs.w;
    r.O = __builtin_amdgcn_perm(r.tabB, r.tabA, sl);
    t = pk_mad(r.O, k.k256, HP);
  } else {
    t = pk_add(r.O & 0xFF00FF00u, HP);
  }
  const uint32_t M = pk_subs(pk_min(t, pk_gate(HP, k.cg)), k.bias);
  const uint32_t H = pk_max(pk_max(M, E), r.F);
  const uint32_t MOd = pk_subs(M, k.oed);
  const uint32_t EN = pk_max(pk_subs(E, k.ed), MOd);
  const uint32_t MOi = SYM ? MOd : pk_subs(M, k.oei);
  const uint32_t Fn = pk_max(pk_subs(r.F, k.ei), MOi);
  // in place (tied operand), so no chunk path moves eh[] between registers;
  // edge chunks copy the entries they must restore in their pre-pass
  asm("v_perm_b32 %0, %1, %2, %3" : "+v"(eh[J]) : "v"(r.H1), "v"(EN), "s"(0x07030501u));
  r.KEY = pk_max(r.KEY, H | JJ);
  r.H1 = H;
  r.F = Fn;
}

// One kPW-column chunk of the row.  A chunk some task's band edge touches
// (its end, or a band-cut column on the left) runs the same cell body with
// its inputs outside [beg, end) zeroed first.  Zero inputs make the body
// compute exactly bwa's edge behaviour: left of beg zeros (so h1 = f = 0
// enter beg), at end the entry {h1, 0} bwa stores, and beyond end only the
// decaying f chain, which stays below the row max (f <= max M - (o + e)), so
// the row's arg-max is unaffected.  The post-pass then puts back the stale
// entries beyond end that bwa leaves untouched, and takes h1 at end (for the
// to-end score).  Bits of the trims' bitmap beyond end are masked per row.
template <int C, int NC, bool SYM>
__device__ __forceinline__ void pair_chunk(uint32_t (&eh)[NC], const uint4* __restrict__ qs, PairRow<NC>& r,
                                           const PairK& k, const uint32_t proc, const uint32_t edges,
                                           const uint32_t cuts) {
  constexpr int j0 = kPW * C, L = (NC - j0) < kPW ? (NC - j0) : kPW;
  static_assert(L % 2 == 0, "column pairs share one score perm");
  if (!((proc >> C) & 1u)) return;
  if constexpr (C + 1 < PCH<NC>) r.sel[(C + 1) & 1] = qs[64 * (C + 1)];
  const bool left = (cuts >> C) & 1u;
  const bool edge = (edges >> C) & 1u;
  uint32_t keep[L];
  if (edge) {
    PAIR_STAT(3, 1);
    const uint32_t endv = launder(r.END);
    [&]<int... S>(std::integer_sequence<int, S...>) __attribute__((always_inline)) {
      ((keep[S] = vcopy(eh[j0 + S]), and_in_place(eh[j0 + S], pk_lt((uint32_t)(j0 + S) * 0x10001u, endv))), ...);  // j < end
    }(std::make_integer_sequence<int, L>{});
    if (left) {
      const uint32_t begv = launder(r.BEGM1);
      [&]<int... S>(std::integer_sequence<int, S...>) __attribute__((always_inline)) {
        (and_in_place(eh[j0 + S], pk_lt(begv, (uint32_t)(j0 + S) * 0x10001u)), ...);  // j >= beg
      }(std::make_integer_sequence<int, L>{});
    }
  } else {
    PAIR_STAT(2, 1);
  }
  [&]<int... S>(std::integer_sequence<int, S...>) __attribute__((always_inline)) {
    (pair_cell<j0 + S, NC, SYM>(eh, r, k), ...);
  }(std::make_integer_sequence<int, L>{});
  if (edge) {
    const uint32_t endv = launder(r.END);
    uint32_t mx = pk_lt((uint32_t)(j0 - 1) * 0x10001u, endv);  // column j0 <= end
    [&]<int... S>(std::integer_sequence<int, S...>) __attribute__((always_inline)) {
      (([&] __attribute__((always_inline)) {
         const uint32_t me = pk_lt((uint32_t)(j0 + S) * 0x10001u, endv);  // j < end
         r.CAP = pbfi(mx ^ me, eh[j0 + S], r.CAP);                          // j == end: {h1, 0}
         bfi_in_place(eh[j0 + S], mx, keep[S]);                             // j > end: stale entry back
         mx = me;
       }()),
       ...);
    }(std::make_integer_sequence<int, L>{});
  }
}

// Non-zero map of chunk C's stored entries: bit S of each half set when column
// j0 + S of that task has h or e != 0; columns beyond the task's end (stale
// entries bwa leaves in place) masked out.
template <int C, int NC>
__device__ __forceinline__ uint32_t chunk_nz(const uint32_t (&eh)[NC], uint32_t one, int endA, int endB) {
  constexpr int j0 = kPW * C, L = (NC - j0) < kPW ? (NC - j0) : kPW;
  uint32_t b = 0;
  [&]<int... S>(std::integer_sequence<int, S...>) __attribute__((always_inline)) {
    ((b |= pk_nz(eh[j0 + S], one) << S), ...);
  }(std::make_integer_sequence<int, L>{});
  const uint32_t ka = __builtin_amdgcn_ubfe(~0u, 0, (uint32_t)min(max(endA + 1 - j0, 0), L));
  const uint32_t kb = __builtin_amdgcn_ubfe(~0u, 0, (uint32_t)min(max(endB + 1 - j0, 0), L));
  return b & (ka | (kb << 16));
}
// ~(last set column) of chunk c's map w (one task's half), ~0u when w == 0:
// a v_min_u32 chain over chunks then keeps the highest column.
__device__ __forceinline__ uint32_t last_col(uint32_t w, int c) {
  uint32_t h;
  asm("v_ffbh_u32 %0, %1" : "=v"(h) : "v"(w));
  const uint32_t none = (uint32_t)((int)h >> 31);
  return bsel(none, ~0u, ~((uint32_t)(kPW * c + 31) - h));
}

// bwa's per-task scalar state.
struct PairTask {
  long long id;
  const uint8_t* tg;
  int qlen, tlen, h0, w;
  int beg, end;
  int mx, max_i, max_j, max_ie, gscore, max_off, ncell;
  bool done;
};

__device__ __forceinline__ void task_load(PairTask& T, const BswDevBatch& b, const BswParams& p, const int32_t* order,
                                          long long k, long long hi) {
  T.done = k >= hi;
  T.id = T.done ? -1 : order[k];
  T.qlen = T.tlen = T.w = 0;
  T.h0 = 1;
  T.tg = b.tbuf;
  if (!T.done) {
    T.qlen = b.qlen[T.id];
    T.tlen = b.tlen[T.id];
    T.h0 = b.h0[T.id];
    T.w = b.w[T.id];
    T.tg = b.tbuf + b.toff[T.id];
  }
  const int max_ins = bwa_max_gap(T.qlen, p.max_mat, p.end_bonus, p.o_ins, p.e_ins);
  T.w = T.w < max_ins ? T.w : max_ins;
  const int max_del = bwa_max_gap(T.qlen, p.max_mat, p.end_bonus, p.o_del, p.e_del);
  T.w = T.w < max_del ? T.w : max_del;
  T.beg = 0;
  T.end = T.qlen;
  T.mx = T.h0;
  T.max_i = T.max_j = T.max_ie = -1;
  T.gscore = -1;
  T.max_off = 0;
  T.ncell = 0;
}

// ---------------------------------------------------------------- bookkeeping
// bwa's per-row scalar logic for both tasks at once: every field is a pair of
// signed 16-bit halves (task A low, B high) and every condition an all-ones
// half mask, so the row start / end costs the same as for one task.  The
// envelope keeps every value in range (tlen < 1024, e_del, e_ins <= 16).
__device__ __forceinline__ i16x2 SI(uint32_t x) { return __builtin_bit_cast(i16x2, x); }
__device__ __forceinline__ uint32_t SU(i16x2 x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ uint32_t s_add(uint32_t a, uint32_t b) { return SU(SI(a) + SI(b)); }
__device__ __forceinline__ uint32_t s_sub(uint32_t a, uint32_t b) { return SU(SI(a) - SI(b)); }
__device__ __forceinline__ uint32_t s_mul(uint32_t a, uint32_t b) { return SU(SI(a) * SI(b)); }
__device__ __forceinline__ uint32_t s_max(uint32_t a, uint32_t b) { return SU(__builtin_elementwise_max(SI(a), SI(b))); }
__device__ __forceinline__ uint32_t s_min(uint32_t a, uint32_t b) { return SU(__builtin_elementwise_min(SI(a), SI(b))); }
// all-ones per half where a == b (one = 0x00010001 at run time)
__device__ __forceinline__ uint32_t s_eq(uint32_t a, uint32_t b, uint32_t one) {
  return U(V(pk_min(a ^ b, one)) - V(one));
}

struct PairState {
  uint32_t QLEN, TLEN, W, H0, BEG, END;
  uint32_t MX, MAXI, MAXJ, MAXIE, GS, MOFF, DONE;
  uint32_t NCA, NCB;  // evaluated cells (32-bit per task)
};

__device__ __forceinline__ int pair_eh_init(const PairTask& T, int j, int h1v, int e_ins) {
  if (j == 0) return T.h0;
  if (j > T.qlen) return 0;
  if (j == 1) return h1v;
  return max(h1v - (j - 1) * e_ins, 0);
}

// 128 consecutive tasks of the sorted schedule (lane l: 2l and 2l + 1), from `base`.
template <int NC, bool SYM>
__device__ __forceinline__ void pair_wave(const BswDevBatch& b, const BswParams& p, const int32_t* __restrict__ order,
                                          const long long base, const long long hi, int32_t* __restrict__ res,
                                          int64_t* __restrict__ cells_out, uint4* __restrict__ qsel,
                                          const uint32_t* __restrict__ ptab) {
  const int lane = threadIdx.x;
  PairTask A, B;
  task_load(A, b, p, order, base + 2 * lane, hi);
  task_load(B, b, p, order, base + 2 * lane + 1, hi);

  // selector dwords [qA_j, qA_j+1, 4 + qB_j, 4 + qB_j+1], four per chunk.
  // Each query is read as the aligned dwords that cover it (every load issued
  // before any use: one memory round trip per wave instead of one per chunk),
  // realigned to column 0 by v_alignbyte, and cut at qlen (columns past qlen
  // read as code 0, as bwa never scores them).
  uint4* __restrict__ qs = qsel + lane;
  {
    constexpr int NQ = PCH<NC> * 2;  // query words: 4 columns each
    const uint8_t* qa = A.done ? b.qbuf : b.qbuf + b.qoff[A.id];
    const uint8_t* qb = B.done ? b.qbuf : b.qbuf + b.qoff[B.id];
    const uint32_t* wa = reinterpret_cast<const uint32_t*>((uintptr_t)qa & ~(uintptr_t)3);
    const uint32_t* wb = reinterpret_cast<const uint32_t*>((uintptr_t)qb & ~(uintptr_t)3);
    const int oa = (int)((uintptr_t)qa & 3), ob = (int)((uintptr_t)qb & 3);
    uint32_t WA[NQ + 1], WB[NQ + 1];
#pragma unroll
    for (int w = 0; w <= NQ; ++w) {
      // aligned dwords holding some query byte (they lie inside the hipMalloc'd buffer)
      WA[w] = 4 * w < oa + A.qlen ? wa[w] : 0u;
      WB[w] = 4 * w < ob + B.qlen ? wb[w] : 0u;
    }
    auto cut = [](uint32_t v, int rem) __attribute__((always_inline)) {  // bytes >= rem zeroed
      return rem >= 4 ? v : rem <= 0 ? 0u : v & ((1u << (8 * rem)) - 1u);
    };
#pragma unroll
    for (int c = 0; c < PCH<NC>; ++c) {
      uint32_t v[4];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int w = 2 * c + h;
        const uint32_t qa4 = cut(__builtin_amdgcn_alignbyte(WA[w + 1], WA[w], (uint32_t)oa), A.qlen - 4 * w);
        const uint32_t qb4 = cut(__builtin_amdgcn_alignbyte(WB[w + 1], WB[w], (uint32_t)ob), B.qlen - 4 * w);
        // columns 4w, 4w+1 and 4w+2, 4w+3: [qA_j, qA_j+1, qB_j, qB_j+1] & 3, B + 4
        v[2 * h] = (__builtin_amdgcn_perm(qb4, qa4, 0x05040100u) & 0x03030303u) | 0x04040000u;
        v[2 * h + 1] = (__builtin_amdgcn_perm(qb4, qa4, 0x07060302u) & 0x03030303u) | 0x04040000u;
      }
      qs[64 * c] = make_uint4(v[0], v[1], v[2], v[3]);
    }
  }
  const PairK k{(uint32_t)p.pair_k256, (uint32_t)p.pair_one, ((uint32_t)p.pair_cg) * 0x10001u, ((uint32_t)p.pair_bias << 8) * 0x10001u,
                ((uint32_t)(p.o_del + p.e_del) << 8) * 0x10001u, ((uint32_t)p.e_del << 8) * 0x10001u,
                ((uint32_t)(p.o_ins + p.e_ins) << 8) * 0x10001u, ((uint32_t)p.e_ins << 8) * 0x10001u};

  uint32_t eh[NC];
  {
    const int oe_ins = p.o_ins + p.e_ins;
    const int h1a = A.h0 > oe_ins ? A.h0 - oe_ins : 0, h1b = B.h0 > oe_ins ? B.h0 - oe_ins : 0;
#pragma unroll
    for (int j = 0; j < NC; ++j)
      eh[j] = ((uint32_t)pair_eh_init(A, j, h1a, p.e_ins) << 8) | ((uint32_t)pair_eh_init(B, j, h1b, p.e_ins) << 24);
  }
  // wave range of band widths (the band-cut column of row i is i - 1 - w)
  const int wlo_w = -wave_max(-min(A.done ? (1 << 20) : A.w, B.done ? (1 << 20) : B.w));
  const int whi_w = wave_max(max(A.done ? -1 : A.w, B.done ? -1 : B.w));

  PairState S;
  S.QLEN = pack2(A.qlen, B.qlen);
  S.TLEN = pack2(A.tlen, B.tlen);
  S.W = pack2(A.w, B.w);
  S.H0 = pack2(A.h0, B.h0);
  S.BEG = 0;
  S.END = S.QLEN;
  S.MX = S.H0;
  S.MAXI = S.MAXJ = S.MAXIE = S.GS = 0xFFFFFFFFu;  // -1, -1
  S.MOFF = 0;
  S.DONE = (A.done ? 0xFFFFu : 0u) | (B.done ? 0xFFFF0000u : 0u);
  S.NCA = S.NCB = 0;
  // Target bytes as the aligned dwords that cover each target, one load per
  // task every four rows (wave-uniform rows), realigned by v_alignbyte: a byte
  // load per task and row made every row touch 128 target lines per wave, and
  // at 8 waves per CU those lines thrash the XCD's L2 (2.84 GB of DRAM reads
  // per C3 batch for 0.28 GB of input).  The dword for rows
  // 4k + 4 .. 4k + 7 is requested at row 4k: four rows of cells hide it.
  const uint32_t* __restrict__ twA = reinterpret_cast<const uint32_t*>((uintptr_t)A.tg & ~(uintptr_t)3);
  const uint32_t* __restrict__ twB = reinterpret_cast<const uint32_t*>((uintptr_t)B.tg & ~(uintptr_t)3);
  const uint32_t toA = (uint32_t)((uintptr_t)A.tg & 3), toB = (uint32_t)((uintptr_t)B.tg & 3);
  // aligned dwords holding some target byte (they lie inside the hipMalloc'd buffer)
  const int nwA = ((int)toA + A.tlen + 3) >> 2, nwB = ((int)toB + B.tlen + 3) >> 2;
  uint32_t LA = nwA > 0 ? twA[0] : 0u, LB = nwB > 0 ? twB[0] : 0u;  // low dword of the coming quad
  uint32_t HA = nwA > 1 ? twA[1] : 0u, HB = nwB > 1 ? twB[1] : 0u;  // its high dword (in flight)
  uint32_t QA = 0, QB = 0;  // this quad's target bytes, row i in the low byte
  const uint32_t ONE = k.one, ED1 = (uint32_t)p.e_del * 0x10001u, EI1 = (uint32_t)p.e_ins * 0x10001u;
  const uint32_t ZD2 = (uint32_t)min(p.zdrop, 32767) * 0x10001u;

  PairRow<NC> r;
  for (int i = 0;; ++i) {
    const uint32_t I2 = (uint32_t)i * 0x10001u;
    const uint32_t ALIVE = ~S.DONE & pk_lt(I2, S.TLEN);
    if (__ballot(ALIVE != 0u) == 0ull) break;
    if ((i & 3) == 0) {
      QA = __builtin_amdgcn_alignbyte(HA, LA, toA);
      QB = __builtin_amdgcn_alignbyte(HB, LB, toB);
      LA = HA;
      LB = HB;
      const int w = (i >> 2) + 2;
      HA = w < nwA ? twA[w] : 0u;
      HB = w < nwB ? twB[w] : 0u;
    }
    const uint32_t tA = QA & 0xFFu, tB = QB & 0xFFu;
    QA >>= 8;
    QB >>= 8;
    // bwa's band: beg = max(beg, i - w), end = min(end, i + w + 1, qlen)
    S.BEG = s_max(S.BEG, s_sub(I2, S.W));
    S.END = s_min(S.END, s_min(s_add(s_add(I2, ONE), S.W), S.QLEN));
    // h1 of the row start: max(h0 - (o_del + e_del (i + 1)), 0) where beg == 0
    const uint32_t ode = (uint32_t)min(p.o_del + p.e_del * (i + 1), 65535) * 0x10001u;
    const uint32_t H1r = pk_subs(S.H0, ode) & pk_lt(S.BEG, ONE);
    const uint32_t WORK = ALIVE & pk_lt(S.BEG, S.END);
    const uint32_t EMPTY = ALIVE ^ WORK;  // beg >= end: bwa stores eh[end] and stops
    const int endA = (int)(int16_t)(S.END & 0xFFFFu), endB = (int)(int16_t)(S.END >> 16);
    // wave range of the working tasks' bands (idle halves as 32767 / -1 by
    // bitop3 selects on the WORK half masks)
    const uint32_t BW = bsel(WORK, S.BEG, 0x7FFF7FFFu), EW = bsel(WORK, S.END, 0x7FFF7FFFu);
    const uint32_t EX = bsel(WORK, S.END, ~0u);
    const int cmin = -wave_max(-min((int)(int16_t)(BW & 0xFFFFu), (int)BW >> 16));
    const int cmax = wave_max(max((int)(int16_t)(EX & 0xFFFFu), (int)EX >> 16));
    const int emin = -wave_max(-min((int)(int16_t)(EW & 0xFFFFu), (int)EW >> 16));
    PAIR_STAT(1, 1);
#ifdef FCS_BSW_STATS
    {  // task-rows of the wave that still work / are alive in this row
      int wk = (int)(WORK & 1u) + (int)((WORK >> 16) & 1u), al = (int)(ALIVE & 1u) + (int)((ALIVE >> 16) & 1u);
      for (int o = 32; o > 0; o >>= 1) wk += __shfl_xor(wk, o), al += __shfl_xor(al, o);
      PAIR_STAT(5, wk);
      PAIR_STAT(6, al);
    }
#endif
    PAIR_STAT(7, cmax >= cmin ? cmax - cmin + 1 : 0);
    r.tabA = ptab[min(tA, 4u)];
    r.tabB = ptab[min(tB, 4u)];
    r.F = 0;
    r.H1 = pk_shl8(H1r);
    r.KEY = 0;
    r.CAP = 0;
    r.BEGM1 = s_sub(S.BEG, ONE);
    r.END = S.END;
    if (cmax >= 0) r.sel[0] = r.sel[1] = qs[64 * (min(max(cmin, 0), NC - 1) / kPW)];
    // chunk classes of this row as wave-uniform bit masks (bit C = chunk C):
    // processed = overlaps [cmin, cmax]; edge = reaches some end (>= emin) or
    // holds a band-cut column [i - 1 - max w, i - 1 - min w]
    uint32_t proc = 0, edges = 0, cuts = 0;
    if (cmax >= cmin) {
      const int cf = max(cmin, 0) / kPW, cl = min(cmax, NC - 1) / kPW;
      proc = (cl >= 31 ? ~0u : (2u << cl) - 1u) & ~((1u << cf) - 1u);
      const int ef = max(emin, 0) / kPW;  // first chunk whose last column >= emin
      edges = proc & ~((1u << min(ef, 31)) - 1u);
      const int cut_lo = i - 1 - whi_w, cut_hi = i - 1 - wlo_w;
      if (cut_hi >= 0) {
        const int kf = max(cut_lo, 0) / kPW, kl = min(cut_hi, NC - 1) / kPW;
        cuts = proc & (kl >= 31 ? ~0u : (2u << kl) - 1u) & ~((1u << kf) - 1u);
      }
      edges |= cuts;
    }
    [&]<int... C>(std::integer_sequence<int, C...>) __attribute__((always_inline)) {
      (pair_chunk<C, NC, SYM>(eh, qs, r, k, proc, edges, cuts), ...);
    }(std::make_integer_sequence<int, PCH<NC>>{});

    // ---- row end (bwa's order): to-end score, cells, m == 0, new max or z-drop, trims
    const uint32_t M8 = U(V(r.KEY) >> (u16x2)(8)), MJ = r.KEY & 0x00FF00FFu;
    // to-end score: a working row reaching qlen (h1 at end) or an empty row with beg == qlen
    const uint32_t CAND = pbfi(WORK, U(V(r.CAP) >> (u16x2)(8)), H1r);
    const uint32_t GATE = (WORK & s_eq(S.END, S.QLEN, ONE)) | (EMPTY & s_eq(S.BEG, S.QLEN, ONE));
    const uint32_t UPD = GATE & ~pk_lt(CAND, S.GS);  // ties go to the later row
    S.GS = pbfi(UPD, CAND, S.GS);
    S.MAXIE = pbfi(UPD, I2, S.MAXIE);
    {
      const uint32_t dc = s_sub(S.END, S.BEG) & WORK;
      S.NCA += dc & 0xFFFFu;
      S.NCB += dc >> 16;
    }
    const uint32_t ZERO = WORK & s_eq(M8, 0u, ONE);
    const uint32_t NEWMAX = WORK & pk_lt(S.MX, M8);
    uint32_t DROP = 0;
    if (p.zdrop > 0) {
      // (i - max_i) - (mj - max_j) > 0: mx - m - d e_del > zdrop; else mx - m + d e_ins > zdrop
      const uint32_t D = s_sub(s_sub(I2, S.MAXI), s_sub(MJ, S.MAXJ));
      const uint32_t base = s_sub(S.MX, M8);
      const uint32_t val = pbfi(pk_lt(0u, D), s_sub(base, s_mul(D, ED1)), s_add(base, s_mul(D, EI1)));
      DROP = WORK & ~NEWMAX & ~ZERO & pk_lt(ZD2, val);
    }
    S.MOFF = pbfi(NEWMAX, s_max(S.MOFF, s_max(s_sub(MJ, I2), s_sub(I2, MJ))), S.MOFF);
    S.MX = pbfi(NEWMAX, M8, S.MX);
    S.MAXI = pbfi(NEWMAX, I2, S.MAXI);
    S.MAXJ = pbfi(NEWMAX, MJ, S.MAXJ);
    S.DONE |= EMPTY | ZERO | DROP;
    const uint32_t TRIM = WORK & ~S.DONE;
    if (__ballot(TRIM != 0u)) {
      // bwa's trims: beg = first entry in [beg, end] with h or e != 0, end = the
      // last one + 2.  Entries left of beg are zero (kept so), so the first one
      // is found by scanning chunks of the stored entries upward from the band's
      // first chunk until every trimming task has one, and the last one downward
      // from the band's last chunk: one chunk each in most rows (the live band
      // moves about a column per row), where a per-cell bitmap cost two VALU in
      // every cell of the row.
      const int cf = max(cmin, 0) / kPW, cl = min(cmax, NC - 1) / kPW;
      const bool ta = (TRIM & 0xFFFFu) != 0u, tb = (TRIM >> 16) != 0u;
      uint32_t fa = ~0u, fb = ~0u;  // first non-zero column, ~0u: none
      uint32_t la = ~0u, lb = ~0u;  // last non-zero column, ~0u: none
      bool go = true;
      [&]<int... C>(std::integer_sequence<int, C...>) __attribute__((always_inline)) {
        (([&] __attribute__((always_inline)) {
           if (!go || C < cf || C > cl) return;
           const uint32_t bits = chunk_nz<C, NC>(eh, ONE, endA, endB);
           fa = min(fa, ffbl_or(bits & 0xFFFFu, (uint32_t)(kPW * C)));
           fb = min(fb, ffbl_or(bits >> 16, (uint32_t)(kPW * C)));
           go = __ballot((ta && fa == ~0u) || (tb && fb == ~0u)) != 0ull;
         }()),
         ...);
      }(std::make_integer_sequence<int, PCH<NC>>{});
      go = true;
      [&]<int... C>(std::integer_sequence<int, C...>) __attribute__((always_inline)) {
        (([&] __attribute__((always_inline)) {
           constexpr int D = PCH<NC> - 1 - C;  // descending
           if (!go || D < cf || D > cl) return;
           const uint32_t bits = chunk_nz<D, NC>(eh, ONE, endA, endB);
           la = min(la, last_col(bits & 0xFFFFu, D));
           lb = min(lb, last_col(bits >> 16, D));
           go = __ballot((ta && la == ~0u) || (tb && lb == ~0u)) != 0ull;
         }()),
         ...);
      }(std::make_integer_sequence<int, PCH<NC>>{});
      // f is ~0u (sign bit set) when the task has no non-zero entry: bwa's
      // beg = end, end = end + 1; l is then ~0u too
      auto trim = [&](uint32_t f, uint32_t l, int endv, int qlen, int& nb, int& ne) __attribute__((always_inline)) {
        const uint32_t none = (uint32_t)((int)f >> 31);
        nb = (int)bsel(none, (uint32_t)endv, f);
        const int last = (int)bsel(none, (uint32_t)(endv - 1), ~l);
        ne = min(last + 2, qlen);
      };
      int nba, nea, nbb, neb;
      trim(fa, la, endA, A.qlen, nba, nea);
      trim(fb, lb, endB, B.qlen, nbb, neb);
      S.BEG = pbfi(TRIM, pack2(nba, nbb), S.BEG);
      S.END = pbfi(TRIM, pack2(nea, neb), S.END);
    }
  }
#ifdef FCS_BSW_STATS
  {
    int tot = (int)(S.NCA + S.NCB);
    for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o);
    PAIR_STAT(4, tot);
    PAIR_STAT(0, 1);
  }
#endif
  auto emit = [&](long long id, int h, uint32_t nc) __attribute__((always_inline)) {
    if (id < 0) return;
    auto f = [&](uint32_t x) { return (int)(int16_t)(h ? (x >> 16) : (x & 0xFFFFu)); };
    int32_t* o = res + 6 * id;
    o[0] = f(S.MX);
    o[1] = f(S.MAXJ) + 1;
    o[2] = f(S.MAXI) + 1;
    o[3] = f(S.MAXIE) + 1;
    o[4] = f(S.GS);
    o[5] = f(S.MOFF);
    if (cells_out) cells_out[id] = nc;
  };
  emit(A.id, 0, S.NCA);
  emit(B.id, 1, S.NCB);
}

}  // namespace

}  // namespace fcs

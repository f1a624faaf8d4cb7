// BWA-MEM banded Smith-Waterman (ksw_extend2 / ksw_global2) on gfx950.
//
// Algorithm: bwa ksw.c, reached from
// /root/reference/src/workers/BWAWorker.cpp:134-166 (bwa-flow --offload).
//
// Mapping (DESIGN.md §Banded SW): one 64-lane wave per extension task.  Lane l
// owns query columns j = l + 64*k (k < NS slots) and keeps bwa's eh[j] = {h, e}
// for those columns in registers, so the "stale eh[] beyond the band" that bwa
// re-reads when the band grows is reproduced exactly.  Target rows are processed
// in bwa's order, one row per iteration:
//   * M and E need only the lane's own column;
//   * F(i,j) = max(F0 - (j-beg)e, max_{beg<=k<j} (t_k - (j-1-k)e)),
//     t_k = max(M_k - (o_ins+e_ins), 0), is an exclusive max-plus prefix scan
//     over the lanes (both E and F open from M in ksw, so the row has no other
//     dependency) — 6 DPP steps + one wave shift per slot;
//   * eh[j].h <- H(i, j-1) is a one-lane DPP shift of the row's H;
//   * row max / arg-max (ties to the larger j), z-drop, and the beg/end band
//     trimming are wave ballots + scalar bit scans, so all control flow is
//     wave-uniform and every integer matches bwa bit for bit.
#include <hip/hip_runtime.h>

#include "bsw_scan.h"
#include "fcship_internal.h"

namespace fcs {

template <int NS>
__device__ void extend_task(const BswDevBatch& b, const BswParams& p, long long task, uint8_t* __restrict__ tl,
                            int32_t* __restrict__ res, int64_t* __restrict__ cells_out) {
  const int lane = lane_id();
  const int qlen = b.qlen[task], tlen = b.tlen[task], h0 = b.h0[task];
  int w = b.w[task];
  const uint8_t* __restrict__ q = b.qbuf + b.qoff[task];
  const uint8_t* __restrict__ tg = b.tbuf + b.toff[task];
  for (int i = lane; i < tlen; i += 64) tl[i] = tg[i];

  const int oe_del = p.o_del + p.e_del, oe_ins = p.o_ins + p.e_ins;
  const int e_del = p.e_del, e_ins = p.e_ins;
  int H[NS], E[NS], plo[NS], phi[NS];
  const int h1v = h0 > oe_ins ? h0 - oe_ins : 0;
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    const int j = lane + 64 * k;
    const int qb = j < qlen ? (int)q[j] : 4;
    plo[k] = (p.mat[0 * 5 + qb] & 0xFF) | ((p.mat[1 * 5 + qb] & 0xFF) << 8) | ((p.mat[2 * 5 + qb] & 0xFF) << 16) |
             ((p.mat[3 * 5 + qb] & 0xFF) << 24);
    phi[k] = p.mat[4 * 5 + qb];
    int hv = 0;
    if (j == 0) hv = h0;
    else if (j == 1 && j <= qlen) hv = h1v;
    else if (j >= 2 && j <= qlen) hv = max(h1v - (j - 1) * e_ins, 0);
    H[k] = hv;
    E[k] = 0;
  }
  {
    const int max_ins = bwa_max_gap(qlen, p.max_mat, p.end_bonus, p.o_ins, e_ins);
    w = w < max_ins ? w : max_ins;
    const int max_del = bwa_max_gap(qlen, p.max_mat, p.end_bonus, p.o_del, e_del);
    w = w < max_del ? w : max_del;
  }
  __syncthreads();

  int mx = h0, max_i = -1, max_j = -1, max_ie = -1, gscore = -1, max_off = 0;
  int beg = 0, end = qlen;
  long long ncell = 0;
  for (int i = 0; i < tlen; ++i) {
    const int tb = first_lane((int)tl[i]);
    if (beg < i - w) beg = i - w;
    if (end > i + w + 1) end = i + w + 1;
    if (end > qlen) end = qlen;
    int h1 = 0;
    if (beg == 0) {
      h1 = h0 - (p.o_del + e_del * (i + 1));
      if (h1 < 0) h1 = 0;
    }
    if (beg >= end) {
      // empty row: bwa still stores eh[end] = {h1, 0}; j == beg here.
#pragma unroll
      for (int k = 0; k < NS; ++k)
        if (lane + 64 * k == end) { H[k] = h1; E[k] = 0; }
      if (beg == qlen) {
        max_ie = gscore > h1 ? max_ie : i;
        gscore = gscore > h1 ? gscore : h1;
      }
      break;  // row max is 0
    }
    ncell += end - beg;
    int M[NS], u[NS], ex[NS], h[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      const int j = lane + 64 * k;
      const bool inb = j >= beg && j < end;
      const int sc = prof_score(plo[k], phi[k], tb);
      M[k] = H[k] ? H[k] + sc : 0;
      const int t = max(M[k] - oe_ins, 0);
      u[k] = inb ? t + j * e_ins : kScanNeg;
    }
    excl_scan<NS>(u, (beg - 1) * e_ins, ex);
    int rowmax = -1;
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      const int j = lane + 64 * k;
      const bool inb = j >= beg && j < end;
      const int f = ex[k] - (j - 1) * e_ins;
      const int hh = max(max(M[k], E[k]), f);
      h[k] = inb ? hh : -1;
      rowmax = max(rowmax, h[k]);
    }
    const int m = wave_max(rowmax);
    // arg-max, ties to the larger j
    int mj = -1;
#pragma unroll
    for (int k = NS - 1; k >= 0; --k) {
      const unsigned long long bm = ballot64(h[k] == m);
      if (mj < 0 && bm) mj = 64 * k + 63 - __builtin_clzll(bm);
    }
    // eh update over [beg, end]
    int carry_h = h1;
    unsigned long long nz[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      const int j = lane + 64 * k;
      const int hs = dpp_wave_shr1_i(carry_h, h[k]);
      const int lastk = read_lane(h[k], 63);
      const int t = max(M[k] - oe_del, 0);
      const int en = max(E[k] - e_del, t);
      if (j >= beg && j <= end) {
        H[k] = (j == beg) ? h1 : hs;
        E[k] = (j == end) ? 0 : en;
      }
      carry_h = lastk;
      nz[k] = ballot64(j >= beg && j <= end && (H[k] != 0 || E[k] != 0));
    }
    if (end == qlen) {
      // h1 after the loop = H(i, qlen-1), now stored at eh[qlen].h
      int hl = 0;
#pragma unroll
      for (int k = 0; k < NS; ++k)
        if ((end >> 6) == k) hl = read_lane(H[k], end & 63);
      max_ie = gscore > hl ? max_ie : i;
      gscore = gscore > hl ? gscore : hl;
    }
    if (m == 0) break;
    if (m > mx) {
      mx = m, max_i = i, max_j = mj;
      const int d = mj > i ? mj - i : i - mj;
      max_off = max_off > d ? max_off : d;
    } else if (p.zdrop > 0) {
      if (i - max_i > mj - max_j) {
        if (mx - m - ((i - max_i) - (mj - max_j)) * e_del > p.zdrop) break;
      } else {
        if (mx - m - ((mj - max_j) - (i - max_i)) * e_ins > p.zdrop) break;
      }
    }
    // band trimming: first non-zero in [beg, end), last non-zero in [beg', end]
    int nb = end, last = -1;
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      unsigned long long bm = nz[k];
      if (nb == end) {
        unsigned long long bb = bm;
        const int eb = end - 64 * k;
        if (eb >= 0 && eb < 64) bb &= ~(1ull << eb);
        if (bb) nb = 64 * k + __builtin_ctzll(bb);
      }
      if (bm) last = 64 * k + 63 - __builtin_clzll(bm);
    }
    beg = nb;
    if (last >= 0) end = last + 2 < qlen ? last + 2 : qlen;
    else end = beg + 1 < qlen ? beg + 1 : qlen;
  }
  if (lane == 0) {
    int32_t* r = res + 6 * task;
    r[0] = mx;
    r[1] = max_j + 1;
    r[2] = max_i + 1;
    r[3] = max_ie + 1;
    r[4] = gscore;
    r[5] = max_off;
    if (cells_out) cells_out[task] = ncell;
  }
}

template <int MAXNS>
__global__ __launch_bounds__(64) void bsw_extend_kernel(const BswDevBatch b, const BswParams p, int32_t* __restrict__ res,
                                                        int64_t* __restrict__ cells, const int32_t* __restrict__ order,
                                                        const int64_t* __restrict__ bounds) {
  extern __shared__ __align__(16) unsigned char tl[];
  const long long lo = bounds[kBswWideBucket], hi = bounds[kBswWideBucket + 1];
  for (long long pos = lo + blockIdx.x; pos < hi; pos += gridDim.x) {
    const long long task = order[pos];
    const int qlen = b.qlen[task];
    const int ns = (qlen + 1 + 63) >> 6;
    if (MAXNS <= 4) {
      switch (ns) {
        case 0:
        case 1: extend_task<1>(b, p, task, tl, res, cells); break;
        case 2: extend_task<2>(b, p, task, tl, res, cells); break;
        case 3: extend_task<3>(b, p, task, tl, res, cells); break;
        default: extend_task<4>(b, p, task, tl, res, cells); break;
      }
    } else {
      if (ns <= 8) extend_task<8>(b, p, task, tl, res, cells);
      else extend_task<16>(b, p, task, tl, res, cells);
    }
    __syncthreads();
  }
}

int launch_bsw_extend_wide(const BswDevBatch& b, const BswParams& p, int max_qlen, int max_tlen, int32_t* res,
                           int64_t* cells, const int32_t* order, const int64_t* bounds, hipStream_t s) {
  if (b.n <= 0) return FCS_OK;
  if (max_qlen > 1023) return fail(FCS_ERR_UNSUPPORTED, "[E::fcship] ksw_extend2: qlen > 1023 unsupported");
  const size_t lds = (size_t)((max_tlen + 64 + 15) / 16) * 16;
  if (lds > 64 * 1024) return fail(FCS_ERR_UNSUPPORTED, "[E::fcship] ksw_extend2: tlen too large");
  // grid-stride over the sorted tail; 2048 waves (2 per SIMD) fill the chip,
  // and an empty tail (the common bwa case) costs only that many exits
  long long grid = b.n;
  const long long cap = 2048;
  if (grid > cap) grid = cap;
  if (max_qlen <= 255)
    hipLaunchKernelGGL(bsw_extend_kernel<4>, dim3((unsigned)grid), dim3(64), lds, s, b, p, res, cells, order, bounds);
  else
    hipLaunchKernelGGL(bsw_extend_kernel<16>, dim3((unsigned)grid), dim3(64), lds, s, b, p, res, cells, order, bounds);
  FCS_HIP_CHECK(hipGetLastError());
  return FCS_OK;
}

// ---------------------------------------------------------------- ksw_global2
// Lane-per-task ksw_global2 for the narrow bands bwa_gen_cigar2 asks for
// (w from the score, typically < 32): the band lives in registers in diagonal
// coordinates, k = j - i + w, so H(i-1, j-1) and H(i, j) share slot k, E(i, j)
// sits at k + 1 of the previous row and F runs up k: every cell of a row uses
// compile-time register indices and bwa's sequential row order, exactly.  A
// row is 2w + 1 cells; rows whose band is cut (by column 0 in the first w rows,
// by qlen at the end, or by a lane's narrower band) run a masked variant that
// keeps bwa's boundary values (H(i, -1) = -(o_del + e_del (i + 1)), E = -inf
// past the band end, F = -inf entering it).  Query codes ride through the band
// as bytes (5 * code, the bit offset of the score in the target's packed
// matrix row) shifted one byte per row.  Directions are stored as nibbles of
// raw compare bits (M < E, max(M, E) < F, E-continue, F-continue), cell c of a
// dword in bits 28 - 4c .. 31 - 4c (each bit is the sign of a difference,
// shifted in by one v_alignbit_b32), one row of the task's band in
// ceil((2w + 1) / 8) dwords, inside the task's own min(qlen, 2w + 1) * tlen
// bytes of the direction matrix; the traceback maps bwa's byte index onto
// them.  Tasks outside these bounds take the wave-per-task kernel below.
//
// Every row runs the same unmasked cell sequence over all NB slots.  Slots
// outside a lane's band compute values no band cell reads, except three, set
// up so the unmasked recurrence reproduces bwa's boundaries:
//   * column -1 (left of the band in the first w rows): its E entering row 0
//     is -(o_del + e_del) and the columns left of it hold -inf, so E, and with
//     it H, run down column -1 as bwa's H(i, -1) = -(o_del + e_del (i + 1)),
//     and the F entering column 0 from it is -inf plus a few gap costs, which
//     no compare against a band cell can tell from bwa's -inf;
//   * slot 2w + 1 of a lane whose band is narrower than NB: its E is reset to
//     -inf after each row (bwa's eh[end].e), the only value it passes back;
//   * columns >= qlen pass nothing back (F runs right, E down its own column,
//     the diagonal right), and the score, bwa's eh[qlen].h, is read from the
//     last row's slot qlen - 1 - i + w.
constexpr int kGLaneMaxNB = 65;
__host__ __device__ __forceinline__ bool glane_ok(int qlen, int tlen, int w, bool mat_ok) {
  const int nb = 2 * w + 1;
  return mat_ok && w >= 2 && nb <= kGLaneMaxNB && qlen >= nb && tlen >= 3 &&
         4LL * ((nb + 7) >> 3) * tlen + 3 <= (long long)nb * tlen;
}
__device__ __forceinline__ uint32_t* glane_zrow0(uint8_t* zbuf, const int64_t* zoff, long long task) {
  return reinterpret_cast<uint32_t*>(((uintptr_t)(zbuf + zoff[task]) + 3) & ~(uintptr_t)3);
}

// Where a lane-path task's nibble dwords live: dword d of row i at
// base + i * rs + d * ds.
//  * interleaved (every existing task of the 64-task wave takes the lane path
//    and their direction regions are contiguous and large enough): the wave's
//    tasks share the union of their regions, dword d of row i of lane L at
//    start + (i * ndw + d) * 64 + L — each row's stores are 64 consecutive
//    dwords, and the traceback walks, which all move up from the last row,
//    read neighbouring lines;
//  * otherwise the task's own region, row i at zrow0 + i * nd.
// Both the DP and the traceback compute it from the same inputs (the wave
// partition is task / 64 in every launch).
struct GLayout {
  uint32_t* base;
  int rs, ds;
};
__device__ __forceinline__ GLayout glane_layout(const BswDevBatch& b, const BswParams& p, uint8_t* zbuf,
                                                const int64_t* __restrict__ zoff, long long task, bool ok) {
  const int lane = (int)(threadIdx.x & 63);
  const bool exists = task < b.n;
  int w = 0, tlen = 0;
  int64_t z0 = 0, zend = 0;
  bool good = !exists || ok;
  if (exists) {
    const int qlen = b.qlen[task];
    w = b.w[task];
    tlen = b.tlen[task];
    z0 = zoff[task];
    zend = z0 + (int64_t)min(qlen, 2 * w + 1) * tlen;
    if (lane < 63 && task + 1 < b.n && zoff[task + 1] != zend) good = false;
  }
  const int ndw = (2 * wave_max(exists ? w : 0) + 1 + 7) >> 3;
  const int tmax = wave_max(tlen);
  const int last = 63 - __builtin_clzll(__ballot(exists));  // highest lane holding a task
  const int64_t start = (int64_t)(((uint64_t)(uint32_t)read_lane((int)(z0 >> 32), 0) << 32) |
                                  (uint32_t)read_lane((int)z0, 0));
  const int64_t end = (int64_t)(((uint64_t)(uint32_t)read_lane((int)(zend >> 32), last) << 32) |
                                (uint32_t)read_lane((int)zend, last));
  const bool il = __ballot(!good) == 0ull && 4LL * 64 * ndw * tmax + 3 <= end - start;
  GLayout L;
  if (il) {
    L.base = reinterpret_cast<uint32_t*>(((uintptr_t)(zbuf + start) + 3) & ~(uintptr_t)3) + lane;
    L.rs = ndw * 64;
    L.ds = 64;
  } else {
    L.base = ok ? glane_zrow0(zbuf, zoff, task) : nullptr;
    L.rs = (2 * w + 1 + 7) >> 3;
    L.ds = 1;
  }
  return L;
}

// bwa's traceback (ksw_global2) of a lane-path task, one lane per task, on its
// nibble rows: bwa's byte (row i, band offset c) is cell k = beg_i + c - i + w
// of nibble row i; c past the row's band end reads 0, as bwa's zeroed bytes
// there do; a column left of the row's band start indexes bwa's flat matrix
// backwards into the rows above (row-major, n_col bytes a row), as bwa does.
// Next traceback state from (state, nibble), 2 bits per entry: from M the
// source (max(M, E) < F ? F : M < E ? E : M), from E / F its continue bit.
// A zero nibble (bwa's zeroed bytes) goes to M from every state, as bwa's 0.
__host__ __device__ constexpr uint64_t glane_next01() {
  uint64_t t = 0;
  for (int nb = 0; nb < 16; ++nb) {
    t |= (uint64_t)((nb & 2) ? 2 : (nb & 1)) << (2 * nb);
    t |= (uint64_t)((nb & 4) ? 1 : 0) << (32 + 2 * nb);
  }
  return t;
}
__host__ __device__ constexpr uint32_t glane_next2() {
  uint32_t t = 0;
  for (int nb = 0; nb < 16; ++nb) t |= (uint32_t)((nb & 8) ? 2 : 0) << (2 * nb);
  return t;
}

// The walk runs in blocks of kTbRows rows, wave-synchronously from the wave's
// top row down: the block's nibble dwords (rows rb .. rb - kTbRows + 1 at the
// dword the lane's band slot was in when the block before started) were
// requested one block ahead and sit in LDS, one 256-byte row of the tile per
// block row (lane L at dword L: every read is conflict-free whatever rows the
// lanes are on).  A step whose cell is that dword of a block row reads it from
// LDS; any other cell (an indel moved the slot across a dword, or the path left
// the band) takes the direct load of the per-cell walk.  The per-row walk
// waited on every row's load (137 us a 250k-task batch, 88 us with every load
// an L2 hit, `r6u`); blocks of 4 rows run 101 us, of 8 / 16 rows 111 / 127 us
// (lanes wait for the block's slowest path), two blocks ahead 112 us (`r6v`-`r6z`).
constexpr int kTbRows = 4;
__device__ __forceinline__ void glane_traceback(const GLayout& L, int qlen, int tlen, int w, int top,
                                                uint32_t* __restrict__ tile, uint32_t* __restrict__ cg, int cap,
                                                int32_t* __restrict__ n_out) {
  const int lane = lane_id();
  const int n_col = min(qlen, 2 * w + 1);
  const long long zsize = (long long)n_col * tlen;
  const int dmax = (2 * w) >> 3;  // the band's last nibble dword
  constexpr uint64_t T01 = glane_next01();
  constexpr uint32_t T2 = glane_next2();
  int crow = -1, cdw = -1;
  uint32_t cval = 0;
  int n = 0, which = 0, curop = -1;
  uint32_t curlen = 0;
  int i = tlen - 1;
  int k = (i + w + 1 < qlen ? i + w + 1 : qlen) - 1;
  // the first block's dwords, then each block's for the next
  int rb = top;
  int ndw = min(max((k - i + w) >> 3, 0), dmax);
  uint32_t nx[kTbRows];
  // global (not flat) loads: a flat load also counts in lgkmcnt, so every LDS
  // read of the block would wait for the next block's requests
  typedef const __attribute__((address_space(1))) uint32_t gu32;
  gu32* const gbase = reinterpret_cast<gu32*>(reinterpret_cast<uintptr_t>(L.base));
  auto request = [&](int row0, int dw) {
    gu32* const p = gbase + dw * L.ds;
#pragma unroll
    for (int j = 0; j < kTbRows; ++j) nx[j] = p[(long long)min(max(row0 - j, 0), tlen - 1) * L.rs];
  };
  request(rb, ndw);
  uint32_t* const mine = tile + lane;
  bool live = i >= 0 && k >= 0;
  while (__ballot(live) != 0ull) {
#pragma unroll
    for (int j = 0; j < kTbRows; ++j) mine[64 * j] = nx[j];
    const int tdw = ndw;
    ndw = min(max((k - i + w) >> 3, 0), dmax);
    request(rb - kTbRows, ndw);
    const int lo = rb - (kTbRows - 1);
    for (;;) {
      const bool act = live && i >= lo;
      if (__ballot(act) == 0ull) break;
      if (!act) continue;
      // bwa's byte (row i, band offset c = k - beg_i) is cell k - i + w of
      // nibble row i; c past the row's band end reads 0, as bwa's zeroed bytes
      // there do; a column left of the row's band start indexes bwa's flat
      // matrix backwards into the rows above (row-major, n_col bytes a row).
      // In band (|k - i| <= w; k < qlen always holds) the cell is slot
      // k - i + w of nibble row i; only a path that left the band takes the
      // general mapping below.
      int kb = k - i + w;
      // the block row's dword from LDS (always inside the tile: lo <= i <= rb)
      uint32_t nb = (mine[64 * (rb - i)] >> (28 - 4 * (kb & 7))) & 15u;
      if (!((unsigned)kb <= (unsigned)(2 * w) && (kb >> 3) == tdw)) {
        int r = i;
        bool have = (unsigned)kb <= (unsigned)(2 * w);
        if (!have) {
          int c = k - (i > w ? i - w : 0);
          if (c < 0 || c >= n_col) {
            const long long zi = (long long)i * n_col + c;
            r = (zi < 0 || zi >= zsize) ? -1 : (int)(zi / n_col);
            c = r < 0 ? 0 : (int)(zi - (long long)r * n_col);
          }
          if (r >= 0) {
            const int beg = r > w ? r - w : 0, end = r + w + 1 < qlen ? r + w + 1 : qlen;
            have = beg + c < end;
            kb = beg + c - r + w;
          }
        }
        nb = 0;
        if (have) {
          const int dw = kb >> 3;
          if (r != crow || dw != cdw) {
            crow = r, cdw = dw;
            cval = gbase[(long long)r * L.rs + dw * L.ds];
          }
          nb = (cval >> (28 - 4 * (kb & 7))) & 15u;
        }
      }
      // next state: one 32-bit table of 2-bit entries per state (no branch)
      const uint32_t tbl = which == 0 ? (uint32_t)T01 : which == 1 ? (uint32_t)(T01 >> 32) : T2;
      which = (int)((tbl >> (2 * nb)) & 3u);
      // state M: diagonal (CIGAR M), E: up (D), F: left (I)
      const int op = (int)((0x18u >> (2 * which)) & 3u);
      i -= which != 2;
      k -= which != 1;
      live = i >= 0 && k >= 0;
      // a run ends: stored while it fits (one branch around the store only)
      const bool ends = op != curop && curop >= 0;
      if (ends && n < cap) cg[n] = curlen << 4 | (uint32_t)curop;
      n += ends;
      curlen = op != curop ? 1u : curlen + 1u;
      curop = op;
    }
    rb -= kTbRows;
  }
  auto push = [&](int op, int len) {
    if (op == curop) {
      curlen += (uint32_t)len;
    } else {
      if (curop >= 0) {
        if (n < cap) cg[n] = curlen << 4 | (uint32_t)curop;
        ++n;
      }
      curop = op;
      curlen = (uint32_t)len;
    }
  };
  if (i >= 0) push(2, i + 1);
  if (k >= 0) push(1, k + 1);
  if (curop >= 0) {
    if (n < cap) cg[n] = curlen << 4 | (uint32_t)curop;
    ++n;
  }
  const int nn = n < cap ? n : cap;
  for (int a = 0; a < nn >> 1; ++a) {
    const uint32_t t = cg[a];
    cg[a] = cg[nn - 1 - a];
    cg[nn - 1 - a] = t;
  }
  *n_out = n;
}

// The row's direction bits are signs of differences (every score stays within
// +-2^30 + 2^10, so a difference never overflows: (uint32)(a - b) >> 31 is
// exactly a < b), shifted into the row's dwords by v_alignbit_b32 (acc << 1 |
// x >> 31, one full-rate instruction per bit; the compiler's compare +
// v_cndmask for the same shift costs two).
__device__ __forceinline__ uint32_t gbit(uint32_t acc, int x) {
  uint32_t r;
  asm("v_alignbit_b32 %0, %1, %2, 31" : "=v"(r) : "v"(acc), "v"(x));
  return r;
}

// a + b + c in one VALU instruction (the compiler splits a - b + c into two)
__device__ __forceinline__ int add3(int a, int b, int c) {
  int r;
  asm("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// The row's scores of four band cells in one v_perm_b32 (the row's five
// scores as table bytes, indexed by the cells' query codes), each added to H by
// one SDWA add of its sign-extended byte.
template <int B>
__device__ __forceinline__ int add_sbyte_c(int h, uint32_t s4) {
  int r;
  asm("v_add_u32_sdwa %0, %1, sext(%2) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_%3"
      : "=v"(r)
      : "v"(h), "v"(s4), "i"(B));
  return r;
}

// The 16-bit form of a row (U): every H / E / F value is held as value +
// kGU16Bias, zero-extended in its 32-bit register, with bwa's MINUS_INF
// standing in as kGU16NegInf.  Its maxes are v_max_u16 (full rate on gfx950;
// v_max_i32 issues at half rate), adds and subtracts stay 32-bit
// (a biased value never leaves [0, 65535], so they are exact and stay
// zero-extended), and the difference of two biased values is the true
// difference, so the direction bits are unchanged.  Taken by a wave whose
// tasks all satisfy glane_u16_ok: every real value and every MINUS_INF-derived
// one then keeps its 32-bit path's value up to the bias (|real| <= 8000,
// MINUS_INF-derived within 8000 of kGU16NegInf), so every compare and every
// output is the same.
constexpr int kGU16Bias = 32768;
constexpr int kGU16NegInf = -24576;
__host__ __device__ __forceinline__ bool glane_u16_ok(int qlen, int tlen, int e_del, int e_ins, int o_del,
                                                      int o_ins) {
  // a path's score moves by at most max(e) + 16 (|mat| <= 16 on the lane path)
  // per row or column, plus the two gap opens
  const long long span = (long long)(qlen + tlen + 2) * ((e_del > e_ins ? e_del : e_ins) + 16) + o_del + o_ins;
  return span <= 8000;
}
template <bool U>
__device__ __forceinline__ int gmax(int a, int b) {
  if constexpr (U) {
    int r;
    asm("v_max_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
  } else {
    return max(a, b);
  }
}
template <bool U>
__host__ __device__ constexpr int gval(int v) {  // a boundary value as the row form holds it
  return U ? (v == kMinusInf ? kGU16NegInf : v) + kGU16Bias : v;
}

template <int NB, bool CIG, bool U>
__device__ __forceinline__ void glane_row(int (&Hd)[NB], int (&Ed)[NB + 1], const uint32_t (&Qb)[(NB + 4) / 4],
                                          uint32_t (&nib)[(NB + 7) / 8], const uint32_t rowlo, const uint32_t rowhi,
                                          const int oe_del, const int oe_ins, const int e_del, const int e_ins) {
  int f = gval<U>(kMinusInf);
  uint32_t acc = 0;
  const int o_del = oe_del - e_del, neg_e_del = -e_del;
  uint32_t s4 = 0;
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    if ((k & 3) == 0) s4 = __builtin_amdgcn_perm(rowhi, rowlo, Qb[k >> 2]);  // bytes: scores of cells k .. k + 3
    int m;
    switch (k & 3) {
      case 0: m = add_sbyte_c<0>(Hd[k], s4); break;
      case 1: m = add_sbyte_c<1>(Hd[k], s4); break;
      case 2: m = add_sbyte_c<2>(Hd[k], s4); break;
      default: m = add_sbyte_c<3>(Hd[k], s4); break;
    }
    const int e0 = Ed[k + 1];
    const int h1 = gmax<U>(m, e0);
    const int h = gmax<U>(h1, f);
    const int ti = m - oe_ins;
    const int fn = f - e_ins;
    if constexpr (CIG) {
      // E from the two differences the direction bits need anyway:
      // max(e0 - e_del, M - oe_del) = e0 - e_del + max(x, 0) with
      // x = M - e0 - o_del, one instruction fewer than forming both terms
      // (the 16-bit form takes the full-rate max of both terms instead)
      const int dme = m - e0;
      const int x = dme - o_del;
      acc = gbit(acc, ti - fn);  // F-continue: f - e_ins > M - oe_ins
      acc = gbit(acc, x);        // E-continue: e0 - e_del > M - oe_del
      acc = gbit(acc, h1 - f);   // max(M, E) < F: H from F
      acc = gbit(acc, dme);      // M < E: H from E
      if ((k & 7) == 7) nib[k >> 3] = acc;
      if constexpr (U) Ed[k] = gmax<U>(e0 - e_del, m - oe_del);
      else Ed[k] = add3(e0, max(x, 0), neg_e_del);
    } else {
      (void)neg_e_del;
      Ed[k] = gmax<U>(e0 - e_del, m - oe_del);
    }
    Hd[k] = h;
    f = gmax<U>(fn, ti);
  }
  if constexpr (CIG && (NB & 7) != 0) nib[NB >> 3] = acc << (4 * (8 - (NB & 7)));  // the row's last cells to the top
}

template <int NB, bool CIG, bool U>
__device__ void glane_run(const BswDevBatch& b, const BswParams& p, long long task, bool ok,
                          int32_t* __restrict__ scores, uint8_t* __restrict__ zbuf, const int64_t* __restrict__ zoff,
                          uint32_t* __restrict__ cigar, const int64_t* __restrict__ cigar_off,
                          const int32_t* __restrict__ cigar_cap, int32_t* __restrict__ n_cigar) {
  constexpr int NQ = (NB + 4) / 4, NW = (NB + 7) / 8;
  int qlen = 0, tlen = 0, w = 0;
  const uint8_t* __restrict__ q = nullptr;
  const uint8_t* __restrict__ tg = nullptr;
  if (ok) {
    qlen = b.qlen[task];
    tlen = b.tlen[task];
    w = b.w[task];
    q = b.qbuf + b.qoff[task];
    tg = b.tbuf + b.toff[task];
  }
  const int tmax = wave_max(tlen);
  const int oe_del = p.o_del + p.e_del, oe_ins = p.o_ins + p.e_ins, e_del = p.e_del, e_ins = p.e_ins;
  const int nb = 2 * w + 1, nd = (nb + 7) >> 3;
  GLayout zl{nullptr, 0, 0};
  if constexpr (CIG) zl = glane_layout(b, p, zbuf, zoff, task, ok);
  uint32_t* zrow = zl.base;
  const bool zil = zl.ds == 64;
  int Hd[NB], Ed[NB + 1];
  uint32_t Qb[NQ], nib[NW];
  // every lane loads every row (a clamped index into a valid buffer) and
  // selects afterwards: a load under a branch makes the compiler wait for all
  // outstanding loads at the next use, which serialised the row-ahead reads
  const uint8_t* __restrict__ qp = ok ? q : b.qbuf;
  const uint8_t* __restrict__ tp = ok ? tg : b.tbuf;
  const int qlast = max(qlen - 1, 0);
  auto qbyte = [&](int j) -> uint32_t {
    const uint32_t v = qp[min(max(j, 0), qlast)];
    return (ok && j >= 0 && j < qlen) ? v : 0u;
  };
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    const int j = k - w;  // column of slot k in row 0; Hd holds "H(-1, j - 1)" = bwa's first-row eh[j].h
    Hd[k] = gval<U>(j == 0 ? 0 : (j >= 1 && j <= w) ? -(p.o_ins + e_ins * j) : kMinusInf);
    Ed[k] = gval<U>(kMinusInf);
  }
  Ed[NB] = gval<U>(kMinusInf);
#pragma unroll
  for (int d = 0; d < NQ; ++d) {
    uint32_t v = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (4 * d + c <= NB) v |= qbyte(4 * d + c - w) << (8 * c);
    Qb[d] = v;
  }
#pragma unroll
  for (int d = 0; d < NW; ++d) nib[d] = 0;
  // column -1's E entering row 0 (slot w - 1 reads Ed[w]): bwa's H(i, -1)
  // chain, -(o_del + e_del (i + 1)), runs down it from here
#pragma unroll
  for (int k = 1; k <= NB; ++k)
    if (k == w) Ed[k] = gval<U>(-(p.o_del + e_del));
  // lanes whose band is narrower than the class: E of slot nb back to -inf
  // after every row (a wave-uniform test; the class's widest lanes need none)
  const bool narrow = __ballot(ok && nb < NB) != 0ull;
  int score = kMinusInf;
  const int kfin = qlen - tlen + w;  // the last row's slot of column qlen - 1
  // Row inputs as byte streams read by aligned dwords, four rows per group
  // (the target byte of row i and the query byte entering the band for row
  // i + 1, position i + NB + 1 - w).  The two dwords a group needs are loaded
  // during the group before and only read (realigned) at its start, so no
  // register holding a load in flight is copied and the loads get a group's
  // compute to land.  (A byte load per lane and row kept the lines of a
  // wave's 64 tasks live, overflowing the XCD's L2 at 4 waves per SIMD, and
  // every row waited on memory.)
  struct Stream {
    const uint32_t* __restrict__ w;
    uint32_t off;
    int last;  // last dword holding a byte of the stream (clamped loads stay inside it)
    uint32_t lo, hi, cur;
    __device__ __forceinline__ void init(const uint8_t* base, int len) {
      off = (uint32_t)((uintptr_t)base & 3);
      w = reinterpret_cast<const uint32_t*>(base - off);  // pointer arithmetic keeps the global address space
      last = max(((int)off + len + 3) / 4 - 1, 0);
      lo = w[0];
      hi = w[min(1, last)];
    }
    // at row 4k: bytes 4k .. 4k + 3 into cur; then group k + 1's dwords requested
    __device__ __forceinline__ void realign() { cur = __builtin_amdgcn_alignbyte(hi, lo, off); }
    __device__ __forceinline__ void fetch(int k) {
      lo = w[min(k + 1, last)];
      hi = w[min(k + 2, last)];
    }
  };
  Stream ts, qs;
  const int qc = NB + 1 - w;  // row i's entering query position is i + qc
  ts.init(tp, ok ? tlen : 1);
  // (a lane whose band never takes a new query byte reads its first byte)
  const bool qin = ok && qc < qlen;
  qs.init(qin ? qp + qc : qp, qin ? qlen - qc : 1);
  // the row's packed score table by the lane's target base: lanes 0..4 hold
  // the five tables, one ds_bpermute fetches lane tb's
  const int ln = lane_id();
  // lane t < 5: target base t's scores of query codes 0..3 (bytes of tabv)
  // and of code 4 (byte 0 of tabh)
  const int tabv = ln < 5 ? (int)((uint32_t)(uint8_t)p.mat[5 * ln] | (uint32_t)(uint8_t)p.mat[5 * ln + 1] << 8 |
                                  (uint32_t)(uint8_t)p.mat[5 * ln + 2] << 16 | (uint32_t)(uint8_t)p.mat[5 * ln + 3] << 24)
                         : 0;
  const int tabh = ln < 5 ? (int)(uint32_t)(uint8_t)p.mat[5 * ln + 4] : 0;
  for (int i0 = 0; i0 < tmax; i0 += 4) {
    // both streams realigned before either requests more (with the CIG pass's
    // stores counted in vmcnt, a wait after a new request would wait for it)
    ts.realign();
    qs.realign();
    asm volatile("" ::: "memory");
    ts.fetch(i0 >> 2);
    qs.fetch(i0 >> 2);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + r;
      if (i >= tmax) break;
      const int tb = (ok && i < tlen) ? (int)((ts.cur >> (8 * r)) & 0xFFu) : 4;
      const uint32_t qn = (ok && i + qc < qlen) ? ((qs.cur >> (8 * r)) & 0xFFu) : 0u;
      const uint32_t rowlo = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * min(tb, 4), tabv);
      const uint32_t rowhi = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * min(tb, 4), tabh);
      glane_row<NB, CIG, U>(Hd, Ed, Qb, nib, rowlo, rowhi, oe_del, oe_ins, e_del, e_ins);
      // (the slot tests are built where they are used: hoisted out of the row
      // loop they would hold one SGPR pair per slot)
      if (narrow) {
        int nbv = nb;
        asm volatile("" : "+v"(nbv));
#pragma unroll
        for (int k = 5; k < NB; k += 2)
          if (k == nbv) Ed[k] = gval<U>(kMinusInf);
      }
      if (ok && i == tlen - 1) {  // bwa's score eh[qlen].h: H(tlen - 1, qlen - 1) when the band reaches it
        int kf = kfin < nb ? kfin : -1;
        asm volatile("" : "+v"(kf));
#pragma unroll
        for (int k = 0; k < NB; ++k)
          if (k == kf) score = Hd[k];
      }
      if constexpr (CIG) {
        // a running row pointer and compile-time dword offsets (the layout's
        // dword stride is 64 or 1, wave-uniform)
        if (ok && i < tlen) {
          if (zil) {
#pragma unroll
            for (int d = 0; d < NW; ++d)
              if (d < nd) zrow[64 * d] = nib[d];
          } else {
#pragma unroll
            for (int d = 0; d < NW; ++d)
              if (d < nd) zrow[d] = nib[d];
          }
        }
        zrow += zl.rs;
      }
      // next row's query bytes: the band moves one column right
#pragma unroll
      for (int d = 0; d < NQ; ++d) Qb[d] = d + 1 < NQ ? __builtin_amdgcn_alignbyte(Qb[d + 1], Qb[d], 1) : Qb[d] >> 8;
      Qb[NB >> 2] = (Qb[NB >> 2] & ~(0xFFu << (8 * (NB & 3)))) | (qn << (8 * (NB & 3)));
    }
  }
  if constexpr (U) {  // back to the 32-bit form: MINUS_INF-derived values keep their offset from it
    if (score != kMinusInf) {
      score -= kGU16Bias;
      if (score < -16384) score = score - kGU16NegInf + kMinusInf;
    }
  }
  if (ok) scores[task] = score;
  // (the traceback runs in bsw_traceback_kernel: a chain of dependent loads per
  // lane, it wants the occupancy this kernel's registers do not leave)
}

// One launch per band class (each with its own register budget): a wave runs
// in the launch whose NB is the smallest of 17 / 33 / 65 holding its widest band.
template <int NB, bool CIG>
__global__ __launch_bounds__(64) void bsw_global_lane_kernel(const BswDevBatch b, const BswParams p,
                                                             int32_t* __restrict__ scores, uint8_t* __restrict__ zbuf,
                                                             const int64_t* __restrict__ zoff,
                                                             uint32_t* __restrict__ cigar,
                                                             const int64_t* __restrict__ cigar_off,
                                                             const int32_t* __restrict__ cigar_cap,
                                                             int32_t* __restrict__ n_cigar) {
  const long long task = (long long)blockIdx.x * 64 + threadIdx.x;
  bool ok = false;
  int w = -1;
  if (task < b.n) {
    w = b.w[task];
    ok = glane_ok(b.qlen[task], b.tlen[task], w, p.lane_ok != 0);
  }
  const int nbw = 2 * wave_max(ok ? w : -1) + 1;
  constexpr int lo = NB == 17 ? 0 : NB == 33 ? 17 : 33;
  if (nbw <= lo || nbw > NB) return;
  // the 16-bit row form when every task of the wave keeps its values in range
  const bool u16 = __ballot(ok && !glane_u16_ok(b.qlen[task], b.tlen[task], p.e_del, p.e_ins, p.o_del, p.o_ins)) == 0ull;
  if (u16) glane_run<NB, CIG, true>(b, p, task, ok, scores, zbuf, zoff, cigar, cigar_off, cigar_cap, n_cigar);
  else glane_run<NB, CIG, false>(b, p, task, ok, scores, zbuf, zoff, cigar, cigar_off, cigar_cap, n_cigar);
}

template <int NS>
__device__ void global_task(const BswDevBatch& b, const BswParams& p, long long task, uint8_t* __restrict__ tl,
                            int32_t* __restrict__ scores, uint8_t* __restrict__ zbuf, const int64_t* __restrict__ zoff) {
  const int lane = lane_id();
  const int qlen = b.qlen[task], tlen = b.tlen[task], w = b.w[task];
  const uint8_t* __restrict__ q = b.qbuf + b.qoff[task];
  const uint8_t* __restrict__ tg = b.tbuf + b.toff[task];
  for (int i = lane; i < tlen; i += 64) tl[i] = tg[i];
  const int oe_del = p.o_del + p.e_del, oe_ins = p.o_ins + p.e_ins;
  const int e_del = p.e_del, e_ins = p.e_ins;
  const int n_col = qlen < 2 * w + 1 ? qlen : 2 * w + 1;
  uint8_t* __restrict__ z = zbuf ? zbuf + zoff[task] : nullptr;
  if (z)  // bwa's traceback may read cells outside the band: they read 0 (the oracle zeroes its matrix too)
    for (long long x = lane; x < (long long)n_col * tlen; x += 64) z[x] = 0;
  int H[NS], E[NS], plo[NS], phi[NS];
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    const int j = lane + 64 * k;
    const int qb = j < qlen ? (int)q[j] : 4;
    plo[k] = (p.mat[0 * 5 + qb] & 0xFF) | ((p.mat[1 * 5 + qb] & 0xFF) << 8) | ((p.mat[2 * 5 + qb] & 0xFF) << 16) |
             ((p.mat[3 * 5 + qb] & 0xFF) << 24);
    phi[k] = p.mat[4 * 5 + qb];
    int hv = kMinusInf;
    if (j == 0) hv = 0;
    else if (j <= qlen && j <= w) hv = -(p.o_ins + e_ins * j);
    H[k] = hv;
    E[k] = kMinusInf;
  }
  __syncthreads();
  for (int i = 0; i < tlen; ++i) {
    const int tb = first_lane((int)tl[i]);
    const int beg = i > w ? i - w : 0;
    const int end = i + w + 1 < qlen ? i + w + 1 : qlen;
    const int h1 = beg == 0 ? -(p.o_del + e_del * (i + 1)) : kMinusInf;
    int M[NS], u[NS], ex[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      const int j = lane + 64 * k;
      const bool inb = j >= beg && j < end;
      M[k] = H[k] + prof_score(plo[k], phi[k], tb);
      u[k] = inb ? (M[k] - oe_ins) + j * e_ins : kScanNeg;
    }
    // F0 = MINUS_INF enters as a virtual column beg-1
    excl_scan<NS>(u, kMinusInf + (beg - 1) * e_ins, ex);
    int carry_h = h1;
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      const int j = lane + 64 * k;
      const bool inb = j >= beg && j < end;
      const int f = ex[k] - (j - 1) * e_ins;
      const int m = M[k], e = E[k];
      int d = m >= e ? 0 : 1;
      int hh = m >= e ? m : e;
      d = hh >= f ? d : 2;
      hh = hh >= f ? hh : f;
      int t = m - oe_del;
      const int e2 = e - e_del;
      d |= e2 > t ? 1 << 2 : 0;
      const int en = e2 > t ? e2 : t;
      t = m - oe_ins;
      const int f2 = f - e_ins;
      d |= f2 > t ? 2 << 4 : 0;
      if (z && inb) z[(long long)i * n_col + (j - beg)] = (uint8_t)d;
      const int hsrc = inb ? hh : 0;
      const int hs = dpp_wave_shr1_i(carry_h, hsrc);
      carry_h = read_lane(hsrc, 63);
      // bwa writes eh[end] = {h1, MINUS_INF} even when the band is empty
      // (beg >= end, h1 then still holds its row-start value).
      if ((j >= beg && j <= end) || j == end) {
        H[k] = (j == beg || beg >= end) ? h1 : hs;
        E[k] = (j == end) ? kMinusInf : en;
      }
    }
  }
  // score = eh[qlen].h
  int sc = 0;
#pragma unroll
  for (int k = 0; k < NS; ++k)
    if ((qlen >> 6) == k) sc = read_lane(H[k], qlen & 63);
  if (lane == 0) scores[task] = sc;
}

template <int MAXNS>
__global__ __launch_bounds__(64) void bsw_global_kernel(const BswDevBatch b, const BswParams p, int32_t* __restrict__ scores,
                                                        uint8_t* __restrict__ zbuf, const int64_t* __restrict__ zoff) {
  extern __shared__ __align__(16) unsigned char tl[];
  // 64 tasks per probe, one per lane: this kernel's tasks (those the lane
  // kernels do not take) found by one ballot, then taken one at a time
  const int lane = (int)threadIdx.x;
  for (long long base = (long long)blockIdx.x * 64; base < b.n; base += (long long)gridDim.x * 64) {
    const long long mine = base + lane;
    const bool wave_task = mine < b.n && !glane_ok(b.qlen[mine], b.tlen[mine], b.w[mine], p.lane_ok != 0);
    unsigned long long todo = __ballot(wave_task);
    while (todo) {
    const long long task = base + __builtin_ctzll(todo);
    todo &= todo - 1;
    const int qlen = b.qlen[task];
    const int ns = (qlen + 1 + 63) >> 6;
    if (MAXNS <= 4) {
      switch (ns) {
        case 0:
        case 1: global_task<1>(b, p, task, tl, scores, zbuf, zoff); break;
        case 2: global_task<2>(b, p, task, tl, scores, zbuf, zoff); break;
        case 3: global_task<3>(b, p, task, tl, scores, zbuf, zoff); break;
        default: global_task<4>(b, p, task, tl, scores, zbuf, zoff); break;
      }
    } else {
      if (ns <= 8) global_task<8>(b, p, task, tl, scores, zbuf, zoff);
      else global_task<16>(b, p, task, tl, scores, zbuf, zoff);
    }
    __syncthreads();
    }
  }
}

// One lane per task walks the direction bytes back from (tlen-1, last column).
__global__ __launch_bounds__(64) void bsw_traceback_kernel(const BswDevBatch b, const BswParams p, uint8_t* __restrict__ zbuf,
                                     const int64_t* __restrict__ zoff, uint32_t* __restrict__ cigar,
                                     const int64_t* __restrict__ cigar_off, const int32_t* __restrict__ cigar_cap,
                                     int32_t* __restrict__ n_cigar) {
  const long long task = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const bool exists = task < b.n;
  const int qlen = exists ? b.qlen[task] : 0, tlen = exists ? b.tlen[task] : 0, w = exists ? b.w[task] : 0;
  // lane-path tasks: their nibble rows, located as bsw_global_lane_kernel
  // wrote them (the same 64-task waves: every lane takes part in the layout's
  // wave votes)
  const bool lane = exists && glane_ok(qlen, tlen, w, p.lane_ok != 0);
  const GLayout zl = glane_layout(b, p, zbuf, zoff, task, lane);
  const int top = wave_max(lane ? tlen - 1 : -1);  // the lane walks' first block (every lane votes)
  __shared__ uint32_t tile[kTbRows * 64];
  if (!exists) return;
  if (lane) {
    glane_traceback(zl, qlen, tlen, w, top, tile, cigar + cigar_off[task], cigar_cap[task], n_cigar + task);
    return;
  }
  const int n_col = qlen < 2 * w + 1 ? qlen : 2 * w + 1;
  const uint8_t* z = zbuf + zoff[task];
  const long long zsize = (long long)n_col * (tlen > 0 ? tlen : 0);
  auto zbyte = [&](long long zi) -> int { return z[zi]; };
  uint32_t* cg = cigar + cigar_off[task];
  const int cap = cigar_cap[task];
  int n = 0, which = 0, curop = -1;
  uint32_t curlen = 0;
  int i = tlen - 1;
  int k = (i + w + 1 < qlen ? i + w + 1 : qlen) - 1;
  // ops are produced last-to-first as runs; each finished run is stored, the
  // array is reversed at the end (bwa push_cigar + reverse).
  auto push = [&](int op, int len) {
    if (op == curop) {
      curlen += (uint32_t)len;
    } else {
      if (curop >= 0) {
        if (n < cap) cg[n] = curlen << 4 | (uint32_t)curop;
        ++n;
      }
      curop = op;
      curlen = (uint32_t)len;
    }
  };
  while (i >= 0 && k >= 0) {
    // cells outside the written band read as 0 (zeroed matrix, bounded index;
    // see oracle/ksw_oracle.c header) instead of bwa's undefined read
    const long long zi = (long long)i * n_col + (k - (i > w ? i - w : 0));
    which = (zi >= 0 && zi < zsize) ? (zbyte(zi) >> (which << 1) & 3) : 0;
    if (which == 0) push(0, 1), --i, --k;
    else if (which == 1) push(2, 1), --i;
    else push(1, 1), --k;
  }
  if (i >= 0) push(2, i + 1);
  if (k >= 0) push(1, k + 1);
  if (curop >= 0) {
    if (n < cap) cg[n] = curlen << 4 | (uint32_t)curop;
    ++n;
  }
  const int nn = n < cap ? n : cap;
  for (int a = 0; a < nn >> 1; ++a) {
    const uint32_t t = cg[a];
    cg[a] = cg[nn - 1 - a];
    cg[nn - 1 - a] = t;
  }
  n_cigar[task] = n;
}

int launch_bsw_global(const BswDevBatch& b, const BswParams& p, int max_qlen, int max_tlen, int32_t* scores,
                      uint8_t* zbuf, int64_t zbytes, const int64_t* zoff, uint32_t* cigar, const int64_t* cigar_off,
                      const int32_t* cigar_cap, int32_t* n_cigar, hipStream_t s) {
  if (b.n <= 0) return FCS_OK;
  if (max_qlen > 1023) return fail(FCS_ERR_UNSUPPORTED, "[E::fcship] ksw_global2: qlen > 1023 unsupported");
  (void)zbytes;  // no arena-wide memset: lane-path tasks write every nibble their traceback reads, and the
                // wave kernel zeroes its own tasks' regions
  const size_t lds = (size_t)((max_tlen + 64 + 15) / 16) * 16;
  if (lds > 64 * 1024) return fail(FCS_ERR_UNSUPPORTED, "[E::fcship] ksw_global2: tlen too large");
  // grid-stride over the sorted tail; 2048 waves (2 per SIMD) fill the chip,
  // and an empty tail (the common bwa case) costs only that many exits
  long long grid = (b.n + 63) / 64;  // one 64-task probe per wave and round
  const long long cap = 2048;
  if (grid > cap) grid = cap;
  // narrow bands: one lane per task (64 consecutive tasks per wave)
  const long long lane_waves = (b.n + 63) / 64;
  if (lane_waves > 0x7FFFFFFFLL) return fail(FCS_ERR_UNSUPPORTED, "[E::fcship] ksw_global2: batch too large");
  auto lane_launch = [&](auto kern) -> int {
    hipLaunchKernelGGL(kern, dim3((unsigned)lane_waves), dim3(64), 0, s, b, p, scores, zbuf, zoff, cigar, cigar_off,
                       cigar_cap, n_cigar);
    FCS_HIP_CHECK(hipGetLastError());
    return FCS_OK;
  };
  int rc;
  if (zbuf) {
    if ((rc = lane_launch(bsw_global_lane_kernel<17, true>)) || (rc = lane_launch(bsw_global_lane_kernel<33, true>)) ||
        (rc = lane_launch(bsw_global_lane_kernel<65, true>)))
      return rc;
  } else {
    if ((rc = lane_launch(bsw_global_lane_kernel<17, false>)) || (rc = lane_launch(bsw_global_lane_kernel<33, false>)) ||
        (rc = lane_launch(bsw_global_lane_kernel<65, false>)))
      return rc;
  }
  if (max_qlen <= 255)
    hipLaunchKernelGGL(bsw_global_kernel<4>, dim3((unsigned)grid), dim3(64), lds, s, b, p, scores, zbuf, zoff);
  else
    hipLaunchKernelGGL(bsw_global_kernel<16>, dim3((unsigned)grid), dim3(64), lds, s, b, p, scores, zbuf, zoff);
  FCS_HIP_CHECK(hipGetLastError());
  if (cigar) {
    const long long nb = (b.n + 63) / 64;
    hipLaunchKernelGGL(bsw_traceback_kernel, dim3((unsigned)nb), dim3(64), 0, s, b, p, zbuf, zoff, cigar, cigar_off,
                       cigar_cap, n_cigar);
    FCS_HIP_CHECK(hipGetLastError());
  }
  return FCS_OK;
}

}  // namespace fcs

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
// Here one 64-lane wave runs one task; lane l owns positions x = l + 64 k
// (k < NK slots), padded to slen * p as bwa's profile is (padding scores 0).
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
// the same wave, all control flow wave-uniform.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "bsw_scan.h"
#include "fcship_internal.h"

namespace fcs {

constexpr int kKswXByte = 0x10000, kKswXStop = 0x20000, kKswXSubo = 0x40000, kKswXStart = 0x80000;
constexpr int kBlockBig = 1 << 20;  // > the range of one block's scan values; block ids < 16

struct AlignRun {
  int score, te, qe, score2, te2;
};

// One ksw_u8 / ksw_i16 run of query q[x] (x < qlen, read through qidx) against
// target t[j] (j < tlen, LDS, read through tidx).  minsc / endsc as bwa's.
template <int NK, class QAt, class TAt>
__device__ AlignRun align_run(const BswParams& p, int qlen, QAt q_at, int tlen, TAt t_at, bool u8, int shift,
                              int max_mat, int minsc, int endsc, uint64_t* __restrict__ blist) {
  const int lane = lane_id();
  const int pl = u8 ? 16 : 8;
  const int slen = (qlen + pl - 1) / pl;
  const int nlen = slen * pl;
  const int oe_del = p.o_del + p.e_del, oe_ins = p.o_ins + p.e_ins, e_del = p.e_del, e_ins = p.e_ins;
  int Hp[NK], E[NK], Hm[NK], plo[NK], phi[NK], blk[NK];
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int x = lane + 64 * k;
    const int qb = x < qlen ? q_at(x) : -1;  // padding: score 0 against every base
    auto sc = [&](int a) { return qb < 0 ? 0 : (int)p.mat[a * 5 + qb]; };
    plo[k] = (sc(0) & 0xFF) | ((sc(1) & 0xFF) << 8) | ((sc(2) & 0xFF) << 16) | ((sc(3) & 0xFF) << 24);
    phi[k] = sc(4);
    blk[k] = slen > 0 ? x / slen : 0;
    Hp[k] = E[k] = Hm[k] = 0;
  }
  int gmax = 0, te = -1, n_b = 0, last_i = -2, last_v = 0;  // b[]'s last entry (column, score): wave-uniform
  for (int i = 0; i < tlen; ++i) {
    const int tb = first_lane(t_at(i));
    int Mp[NK], u1[NK], u2[NK];
    int carry = 0;  // H(i - 1, x - 1) for lane 0 of slot k: lane 63 of slot k - 1
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int x = lane + 64 * k;
      const int hd = dpp_wave_shr1_i(carry, Hp[k]);
      carry = read_lane(Hp[k], 63);
      const int s = prof_score(plo[k], phi[k], tb);
      int m = u8 ? max(min(hd + s + shift, 255) - shift, 0) : max(min(hd + s, 32767), -32768);
      m = max(m, E[k]);
      Mp[k] = m;
      const bool in = x < nlen;
      u1[k] = in ? m - oe_ins + x * e_ins + blk[k] * kBlockBig : kScanNeg;
      u2[k] = in ? m - oe_ins + x * e_ins : kScanNeg;
    }
    int ex1[NK], ex2[NK];
    excl_scan<NK>(u1, kScanNeg, ex1);
    excl_scan<NK>(u2, kScanNeg, ex2);
    int imax = 0;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int x = lane + 64 * k;
      const bool in = x < nlen;
      const bool first = slen == 0 || x % slen == 0;
      const int f1 = first ? 0 : max(0, ex1[k] - blk[k] * kBlockBig - (x - 1) * e_ins);
      const int h1 = max(Mp[k], f1);
      const int f2 = x == 0 ? 0 : max(0, ex2[k] - (x - 1) * e_ins);
      E[k] = in ? max(max(E[k] - e_del, 0), max(h1 - oe_del, 0)) : 0;
      Hp[k] = in ? max(h1, f2) : 0;
      imax = max(imax, in ? h1 : 0);
    }
    imax = wave_max(imax);
    if (imax >= minsc) {  // bwa's b[]: append, or raise the last entry when it holds the previous column
      if (n_b == 0 || last_i + 1 != i) {
        if (lane == 0) blist[n_b] = (uint64_t)(uint32_t)imax << 32 | (uint32_t)i;
        ++n_b;
        last_i = i, last_v = imax;
      } else if (last_v < imax) {
        if (lane == 0) blist[n_b - 1] = (uint64_t)(uint32_t)imax << 32 | (uint32_t)i;
        last_i = i, last_v = imax;
      }
    }
    if (imax > gmax) {
      gmax = imax;
      te = i;
#pragma unroll
      for (int k = 0; k < NK; ++k) Hm[k] = Hp[k];
      if ((u8 && gmax + shift >= 255) || gmax >= endsc) break;
    }
  }
  AlignRun r{u8 ? (gmax + shift < 255 ? gmax : 255) : gmax, te, -1, -1, -1};
  if (!u8 || r.score != 255) {
    int mx = -1;
#pragma unroll
    for (int k = 0; k < NK; ++k)
      if (lane + 64 * k < nlen) mx = max(mx, Hm[k]);
    mx = wave_max(mx);
    int qe = 0x7FFFFFFF;  // the smallest position holding the column maximum (bwa's scan keeps it)
#pragma unroll
    for (int k = 0; k < NK; ++k)
      if (lane + 64 * k < nlen && Hm[k] == mx) qe = min(qe, lane + 64 * k);
    r.qe = -wave_max(-qe);
    if (n_b > 0) {
      __syncthreads();  // lane 0's b[] stores before every lane reads them
      const int w = (r.score + max_mat - 1) / max_mat;
      const int low = te - w, high = te + w;
      int best = -1, bte = -1;
      for (int j = lane; j < n_b; j += 64) {  // the first entry (column order) of the largest score outside the window
        const uint64_t e = blist[j];
        const int c = (int)(uint32_t)e, v = (int)(e >> 32);
        if ((c < low || c > high) && v > best) best = v, bte = c;
      }
      const int vmax = wave_max(best);
      if (vmax > -1) {
        const int c = bte >= 0 && best == vmax ? bte : 0x7FFFFFFF;
        r.score2 = vmax;
        r.te2 = -wave_max(-c);
      }
    }
  }
  return r;
}

template <int NK>
__global__ __launch_bounds__(64) void bsw_align_kernel(const BswDevBatch b, const BswParams p,
                                                       const int32_t* __restrict__ xtra, int32_t* __restrict__ out,
                                                       int max_tlen) {
  extern __shared__ __align__(16) unsigned char smem[];
  uint64_t* const blist = reinterpret_cast<uint64_t*>(smem);
  uint8_t* const tl = smem + 8 * (size_t)max_tlen;
  const int lane = lane_id();
  // bwa's shift (u8 bias) and max_mat from the 5 x 5 matrix, as ksw_qinit
  int mn = 127, mxm = 0;
  for (int a = 0; a < 25; ++a) mn = min(mn, (int)p.mat[a]), mxm = max(mxm, (int)p.mat[a]);
  const int shift = (256 - (int)(uint8_t)(int8_t)mn) & 0xFF;
  for (long long task = blockIdx.x; task < b.n; task += gridDim.x) {
    const int qlen = b.qlen[task], tlen = b.tlen[task], xt = xtra[task];
    const uint8_t* __restrict__ q = b.qbuf + b.qoff[task];
    const uint8_t* __restrict__ tg = b.tbuf + b.toff[task];
    for (int i = lane; i < tlen; i += 64) tl[i] = tg[i];
    __syncthreads();
    const bool u8 = (xt & kKswXByte) != 0;
    const int minsc = (xt & kKswXSubo) ? xt & 0xffff : 0x10000;
    const int endsc = (xt & kKswXStop) ? xt & 0xffff : 0x10000;
    AlignRun r = align_run<NK>(
        p, qlen, [&](int x) { return (int)q[x]; }, tlen, [&](int j) { return (int)tl[j]; }, u8, shift, mxm, minsc,
        endsc, blist);
    int tb = -1, qb = -1;
    if ((xt & kKswXStart) && !((xt & kKswXSubo) && r.score < (xt & 0xffff))) {
      // bwa: reverse query[0, qe] and target[0, te] in place (the rest of the
      // target unchanged, full tlen), stop at the first score, no b[] list
      const int qe = r.qe, te = r.te;
      const AlignRun rr = align_run<NK>(
          p, qe + 1, [&](int x) { return (int)q[qe - x]; }, tlen,
          [&](int j) { return (int)tl[j <= te ? te - j : j]; }, u8, shift, mxm, 0x10000, r.score, blist);
      if (rr.score == r.score) tb = r.te - rr.te, qb = r.qe - rr.qe;
    }
    if (lane == 0) {
      int32_t* o = out + 7 * task;
      o[0] = r.score, o[1] = r.te, o[2] = r.qe, o[3] = r.score2, o[4] = r.te2, o[5] = tb, o[6] = qb;
    }
    __syncthreads();  // the next task rewrites the target and the b[] list
  }
}

int launch_bsw_align(const BswDevBatch& b, const BswParams& p, const int32_t* xtra, int max_qlen, int max_tlen,
                     int32_t* out, hipStream_t s) {
  if (b.n <= 0) return FCS_OK;
  if (max_qlen > 1024) return fail(FCS_ERR_UNSUPPORTED, "[E::fcship] ksw_align2: qlen > 1024 unsupported");
  const size_t lds = 8 * (size_t)max(max_tlen, 1) + (size_t)((max_tlen + 15) / 16) * 16;
  if (lds > 64 * 1024) return fail(FCS_ERR_UNSUPPORTED, "[E::fcship] ksw_align2: tlen too large");
  const unsigned grid = (unsigned)std::min<long long>(b.n, 4096);
  // slots of 64 positions for slen * p (p = 16 u8 / 8 i16: at most qlen + 15)
  const int nlen = max_qlen + 15;
  if (nlen <= 256)
    hipLaunchKernelGGL(bsw_align_kernel<4>, dim3(grid), dim3(64), lds, s, b, p, xtra, out, max_tlen);
  else
    hipLaunchKernelGGL(bsw_align_kernel<17>, dim3(grid), dim3(64), lds, s, b, p, xtra, out, max_tlen);
  FCS_HIP_CHECK(hipGetLastError());
  return FCS_OK;
}

}  // namespace fcs

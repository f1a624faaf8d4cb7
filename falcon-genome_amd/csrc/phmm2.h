// PairHMM fp32 forward pass, two read rows per lane (included by
// phmm_kernels.hip after the one-row kernel's helpers).
//
// Same wave shape as phmm_kernel (four pairs per wave, one per 16-lane DPP
// row, an LDS boundary ring per pair), but lane l owns read rows 2l + 1 and
// 2l + 2 of a 32-row stripe ("row a" and "row b"), row b one column behind
// row a.  Every recurrence value is a float pair {row a, row b} and the whole
// cell update is seven packed FP32 instructions (v_pk_mul_f32 / v_pk_fma_f32)
// for the two cells.  Row a takes its inputs from row b of the lane below by
// DPP row_shr:1 (lane 0: from the ring), row b from row a of the same lane one
// step earlier.  The inputs are built in place as swapped pairs {b, a} in the
// previous step's output registers and read through op_sel, so a step is
//   2 DPP + 2 lane-0 selects (X, I of row a) + 2 x 2 for the emission priors
//   + 7 packed FP, one ring read, one hap-code read, and lane 15's ring write
//   (one ds_write2_b32 under a 2-SALU exec mask)
// for TWO cells, ~25 instructions; the one-row kernel spends ~19 per cell
// (11-13 VALU + 3 LDS + 2 SALU + waits) and is bound by per-wave instruction
// issue (SQ_ACTIVE_INST_ANY counts a quad-cycle per instruction of any kind;
// profiles/r1/stalls), not by the VALU pipe.  Costs: stripes of 32 rows
// (R = 101 runs 128 rows, not 112), a 31-step fill instead of 15, and 3 waves
// per SIMD instead of 4.  C2: 2.43 -> 2.64 TCUPS (gpurun_out/abp4).
//
// Columns: at step t row a computes c = t - 2l, row b c - 1.  Ring slot =
// column + 16 as in the one-row kernel (nslot >= H + 65); hap slot = column +
// 32 (lane 15 reads column t - 30 + PFD), nslot + 16 hap bytes per pair.
// Lane 15 writes row b's X(r, c), I(r + 1, c) (c = t - 31) to ring slot
// t - 15 from the second block on (the first block's columns are negative).
#pragma once

// 3 waves per SIMD (<= 168 VGPRs; LDS allows ~3.5 at H ~ 225): capped at 128
// VGPRs for 4 the kernel spills 33 VGPRs to scratch.
constexpr int kPhmm2Waves = 3;

namespace fcs {

typedef float pf2 __attribute__((ext_vector_type(2)));

struct RowP2 {
  pf2 e1, e3, my, yy;  // own rows a, b: emission priors, deletion transitions (my * gm of the row below)
  pf2 mm, gm, mx, xx;  // the rows below a and b: match/gap-to-match, insertion transitions
  int ra, rb;          // read base bytes (byte-compare groups)
  int ma, mb;          // hap-code match masks (base_mask)
};

__device__ __forceinline__ RowP2 row_params2(const PhmmTables<float>& tab, const RawRow& a, const RawRow& b) {
  const RowP<float> pa = row_params<float, false>(tab, a), pb = row_params<float, false>(tab, b);
  RowP2 p;
  p.e1 = pf2{pa.e1, pb.e1};
  p.e3 = pf2{pa.e3, pb.e3};
  p.my = pf2{pa.my, pb.my};
  p.yy = pf2{pa.yy, pb.yy};
  p.mm = pf2{pa.mm, pb.mm};
  p.gm = pf2{pa.gm, pb.gm};
  p.mx = pf2{pa.mx, pb.mx};
  p.xx = pf2{pa.xx, pb.xx};
  p.ra = pa.rbase;
  p.rb = pb.rbase;
  p.ma = pa.rmask;
  p.mb = pb.rmask;
  return p;
}

struct Lane2 {
  pf2 Mo, Do;  // own M, D' at the previous column
  pf2 Xp;      // X inputs for this step's M (received last step)
  pf2 Xn, In;  // last step's outputs: X(r, c), I(r + 1, c) of rows a, b
  int hbp;     // row a's hap code of the last step = row b's of this step
};

// 32-bit LDS address of a pointer into dynamic shared memory.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

__device__ __forceinline__ float prior_code(int mask, int hb, float e1, float e3) {
  int bit;
  asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(bit) : "v"(mask), "v"(hb));  // hb < 256: no masking of the offset
  return sel_bits((uint32_t)bit, e1, e3);
}

template <bool SUM, bool BC, bool COND, bool WRITE, int S>
__device__ __forceinline__ void phmm2_step(Lane2& L, PhRing<float> (&pf)[PFD], int (&hq)[PFD],
                                           const unsigned char* __restrict__ hapl, const RowP2& p,
                                           PhRing<float>* __restrict__ ring, const int t0, const int sl2,
                                           const bool lane0, const bool top, const int lim_a, const int lim_b,
                                           pf2& accM, pf2& accI, const uint32_t wbase, const int tdyn = 0) {
  const int t = S >= 0 ? t0 + S : tdyn;
  const PhRing<float> cur = pf[0];
  const int hba = hq[0];
#pragma unroll
  for (int k = 0; k + 1 < PFD; ++k) {
    pf[k] = pf[k + 1];
    hq[k] = hq[k + 1];
  }
  pf[PFD - 1] = ring[t + 16 + PFD];       // lane-0 input for column t + PFD
  hq[PFD - 1] = hapl[t + 32 + PFD - sl2];  // row a's hap code for column t + PFD - 2l
  const int hbb = L.hbp;
  L.hbp = hba;
  // row a <- row b of the lane below (lane 0: the ring); row b <- row a, one step back
  // X and I inputs as swapped pairs {row b, row a} built in place in last
  // step's output pairs: row a's half is the DPP'd row b of the lane below
  // (lane 0: the ring), row b's half is this lane's own row a, already there;
  // the packed ops read them with op_sel swapped (no register moves).
  pf2 Xsw = L.Xn, Isw = L.In;
  Xsw.y = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(L.Xn.y), kDppRowShr1, 0xF, 0xF, true));
  Isw.y = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(L.In.y), kDppRowShr1, 0xF, 0xF, true));
  Xsw.y = lane0 ? cur.X : Xsw.y;
  Isw.y = lane0 ? cur.I : Isw.y;
  const pf2 I = __builtin_shufflevector(Isw, Isw, 1, 0);
  pf2 prior;
  if constexpr (BC) {
    prior.x = (hba == p.ra || hba == 'N') ? p.e1.x : p.e3.x;
    prior.y = (hbb == p.rb || hbb == 'N') ? p.e1.y : p.e3.y;
  } else {
    prior.x = prior_code(p.ma, hba, p.e1.x, p.e3.x);
    prior.y = prior_code(p.mb, hbb, p.e1.y, p.e3.y);
  }
  const pf2 M = __builtin_shufflevector(L.Xp, L.Xp, 1, 0) * prior;
  const pf2 D = __builtin_elementwise_fma(L.Mo, p.my, L.Do * p.yy);
  const pf2 Xn = __builtin_elementwise_fma(M, p.mm, __builtin_elementwise_fma(I, p.gm, D));
  const pf2 In = __builtin_elementwise_fma(M, p.mx, I * p.xx);
  if constexpr (WRITE) {
    if (top) {  // row b of lane 15, column t - 31 -> slot t - 15
      // one ds_write2_b32 of the two halves: a 64-bit store would need them
      // moved into one register pair first (two v_mov per step).  LDS ops of
      // a wave complete in order, so the compiler's lgkmcnt waits (which do
      // not count this store) stay correct.
      if constexpr (S >= 0)
        asm volatile("ds_write2_b32 %0, %1, %2 offset0:%3 offset1:%4"
                     :
                     : "v"(wbase), "v"(Xn.y), "v"(In.y), "i"(2 * S), "i"(2 * S + 1)
                     : "memory");
      else
        asm volatile("ds_write2_b32 %0, %1, %2 offset1:1" : : "v"(lds_addr(ring + (t - 15))), "v"(Xn.y), "v"(In.y)
                     : "memory");
    }
  }
  if constexpr (SUM) {
    // The summing row runs with my = yy = 1, so D is its running M sum; both
    // halves accumulate I every step (the non-summing half is dropped) and the
    // sum over columns 1..H is captured, branch-free, at the step of column H.
    accI += I;
    if constexpr (COND) {
      const float sa = accI.x + (D.x + M.x), sb = accI.y + (D.y + M.y);
      accM.x = (t == lim_a) ? sa : accM.x;
      accM.y = (t == lim_b) ? sb : accM.y;
    }
  }
  L.Xp = Xsw;
  L.Xn = Xn;
  L.In = In;
  L.Mo = M;
  L.Do = D;
}

template <bool SUM, bool BC, bool COND, bool WRITE>
__device__ __forceinline__ void phmm2_block(Lane2& L, PhRing<float> (&pf)[PFD], int (&hq)[PFD],
                                            const unsigned char* __restrict__ hapl, const RowP2& p,
                                            PhRing<float>* __restrict__ ring, const int t0, const int sl2,
                                            const bool lane0, const bool top, const int lim_a, const int lim_b,
                                            pf2& accM, pf2& accI) {
  if constexpr (COND) {
    // the blocks holding a summing row's last column (a few per summing
    // stripe): one step at a time, so their captures do not hold 16 steps'
    // compares and extra values live through the unrolled code
#pragma unroll 1
    for (int u = 0; u < 16; ++u)
      phmm2_step<SUM, BC, COND, WRITE, -1>(L, pf, hq, hapl, p, ring, t0, sl2, lane0, top, lim_a, lim_b, accM, accI,
                                           0, t0 + u);
    return;
  }
  const uint32_t wbase = lds_addr(ring + (t0 - 15));  // ring slot t0 - 15: this block's first write
  [&]<int... S>(std::integer_sequence<int, S...>) {
    (phmm2_step<SUM, BC, COND, WRITE, S>(L, pf, hq, hapl, p, ring, t0, sl2, lane0, top, lim_a, lim_b, accM, accI,
                                         wbase),
     ...);
  }(std::make_integer_sequence<int, 16>{});
}

template <bool SUM, bool BC>
__device__ __forceinline__ void phmm2_stripe(const RowP2& p, PhRing<float>* __restrict__ ring,
                                             const unsigned char* __restrict__ hapl, const int sl, const int nblk,
                                             const int lim_a, const int lim_b, const int ulim, pf2& accM, pf2& accI,
                                             const PhmmTables<float>& tab, const RawRow& na, const RawRow& nb,
                                             RowP2& np, const bool top) {
  const bool lane0 = sl == 0;
  const int sl2 = 2 * sl;
  Lane2 L;
  L.Mo = L.Do = L.Xp = L.Xn = L.In = pf2{0.f, 0.f};
  L.hbp = 6;
  PhRing<float> pf[PFD];
  int hq[PFD];
#pragma unroll
  for (int k = 0; k < PFD; ++k) {
    pf[k] = ring[16 + k];
    hq[k] = hapl[32 + k - sl2];
  }
  // block 0: every row-b column of lane 15 is negative, nothing to write
  if (!SUM || 15 < ulim)
    phmm2_block<SUM, BC, false, false>(L, pf, hq, hapl, p, ring, 0, sl2, lane0, top, lim_a, lim_b, accM, accI);
  else
    phmm2_block<SUM, BC, true, false>(L, pf, hq, hapl, p, ring, 0, sl2, lane0, top, lim_a, lim_b, accM, accI);
  np = row_params2(tab, na, nb);
  for (int blk = 1; blk < nblk; ++blk) {
    if (!SUM || 16 * blk + 15 < ulim)
      phmm2_block<SUM, BC, false, true>(L, pf, hq, hapl, p, ring, 16 * blk, sl2, lane0, top, lim_a, lim_b, accM, accI);
    else
      phmm2_block<SUM, BC, true, true>(L, pf, hq, hapl, p, ring, 16 * blk, sl2, lane0, top, lim_a, lim_b, accM, accI);
  }
}

// LDS layout of one wave: four rings, then four hap-code arrays.
__host__ __device__ constexpr int ring2_stride(int nslot) { return nslot * 8; }
__host__ __device__ constexpr int hap2_stride(int nslot) { return nslot + 16; }
__host__ __device__ constexpr int phmm2_lds(int nslot) { return 4 * (ring2_stride(nslot) + hap2_stride(nslot)); }

// Forward pass (fp32, FMA order) of one hap-length class; nslot >= H + 66.
__global__ __launch_bounds__(64, kPhmm2Waves) void phmm2_kernel(const PhmmDevBatch b, const int32_t* __restrict__ order,
                                                      const int64_t* __restrict__ bounds, const int cls,
                                                      const int nslot, const PhmmTables<float> tab,
                                                      double* __restrict__ out, int32_t* __restrict__ rescue_list,
                                                      unsigned long long* __restrict__ rescue_count, const float thr,
                                                      const int use_rescue) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  const int lane = threadIdx.x;
  const int seg = lane >> 4;
  const int sl = lane & 15;
  PhRing<float>* const ring = reinterpret_cast<PhRing<float>*>(smem_raw + seg * ring2_stride(nslot));
  const int nhap = nslot + 16;
  unsigned char* const hapl = smem_raw + (size_t)4 * ring2_stride(nslot) + seg * hap2_stride(nslot);
  const bool top = sl == 15;
  order += bounds[cls];
  const long long count = bounds[cls + 1] - bounds[cls];
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
    const int nstr = active ? (R + 31) >> 5 : 0;
    const int Hmax = wave_max(active ? H : 0);
    const int nstr_max = wave_max(nstr);
    if (nstr_max == 0) continue;

    // ring <- row 0 as seen by row 1, hap codes by column + 16 (as phmm_kernel)
    const float init = active ? tab.init_const / (float)H : 0.f;
    const float x0 = active ? init * tab.dmatch[b.gq[ro] & 127] : 0.f;
    __syncthreads();
    for (int s = sl; s < nslot; s += 16) {
      const int c = s - 16;
      PhRing<float> v;
      v.X = (c >= 0 && c <= H) ? x0 : 0.f;
      v.I = 0.f;
      ring[s] = v;
    }
    // hap codes by column + 32: eight slots per lane per batch, loads first
    bool other = false;
    constexpr int kHB = 8;
    for (int s0 = sl; s0 < nhap; s0 += 16 * kHB) {
      unsigned char raw[kHB];
#pragma unroll
      for (int u = 0; u < kHB; ++u) {
        const int c = s0 + 16 * u - 32;
        raw[u] = (active && c >= 1 && c <= H) ? b.hb[ho + c - 1] : (unsigned char)0;
      }
#pragma unroll
      for (int u = 0; u < kHB; ++u) {
        const int s = s0 + 16 * u, c = s - 32;
        if (s < nhap) {
          const bool in = active && c >= 1 && c <= H;
          const unsigned char code = in ? base_code(raw[u]) : (unsigned char)6;
          other |= code == 5;
          hapl[s] = code;
        }
      }
    }
    const bool bytecmp = __ballot(other) != 0ull;
    if (bytecmp)
      for (int s = sl; s < nhap; s += 16) {
        const int c = s - 32;
        hapl[s] = (active && c >= 1 && c <= H) ? b.hb[ho + c - 1] : (unsigned char)0;
      }
    __syncthreads();

    const int Ra = active ? R : 0;
    RowP2 prm = row_params2(tab, load_raw(b, Ra, ro, 2 * sl), load_raw(b, Ra, ro, 2 * sl + 1));
    pf2 accM{0.f, 0.f}, accI{0.f, 0.f};
    const int sum_stripe = active ? (R - 1) >> 5 : -1;
    const int sum_lane = active ? ((R - 1) & 31) >> 1 : -1;
    const int sum_half = active ? (R - 1) & 1 : -1;
    for (int st = 0; st < nstr_max; ++st) {
      const RawRow na = load_raw(b, Ra, ro, (st + 1) * 32 + 2 * sl);
      const RawRow nb = load_raw(b, Ra, ro, (st + 1) * 32 + 2 * sl + 1);
      RowP2 nprm;
      const bool seg_sums = (st == sum_stripe);
      const int any_sum = wave_max(seg_sums ? 1 : 0);
      if (any_sum) {
        const bool mine = seg_sums && sl == sum_lane;
        const int cont = wave_max((active && nstr > st + 1) ? 1 : 0);
        const int mylim = mine ? H + 2 * sl + sum_half : -1;  // step of the summing row's last column
        const int lim_a = (mine && sum_half == 0) ? mylim : -1;
        const int lim_b = (mine && sum_half == 1) ? mylim : -1;
        const int ulim = -wave_max(mine ? -mylim : -0x7FFFFFFF);
        accM = accI = pf2{0.f, 0.f};
        const int tend = cont ? Hmax + 31 : wave_max(mine ? mylim : 0);
        RowP2 sp = prm;
        if (lim_a >= 0) sp.my.x = sp.yy.x = 1.f;
        if (lim_b >= 0) sp.my.y = sp.yy.y = 1.f;
        if (bytecmp)
          phmm2_stripe<true, true>(sp, ring, hapl, sl, (tend + 16) >> 4, lim_a, lim_b, ulim, accM, accI, tab, na, nb,
                                   nprm, top);
        else
          phmm2_stripe<true, false>(sp, ring, hapl, sl, (tend + 16) >> 4, lim_a, lim_b, ulim, accM, accI, tab, na,
                                    nb, nprm, top);
        if (mine) {
          const float sum = sum_half ? accM.y : accM.x;
          if (use_rescue && sum < thr) {
            const unsigned long long k = atomicAdd(rescue_count, 1ull);
            rescue_list[k] = p;
            out[p] = __builtin_nan("");
          } else {
            out[p] = (double)(log10f(sum) - tab.log10_init);
          }
        }
      } else {
        if (bytecmp)
          phmm2_stripe<false, true>(prm, ring, hapl, sl, (Hmax + 47) >> 4, -1, -1, -1, accM, accI, tab, na, nb, nprm,
                                    top);
        else
          phmm2_stripe<false, false>(prm, ring, hapl, sl, (Hmax + 47) >> 4, -1, -1, -1, accM, accI, tab, na, nb,
                                     nprm, top);
      }
      prm = nprm;
    }
  }
}

}  // namespace fcs

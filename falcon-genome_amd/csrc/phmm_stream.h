// PairHMM fp32 forward pass with row-streamed segments (included by
// phmm_kernels.hip after phmm2.h).
//
// phmm2_kernel gives each 16-lane segment one pair and runs its rows in
// stripes of 32 (two rows per lane), so a read of R = 101 rows occupies 128:
// the last stripe computes 5 useful rows at the price of 32 (C2: 35% of the
// cell slots idle).  Here a segment runs a STREAM of K pairs back to back:
// the stream's rows are cut into 32-row stripes regardless of pair
// boundaries, so a stripe may finish one pair in its low lanes and start the
// next in its high lanes.  Only the stream's very end is quantised.
//
// Per pair the stream holds, in two-row units (lane row a, row b):
//   [pad if R is even] rows 1..R, V
// where V is a virtual row R + 1 that sums the last row.  The step is exactly
// phmm2's (seven packed FP32 ops per two cells, same DPP hand-off and LDS
// boundary ring); only the per-row constants change:
//   * row 1 starts the pair: its lane reads the row-0 boundary from a 64-entry
//     LDS constant Z ({1, 0} at columns >= 0, {0, 0} below) instead of the
//     lane below / ring, and its emission priors are pre-multiplied by
//     x0 = (2^120 / H) * gm_1, so M(1, c) = (prior * x0) * 1 = prior * x0
//     bitwise as in phmm2 (whose ring holds x0 itself);
//   * the pad row (R even) passes Z through one column later (prior 1, mm 1,
//     everything else 0), so row 1 sits in a row b and V again in a row b;
//   * row R hands the row below X = M + I (mm = gm = 1, D killed by my = 0) and
//     I = 0;
//   * V (prior 1, my = yy = 1, mm = gm = 1) keeps D = running sum of its M =
//     sum over c of (M + I)(R, c) in column order, and hands X = M + D: at its
//     column H + 1 that is sum_{c = 1..H} (M + I)(R, c).  The capture is one
//     compare-select in the (at most two) 16-step blocks that hold some V
//     lane's column H + 1 — no per-step accumulator anywhere.
// Lane 0 of a stripe continues its pair from the segment's LDS ring that lane
// 15 wrote in the previous stripe, exactly as in phmm2.  A pair spans >= 17
// units (R >= 33, enforced by the schedule), so a stripe holds at most two
// pairs of a segment and the segment keeps two hap-code buffers (pair parity).
// Ring, hap codes and Z are read a few columns past a pair's end and before
// its start; those columns only feed columns > H or multiply exact zeros, so
// their content is irrelevant and the arrays are sized to the written ranges.
// Pairs whose haplotype holds bytes outside A/C/G/T/N (the hap codes cannot
// express GKL's byte compare) are handed to a fallback list that the one-row
// kernel recomputes; their streamed results are discarded.
#pragma once

namespace fcs {

constexpr int kStreamHalf = 8;   // a stripe's last block runs 8 steps when that suffices
constexpr int kStreamPfd = 2;    // LDS read-ahead (steps) of the ring and hap-code reads
constexpr int kStreamMinR = 33;  // a pair spans >= 17 units: at most two pairs per stripe and segment
constexpr int kStreamMaxR = 0xFFFF;  // a segment packs R | H << 16 between stripes; longer reads take phmm2
constexpr int kStreamMaxK = 8;   // pairs per segment stream
constexpr uint64_t kTopLanes = 0x8000800080008000ull;  // lane 15 of each 16-lane segment
// Hap-length bounds of the stream classes: LDS <= 13,312 B per wave (3 waves per
// SIMD at the 512-byte allocation granularity), <= 20 KB (2), and the 160 KB
// limit.  Classes 0 and 1 both run at 3 waves per SIMD: at 4 (10,240 B) the
// kernel's 128-VGPR budget spilled 9 VGPRs and measured the same time as 3
// (DESIGN §4.1); class 0 keeps its smaller LDS footprint.
__host__ __device__ constexpr int stream_class_hmax(int c) {
  return c == 0 ? 224 : c == 1 ? 300 : c == 2 ? 472 : 3700;
}
// Waves per SIMD the class's launch bounds ask for (its LDS allows as many).
__host__ __device__ constexpr int stream_class_waves(int c) { return c <= 1 ? 3 : c == 2 ? 2 : 1; }
__host__ __device__ inline int stream_class(int H) {
  for (int c = 0; c < kStreamClasses; ++c)
    if (H <= stream_class_hmax(c)) return c;
  return -1;
}
// LDS per wave: Z (64 ring entries) | four rings of hmax + 18 slots (slot =
// column; a stripe runs to step 16 * ceil((H + 33) / 16) - 1 <= H + 47, so lane
// 15 writes columns 1 .. hmax + 16) | eight hap-code buffers of hmax + 10 bytes
// (column c at 3 + (address & 3) + c: whole aligned dwords of the hap bytes are
// converted in place) | 64 bytes of read-ahead tail.
__host__ __device__ constexpr int stream_nslot(int hmax) { return hmax + 18; }
__host__ __device__ constexpr int stream_hstride(int hmax) { return (hmax + 12) & ~3; }
__host__ __device__ constexpr int stream_lds(int hmax) {
  return 512 + 4 * 8 * stream_nslot(hmax) + 8 * stream_hstride(hmax) + 64;
}

// Per-row constants of one half (role: 0 idle, 1 pad, 2 row r < R, 3 row R, 4 V).
struct SRowC {
  float e1, e3, my, yy, mm, gm, mx, xx;
  int mask;
};

// Branch-free (selects only): an SRowC assembled in role branches was merged
// through a 36-byte stack copy, i.e. a scratch store + reload per stripe
// (0.5-0.8 GB of scratch traffic per C2 pass, profiles/r2/r2d_*).
__device__ __forceinline__ SRowC srow_params(const PhmmTables<float>& tab, const RawRow& raw, int role, bool first,
                                             float init_h) {
  const RowP<float> q = row_params<float, false>(tab, raw);
  const bool real = role == 2 || role == 3;  // rows 1..R
  const bool mid = role == 2;                // rows 1..R-1
  const bool last = role == 3;               // row R hands X = M + I, I = 0; D is never needed by anyone
  const bool v = role == 4;                  // V: D = running sum of M; X = M + D
  const bool pad = role == 1;                // pad: X = prior * Xp = Z one column on, I = 0, D = 0
  // row 1: M(1, c) = prior * x0 (x0 = X(0, c - 1) for c - 1 >= 0); x * 1.f is exact elsewhere.
  // init_h = 2^120 / H, divided once per pair at batch start (two divisions per
  // stripe here were ~54 VALU of the stripe's ~700)
  const float x0 = first ? init_h * tab.dmatch[raw.gq & 127] : 1.f;
  const float one_vp = (v || pad) ? 1.f : 0.f;
  SRowC c;
  c.e1 = real ? q.e1 * x0 : one_vp;
  c.e3 = real ? q.e3 * x0 : one_vp;
  c.my = mid ? q.my : v ? 1.f : 0.f;
  c.yy = real ? q.yy : v ? 1.f : 0.f;
  c.mm = mid ? q.mm : (last || v || pad) ? 1.f : 0.f;
  c.gm = mid ? q.gm : (last || v) ? 1.f : 0.f;
  c.mx = mid ? q.mx : 0.f;
  c.xx = mid ? q.xx : 0.f;
  c.mask = real ? q.rmask : 0;
  return c;
}

__device__ __forceinline__ RowP2 srow_pack(const SRowC a, const SRowC b) {
  RowP2 p;
  p.e1 = pf2{a.e1, b.e1};
  p.e3 = pf2{a.e3, b.e3};
  p.my = pf2{a.my, b.my};
  p.yy = pf2{a.yy, b.yy};
  p.mm = pf2{a.mm, b.mm};
  p.gm = pf2{a.gm, b.gm};
  p.mx = pf2{a.mx, b.mx};
  p.xx = pf2{a.xx, b.xx};
  p.ra = p.rb = 0;
  p.ma = a.mask;
  p.mb = b.mask;
  return p;
}

// Where one lane sits in a stripe: pair (index k in its segment, batch index
// p), unit u of the pair, its rows and their roles.
struct SLane {
  int k, p, R, H, u;
  float ih;  // 2^120 / H (GKL's initial D row value), computed once per pair
  int64_t ro;
  int role_a, role_b, ra, rb;  // rb = ra + 1; rows are 1-based, 0 = pad
  bool act;
};

__device__ __forceinline__ int srole(int r, int R) { return r == 0 ? 1 : r < R ? 2 : r == R ? 3 : 4; }

// One step: phmm2_step without the byte-compare and summing variants; the
// boundary source is this block's per-lane pointer `rd` (ring or Z) and COND
// captures the V lanes' X at their column H + 1.
// Start-lane select as one full-rate v_bitop3_b32 on a per-lane mask VGPR:
// v_cndmask_b32 on an SGPR lane mask issues at half the rate (4 cycles per
// wave64 instruction on gfx950 vs 2; tools/micro/valu_rate.hip, profiles/r3/r3m).
__device__ __forceinline__ float sel_v(uint32_t m, float a, float b) {
  float r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xe4" : "=v"(r) : "v"(a), "v"(b), "v"(m));
  return r;
}

template <bool COND, bool WRITE, int S, int PF>
__device__ __forceinline__ void pstream_step(Lane2& L, PhRing<float> (&pf)[PF], int (&hq)[PF],
                                             const unsigned char* __restrict__ hp, const PhRing<float>* __restrict__ rd,
                                             const RowP2& p, const uint32_t smask, const int t0, const int dl,
                                             float& acc, const uint32_t wbase) {
  const int t = t0 + S;
  const PhRing<float> cur = pf[0];
  const int hba = hq[0];
#pragma unroll
  for (int k = 0; k + 1 < PF; ++k) {
    pf[k] = pf[k + 1];
    hq[k] = hq[k + 1];
  }
  pf[PF - 1] = rd[S];  // boundary input for step t + PF
  hq[PF - 1] = hp[t];  // row a's hap code for column t + PF - 2l
  const int hbb = L.hbp;
  L.hbp = hba;
  pf2 Xsw = L.Xn, Isw = L.In;
  Xsw.y = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(L.Xn.y), kDppRowShr1, 0xF, 0xF, true));
  Isw.y = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(L.In.y), kDppRowShr1, 0xF, 0xF, true));
  Xsw.y = sel_v(smask, cur.X, Xsw.y);
  Isw.y = sel_v(smask, cur.I, Isw.y);
  const pf2 I = __builtin_shufflevector(Isw, Isw, 1, 0);
  pf2 prior;
  prior.x = prior_code(p.ma, hba, p.e1.x, p.e3.x);
  prior.y = prior_code(p.mb, hbb, p.e1.y, p.e3.y);
  const pf2 M = __builtin_shufflevector(L.Xp, L.Xp, 1, 0) * prior;
  const pf2 D = __builtin_elementwise_fma(L.Mo, p.my, L.Do * p.yy);
  const pf2 Xn = __builtin_elementwise_fma(M, p.mm, __builtin_elementwise_fma(I, p.gm, D));
  const pf2 In = __builtin_elementwise_fma(M, p.mx, I * p.xx);
  if constexpr (WRITE) {
    // row b of lane 15, column t - 31 -> ring slot t - 31: EXEC narrowed to the
    // four lanes 15 inside the statement, so the step stays one basic block (a
    // branch per step cost six SALU, and values carried across the blocks were
    // re-zero-extended at each use)
    uint64_t keep;
    asm volatile(
        "s_mov_b64 %0, exec\n\t"
        "s_mov_b64 exec, %4\n\t"
        "ds_write2_b32 %1, %2, %3 offset0:%5 offset1:%6\n\t"
        "s_mov_b64 exec, %0"
        : "=&s"(keep)
        : "v"(wbase), "v"(Xn.y), "v"(In.y), "s"(kTopLanes), "i"(2 * S), "i"(2 * S + 1)
        : "memory");
  }
  else
    asm volatile("" ::: "memory");  // keep each step's LDS reads in their step (hoisted, they cost registers)
  if constexpr (COND)  // V lanes: take X at the step dl = lim - t0 (a compare-select in place, not
                       // sixteen compares hoisted into SGPR pairs; the VOP3 form of the select:
                       // the VOP2 form reading VCC issues at ~1/5 of its rate on gfx950,
                       // tools/micro/valu_rate.hip)
    asm volatile("v_cmp_eq_u32 vcc, %2, %3\n\tv_cndmask_b32_e64 %0, %0, %1, vcc"
                 : "+v"(acc)
                 : "v"(Xn.y), "i"(S), "v"(dl)
                 : "vcc");
  L.Xp = Xsw;
  L.Xn = Xn;
  L.In = In;
  L.Mo = M;
  L.Do = D;
}

template <bool COND, bool WRITE, int PF, int NS = 16>
__device__ __forceinline__ void pstream_block(Lane2& L, PhRing<float> (&pf)[PF], int (&hq)[PF],
                                              const unsigned char* __restrict__ hp,
                                              const PhRing<float>* __restrict__ rd, const RowP2& p,
                                              const uint32_t smask, const int t0, const int dl, float& acc,
                                              const uint32_t wbase) {
  [&]<int... S>(std::integer_sequence<int, S...>) {
    (pstream_step<COND, WRITE, S, PF>(L, pf, hq, hp, rd, p, smask, t0, dl, acc, wbase), ...);
  }(std::make_integer_sequence<int, NS>{});
}

// Hap bytes -> codes (A,C,G,T,N = 0..4), four per dword: (b >> 1) & 7 is
// distinct for A, C, T, G, N (0, 1, 2, 3, 7) and v_perm looks the code up; a
// byte whose code does not map back to itself is outside A/C/G/T/N.
__device__ __forceinline__ uint32_t hap_codes4(uint32_t x, uint32_t valid, bool& other) {
  const uint32_t sel = (x >> 1) & 0x07070707u;
  const uint32_t code = __builtin_amdgcn_perm(0x04050505u, 0x02030100u, sel);
  const uint32_t back = __builtin_amdgcn_perm(0x0000004Eu, 0x54474341u, code);
  other |= ((back ^ x) & valid) != 0u;
  return code;
}

template <int LB>
__global__ __launch_bounds__(64, LB) void phmm3_kernel(
    const PhmmDevBatch b, const int32_t* __restrict__ order, const int64_t* __restrict__ bounds, const int cls,
    const int K, const int tail_pairs, const int nslot, const int hstride, const PhmmTables<float> tab,
    double* __restrict__ out, int32_t* __restrict__ rescue_list, unsigned long long* __restrict__ rescue_count,
    const float thr, const int use_rescue, int32_t* __restrict__ fb_list, unsigned long long* __restrict__ fb_count) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  const int lane = threadIdx.x;
  const int seg = lane >> 4;
  const int sl = lane & 15;
  const int sbase = lane & 48;
  const int sl2 = 2 * sl;
  constexpr int PF = kStreamPfd;
  PhRing<float>* const Z = reinterpret_cast<PhRing<float>*>(smem_raw);
  PhRing<float>* const ring = reinterpret_cast<PhRing<float>*>(smem_raw + 512) + seg * nslot;
  unsigned char* const hbufs = smem_raw + 512 + 32 * nslot + 2 * seg * hstride;  // this segment's two buffers
  {
    PhRing<float> z;
    z.X = lane >= 32 ? 1.f : 0.f;
    z.I = 0.f;
    Z[lane] = z;
    if (sl == 0) {  // column 0 of the boundary is always {0, 0}; lane 15 never writes it
      PhRing<float> o;
      o.X = o.I = 0.f;
      ring[0] = o;
    }
  }
  const int64_t cbeg = bounds[cls];
  const long long count = bounds[cls + 1] - cbeg;
  order += cbeg;
  // Batches: K pairs per segment, except the range's last tail_pairs (its
  // shortest haplotypes), one pair per segment, so the launch ends on short waves.
  const long long tailn = count < (long long)tail_pairs ? count : (long long)tail_pairs;
  const long long headn = count - tailn;
  const long long per = 4LL * K;
  const long long nb_head = (headn + per - 1) / per;
  const long long nbatch = nb_head + (tailn + 3) / 4;

  for (long long w = blockIdx.x; w < nbatch; w += gridDim.x) {
    const bool head = w < nb_head;
    const int Kb = head ? K : 1;
    const long long bstart = head ? w * per : headn + (w - nb_head) * 4;
    const long long bend = head ? min(headn, bstart + per) : min(count, bstart + 4);
    // Segment table: lane k of the segment holds pair k of its stream.
    const long long idx = bstart + 4LL * sl + seg;
    const int pm = (sl < Kb && idx < bend) ? order[idx] : -1;
    int Rm = 0, Hm = 0, Um = 0;
    float Im = 0.f;
    int64_t rom = 0, hom = 0;
    if (pm >= 0) {
      const int ri = b.pair_read[pm], hi = b.pair_hap[pm];
      Rm = b.read_len[ri];
      Hm = b.hap_len[hi];
      rom = b.read_off[ri];
      hom = b.hap_off[hi];
      Um = (Rm + 2) >> 1;
      Im = tab.init_const / (float)Hm;
    }
    int ube = Um;  // inclusive prefix sum of units over the segment
    ube += __builtin_amdgcn_update_dpp(0, ube, kDppRowShr1, 0xF, 0xF, false);
    ube += __builtin_amdgcn_update_dpp(0, ube, kDppRowShr2, 0xF, 0xF, false);
    ube += __builtin_amdgcn_update_dpp(0, ube, kDppRowShr4, 0xF, 0xF, false);
    ube += __builtin_amdgcn_update_dpp(0, ube, kDppRowShr8, 0xF, 0xF, false);
    const int ubb = ube - Um;
    const int total = __shfl(ube, sbase + 15);
    const int nstr = (wave_max(total) + 15) >> 4;
    unsigned other = 0;  // bit k: pair k's haplotype needs the byte-compare fallback (segment-uniform)

    // Lane position in stripe st from the pair cursor kc of stripe st - 1
    // (advanced by at most one pair: every pair spans more than 16 units).
    int kc = 0;
    auto locate = [&](int st) {
      SLane s;
      const int g = 16 * st + sl;
      {
        const int e = __shfl(ube, sbase + min(kc, 15));
        if (kc < Kb && g >= e) ++kc;
      }
      const int kk = min(kc, 15);
      s.k = kc;
      s.act = g < total;
      s.p = __shfl(pm, sbase + kk);
      s.R = __shfl(Rm, sbase + kk);
      s.H = __shfl(Hm, sbase + kk);
      s.ih = __shfl(Im, sbase + kk);
      const int lo = __shfl((int)rom, sbase + kk), hi = __shfl((int)(rom >> 32), sbase + kk);
      s.ro = (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
      s.u = g - __shfl(ubb, sbase + kk);
      const int pad = (s.R & 1) ^ 1;
      s.ra = 2 * s.u + 1 - pad;
      s.rb = s.ra + 1;
      s.role_a = s.act ? srole(s.ra, s.R) : 0;
      s.role_b = s.act ? srole(s.rb, s.R) : 0;
      return s;
    };
    auto raw_of = [&](const SLane& s, int r, int role) {
      return (role == 2 || role == 3) ? load_raw(b, s.R, s.ro, r - 1) : RawRow{-1, 0, 0, 0, 0, 0, 0};
    };
    // The stripe-to-stripe lane state in three registers: p, R | H << 16 and
    // act | k << 1 | hap alignment << 5 | u << 7.
    struct SPack {
      int p, rh, w;
      float ih;
    };
    auto pack = [&](const SLane& s) {
      SPack q;
      q.p = s.p;
      q.rh = s.R | (s.H << 16);
      q.ih = s.ih;
      const uint8_t* const ha = b.hb + (int64_t)(uint32_t)__shfl((int)hom, sbase + min(s.k, 15));
      const int al = (int)((uintptr_t)ha & 3);  // only its address: a lane past the stream may point anywhere
      q.w = (s.act ? 1 : 0) | (s.k << 1) | (al << 5) | (s.u << 7);
      return q;
    };
    auto unpack = [&](const SPack& q) {
      SLane s;
      s.p = q.p;
      s.R = q.rh & 0xFFFF;
      s.H = q.rh >> 16;
      s.ih = q.ih;
      s.act = q.w & 1;
      s.k = (q.w >> 1) & 15;
      s.u = q.w >> 7;
      s.ro = 0;
      const int pad = (s.R & 1) ^ 1;
      s.ra = 2 * s.u + 1 - pad;
      s.rb = s.ra + 1;
      s.role_a = s.act ? srole(s.ra, s.R) : 0;
      s.role_b = s.act ? srole(s.rb, s.R) : 0;
      return s;
    };
    auto params_of = [&](const SLane& s, const RawRow& a, const RawRow& bb) {
      return srow_pack(srow_params(tab, a, s.role_a, s.ra == 1, s.ih),
                       srow_params(tab, bb, s.role_b, s.rb == 1, s.ih));
    };

    // Haplotype codes of the pair that starts in the coming stripe (at most one
    // per segment): located a stripe ahead, loaded as the aligned dwords that
    // cover its bytes when the stripe starts (holding five prefetched dwords
    // per lane through a stripe measured 2% slower: VGPR pressure).  Its buffer
    // (pair parity) was last used by the pair two back, which ended in an
    // earlier stripe.  Column c of pair k sits at hbuf(k) + 3 + al + c.
    int hk = -1, hH = 0;
    const uint8_t* ha = nullptr;
    auto hap_issue = [&](int st_next, const SLane& first_lane15) {
      // first_lane15: lane 15's position in stripe st_next (shuffled below)
      const int k15 = __shfl(first_lane15.k, sbase + 15);
      const int u15 = __shfl(first_lane15.u, sbase + 15);
      const bool a15 = __shfl((int)first_lane15.act, sbase + 15) != 0;
      const int kk = min(k15, 15);
      hk = (a15 && u15 < 16 && k15 < Kb) ? k15 : -1;  // started within stripe st_next
      hH = __shfl(Hm, sbase + kk);
      const int lo = __shfl((int)hom, sbase + kk), hi = __shfl((int)(hom >> 32), sbase + kk);
      ha = b.hb + (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
    };
    auto hap_commit = [&] {
      bool oth = false;
      if (hk >= 0) {
        const int al = (int)((uintptr_t)ha & 3);
        uint32_t* const dst = reinterpret_cast<uint32_t*>(hbufs + (hk & 1) * hstride + 4);
        const uint32_t* const src = reinterpret_cast<const uint32_t*>(ha - al);
        const int nb = al + hH;  // bytes from the aligned start; valid ones are [al, nb)
        auto put = [&](int j, uint32_t x) {
          const int lo = 4 * j, hi = lo + 4;
          uint32_t valid = 0xFFFFFFFFu;
          if (lo < al) valid &= 0xFFFFFFFFu << (8 * (al - lo));
          if (hi > nb) valid &= 0xFFFFFFFFu >> (8 * (hi - nb));
          dst[j] = hap_codes4(x, valid, oth);
        };
        constexpr int kB = 5;  // dwords per lane per round trip (320 bytes per segment)
        for (int j0 = sl; 4 * j0 < nb; j0 += 16 * kB) {
          uint32_t x[kB];
#pragma unroll
          for (int i = 0; i < kB; ++i) x[i] = 4 * (j0 + 16 * i) < nb ? src[j0 + 16 * i] : 0u;
#pragma unroll
          for (int i = 0; i < kB; ++i)
            if (4 * (j0 + 16 * i) < nb) put(j0 + 16 * i, x[i]);
        }
      }
      const unsigned long long bal = __ballot(oth);
      if (hk >= 0 && ((bal >> sbase) & 0xFFFFull)) other |= 1u << hk;
    };

    SPack cur_pk;
    RowP2 prm;
    {
      const SLane s0 = locate(0);
      cur_pk = pack(s0);
      prm = params_of(s0, raw_of(s0, s0.ra, s0.role_a), raw_of(s0, s0.rb, s0.role_b));
      hap_issue(0, s0);
    }
    for (int st = 0; st < nstr; ++st) {
      const SLane cur = unpack(cur_pk);
      hap_commit();
      __syncthreads();

      // This lane's role in the stripe.
      const bool start = cur.act && (sl == 0 || cur.u == 0);
      const uint32_t smask = start ? ~0u : 0u;
      const bool is_z = cur.act && cur.u == 0;
      const int zsh = (cur.role_a == 1) ? 1 : 0;  // the pad row reads Z one column on
      const int lim = (cur.role_b == 4) ? cur.H + sl2 + 2 : -1;  // V at its column H + 1
      const int need = cur.act ? cur.H + sl2 + 3 : 0;
      // 16-step blocks, and an 8-step block when the stripe's last block would
      // need no more than 8 steps
      const int nmax = wave_max(need);
      const int nblk = (nmax >> 4) + ((nmax & 15) > kStreamHalf ? 1 : 0);
      const bool half = (nmax & 15) != 0 && (nmax & 15) <= kStreamHalf;
      const int hoff = 3 + ((cur_pk.w >> 5) & 3);
      const unsigned char* const hp =
          (cur.act ? hbufs + (cur.k & 1) * hstride + hoff : hbufs) + PF - sl2;  // hp[t]: column t + PF - 2l

      // Next stripe: its lane state, raw rows and new haplotype, all in flight
      // during this stripe.
      RawRow na, nb;
      SPack nxt_pk;
      {
        const SLane nxt = locate(st + 1);
        na = raw_of(nxt, nxt.ra, nxt.role_a);
        nb = raw_of(nxt, nxt.rb, nxt.role_b);
        nxt_pk = pack(nxt);
        hap_issue(st + 1, nxt);
      }

      Lane2 L;
      L.Mo = L.Do = L.Xp = L.Xn = L.In = pf2{0.f, 0.f};
      // the boundary value "received at step -1": Z one column on at column
      // -2l for a pad row, 0 for every other source (columns < 0)
      L.Xp.y = (is_z && zsh && sl == 0) ? 1.f : 0.f;
      L.hbp = 6;
      PhRing<float> pf[PF];
      int hq[PF];
#pragma unroll
      for (int q = 0; q < PF; ++q) pf[q] = is_z ? Z[32 + q - sl2 + zsh] : ring[q];
#pragma unroll
      for (int q = 0; q < PF; ++q) hq[q] = hp[q - PF];
      float acc = 0.f;
      // Per block: the boundary source (ring, or Z for a lane whose pair starts
      // in this stripe: Z[32 + c] is X = 1 for c >= 0, so past column 0 every
      // block reads Z[32 ..]), the ring-write base, and whether some V lane
      // captures its sum in the block (a wave-uniform branch to the COND body).
      const int lblk = lim >> 4;  // the block holding this lane's capture (-1: none)
      const int zb = PF - sl2 + zsh;
      auto rd_of = [&](int t0) { return is_z ? Z + 32 + min(t0 + zb, 0) : ring + t0 + PF; };
      auto wbase_of = [&](int t0) { return lds_addr(ring + (t0 - 31)); };
      int blk = 0;
      for (; blk < nblk && blk < 2; ++blk) {  // lane 15 writes from block 2 on (its columns are negative before)
        const int t0 = 16 * blk;
        if (__ballot(lblk == blk) != 0ull)
          pstream_block<true, false, PF>(L, pf, hq, hp, rd_of(t0), prm, smask, t0, lim - t0, acc, 0u);
        else
          pstream_block<false, false, PF>(L, pf, hq, hp, rd_of(t0), prm, smask, t0, lim - t0, acc, 0u);
      }
      // two blocks per iteration when neither captures: half the per-block
      // bookkeeping and loop-carried register copies per step
      for (; blk + 1 < nblk; blk += 2) {
        const int t0 = 16 * blk;
        if (__ballot((unsigned)(lblk - blk) < 2u) != 0ull) {
          pstream_block<true, true, PF>(L, pf, hq, hp, rd_of(t0), prm, smask, t0, lim - t0, acc, wbase_of(t0));
          pstream_block<true, true, PF>(L, pf, hq, hp, rd_of(t0 + 16), prm, smask, t0 + 16, lim - t0 - 16, acc,
                                        wbase_of(t0 + 16));
        } else {
          pstream_block<false, true, PF, 32>(L, pf, hq, hp, rd_of(t0), prm, smask, t0, 0, acc, wbase_of(t0));
        }
      }
      if (blk < nblk) {
        const int t0 = 16 * blk;
        if (__ballot(lblk == blk) != 0ull)
          pstream_block<true, true, PF>(L, pf, hq, hp, rd_of(t0), prm, smask, t0, lim - t0, acc, wbase_of(t0));
        else
          pstream_block<false, true, PF>(L, pf, hq, hp, rd_of(t0), prm, smask, t0, 0, acc, wbase_of(t0));
      }
      if (half) {
        const int t0 = 16 * nblk;
        const bool cond = __ballot(lim >= t0 && lim < t0 + 8) != 0ull;
        if (nblk >= 2) {
          if (cond)
            pstream_block<true, true, PF, 8>(L, pf, hq, hp, rd_of(t0), prm, smask, t0, lim - t0, acc, wbase_of(t0));
          else
            pstream_block<false, true, PF, 8>(L, pf, hq, hp, rd_of(t0), prm, smask, t0, 0, acc, wbase_of(t0));
        } else {
          if (cond)
            pstream_block<true, false, PF, 8>(L, pf, hq, hp, rd_of(t0), prm, smask, t0, lim - t0, acc, 0u);
          else
            pstream_block<false, false, PF, 8>(L, pf, hq, hp, rd_of(t0), prm, smask, t0, 0, acc, 0u);
        }
      }
      if (lim >= 0) {
        const int p = cur.p;
        if ((other >> cur.k) & 1u) {
          const unsigned long long k = atomicAdd(fb_count, 1ull);
          fb_list[k] = p;
          out[p] = __builtin_nan("");
        } else if (use_rescue && acc < thr) {
          const unsigned long long k = atomicAdd(rescue_count, 1ull);
          rescue_list[k] = p;
          out[p] = __builtin_nan("");
        } else {
          out[p] = (double)(log10f(acc) - tab.log10_init);
        }
      }
      // the next stripe's constants, at the stripe end: computed after block
      // 0 (as phmm2 does) their values add ~60 VGPRs of pressure
      prm = params_of(unpack(nxt_pk), na, nb);
      cur_pk = nxt_pk;
    }
    __syncthreads();  // the next batch rewrites the hap buffers
  }
}

}  // namespace fcs

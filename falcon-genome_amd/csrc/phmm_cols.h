// PairHMM fp32 forward pass with COLUMN-BLOCKED lanes and continuous row
// streams (included by phmm_kernels.hip after phmm_stream.h).
//
// phmm3 (phmm_stream.h) gives each lane two read rows of a 32-row stripe and
// sweeps the haplotype columns over time, so every stripe pays a 31-step
// skew fill/drain and a ~700-VALU stripe setup (10.4 VALU per
// cell, of which the steady steps are 7.5).  Here the roles are transposed:
//   * lane l of a 16-lane segment OWNS the haplotype columns l*C + 1 ..
//     l*C + C (C per launch class, H <= 16 C - 1) and keeps their state in
//     registers: X(r, c) (the diagonal hand-off M*mm' + I*gm' + D*gm') and
//     I(r + 1, c) of the row it finished last;
//   * each step the lane runs ONE read row across its C columns (row g = t - l
//     of the segment's row stream: one row of skew per lane), so a step is C
//     cells of straight-line code with no per-cell lane traffic: the only
//     cross-lane values are the lane below's X(g - 1, l*C) and the deletion
//     chain D entering column l*C + 1 (two DPP row_shr:1 per value);
//   * the two halves of every packed register are two INDEPENDENT pairs
//     ("half-streams" A and B), so all seven FP ops of a cell are v_pk_*_f32
//     on two cells, with no swaps;
//   * row parameters (8 per row and half) come from a 32-row LDS ring that the
//     segment's 16 lanes fill 8 rows ahead (one (row, half) item per lane every
//     8 steps): no per-stripe setup.
// Each half-stream runs K pairs back to back as one row stream per pair
// [rows 1..R, V, Z]: V sums the last row (as in phmm3: prior 1 on the
// haplotype's columns and on column H + 1, 0 past it, D = running sum), and
// Z resets every column to the row-0 boundary of the next pair (X = 1 with
// row 1's priors pre-multiplied by (2^120 / H) * gm_1, I = 0) through a D
// chain of ones started at lane 0.  The sum therefore leaves lane 15 as the
// D entering column 16 C + 1 of the V row: no column search.  There is no
// fill or drain inside a stream, only at its end (15 steps per stream).
// Per cell the arithmetic is phmm3's exactly (same operations, same order),
// so the results are bitwise those of the row-streamed kernel.
#pragma once

namespace fcs {

constexpr int kColsClasses = 8;
constexpr int kColsMinR = 33;  // the next pair's haplotype codes are converted >= 16 rows after a switch
// Columns per lane of launch class c (longest haplotypes first): H <= 16 C - 1.
__host__ __device__ constexpr int cols_C(int c) { return c == 0 ? 19 : 18 - c; }  // 19, 17, 16, .., 11
__host__ __device__ constexpr int cols_hmax(int c) { return 16 * cols_C(c) - 1; }
// The smallest class that holds H (-1: none).
__host__ __device__ inline int cols_class(int H) {
  for (int c = kColsClasses - 1; c >= 0; --c)
    if (H <= cols_hmax(c)) return c;
  return -1;
}
// LDS per wave: a 32-row ring per segment of six 16-byte chunks per row:
// {e1, e3}, {my, yy}, {mm, gm}, {mx, xx} as {A, B} pairs, the match tables
// {Tlo A, Tlo B, Thi A, Thi B} and the Z flags {A, B, A, B} (floats).  The
// layout is chunk-major, then segment, then slot (16 B entries): the 16 lanes
// of a segment read 16 consecutive slots of a chunk, 256 contiguous bytes
// (row-major records 256 B apart per slot put all 16 lanes on the same banks:
// 7.4 conflict cycles per LDS cycle; segment-minor entries, 64 B apart, 4.5).
constexpr int kColsRing = 32;
constexpr int kColsChunks = 6;
constexpr int kColsChunkBytes = kColsRing * 4 * 16;  // one chunk of every (slot, segment)
constexpr int kColsCapOff = kColsChunks * kColsChunkBytes;  // lane 15's D per step of a block
constexpr int kColsTabOff = kColsCapOff + 4 * 8 * 8;  // ph2pr | dmatch | dmis (3 x 128 floats) for the ring items
constexpr int kColsLds = kColsTabOff + 3 * 128 * 4;

// A constant materialised where it is used: left to the compiler, the
// constants of the code conversion and the item builder are hoisted out of
// every loop and held in VGPRs for the whole kernel.
__device__ __forceinline__ uint32_t vconst(uint32_t k) {
  uint32_t r;
  asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "i"(k));
  return r;
}

// One (row, half) item of the ring.
struct ColsItem {
  float e1, e3, my, yy, mm, gm, mx, xx;
  uint32_t tlo, thi;
  float z;
};

// Roles: 0 = Z (reset row, also before and after the stream), 2 = row r < R,
// 3 = row R, 4 = V.  Match tables for v_perm on the column codes (A, C, G, T
// = 0..3 in Tlo, hap N = 4, column H + 1 = 5, past it = 6 in Thi): byte = 1
// on a match.
__device__ __forceinline__ ColsItem cols_item(const PhmmTables<float>& tab, const RawRow& raw, int role, bool first,
                                              float ih) {
  ColsItem c;
  if (role == 2 || role == 3) {
    const RowP<float> q = row_params<float, false>(tab, raw);
    const float x0 = first ? ih * tab.dmatch[raw.gq & 127] : 1.f;
    const bool last = role == 3;
    c.e1 = q.e1 * x0;
    c.e3 = q.e3 * x0;
    c.my = last ? 0.f : q.my;
    c.yy = q.yy;
    c.mm = last ? 1.f : q.mm;
    c.gm = last ? 1.f : q.gm;
    c.mx = last ? 0.f : q.mx;
    c.xx = last ? 0.f : q.xx;
    const int bc = base_code((unsigned char)raw.rb);
    c.tlo = bc < 4 ? 1u << (8 * bc) : bc == 4 ? vconst(0x01010101u) : 0u;
    c.thi = 0x00000001u;
    c.z = 0.f;
  } else if (role == 4) {  // V: prior 1 on codes 0..5, 0 past column H + 1; D = running sum of M
    c.e1 = 1.f;
    c.e3 = 0.f;
    c.my = c.yy = c.mm = c.gm = 1.f;
    c.mx = c.xx = 0.f;
    c.tlo = vconst(0x01010101u);
    c.thi = vconst(0x00000101u);
    c.z = 0.f;
  } else {  // Z: M = 0, D = 1 (from lane 0's boundary), X = D = 1, I = 0
    c.e1 = c.e3 = c.my = c.mm = c.gm = c.mx = c.xx = 0.f;
    c.yy = 1.f;
    c.tlo = c.thi = 0u;
    c.z = 1.f;
  }
  return c;
}

__device__ __forceinline__ void cols_put(unsigned char* smem, int slot, int seg, int h, const ColsItem& c) {
  float* const p = reinterpret_cast<float*>(smem + (seg * kColsRing + slot) * 16) + h;
  constexpr int F = kColsChunkBytes / 4;  // floats per chunk
  p[0] = c.e1;
  p[2] = c.e3;
  p[F] = c.my;
  p[F + 2] = c.yy;
  p[2 * F] = c.mm;
  p[2 * F + 2] = c.gm;
  p[3 * F] = c.mx;
  p[3 * F + 2] = c.xx;
  uint32_t* const q = reinterpret_cast<uint32_t*>(p);
  q[4 * F] = c.tlo;
  q[4 * F + 2] = c.thi;
  q[5 * F] = __float_as_uint(c.z);
  q[5 * F + 2] = __float_as_uint(c.z);
}

// Column codes of one lane's block (hap indices i0 .. i0 + C - 1, i.e. columns
// i0 + 1 ..) from the aligned dwords raw[] starting `al` bytes before i0:
// A,C,G,T,N = 0..4, index H (column H + 1) = 5, past it = 6.  `other`: a byte
// of the haplotype outside A/C/G/T/N.
template <int NW>
__device__ __forceinline__ void cols_convert(const uint32_t (&raw)[NW + 1], int al, int i0, int H, uint32_t (&code)[NW],
                                             bool& other) {
#pragma unroll
  for (int d = 0; d < NW; ++d) {
    const uint32_t x = __builtin_amdgcn_alignbyte(raw[d + 1], raw[d], (uint32_t)al);
    const int rel = H - (i0 + 4 * d);  // byte of index H (column H + 1) when in [0, 4)
    const int nv = min(max(rel, 0), 4);  // valid haplotype bytes in this dword
    const uint32_t vmask = nv >= 4 ? 0xFFFFFFFFu : (1u << (8 * nv)) - 1u;
    // hap_codes4 (phmm_stream.h) with its table constants materialised here
    const uint32_t sel = (x >> 1) & vconst(0x07070707u);
    uint32_t c = __builtin_amdgcn_perm(vconst(0x04050505u), vconst(0x02030100u), sel);
    const uint32_t back = __builtin_amdgcn_perm(vconst(0x0000004Eu), vconst(0x54474341u), c);
    other |= ((back ^ x) & vmask) != 0u;
    c = (c & vmask) | (vconst(0x06060606u) & ~vmask);
    if (rel >= 0 && rel < 4) c = (c & ~(0xFFu << (8 * rel))) | (0x05u << (8 * rel));
    code[d] = c;
  }
}

// Aligned dwords covering a lane's C haplotype bytes (only those holding a
// byte of the haplotype are read: the buffer ends inside the last one).
template <int NW>
__device__ __forceinline__ void cols_load(const uint8_t* __restrict__ hb, int64_t ho, int H, int i0, uint32_t (&raw)[NW + 1],
                                          int& al) {
  const int64_t s = ho + i0;
  al = (int)(s & 3);
  const int64_t base = s - al;
  const uint32_t* const src = reinterpret_cast<const uint32_t*>(hb + base);
#pragma unroll
  for (int d = 0; d <= NW; ++d) raw[d] = (base + 4 * d < ho + H && H > 0) ? src[d] : 0u;
}

template <int C>
__global__ __launch_bounds__(64, 2) void phmm4_kernel(
    const PhmmDevBatch b, const int32_t* __restrict__ order, const int64_t* __restrict__ bounds, const int cls,
    const int K, const int tail_pairs, const PhmmTables<float> gtab, double* __restrict__ out,
    int32_t* __restrict__ rescue_list, unsigned long long* __restrict__ rescue_count, const float thr,
    const int use_rescue, int32_t* __restrict__ fb_list, unsigned long long* __restrict__ fb_count) {
  constexpr int NW = (C + 3) / 4;  // code dwords per half
  extern __shared__ __align__(16) unsigned char smem_raw[];
  const int lane = threadIdx.x;
  const int seg = lane >> 4;
  const int sl = lane & 15;
  const int sbase = lane & 48;
  const int th = sl >> 3, tk = sl & 7;  // this lane's entry of the segment table: half th, pair tk
  const int i0 = sl * C;                // first haplotype index of this lane's columns
  const int64_t cbeg = bounds[cls];
  const long long count = bounds[cls + 1] - cbeg;
  order += cbeg;
  // the ring items' small tables in LDS (matchToMatch stays in global
  // memory): their lookups wait on LDS instead of the L2 (+1%)
  PhmmTables<float> tab = gtab;
  {
    float* const t = reinterpret_cast<float*>(smem_raw + kColsTabOff);
    for (int i = lane; i < 128; i += 64) {
      t[i] = gtab.ph2pr[i];
      t[128 + i] = gtab.dmatch[i];
      t[256 + i] = gtab.dmis[i];
    }
    tab.ph2pr = t;
    tab.dmatch = t + 128;
    tab.dmis = t + 256;
  }
  // Batches: 8 half-streams per wave, K pairs each, except the range's last
  // tail_pairs (shortest haplotypes), one pair per half-stream.
  const long long tailn = count < (long long)tail_pairs ? count : (long long)tail_pairs;
  const long long headn = count - tailn;
  const long long per = 8LL * K;
  const long long nb_head = (headn + per - 1) / per;
  const long long nbatch = nb_head + (tailn + 7) / 8;

  for (long long w = blockIdx.x; w < nbatch; w += gridDim.x) {
    const bool head = w < nb_head;
    const int Kb = head ? K : 1;
    const long long bstart = head ? w * per : headn + (w - nb_head) * 8;
    const long long bend = head ? min(headn, bstart + per) : min(count, bstart + 8);
    // Segment table: lane (th, tk) holds pair tk of half-stream th (half-
    // streams 2 seg, 2 seg + 1 of the batch take every 8th pair).
    const long long idx = bstart + 2 * seg + th + 8LL * tk;
    const int pm = (tk < Kb && idx < bend) ? order[idx] : -1;
    int Rm = 0, Hm = 0;
    int64_t rom = 0, hom = 0;
    float Im = 0.f;
    if (pm >= 0) {
      const int ri = b.pair_read[pm], hi = b.pair_hap[pm];
      Rm = b.read_len[ri];
      Hm = b.hap_len[hi];
      rom = b.read_off[ri];
      hom = b.hap_off[hi];
      Im = tab.init_const / (float)Hm;
    }
    const int len = pm >= 0 ? Rm + 2 : 0;  // rows 1..R, V, Z
    int incl = len;
#pragma unroll
    for (int d = 1; d < 8; d <<= 1) {
      const int v = __shfl_up(incl, d, 8);
      if (tk >= d) incl += v;
    }
    const int Gm = incl - len;  // first stream row of the pair
    const int totA = __builtin_amdgcn_ds_bpermute(4 * (sbase + 7), incl);
    const int totB = __builtin_amdgcn_ds_bpermute(4 * (sbase + 15), incl);
    const int nsteps = ((wave_max(max(totA, totB)) + 15) + 7) & ~7;
    // Table accessors (uniform control flow: every lane executes the shuffle).
    // sb is sbase laundered once per block (asm below), so the shuffle
    // addresses are computed where they are used instead of being hoisted out
    // of the loops as long-lived registers.
    int sb = sbase * 4;  // byte address of the segment's lane 0 for ds_bpermute
    auto bp = [&](int v, int h, int k) {
      return __builtin_amdgcn_ds_bpermute(sb + 4 * (8 * h + min(k, 7)), v);
    };
    auto tG = [&](int h, int k) { return bp(Gm, h, k); };
    auto tR = [&](int h, int k) { return bp(Rm, h, k); };
    auto tH = [&](int h, int k) { return bp(Hm, h, k); };
    auto tP = [&](int h, int k) { return bp(pm, h, k); };
    auto tI = [&](int h, int k) { return __int_as_float(bp(__float_as_int(Im), h, k)); };
    auto t64 = [&](int64_t v, int h, int k) {
      const int lo = bp((int)v, h, k), hi = bp((int)(v >> 32), h, k);
      return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
    };
    auto valid = [&](int h, int k) {  // the shuffle runs in every lane whatever k is
      const int pv = tP(h, k);
      return k < Kb && pv >= 0;
    };

    // Haplotype codes per half: cur (in use), nxt (the next pair of the
    // half-stream, taken by lane l at stream row swr[h], i.e. step swr + l),
    // nk[h] = the pair held in nxt.  other[h]: bit k = pair k of the half has
    // a haplotype byte outside A/C/G/T/N (segment-uniform).
    uint32_t cur[2][NW], nxt[2][NW];
    int nk[2], swr[2];
    unsigned other[2] = {0u, 0u};
    auto fetch_codes = [&](int h, int k, uint32_t (&dst)[NW]) {  // uniform: every lane of the wave calls it
      const bool ok = valid(h, k);
      const int Hk = tH(h, k);
      const int H = ok ? Hk : 0;
      const int64_t ho = t64(hom, h, k);
      uint32_t raw[NW + 1];
      int al;
      cols_load<NW>(b.hb, ok ? ho : 0, H, i0, raw, al);
      bool oth = false;
      cols_convert<NW>(raw, al, i0, H, dst, oth);
      const unsigned long long bal = __ballot(oth && ok);
      if (((bal >> sbase) & 0xFFFFull) != 0ull) other[h] |= 1u << k;
    };
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int d = 0; d < NW; ++d) cur[h][d] = 0x06060606u;
      fetch_codes(h, 0, nxt[h]);
      nk[h] = 0;
      swr[h] = valid(h, 0) ? tG(h, 0) : 0x3FFFFFFF;
    }
    // Captures: lane 15 takes half h's sum at the V row of pair kc[h]
    // (stream row cap[h], pair index capp[h], fallback flag from other[h]).
    int kc[2] = {0, 0};
    int cap[2], capp[2];
    auto load_cap = [&](int h) {
      const bool ok = valid(h, kc[h]);
      const int v = tG(h, kc[h]) + tR(h, kc[h]);
      cap[h] = ok ? v : -0x3FFFFFFF;  // stream row of the V row
      capp[h] = tP(h, kc[h]);
    };
    load_cap(0);
    load_cap(1);

    // The ring's items (row g of half th per lane) in two stages one block
    // apart, so the read bytes' HBM latency is not paid inside a block:
    // stage A locates the row and issues its byte loads, stage B (eight steps
    // later) builds the item from them and writes it.
    int kp = 0;  // stage A's cursor: the pair of half th holding this lane's item row
    RawRow praw{-1, 0, 0, 0, 0, 0, 0};
    int prole = 0;  // role | first << 4
    float pih = 0.f;
    // the cursor pair's table entries, cached: the shuffles run only in the
    // blocks where some lane's cursor moves (about one block in 13 on C2)
    bool kok = false, nok = false;
    int kG = 0, kR = 0, nG = 0;
    float kI = 0.f;
    int64_t kro = 0;
    auto load_cursor = [&] {
      kok = valid(th, kp);
      kG = tG(th, kp);
      kR = tR(th, kp);
      kI = tI(th, kp);
      kro = t64(rom, th, kp);
      nok = valid(th, kp + 1);
      nG = tG(th, kp + 1);
    };
    load_cursor();
    auto stage_a = [&](int base) {
      const int g = base + tk;
      const bool adv = nok && g >= nG;  // pairs span >= 35 rows: at most one advance per 8 rows
      if (__ballot(adv) != 0ull) {
        if (adv) ++kp;
        load_cursor();
      }
      const bool ok = kok;
      const int G = kG, R = kR;
      pih = kI;
      const int64_t ro = kro;
      const int r = g - G;
      int role = 0;
      if (ok && r >= 0 && r < R) role = r == R - 1 ? 3 : 2;
      else if (ok && r == R) role = 4;
      prole = role | (r == 0 ? 16 : 0);
      praw = (role == 2 || role == 3) ? load_raw(b, R, ro, r) : RawRow{-1, 0, 0, 0, 0, 0, 0};
    };
    auto stage_b = [&](int base) {
      cols_put(smem_raw, (base + tk) & (kColsRing - 1), seg, th,
               cols_item(tab, praw, prole & 15, (prole & 16) != 0, pih));
    };
    {  // ring prologue: rows -16..-1 are Z (slots 16..31), rows 0..7 built, rows 8..15 requested
      ColsItem z = cols_item(tab, RawRow{-1, 0, 0, 0, 0, 0, 0}, 0, false, 0.f);
      cols_put(smem_raw, 16 + tk, seg, th, z);
      cols_put(smem_raw, 24 + tk, seg, th, z);
      stage_a(0);
      stage_b(0);
      stage_a(8);
    }

    // Lane state: the columns' X and I after a Z row; the D chain and the
    // lane below's X as if it had run Z rows.
    pf2 Xn[C], In[C];
#pragma unroll
    for (int j = 0; j < C; ++j) {
      Xn[j] = pf2{1.f, 1.f};
      In[j] = pf2{0.f, 0.f};
    }
    pf2 dn = pf2{1.f, 1.f}, xo = pf2{1.f, 1.f}, xin = pf2{1.f, 1.f};
    const uint32_t segoff = (uint32_t)seg * (kColsRing * 16u) + lds_addr(smem_raw);

    for (int t0 = 0; t0 < nsteps; t0 += 8) {
      asm volatile("" : "+v"(sb));
      // Next pair's codes: once every lane took the pair in nxt (its row swr
      // was reached by lane 15 before this block), convert the one after it.
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const bool ev = swr[h] + 16 <= t0 && nk[h] + 1 < Kb;
        if (__ballot(ev) != 0ull) {  // uniform: fetch_codes shuffles
          uint32_t tmp[NW];
          fetch_codes(h, nk[h] + 1, tmp);
          const bool vn = valid(h, nk[h] + 1);
          const int gn = tG(h, nk[h] + 1);
          if (ev) {
#pragma unroll
            for (int d = 0; d < NW; ++d) nxt[h][d] = tmp[d];
            ++nk[h];
            swr[h] = vn ? gn : 0x3FFFFFFF;
          }
        }
        if (swr[h] + 16 <= t0 && nk[h] + 1 >= Kb) swr[h] = 0x3FFFFFFF;  // last pair taken
      }
      // The ring's rows t0 + 8 .. t0 + 15 (slots of rows t0 - 24 .. t0 - 17,
      // read last in the previous block), requested one block ago; then the
      // requests for rows t0 + 16 .. t0 + 23.
      stage_b(t0 + 8);
      stage_a(t0 + 16);
      // This block's captures (lane 15 at the V row of pair kc[h]) and switches.
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const bool adv = cap[h] >= 0 && cap[h] + 15 < t0;  // lane 15 passed the V row in an earlier block
        if (__ballot(adv) != 0ull) {
          if (adv) ++kc[h];
          load_cap(h);
        }
      }
      bool capo[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) capo[h] = (other[h] >> kc[h]) & 1u;
      const int g0 = t0 - sl;  // this lane's row at the block's first step
      const bool any_cap = __ballot(sl == 15 && ((unsigned)(cap[0] - g0) < 8u || (unsigned)(cap[1] - g0) < 8u)) != 0ull;
      // steps of this block at which some lane takes its next haplotype codes
      // (lane l of segment s switches half h at step swr - t0 + l): a uniform
      // 8-bit mask, tested per step by the scalar unit only
      unsigned swmask = 0u;
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int lo = __builtin_amdgcn_readlane(swr[h], 16 * q) - t0;  // steps lo .. lo + 15
          if (lo < 8 && lo + 15 >= 0) {
            const int a = max(lo, 0), bnd = min(lo + 15, 7);
            swmask |= ((2u << bnd) - 1u) & ~((1u << a) - 1u);
          }
        }
      const uint32_t xs = (uint32_t)(g0 & (kColsRing - 1)) * 16u;
      const uint32_t capa = lds_addr(smem_raw) + kColsCapOff + seg * 64;

      auto step = [&](auto S_) {
        constexpr int S = decltype(S_)::value;
        const int g = g0 + S;
        if (swmask & (1u << S)) {  // uniform
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const bool take = g == swr[h];
#pragma unroll
            for (int d = 0; d < NW; ++d) {  // the VOP3 select: the VOP2 form issues at ~1/5 rate
              uint32_t r;
              asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(cur[h][d]), "v"(nxt[h][d]), "s"(__ballot(take)));
              cur[h][d] = r;
            }
          }
        }
        // this row's records (the barrier keeps each step's LDS reads in their
        // step: hoisted ahead, eight steps' records would hold ~190 VGPRs)
        asm volatile("" ::: "memory");
        const uint32_t pa = ((xs + (uint32_t)(S * 16)) & (uint32_t)((kColsRing - 1) * 16)) + segoff;
        typedef float f4 __attribute__((ext_vector_type(4)));
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        auto ld4 = [&](int chunk) {
          return *reinterpret_cast<const __attribute__((address_space(3))) f4*>((uintptr_t)(pa + chunk * kColsChunkBytes));
        };
        const f4 r0 = ld4(0), r1 = ld4(1), r2 = ld4(2), r3 = ld4(3);
        const u4 cr = *reinterpret_cast<const __attribute__((address_space(3))) u4*>((uintptr_t)(pa + 4 * kColsChunkBytes));
        const pf2 z1 = *reinterpret_cast<const __attribute__((address_space(3))) pf2*>((uintptr_t)(pa + 5 * kColsChunkBytes));
        const pf2 z2 = *reinterpret_cast<const __attribute__((address_space(3))) pf2*>((uintptr_t)(pa + 5 * kColsChunkBytes + 8));
        const pf2 e1 = pf2{r0.x, r0.y}, e3 = pf2{r0.z, r0.w}, my = pf2{r1.x, r1.y}, yy = pf2{r1.z, r1.w};
        const pf2 mm = pf2{r2.x, r2.y}, gm = pf2{r2.z, r2.w}, mx = pf2{r3.x, r3.y}, xx = pf2{r3.z, r3.w};
        // the lane below's D into column l*C + 1 (lane 0: 1 on Z rows, else
        // 0) and its X(g, l*C) for the next row (lane 0: X(g, 0) = 1 after a Z row)
        pf2 din, xnx;
        din.x = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(z1.x), __float_as_int(dn.x), kDppRowShr1, 0xF, 0xF, false));
        din.y = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(z1.y), __float_as_int(dn.y), kDppRowShr1, 0xF, 0xF, false));
        xnx.x = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(z2.x), __float_as_int(xo.x), kDppRowShr1, 0xF, 0xF, false));
        xnx.y = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(z2.y), __float_as_int(xo.y), kDppRowShr1, 0xF, 0xF, false));
        const pf2 xcur = xin;
        xin = xnx;
        uint32_t mA = 0, mB = 0;
        // prior(j) after `dep`: every per-column input is tied to the previous
        // column's D by an empty asm, so the columns run in order.  Left free,
        // the scheduler hoists all C columns' I * xx, priors and M products to
        // the top of the step (~6 extra VGPRs per column: 256 VGPRs and spills
        // at C = 16).
        auto prior = [&](int j, const pf2 dep) {
          if ((j & 3) == 0) {
            mA = __builtin_amdgcn_perm(cr.z, cr.x, cur[0][j >> 2]);
            mB = __builtin_amdgcn_perm(cr.w, cr.y, cur[1][j >> 2]);
          }
          int a, c;
          asm volatile("v_bfe_i32 %0, %2, %3, 1\n\tv_bfe_i32 %1, %4, %3, 1"
                       : "=&v"(a), "=&v"(c)
                       : "v"(mA), "i"(8 * (j & 3)), "v"(mB), "v"(dep));
          return pf2{sel_v((uint32_t)a, e1.x, e3.x), sel_v((uint32_t)c, e1.y, e3.y)};
        };
        pf2 Mn = xcur * prior(0, xcur);
        pf2 D = din, Mp = pf2{0.f, 0.f}, Dp = pf2{0.f, 0.f};
#pragma unroll
        for (int j = 0; j < C; ++j) {
          const pf2 M = Mn;
          if (j > 0) D = __builtin_elementwise_fma(Mp, my, Dp * yy);
          pf2 I = In[j], Xo = Xn[j];
          asm volatile("" : "+v"(I), "+v"(Xo) : "v"(D));
          if (j + 1 < C) Mn = Xo * prior(j + 1, D);
          pf2 xn = __builtin_elementwise_fma(M, mm, __builtin_elementwise_fma(I, gm, D));
          pf2 in = __builtin_elementwise_fma(M, mx, I * xx);
          asm volatile("" : "+v"(xn), "+v"(in));  // and its outputs leave it in order
          Xn[j] = xn;
          In[j] = in;
          Mp = M;
          Dp = D;
        }
        dn = __builtin_elementwise_fma(Mp, my, Dp * yy);
        xo = Xn[C - 1];
        // lane 15's D entering column 16 C + 1, kept per step in LDS (EXEC
        // narrowed to the lanes 15 inside the statement, no branch): at a V row
        // it is the half's sum, taken after the block
        uint64_t keep;
        const uint32_t cpa = capa + 0u;  // a local: asm operands of a generic lambda cannot name captured consts
        const pf2 dnv = dn;
        asm volatile(
            "s_mov_b64 %0, exec\n\t"
            "s_mov_b64 exec, %3\n\t"
            "ds_write_b64 %1, %2 offset:%4\n\t"
            "s_mov_b64 exec, %0"
            : "=&s"(keep)
            : "v"(cpa), "v"(dnv), "s"(kTopLanes), "i"(8 * S)
            : "memory");
      };
      [&]<int... S>(std::integer_sequence<int, S...>) {
        (step(std::integral_constant<int, S>{}), ...);
      }(std::make_integer_sequence<int, 8>{});
      if (any_cap) {
        // lane 15 at a V row: the D entering column 16 C + 1 is the half's sum
#pragma unroll
        for (int h = 0; h < 2; ++h)
          if (sl == 15 && (unsigned)(cap[h] - g0) < 8u) {
            const pf2 v = *reinterpret_cast<const pf2*>(smem_raw + kColsCapOff + seg * 64 + 8 * (cap[h] - g0));
            const float acc = h ? v.y : v.x;
            const int p = capp[h];
            if (capo[h]) {
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
      }
    }
  }
}

}  // namespace fcs

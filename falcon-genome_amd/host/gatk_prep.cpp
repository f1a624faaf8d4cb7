#include "gatk_prep.h"

#include <algorithm>
#include <array>
#include <cmath>
#include <cstring>

#include <emmintrin.h>

#include "common.h"

namespace fcsg {

namespace {

constexpr int kMaxStrUnit = 8, kMaxRepeatLen = 20;

bool equal_range(const char* a, const char* b, int n) { return std::memcmp(a, b, (size_t)n) == 0; }

// GATKVariantContextUtils.findNumberOfRepetitions: copies of unit (len u) at
// the start (leading) or the end of test[0, n).
int repetitions(const char* unit, int u, const char* test, int n, bool leading) {
  int reps = 0;
  const int diff = n - u;
  if (leading) {
    for (int s = 0; s <= diff; s += u) {
      if (!equal_range(test + s, unit, u)) return reps;
      ++reps;
    }
  } else {
    for (int s = diff; s >= 0; s -= u) {
      if (!equal_range(test + s, unit, u)) return reps;
      ++reps;
    }
  }
  return reps;
}

}  // namespace

PcrIndelModel parse_pcr_indel_model(const std::string& s) {
  std::string u;
  for (char c : s) u += (char)std::toupper((unsigned char)c);
  if (u == "NONE") return PcrIndelModel::NONE;
  if (u == "HOSTILE") return PcrIndelModel::HOSTILE;
  if (u == "AGGRESSIVE") return PcrIndelModel::AGGRESSIVE;
  if (u == "CONSERVATIVE") return PcrIndelModel::CONSERVATIVE;
  throw invalidParam("pcr indel model '" + s + "' (NONE, HOSTILE, AGGRESSIVE, CONSERVATIVE)");
}

int tandem_repeat_units(const std::string& bases, int offset) {
  const char* r = bases.data();
  const int n = (int)bases.size();
  int max_bw = 0;
  std::string best_bw(1, r[offset]);
  for (int str = 1; str <= kMaxStrUnit; ++str) {
    if (offset + 1 - str < 0) break;
    max_bw = repetitions(r + offset - str + 1, str, r, offset + 1, false);
    if (max_bw > 1) {
      best_bw.assign(r + offset - str + 1, (size_t)str);
      break;
    }
  }
  int max_rl = max_bw;
  if (offset < n - 1) {
    std::string best_fw(1, r[offset + 1]);
    int max_fw = 0;
    for (int str = 1; str <= kMaxStrUnit; ++str) {
      if (offset + str + 1 > n) break;
      max_fw = repetitions(r + offset + 1, str, r + offset + 1, n - offset - 1, true);
      if (max_fw > 1) {
        best_fw.assign(r + offset + 1, (size_t)str);
        break;
      }
    }
    if (best_fw == best_bw) {
      max_rl = max_bw + max_fw;
    } else {
      // the backward run of the forward unit (TTCTT(C)CCC: (C)4, not (TTC)2)
      max_bw = repetitions(best_fw.data(), (int)best_fw.size(), r, offset + 1, false);
      max_rl = max_fw + max_bw;
    }
  }
  return max_rl > kMaxRepeatLen ? kMaxRepeatLen : max_rl;
}

void tandem_repeat_runs(const char* r, int n, uint8_t* out) {
  // Every repetitions() call above becomes a lookup into two tables of match
  // runs, one row of eight unit lengths u = 1 .. 8 per position (16-byte SSE2
  // lanes, saturating at 255 — far past the cap of 20 copies):
  //   bk[k][8 - u] = the number of consecutive k' = k, k - 1, ... with
  //                  r[k' - u] == r[k'];
  //   fw[j][u - 1] = the number of consecutive j' = j, j + 1, ... with
  //                  r[j'] == r[j' + u].
  // A unit of length u ending at o has k further copies behind it exactly when
  // bk[o][8 - u] >= k u, a unit starting at o + 1 k further copies ahead when
  // fw[o + 1][u - 1] >= k u; the first u with a second copy is a bit scan of
  // the lanes >= u.  Positions outside the read hold pairwise distinct
  // sentinels that match no base.
  if (n <= 1) return;
  constexpr int U = kMaxStrUnit;
  static_assert(U == 8, "one 8-byte row per position");
  static const auto kDiv = [] {
    std::array<std::array<uint8_t, 256>, U + 1> t{};
    for (int u = 1; u <= U; ++u)
      for (int x = 0; x < 256; ++x) t[u][x] = (uint8_t)std::min(x / u, 255);
    return t;
  }();
  thread_local std::vector<char> tl_seq;
  thread_local std::vector<uint8_t> tl_bk, tl_fw;
  std::vector<char>& vs = tl_seq;
  std::vector<uint8_t>& vb = tl_bk;
  std::vector<uint8_t>& vf = tl_fw;
  vs.resize((size_t)n + 2 * U + 8);
  for (int k = 0; k < U; ++k) vs[k] = (char)(9 + k);  // before the read: 9 .. 16
  std::memcpy(vs.data() + U, r, (size_t)n);
  for (int k = 0; k < U + 8; ++k) vs[U + n + k] = (char)(1 + (k & 7));  // after: 1 .. 8 (only 8 are compared)
  vb.resize((size_t)(n + 1) * U + 8);
  vf.resize((size_t)(n + 1) * U + 8);
  const char* q = vs.data() + U;
  uint8_t* const bk = vb.data();
  uint8_t* const fw = vf.data();
  const __m128i zero = _mm_setzero_si128(), one = _mm_set1_epi8(1);
  __m128i run = zero;
  for (int k = 0; k < n; ++k) {  // lane c: q[k - 8 + c] == q[k], u = 8 - c
    const __m128i prev = _mm_loadl_epi64((const __m128i*)(q + k - 8));
    const __m128i eq = _mm_cmpeq_epi8(prev, _mm_set1_epi8(q[k]));
    run = _mm_and_si128(_mm_adds_epu8(run, one), eq);
    _mm_storel_epi64((__m128i*)(bk + (size_t)k * U), run);
  }
  run = zero;
  _mm_storel_epi64((__m128i*)(fw + (size_t)n * U), zero);
  for (int j = n - 1; j >= 0; --j) {  // lane i: q[j + 1 + i] == q[j], u = i + 1
    const __m128i next = _mm_loadl_epi64((const __m128i*)(q + j + 1));
    const __m128i eq = _mm_cmpeq_epi8(next, _mm_set1_epi8(q[j]));
    run = _mm_and_si128(_mm_adds_epu8(run, one), eq);
    _mm_storel_epi64((__m128i*)(fw + (size_t)j * U), run);
  }
  const __m128i ub = _mm_setr_epi8(8, 7, 6, 5, 4, 3, 2, 1, 0, 0, 0, 0, 0, 0, 0, 0);
  const __m128i uf = _mm_setr_epi8(1, 2, 3, 4, 5, 6, 7, 8, 0, 0, 0, 0, 0, 0, 0, 0);
  for (int o = 0; o + 1 < n; ++o) {
    const __m128i rb = _mm_loadl_epi64((const __m128i*)(bk + (size_t)o * U));
    const __m128i rf = _mm_loadl_epi64((const __m128i*)(fw + (size_t)(o + 1) * U));
    // lanes whose run covers one more copy: u - run saturates to 0
    const unsigned mb = (unsigned)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_subs_epu8(ub, rb), zero)) & 0xFF;
    const unsigned mf = (unsigned)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_subs_epu8(uf, rf), zero)) & 0xFF;
    // smallest u: the highest back lane, the lowest forward lane; none: the
    // single base with one copy (its run reads 0)
    const int bu = mb ? 8 - (31 - __builtin_clz(mb)) : 1;
    const int fu = mf ? 1 + __builtin_ctz(mf) : 1;
    const int max_bw = 1 + kDiv[bu][bk[(size_t)o * U + 8 - bu]];
    const int max_fw = 1 + kDiv[fu][fw[(size_t)(o + 1) * U + fu - 1]];
    // the forward unit r[o+1, o+fu] equals the backward one r[o-bu+1, o]
    // exactly when r[o'] == r[o' + fu] for o' = o .. o - fu + 1; otherwise
    // count the forward unit's copies behind o
    const int bf = bk[(size_t)(o + fu) * U + 8 - fu];
    const int same = (bf >= fu) & (fu == bu);
    const int rl = max_fw + same * max_bw + (1 - same) * kDiv[fu][bf];
    out[o] = (uint8_t)std::min(rl, kMaxRepeatLen);
  }
}

int pcr_indel_cap(int repeat_len, PcrIndelModel m) {
  if (m == PcrIndelModel::NONE) return 255;
  const double rate = m == PcrIndelModel::HOSTILE ? 1.0 : m == PcrIndelModel::AGGRESSIVE ? 2.0 : 3.0;
  // MathUtils.fastRound(40.0 - exp(rl / (rate * pi)) + 1.0), at least 10
  const double v = 40.0 - std::exp((double)repeat_len / (rate * M_PI)) + 1.0;
  const int r = v > 0 ? (int)(v + 0.5) : (int)(v - 0.5);
  return std::max(10, r);
}

void gatk_prepare_read(const char* bases, const uint8_t* quals, const char* bi, const char* bd, size_t n, int mapq,
                       uint8_t* out, int thr, PcrIndelModel pcr) {
  // the model's cap per repeat run length, one table per model
  static const auto kCaps = [] {
    std::array<std::array<uint8_t, kMaxRepeatLen + 1>, 4> t{};
    for (int m = 0; m < 4; ++m)
      for (int r = 0; r <= kMaxRepeatLen; ++r) t[m][r] = (uint8_t)std::min(255, pcr_indel_cap(r, (PcrIndelModel)m));
    return t;
  }();
  uint8_t* const ob = out;
  uint8_t* const oq = out + n;
  uint8_t* const oi = out + 2 * n;
  uint8_t* const od = out + 3 * n;
  std::memcpy(ob, bases, n);
  std::memset(out + 4 * n, kGatkGcp, n);
  const int cap = std::max(0, std::min(mapq, 255));
  // gap-open quals: the tag (phred+33) or 45, capped by the PCR model at
  // positions 0 .. n - 2, then floored at 6 (as the vector form above did:
  // the cap applies to the tag value's low byte)
  const uint8_t* runs = nullptr;
  if (pcr != PcrIndelModel::NONE && n > 1) {
    thread_local std::vector<uint8_t> tl_runs;
    tl_runs.resize(n);
    tandem_repeat_runs(bases, (int)n, tl_runs.data());
    runs = tl_runs.data();
  }
  const uint8_t* caps = kCaps[(int)pcr].data();
  for (size_t i = 0; i < n; ++i) {
    int ins = bi ? (int)(uint8_t)bi[i] - 33 : kGatkDefaultGop;
    int del = bd ? (int)(uint8_t)bd[i] - 33 : kGatkDefaultGop;
    if (runs && i + 1 < n) {
      const int c = caps[runs[i]];
      ins = std::min(ins & 0xFF, c);
      del = std::min(del & 0xFF, c);
    }
    int q = std::min<int>(quals[i], cap);
    if (q < thr) q = kGatkMinUsableQ;
    oq[i] = (uint8_t)q;
    oi[i] = (uint8_t)std::max(ins, kGatkMinUsableQ);
    od[i] = (uint8_t)std::max(del, kGatkMinUsableQ);
  }
}

void gatk_prepare_read(const std::string& bases, const std::vector<uint8_t>& quals, const std::string& bi,
                       const std::string& bd, int mapq, PreparedRead& out, int thr, PcrIndelModel pcr) {
  const size_t n = bases.size();
  if (quals.size() != n) throw invalidParam("read quals and bases differ in length");
  if ((!bi.empty() && bi.size() != n) || (!bd.empty() && bd.size() != n))
    throw invalidParam("BI/BD tag length differs from the read length");
  std::vector<uint8_t> rows(5 * n);
  gatk_prepare_read(bases.data(), quals.data(), bi.empty() ? nullptr : bi.data(), bd.empty() ? nullptr : bd.data(), n,
                    mapq, rows.data(), thr, pcr);
  for (int k = 0; k < 5; ++k) {
    std::vector<uint8_t>& v = k == 0 ? out.bases : k == 1 ? out.base_q : k == 2 ? out.ins_q : k == 3 ? out.del_q : out.gcp;
    v.assign(rows.begin() + (std::ptrdiff_t)(k * n), rows.begin() + (std::ptrdiff_t)((k + 1) * n));
  }
}

}  // namespace fcsg

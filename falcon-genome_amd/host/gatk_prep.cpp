#include "gatk_prep.h"

#include <algorithm>
#include <cmath>
#include <cstring>

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

int pcr_indel_cap(int repeat_len, PcrIndelModel m) {
  if (m == PcrIndelModel::NONE) return 255;
  const double rate = m == PcrIndelModel::HOSTILE ? 1.0 : m == PcrIndelModel::AGGRESSIVE ? 2.0 : 3.0;
  // MathUtils.fastRound(40.0 - exp(rl / (rate * pi)) + 1.0), at least 10
  const double v = 40.0 - std::exp((double)repeat_len / (rate * M_PI)) + 1.0;
  const int r = v > 0 ? (int)(v + 0.5) : (int)(v - 0.5);
  return std::max(10, r);
}

void gatk_prepare_read(const std::string& bases, const std::vector<uint8_t>& quals, const std::string& bi,
                       const std::string& bd, int mapq, PreparedRead& out, int thr, PcrIndelModel pcr) {
  const size_t n = bases.size();
  if (quals.size() != n) throw invalidParam("read quals and bases differ in length");
  if ((!bi.empty() && bi.size() != n) || (!bd.empty() && bd.size() != n))
    throw invalidParam("BI/BD tag length differs from the read length");
  out.bases.assign(bases.begin(), bases.end());
  out.base_q.resize(n);
  out.ins_q.resize(n);
  out.del_q.resize(n);
  out.gcp.assign(n, (uint8_t)kGatkGcp);
  const int cap = std::max(0, std::min(mapq, 255));
  std::vector<int> ins(n), del(n);
  for (size_t i = 0; i < n; ++i) {
    ins[i] = bi.empty() ? kGatkDefaultGop : (int)(uint8_t)bi[i] - 33;
    del[i] = bd.empty() ? kGatkDefaultGop : (int)(uint8_t)bd[i] - 33;
  }
  if (pcr != PcrIndelModel::NONE) {
    int cache[kMaxRepeatLen + 1];
    for (int r = 0; r <= kMaxRepeatLen; ++r) cache[r] = pcr_indel_cap(r, pcr);
    for (size_t i = 1; i < n; ++i) {  // applyPCRErrorModel: positions 0 .. n - 2
      const int c = cache[tandem_repeat_units(bases, (int)i - 1)];
      ins[i - 1] = std::min(ins[i - 1] & 0xFF, c);
      del[i - 1] = std::min(del[i - 1] & 0xFF, c);
    }
  }
  for (size_t i = 0; i < n; ++i) {
    int q = std::min<int>(quals[i], cap);
    if (q < thr) q = kGatkMinUsableQ;
    out.base_q[i] = (uint8_t)q;
    out.ins_q[i] = (uint8_t)std::max(ins[i], kGatkMinUsableQ);
    out.del_q[i] = (uint8_t)std::max(del[i], kGatkMinUsableQ);
  }
}

}  // namespace fcsg

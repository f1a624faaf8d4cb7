#include "gatk_prep.h"

#include <algorithm>

#include "common.h"

namespace fcsg {

void gatk_prepare_read(const std::string& bases, const std::vector<uint8_t>& quals, const std::string& bi,
                       const std::string& bd, int mapq, PreparedRead& out, int thr) {
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
  for (size_t i = 0; i < n; ++i) {
    int q = std::min<int>(quals[i], cap);
    if (q < thr) q = kGatkMinUsableQ;
    out.base_q[i] = (uint8_t)q;
    const int iq = bi.empty() ? kGatkDefaultGop : (int)(uint8_t)bi[i] - 33;
    const int dq = bd.empty() ? kGatkDefaultGop : (int)(uint8_t)bd[i] - 33;
    out.ins_q[i] = (uint8_t)std::max(iq, kGatkMinUsableQ);
    out.del_q[i] = (uint8_t)std::max(dq, kGatkMinUsableQ);
  }
}

}  // namespace fcsg

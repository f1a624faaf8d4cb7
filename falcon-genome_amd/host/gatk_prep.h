// Caller-side read preparation for the PairHMM ("caller-side
// preprocessing the build must reproduce" [EXT] — GATK
// PairHMMLikelihoodCalculationEngine; not in /root/reference, parity unpinned):
//
//   * base quality capped at the read's mapping quality;
//   * base qualities below the threshold (18) become MIN_USABLE_Q_SCORE (6);
//   * insertion / deletion gap-open quals from the BI / BD tags (phred+33
//     strings), 45 when the tag is absent, then floored at 6;
//   * gap continuation penalty 10 at every position.
//
// The result is exactly what fcs_phmm_read expects (include/fcship.h).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace fcsg {

constexpr int kGatkBaseQualThreshold = 18;
constexpr int kGatkMinUsableQ = 6;
constexpr int kGatkDefaultGop = 45;
constexpr int kGatkGcp = 10;

struct PreparedRead {
  std::vector<uint8_t> bases, base_q, ins_q, del_q, gcp;
};

// bases: read bases (ASCII); quals: phred (no offset); bi / bd: BI / BD tag
// strings (phred+33) or empty when absent; mapq: mapping quality.
void gatk_prepare_read(const std::string& bases, const std::vector<uint8_t>& quals, const std::string& bi,
                       const std::string& bd, int mapq, PreparedRead& out,
                       int base_qual_threshold = kGatkBaseQualThreshold);

}  // namespace fcsg

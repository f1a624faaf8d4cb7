// Caller-side read preparation for the PairHMM ("caller-side
// preprocessing the build must reproduce" [EXT] — GATK
// PairHMMLikelihoodCalculationEngine; not in /root/reference, parity unpinned):
//
//   * base quality capped at the read's mapping quality;
//   * base qualities below the threshold (18) become MIN_USABLE_Q_SCORE (6);
//   * insertion / deletion gap-open quals from the BI / BD tags (phred+33
//     strings), 45 when the tag is absent, then floored at 6;
//   * gap continuation penalty 10 at every position;
//   * GATK's PCR indel error model (--pcr-indel-model, default CONSERVATIVE),
//     applied to the gap-open quals before the floor: at position i - 1
//     (i = 1 .. n - 1) both are capped at max(10, round(41 - exp(rl / (f pi))))
//     where rl <= 20 is the tandem-repeat run around i - 1 (repeat units up to
//     8 bases) and f = 1 / 2 / 3 for HOSTILE / AGGRESSIVE / CONSERVATIVE
//     (GATK PairHMMLikelihoodCalculationEngine.applyPCRErrorModel and
//     findTandemRepeatUnits, restated from the published GATK 4 source [EXT];
//     parity unpinned).
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

enum class PcrIndelModel { NONE = 0, HOSTILE = 1, AGGRESSIVE = 2, CONSERVATIVE = 3 };
PcrIndelModel parse_pcr_indel_model(const std::string& s);  // throws invalidParam

// GATK's tandem repeat run length at `offset` (capped at 20).
int tandem_repeat_units(const std::string& bases, int offset);
// The same for every offset 0 .. n - 2 at once (out[0, n - 1)), in O(8 n)
// from per-unit-length runs of r[j] == r[j + u]; the read-preparation path.
void tandem_repeat_runs(const char* bases, int n, uint8_t* out);
// The model's gap-open cap for a repeat run length.
int pcr_indel_cap(int repeat_len, PcrIndelModel m);

struct PreparedRead {
  std::vector<uint8_t> bases, base_q, ins_q, del_q, gcp;
};

// The five prepared rows of one read, n bytes each, back to back at out:
// bases, base_q, ins_q, del_q, gcp (the caller's arena form; no allocation).
// bi / bd: n phred+33 bytes, or null when the tag is absent.
void gatk_prepare_read(const char* bases, const uint8_t* quals, const char* bi, const char* bd, size_t n, int mapq,
                       uint8_t* out, int base_qual_threshold = kGatkBaseQualThreshold,
                       PcrIndelModel pcr = PcrIndelModel::CONSERVATIVE);

// bases: read bases (ASCII); quals: phred (no offset); bi / bd: BI / BD tag
// strings (phred+33) or empty when absent; mapq: mapping quality.
void gatk_prepare_read(const std::string& bases, const std::vector<uint8_t>& quals, const std::string& bi,
                       const std::string& bd, int mapq, PreparedRead& out,
                       int base_qual_threshold = kGatkBaseQualThreshold,
                       PcrIndelModel pcr = PcrIndelModel::CONSERVATIVE);

}  // namespace fcsg

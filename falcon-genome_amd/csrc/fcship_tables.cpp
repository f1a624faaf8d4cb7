// Host construction of the GKL PairHMM constant tables (Context<float> /
// Context<double>), uploaded once per device by fcship_api.cpp.
//
// These are part of the algorithm, not a check: the kernels read them instead
// of evaluating powf/log on the device so that every table entry is the value
// the upstream CPU code computes with the host libm.  Formulas: SURVEY.md
// Appendix A.1 (GKL ContextBase::initializeJacobianLogTable /
// initializeMatchToMatchProb / approximateLog10SumLog10, Context<T>() ph2pr).
#include <cmath>
#include <vector>

#include "fcship_internal.h"

namespace fcs {
namespace {

constexpr double kJacStep = 0.0001;
constexpr double kJacTol = 8.0;
constexpr int kJacSize = 80001;  // (int)(kJacTol / kJacStep) + 1

struct JacTable {
  std::vector<double> d;
  std::vector<float> f;
  JacTable() : d(kJacSize + 2), f(kJacSize + 2) {
    for (int k = 0; k < kJacSize + 2; ++k) {
      d[k] = std::log10(1.0 + std::pow(10.0, -static_cast<double>(k) * kJacStep));
      f[k] = static_cast<float>(d[k]);
    }
  }
};

const JacTable& jac() {
  static const JacTable t;
  return t;
}

// approximateLog10SumLog10 evaluated in NUMBER precision.
template <typename N>
N approx_log10_sum(N a, N b) {
  if (a > b) std::swap(a, b);  // b is the larger
  const N diff = b - a;
  if (diff >= static_cast<N>(kJacTol)) return b;
  const N scaled = static_cast<N>(diff * static_cast<N>(1.0 / kJacStep));
  const int ind = scaled > N(0) ? static_cast<int>(scaled + N(0.5)) : static_cast<int>(scaled - N(0.5));
  if constexpr (sizeof(N) == 4)
    return b + jac().f[ind];
  else
    return b + jac().d[ind];
}

template <typename N>
void build(N* ph2pr, N* dmatch, N* dmis, N* mm) {
  for (int x = 0; x < 128; ++x) {
    if constexpr (sizeof(N) == 4)
      ph2pr[x] = powf(10.f, -static_cast<float>(x) / 10.f);
    else
      ph2pr[x] = std::pow(10.0, -static_cast<double>(x) / 10.0);
    dmatch[x] = N(1) - ph2pr[x];
    dmis[x] = ph2pr[x] / N(3);
  }
  const double inv_ln10 = 1.0 / std::log(10.0);
  // matchToMatch for max qual <= 127 (quals are masked & 127 before lookup).
  for (int hi = 0, off = 0; hi <= 127; off += ++hi) {
    for (int lo = 0; lo <= hi; ++lo) {
      const double s = static_cast<double>(
          approx_log10_sum<N>(static_cast<N>(-0.1 * hi), static_cast<N>(-0.1 * lo)));
      const double l = std::log1p(-std::fmin(1.0, std::pow(10.0, s))) * inv_ln10;
      mm[off + lo] = static_cast<N>(std::pow(10.0, l));
    }
  }
}

}  // namespace

void build_phmm_tables_f(float* ph2pr, float* dmatch, float* dmis, float* mm) { build<float>(ph2pr, dmatch, dmis, mm); }
void build_phmm_tables_d(double* ph2pr, double* dmatch, double* dmis, double* mm) {
  build<double>(ph2pr, dmatch, dmis, mm);
}

}  // namespace fcs

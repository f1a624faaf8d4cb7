// Wave-level helpers shared by the wave-per-task Smith-Waterman kernels
// (bsw_kernels.hip: ksw_extend2 / ksw_global2; bsw_align.hip: ksw_align2).
#pragma once

#include "fcship_internal.h"

namespace fcs {

static constexpr int kMinusInf = -0x40000000;                    // ksw.c MINUS_INF
static constexpr int kScanNeg = (-2147483647 - 1) + (1 << 24);  // below any reachable scan value

__device__ __forceinline__ unsigned long long ballot64(bool v) { return __ballot(v); }

// Exclusive prefix max of u across slots (column order: slot k of lane l is
// column l + 64 k), seeded with carry.
template <int NS>
__device__ __forceinline__ void excl_scan(const int (&u)[NS], int carry, int (&ex)[NS]) {
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    const int incl = wave_incl_max(u[k], kScanNeg);
    int e = dpp_wave_shr1_i(carry, incl);
    ex[k] = max(e, carry);
    carry = max(carry, read_lane(incl, 63));
  }
}

// Query profile for column j: bytes mat[t*5 + q_j] for t = 0..3 packed, and t = 4.
__device__ __forceinline__ int prof_score(int lo, int hi, int tb) {
  return tb < 4 ? (int)(int8_t)(lo >> (tb << 3)) : hi;
}

}  // namespace fcs

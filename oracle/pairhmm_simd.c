/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by, or called
 * from the product library (libfcship.so).  Only bench.py's cpu_baseline leg
 * and tests/ load it, as the CPU baseline and as a checker of itself.
 *
 * A GKL-style AVX-512 PairHMM for the CPU baseline: the
 * "GATK AVX path" the north_star names is Intel GKL's IntelPairHmm, which is
 * not vendored in /root/reference (reached from
 * /root/reference/src/workers/HTCWorker.cpp:51-85 through GATK's
 * --native-pair-hmm-threads).  GKL vectorises each read x haplotype pair
 * along anti-diagonals: a stripe of VEC consecutive read rows sits in the
 * lanes of one vector, every step advances each lane by one haplotype column,
 * and the M/X/Y values of the row above reach a lane by shifting the vector
 * one lane up (lane 0 takes the previous stripe's last row, kept in three
 * column arrays).  Float pass in 16-lane vectors, results below 1e-28f redone
 * in double in 8-lane vectors — GKL's computeLikelihoodsNative flow.
 *
 * Cell arithmetic and summation order are those of oracle_phmm_prob_f/_d
 * (pairhmm_oracle.c: M = ((M*mm + X*gm) + Y*gm)*prior, X = M*mx + X*xx,
 * Y = M*my + Y*yy, final sumM + sumX in column order) with no FMA
 * (-ffp-contract=off), so every value is bit-identical to the scalar oracle;
 * tests/test_oracle_simd.py holds it to that.  Compiled with per-function
 * target attributes; oracle_phmm_simd_batch returns -1 when the host CPU has
 * no AVX-512F (the caller then times the scalar oracle and says so).
 */
#include <immintrin.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* Tables shared with pairhmm_oracle.c (same library). */
const float* oracle_phmm_ph2pr_f(void);
const double* oracle_phmm_ph2pr_d(void);
float oracle_phmm_mm_f(int i, int d);
double oracle_phmm_mm_d(int i, int d);
void oracle_phmm_init(void);

#define PAD 32 /* front/back padding of the boundary-row arrays: masked stores of the last lane
                  * start up to 2 x (lanes - 1) columns before column 1 */

/* Per-row parameters of one stripe: match-to-match, gap-to-match (1-gcp),
 * match-to-ins, match-to-del, gap extension (ins and del share gcp), prior
 * on a match and on a mismatch. */
#define STRIPE_PARAMS(T, VEC, PH2PR, MMF)                                      \
  T amm[VEC], agm[VEC], amx[VEC], axx[VEC], amy[VEC], aem[VEC], aex[VEC];      \
  int32_t arb[VEC], arn[VEC];                                                  \
  for (int l = 0; l < VEC; l++) {                                              \
    if (l < nl) {                                                              \
      const int r = r0 + l;                                                    \
      const int qi = iq[r] & 127, qd = dq[r] & 127, qc = gq[r] & 127;         \
      const T e = PH2PR[bq[r] & 127];                                          \
      amm[l] = MMF(qi, qd);                                                    \
      agm[l] = (T)1 - PH2PR[qc];                                               \
      amx[l] = PH2PR[qi];                                                      \
      amy[l] = PH2PR[qd];                                                      \
      axx[l] = PH2PR[qc];                                                      \
      aem[l] = (T)1 - e;                                                       \
      aex[l] = e / (T)3;                                                       \
      arb[l] = rb[r];                                                          \
      arn[l] = rb[r] == 'N';                                                   \
    } else {                                                                   \
      amm[l] = agm[l] = amx[l] = amy[l] = axx[l] = aem[l] = aex[l] = (T)0;     \
      arb[l] = -2;                                                             \
      arn[l] = 0;                                                              \
    }                                                                          \
  }

__attribute__((target("avx512f,avx512dq,avx512vl")))
static float prob_f512(const uint8_t* rb, const uint8_t* bq, const uint8_t* iq, const uint8_t* dq,
                       const uint8_t* gq, int R, const uint8_t* hb, int H, float* work) {
  enum { VEC = 16 };
  const float* ph2pr = oracle_phmm_ph2pr_f();
  /* previous stripe's last row (read) and this stripe's (written), swapped per stripe */
  const size_t stride = (size_t)H + 2 * PAD + 2;
  float* Mb = work + PAD;
  float* Xb = Mb + stride;
  float* Yb = Xb + stride;
  float* Mw = Yb + stride;
  float* Xw = Mw + stride;
  float* Yw = Xw + stride;
  const float init = ldexpf(1.f, 120) / (float)H;
  for (int c = -PAD; c <= H + PAD; c++) Mb[c] = Xb[c] = Yb[c] = Mw[c] = Xw[c] = Yw[c] = 0.f;
  for (int c = 0; c <= H; c++) Yb[c] = init;
  for (int r0 = 0; r0 < R; r0 += VEC) {
    const int nl = R - r0 < VEC ? R - r0 : VEC;
    STRIPE_PARAMS(float, VEC, ph2pr, oracle_phmm_mm_f)
    const __m512 mm = _mm512_loadu_ps(amm), gm = _mm512_loadu_ps(agm), mx = _mm512_loadu_ps(amx);
    const __m512 xx = _mm512_loadu_ps(axx), my = _mm512_loadu_ps(amy);
    const __m512 em = _mm512_loadu_ps(aem), ex = _mm512_loadu_ps(aex);
    const __m512i rv = _mm512_loadu_si512(arb);
    const __mmask16 rn = _mm512_test_epi32_mask(_mm512_loadu_si512(arn), _mm512_set1_epi32(1));
    const __m512i nv = _mm512_set1_epi32('N');
    __m512 M1 = _mm512_setzero_ps(), X1 = M1, Y1 = M1, M2 = M1, X2 = M1, Y2 = M1;
    __m512i hv = _mm512_set1_epi32(-1);
    const int last = nl - 1;
    const unsigned live = (1u << nl) - 1u;
    for (int s = 1; s <= H + last; s++) {
      /* lane l holds column c = s - l of row r0 + l + 1 */
      hv = _mm512_alignr_epi32(hv, _mm512_set1_epi32(s <= H ? hb[s - 1] : -1), 15);
      const __m512 um2 = _mm512_castsi512_ps(_mm512_alignr_epi32(_mm512_castps_si512(M2),
                                                                 _mm512_castps_si512(_mm512_set1_ps(Mb[s - 1])), 15));
      const __m512 ux2 = _mm512_castsi512_ps(_mm512_alignr_epi32(_mm512_castps_si512(X2),
                                                                 _mm512_castps_si512(_mm512_set1_ps(Xb[s - 1])), 15));
      const __m512 uy2 = _mm512_castsi512_ps(_mm512_alignr_epi32(_mm512_castps_si512(Y2),
                                                                 _mm512_castps_si512(_mm512_set1_ps(Yb[s - 1])), 15));
      const __m512 um1 = _mm512_castsi512_ps(_mm512_alignr_epi32(_mm512_castps_si512(M1),
                                                                 _mm512_castps_si512(_mm512_set1_ps(Mb[s])), 15));
      const __m512 ux1 = _mm512_castsi512_ps(_mm512_alignr_epi32(_mm512_castps_si512(X1),
                                                                 _mm512_castps_si512(_mm512_set1_ps(Xb[s])), 15));
      const int lo = s - H > 0 ? s - H : 0;           /* lanes with c <= H */
      const int hi = s - 1 < last ? s - 1 : last;     /* lanes with c >= 1 */
      const __mmask16 valid = (__mmask16)(live & ((2u << hi) - 1u) & ~((1u << lo) - 1u));
      const __mmask16 match = _mm512_cmpeq_epi32_mask(hv, rv) | _mm512_cmpeq_epi32_mask(hv, nv) | rn;
      const __m512 prior = _mm512_maskz_mov_ps(valid, _mm512_mask_blend_ps(match, ex, em));
      __m512 t = _mm512_mul_ps(um2, mm);
      t = _mm512_add_ps(t, _mm512_mul_ps(ux2, gm));
      t = _mm512_add_ps(t, _mm512_mul_ps(uy2, gm));
      const __m512 Mn = _mm512_mul_ps(t, prior);
      const __m512 Xn = _mm512_maskz_add_ps(valid, _mm512_mul_ps(um1, mx), _mm512_mul_ps(ux1, xx));
      const __m512 Yn = _mm512_maskz_add_ps(valid, _mm512_mul_ps(M1, my), _mm512_mul_ps(Y1, xx));
      M2 = M1; X2 = X1; Y2 = Y1;
      M1 = Mn; X1 = Xn; Y1 = Yn;
      /* the stripe's last row becomes the next stripe's boundary: lane `last`
       * holds column s - last (columns <= 0 land in the front padding) */
      const __mmask16 lm = (__mmask16)(1u << last);
      _mm512_mask_storeu_ps(Mw + s - 2 * last, lm, Mn);
      _mm512_mask_storeu_ps(Xw + s - 2 * last, lm, Xn);
      _mm512_mask_storeu_ps(Yw + s - 2 * last, lm, Yn);
    }
    Mw[0] = 0.f; Xw[0] = 0.f; Yw[0] = 0.f;
    float* t;
    t = Mb; Mb = Mw; Mw = t;
    t = Xb; Xb = Xw; Xw = t;
    t = Yb; Yb = Yw; Yw = t;
  }
  float sumM = 0.f, sumX = 0.f;
  for (int c = 1; c <= H; c++) { sumM += Mb[c]; sumX += Xb[c]; }
  return sumM + sumX;
}

__attribute__((target("avx512f,avx512dq,avx512vl")))
static double prob_d512(const uint8_t* rb, const uint8_t* bq, const uint8_t* iq, const uint8_t* dq,
                        const uint8_t* gq, int R, const uint8_t* hb, int H, double* work) {
  enum { VEC = 8 };
  const double* ph2pr = oracle_phmm_ph2pr_d();
  /* previous stripe's last row (read) and this stripe's (written), swapped per stripe */
  const size_t stride = (size_t)H + 2 * PAD + 2;
  double* Mb = work + PAD;
  double* Xb = Mb + stride;
  double* Yb = Xb + stride;
  double* Mw = Yb + stride;
  double* Xw = Mw + stride;
  double* Yw = Xw + stride;
  const double init = ldexp(1.0, 1020) / (double)H;
  for (int c = -PAD; c <= H + PAD; c++) Mb[c] = Xb[c] = Yb[c] = Mw[c] = Xw[c] = Yw[c] = 0.0;
  for (int c = 0; c <= H; c++) Yb[c] = init;
  for (int r0 = 0; r0 < R; r0 += VEC) {
    const int nl = R - r0 < VEC ? R - r0 : VEC;
    STRIPE_PARAMS(double, VEC, ph2pr, oracle_phmm_mm_d)
    int64_t brb[VEC];
    for (int l = 0; l < VEC; l++) brb[l] = arb[l];
    const __m512d mm = _mm512_loadu_pd(amm), gm = _mm512_loadu_pd(agm), mx = _mm512_loadu_pd(amx);
    const __m512d xx = _mm512_loadu_pd(axx), my = _mm512_loadu_pd(amy);
    const __m512d em = _mm512_loadu_pd(aem), ex = _mm512_loadu_pd(aex);
    const __m512i rv = _mm512_loadu_si512(brb);
    __mmask8 rn = 0;
    for (int l = 0; l < VEC; l++) rn |= (__mmask8)(arn[l] << l);
    const __m512i nv = _mm512_set1_epi64('N');
    __m512d M1 = _mm512_setzero_pd(), X1 = M1, Y1 = M1, M2 = M1, X2 = M1, Y2 = M1;
    __m512i hv = _mm512_set1_epi64(-1);
    const int last = nl - 1;
    const unsigned live = (1u << nl) - 1u;
#define SH8(v, x) _mm512_castsi512_pd(_mm512_alignr_epi64(_mm512_castpd_si512(v), \
                                                          _mm512_castpd_si512(_mm512_set1_pd(x)), 7))
    for (int s = 1; s <= H + last; s++) {
      hv = _mm512_alignr_epi64(hv, _mm512_set1_epi64(s <= H ? hb[s - 1] : -1), 7);
      const __m512d um2 = SH8(M2, Mb[s - 1]), ux2 = SH8(X2, Xb[s - 1]), uy2 = SH8(Y2, Yb[s - 1]);
      const __m512d um1 = SH8(M1, Mb[s]), ux1 = SH8(X1, Xb[s]);
      const int lo = s - H > 0 ? s - H : 0;
      const int hi = s - 1 < last ? s - 1 : last;
      const __mmask8 valid = (__mmask8)(live & ((2u << hi) - 1u) & ~((1u << lo) - 1u));
      const __mmask8 match = _mm512_cmpeq_epi64_mask(hv, rv) | _mm512_cmpeq_epi64_mask(hv, nv) | rn;
      const __m512d prior = _mm512_maskz_mov_pd(valid, _mm512_mask_blend_pd(match, ex, em));
      __m512d t = _mm512_mul_pd(um2, mm);
      t = _mm512_add_pd(t, _mm512_mul_pd(ux2, gm));
      t = _mm512_add_pd(t, _mm512_mul_pd(uy2, gm));
      const __m512d Mn = _mm512_mul_pd(t, prior);
      const __m512d Xn = _mm512_maskz_add_pd(valid, _mm512_mul_pd(um1, mx), _mm512_mul_pd(ux1, xx));
      const __m512d Yn = _mm512_maskz_add_pd(valid, _mm512_mul_pd(M1, my), _mm512_mul_pd(Y1, xx));
      M2 = M1; X2 = X1; Y2 = Y1;
      M1 = Mn; X1 = Xn; Y1 = Yn;
      const __mmask8 lm = (__mmask8)(1u << last);
      _mm512_mask_storeu_pd(Mw + s - 2 * last, lm, Mn);
      _mm512_mask_storeu_pd(Xw + s - 2 * last, lm, Xn);
      _mm512_mask_storeu_pd(Yw + s - 2 * last, lm, Yn);
    }
#undef SH8
    Mw[0] = 0.0; Xw[0] = 0.0; Yw[0] = 0.0;
    double* t;
    t = Mb; Mb = Mw; Mw = t;
    t = Xb; Xb = Xw; Xw = t;
    t = Yb; Yb = Yw; Yw = t;
  }
  double sumM = 0.0, sumX = 0.0;
  for (int c = 1; c <= H; c++) { sumM += Mb[c]; sumX += Xb[c]; }
  return sumM + sumX;
}

int oracle_phmm_simd_available(void) {
  __builtin_cpu_init();
  return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512dq") &&
         __builtin_cpu_supports("avx512vl");
}

/*
 * Same interface and outputs as oracle_phmm_batch (pairhmm_oracle.c).  OpenMP
 * over pairs, one boundary-row workspace per thread.  Returns 0, or -1 when
 * the CPU lacks AVX-512 (nothing computed).
 */
int oracle_phmm_simd_batch(const uint8_t* rb, const uint8_t* bq, const uint8_t* iq, const uint8_t* dq,
                           const uint8_t* gq, const int64_t* read_off, const int32_t* read_len,
                           const uint8_t* hb, const int64_t* hap_off, const int32_t* hap_len,
                           const int32_t* pair_read, const int32_t* pair_hap, int64_t n_pairs,
                           float* out_raw_f, double* out_log10, int32_t* used_double, int n_threads) {
  if (!oracle_phmm_simd_available()) return -1;
  oracle_phmm_init();
  int hmax = 1;
  for (int64_t p = 0; p < n_pairs; p++)
    if (hap_len[pair_hap[p]] > hmax) hmax = hap_len[pair_hap[p]];
  const size_t wsz = 6 * ((size_t)hmax + 2 * PAD + 2);
  const double log_init_d = log10(ldexp(1.0, 1020));
  const float log_init_f = log10f(ldexpf(1.f, 120));
#ifdef _OPENMP
#pragma omp parallel num_threads(n_threads > 0 ? n_threads : 1)
#endif
  {
    float* wf = (float*)malloc(wsz * sizeof(float));
    double* wd = (double*)malloc(wsz * sizeof(double));
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 64)
#endif
    for (int64_t p = 0; p < n_pairs; p++) {
      const int ri = pair_read[p], hi = pair_hap[p];
      const int64_t ro = read_off[ri], ho = hap_off[hi];
      const int R = read_len[ri], H = hap_len[hi];
      float f = 0.f;
      if (R > 0 && H > 0) f = prob_f512(rb + ro, bq + ro, iq + ro, dq + ro, gq + ro, R, hb + ho, H, wf);
      if (out_raw_f) out_raw_f[p] = f;
      int ud = 0;
      double v;
      if (f < 1e-28f) {
        const double d = (R > 0 && H > 0) ? prob_d512(rb + ro, bq + ro, iq + ro, dq + ro, gq + ro, R, hb + ho, H, wd)
                                          : 0.0;
        v = log10(d) - log_init_d;
        ud = 1;
      } else {
        v = (double)(log10f(f) - log_init_f);
      }
      if (out_log10) out_log10[p] = v;
      if (used_double) used_double[p] = ud;
    }
    free(wf);
    free(wd);
  }
  return 0;
}

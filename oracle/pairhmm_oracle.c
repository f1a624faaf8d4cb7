/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by, or called
 * from the product library (libfcship.so).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it, and only as the checker.
 *
 * CPU restatement of the GATK PairHMM forward algorithm as run by
 * `fcs-genome htc` / `fcs-genome mutect2`.
 *
 * Where the reference reaches it: the reference repo never contains the
 * arithmetic; it launches GATK (`java -jar GATK HaplotypeCaller ...
 * --native-pair-hmm-threads=N`) from HTCWorker::setup
 * (/root/reference/src/workers/HTCWorker.cpp:51-85) and
 * Mutect2Worker::setup (/root/reference/src/workers/Mutect2Worker.cpp:113-120);
 * the FPGA variant goes through the Blaze NAM daemon started at
 * /root/reference/src/worker-htc.cpp:100-112.  The algorithm therefore lives in
 * third-party code that is NOT vendored in /root/reference:
 *   - Intel GKL (com.intel.gkl, PairHMM native library: Context<NUMBER>,
 *     compute_full_prob<NUMBER>, IntelPairHmm computeLikelihoodsNative) — the
 *     "GATK AVX path" the north_star names.  Version unpinned by the reference
 *     (no build file pins it; GATK build v3.7-2-g53263cf per
 *     /root/reference/test/resource/gatk-error1/base-recalibration-20180730-180306.log.0:2).
 *   - GATK LoglessPairHMM / PairHMMModel (Java, double precision) — the CPU
 *     Java path of config C1.
 * Both are restated here from their published algorithms.
 *
 * PARITY UNPINNED: the reference holds no PairHMM golden vectors, no
 * known-answer tests and no fixtures for this path, and the
 * upstream code cannot be built or run here (no Java, GKL not vendored).  This
 * restatement is cross-checked instead by an independent arbitrary-precision
 * evaluation (tests/test_oracle_pairhmm.py, mpmath) and by the Java-semantics
 * double variant below.
 *
 * Semantics restated (GKL Context<float>/Context<double>):
 *   ph2pr[q]            = 10^(-q/10)  (powf for float, pow for double), q = qual & 127
 *   jacobianLogTable[k] = log10(1 + 10^(-k*1e-4)),  k = 0 .. 8.0/1e-4
 *   approximateLog10SumLog10(a,b) = max + table[round(|a-b|*1e4)] (|a-b| < 8), in NUMBER
 *   matchToMatch(i,d)   = 10^(log1p(-min(1, 10^approxSum(-0.1*max,-0.1*min))) / ln10)
 *   INITIAL_CONSTANT    = 2^120 (float) / 2^1020 (double)
 *   M[r][c] = prior * ((M[r-1][c-1]*mm + X[r-1][c-1]*gm) + Y[r-1][c-1]*gm)
 *   X[r][c] = M[r-1][c]*mx + X[r-1][c]*xx        (insertion: consumes a read base)
 *   Y[r][c] = M[r][c-1]*my + Y[r][c-1]*yy        (deletion: consumes a hap base)
 *   prior   = (read==hap || read=='N' || hap=='N') ? 1-ph2pr[q] : ph2pr[q]/3
 *   Y[0][c] = INITIAL_CONSTANT / H ;  result = sum_c M[R][c] + sum_c X[R][c]
 *   rescue : if float result < 1e-28f, redo in double
 *   log10  : float  -> (double)(log10f(res) - log10f(2^120))
 *            double -> log10(res) - log10(2^1020)
 *
 * [EXT] decisions where GKL itself cannot be consulted here (each one PARITY
 * UNPINNED; DESIGN.md §2 carries the same list):
 *   - Bytes outside A/C/G/T/N.  GKL's AVX kernels first map bases through a
 *     ConvertChar table (A,C,T,G,N -> small codes); from memory its other
 *     entries are zero, which would make an unknown byte compare like 'A' (and
 *     lowercase bases likewise).  That recollection cannot be verified (GKL is
 *     not vendored, no network), so this oracle and the product keep GATK's
 *     Java semantics (LoglessPairHMM: plain byte equality, 'N' a wildcard on
 *     either side), which GKL is contractually tested against.  Reads and
 *     haplotypes reaching the PairHMM from HaplotypeCaller are A/C/G/T/N in
 *     practice; tests/test_pairhmm_gpu.py::test_bytes_outside_acgtn pins the
 *     chosen rule on the GPU.
 *   - FTZ/DAZ.  Whether GKL runs its float pass with flush-to-zero is unknown
 *     here.  It stays inside the 1e-5 bar: a float sum below 1e-28 (scaled
 *     by 2^120) is recomputed in double anyway, and flushing denormal cells
 *     (< 1.2e-38 each, path gains <= 1) moves an accepted sum by at most
 *     R*H*1.2e-38, about 4e-34 for a 101 x 300 pair, i.e. < 4e-6 of any sum
 *     >= 1e-28.  This oracle keeps denormals (IEEE default); so does the GPU
 *     kernel.
 *   - GATK's PCR indel error model (--pcr-indel-model, CONSERVATIVE default)
 *     rewrites the ins/del GOPs before they reach the PairHMM; it is applied by
 *     the caller's read preparation (falcon-genome_amd/host/gatk_prep.cpp), not
 *     here: this oracle consumes prepared qualities, as GKL does.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define OR_MAX_QUAL 254
#define OR_JAC_TOL 8.0
#define OR_JAC_STEP 0.0001
#define OR_JAC_SIZE 80001 /* (int)(OR_JAC_TOL / OR_JAC_STEP) + 1 */
#define OR_MM_SIZE (((OR_MAX_QUAL + 1) * (OR_MAX_QUAL + 2)) >> 1)
#define OR_MIN_ACCEPTED 1e-28f

static float  jac_f[OR_JAC_SIZE + 2];
static double jac_d[OR_JAC_SIZE + 2];
static float  ph2pr_f[128];
static double ph2pr_d[128];
static float  mm_f[OR_MM_SIZE];
static double mm_d[OR_MM_SIZE];
static double jv_qual2err[256]; /* Java QualityUtils.qualToErrorProb cache */
static double jv_mm[OR_MM_SIZE]; /* Java PairHMMModel.matchToMatchProb */
static int tables_ready = 0;

static int fast_round_f(float v) { return v > 0.f ? (int)(v + 0.5f) : (int)(v - 0.5f); }
static int fast_round_d(double v) { return v > 0.0 ? (int)(v + 0.5) : (int)(v - 0.5); }

/* GKL ContextBase<float>::approximateLog10SumLog10, evaluated in float. */
static float approx_sum_f(float small, float big) {
  if (small > big) { float t = big; big = small; small = t; }
  float diff = big - small;
  if (diff >= (float)OR_JAC_TOL) return big;
  int ind = fast_round_f((float)(diff * (float)(1.0 / OR_JAC_STEP)));
  return big + jac_f[ind];
}

/* Same, evaluated in double (GKL ContextBase<double>; also GATK MathUtils). */
static double approx_sum_d(double small, double big) {
  if (small > big) { double t = big; big = small; small = t; }
  double diff = big - small;
  if (diff >= OR_JAC_TOL) return big;
  int ind = fast_round_d(diff * (1.0 / OR_JAC_STEP));
  return big + jac_d[ind];
}

void oracle_phmm_init(void) {
  if (tables_ready) return;
  for (int k = 0; k < OR_JAC_SIZE + 2; k++) {
    double v = log10(1.0 + pow(10.0, -((double)k) * OR_JAC_STEP));
    jac_d[k] = v;
    jac_f[k] = (float)v;
  }
  for (int x = 0; x < 128; x++) {
    ph2pr_f[x] = powf(10.f, -((float)x) / 10.f);
    ph2pr_d[x] = pow(10.0, -((double)x) / 10.0);
  }
  const double inv_ln10 = 1.0 / log(10.0);
  for (int i = 0, off = 0; i <= OR_MAX_QUAL; off += ++i) {
    for (int j = 0; j <= i; j++) {
      double s_f = (double)approx_sum_f((float)(-0.1 * i), (float)(-0.1 * j));
      double l_f = log1p(-fmin(1.0, pow(10.0, s_f))) * inv_ln10;
      mm_f[off + j] = (float)pow(10.0, l_f);
      double s_d = approx_sum_d(-0.1 * i, -0.1 * j);
      double l_d = log1p(-fmin(1.0, pow(10.0, s_d))) * inv_ln10;
      mm_d[off + j] = pow(10.0, l_d);
      jv_mm[off + j] = mm_d[off + j];
    }
  }
  for (int q = 0; q < 256; q++) jv_qual2err[q] = pow(10.0, ((double)q) / -10.0);
  tables_ready = 1;
}

static float mm_prob_f(int ins, int del) {
  int mn = del, mx = ins;
  if (ins <= del) { mn = ins; mx = del; }
  if (mx > OR_MAX_QUAL)
    return 1.f - powf(10.f, approx_sum_f(-0.1f * mn, -0.1f * mx));
  return mm_f[((mx * (mx + 1)) >> 1) + mn];
}

static double mm_prob_d(int ins, int del) {
  int mn = del, mx = ins;
  if (ins <= del) { mn = ins; mx = del; }
  if (mx > OR_MAX_QUAL)
    return 1.0 - pow(10.0, approx_sum_d(-0.1 * mn, -0.1 * mx));
  return mm_d[((mx * (mx + 1)) >> 1) + mn];
}

/* Exported table views, used only by tests to cross-check the product's own
 * host-computed tables and the mpmath restatement. */
const float* oracle_phmm_ph2pr_f(void) { oracle_phmm_init(); return ph2pr_f; }
const double* oracle_phmm_ph2pr_d(void) { oracle_phmm_init(); return ph2pr_d; }
float oracle_phmm_mm_f(int i, int d) { oracle_phmm_init(); return mm_prob_f(i, d); }
double oracle_phmm_mm_d(int i, int d) { oracle_phmm_init(); return mm_prob_d(i, d); }

static int is_match(uint8_t r, uint8_t h) { return r == h || r == 'N' || h == 'N'; }

/*
 * GKL compute_full_prob<float>, restated as a row sweep with the operation
 * order of GKL's vector kernel (computeMXY): M = ((M*mm + X*gm) + Y*gm)*prior,
 * result = sumM + sumX accumulated in column order.  Compiled with
 * -ffp-contract=off so no FMA is introduced.
 */
float oracle_phmm_prob_f(const uint8_t* rb, const uint8_t* bq, const uint8_t* iq,
                         const uint8_t* dq, const uint8_t* gq, int R,
                         const uint8_t* hb, int H) {
  oracle_phmm_init();
  if (R <= 0 || H <= 0) return 0.f;
  const int COLS = H + 1;
  float* pm = (float*)calloc(3 * (size_t)COLS, sizeof(float));
  float* cm = (float*)calloc(3 * (size_t)COLS, sizeof(float));
  float *Mp = pm, *Xp = pm + COLS, *Yp = pm + 2 * COLS;
  float *Mc = cm, *Xc = cm + COLS, *Yc = cm + 2 * COLS;
  const float init = ldexpf(1.f, 120) / (float)H;
  for (int c = 0; c < COLS; c++) { Mp[c] = 0.f; Xp[c] = 0.f; Yp[c] = init; }
  float sumM = 0.f, sumX = 0.f;
  for (int r = 1; r <= R; r++) {
    const int qi = iq[r - 1] & 127, qd = dq[r - 1] & 127, qc = gq[r - 1] & 127;
    const float mm = mm_prob_f(qi, qd);
    const float gm = 1.f - ph2pr_f[qc];
    const float mx = ph2pr_f[qi], xx = ph2pr_f[qc];
    const float my = ph2pr_f[qd], yy = ph2pr_f[qc];
    const float e = ph2pr_f[bq[r - 1] & 127];
    const float e_match = 1.f - e, e_mis = e / 3.f;
    Mc[0] = 0.f; Xc[0] = 0.f; Yc[0] = 0.f;
    for (int c = 1; c < COLS; c++) {
      const float prior = is_match(rb[r - 1], hb[c - 1]) ? e_match : e_mis;
      float t = Mp[c - 1] * mm;
      t = t + Xp[c - 1] * gm;
      t = t + Yp[c - 1] * gm;
      Mc[c] = t * prior;
      Xc[c] = Mp[c] * mx + Xp[c] * xx;
      Yc[c] = Mc[c - 1] * my + Yc[c - 1] * yy;
    }
    float* tmp;
    tmp = Mp; Mp = Mc; Mc = tmp;
    tmp = Xp; Xp = Xc; Xc = tmp;
    tmp = Yp; Yp = Yc; Yc = tmp;
  }
  for (int c = 1; c < COLS; c++) { sumM += Mp[c]; sumX += Xp[c]; }
  free(pm); free(cm);
  return sumM + sumX;
}

/* GKL compute_full_prob<double> (the rescue pass). */
double oracle_phmm_prob_d(const uint8_t* rb, const uint8_t* bq, const uint8_t* iq,
                          const uint8_t* dq, const uint8_t* gq, int R,
                          const uint8_t* hb, int H) {
  oracle_phmm_init();
  if (R <= 0 || H <= 0) return 0.0;
  const int COLS = H + 1;
  double* pm = (double*)calloc(3 * (size_t)COLS, sizeof(double));
  double* cm = (double*)calloc(3 * (size_t)COLS, sizeof(double));
  double *Mp = pm, *Xp = pm + COLS, *Yp = pm + 2 * COLS;
  double *Mc = cm, *Xc = cm + COLS, *Yc = cm + 2 * COLS;
  const double init = ldexp(1.0, 1020) / (double)H;
  for (int c = 0; c < COLS; c++) { Mp[c] = 0.0; Xp[c] = 0.0; Yp[c] = init; }
  double sumM = 0.0, sumX = 0.0;
  for (int r = 1; r <= R; r++) {
    const int qi = iq[r - 1] & 127, qd = dq[r - 1] & 127, qc = gq[r - 1] & 127;
    const double mm = mm_prob_d(qi, qd);
    const double gm = 1.0 - ph2pr_d[qc];
    const double mx = ph2pr_d[qi], xx = ph2pr_d[qc];
    const double my = ph2pr_d[qd], yy = ph2pr_d[qc];
    const double e = ph2pr_d[bq[r - 1] & 127];
    const double e_match = 1.0 - e, e_mis = e / 3.0;
    Mc[0] = 0.0; Xc[0] = 0.0; Yc[0] = 0.0;
    for (int c = 1; c < COLS; c++) {
      const double prior = is_match(rb[r - 1], hb[c - 1]) ? e_match : e_mis;
      double t = Mp[c - 1] * mm;
      t = t + Xp[c - 1] * gm;
      t = t + Yp[c - 1] * gm;
      Mc[c] = t * prior;
      Xc[c] = Mp[c] * mx + Xp[c] * xx;
      Yc[c] = Mc[c - 1] * my + Yc[c - 1] * yy;
    }
    double* tmp;
    tmp = Mp; Mp = Mc; Mc = tmp;
    tmp = Xp; Xp = Xc; Xc = tmp;
    tmp = Yp; Yp = Yc; Yc = tmp;
  }
  for (int c = 1; c < COLS; c++) { sumM += Mp[c]; sumX += Xp[c]; }
  free(pm); free(cm);
  return sumM + sumX;
}

/*
 * GKL IntelPairHmm computeLikelihoodsNative per-testcase logic:
 *   float pass; if result < MIN_ACCEPTED (1e-28f) -> double pass.
 * *used_double reports which pass produced the value.
 */
double oracle_phmm_log10(const uint8_t* rb, const uint8_t* bq, const uint8_t* iq,
                         const uint8_t* dq, const uint8_t* gq, int R,
                         const uint8_t* hb, int H, int* used_double) {
  oracle_phmm_init();
  float f = oracle_phmm_prob_f(rb, bq, iq, dq, gq, R, hb, H);
  if (f < OR_MIN_ACCEPTED) {
    double d = oracle_phmm_prob_d(rb, bq, iq, dq, gq, R, hb, H);
    if (used_double) *used_double = 1;
    return log10(d) - log10(ldexp(1.0, 1020));
  }
  if (used_double) *used_double = 0;
  return (double)(log10f(f) - log10f(ldexpf(1.f, 120)));
}

/*
 * GATK LoglessPairHMM (Java, double): INITIAL_CONDITION = 2^1020, transition
 * probabilities from PairHMMModel.qualToTransProbs (no &127 masking, quals as
 * unsigned bytes), priors from QualityUtils.qualToProb/qualToErrorProb,
 * per-cell M = prior*(M*mm + X*gm + Y*gm) evaluated left to right, final sum
 * over j of (M + X) in one accumulator.
 */
double oracle_phmm_java_log10(const uint8_t* rb, const uint8_t* bq, const uint8_t* iq,
                              const uint8_t* dq, const uint8_t* gq, int R,
                              const uint8_t* hb, int H) {
  oracle_phmm_init();
  if (R <= 0 || H <= 0) return -INFINITY;
  const int COLS = H + 1;
  double* pm = (double*)calloc(3 * (size_t)COLS, sizeof(double));
  double* cm = (double*)calloc(3 * (size_t)COLS, sizeof(double));
  double *Mp = pm, *Xp = pm + COLS, *Yp = pm + 2 * COLS;
  double *Mc = cm, *Xc = cm + COLS, *Yc = cm + 2 * COLS;
  const double init_cond = ldexp(1.0, 1020);
  for (int c = 0; c < COLS; c++) { Mp[c] = 0.0; Xp[c] = 0.0; Yp[c] = init_cond / (double)H; }
  for (int r = 1; r <= R; r++) {
    const int qi = iq[r - 1], qd = dq[r - 1], qc = gq[r - 1];
    int mn = qi <= qd ? qi : qd, mxq = qi <= qd ? qd : qi;
    const double mm = (mxq > OR_MAX_QUAL)
        ? 1.0 - pow(10.0, approx_sum_d(-0.1 * mn, -0.1 * mxq))
        : jv_mm[((mxq * (mxq + 1)) >> 1) + mn];
    const double mx = jv_qual2err[qi], my = jv_qual2err[qd];
    const double gm = 1.0 - jv_qual2err[qc], xx = jv_qual2err[qc], yy = jv_qual2err[qc];
    const double e = jv_qual2err[bq[r - 1]];
    Mc[0] = 0.0; Xc[0] = 0.0; Yc[0] = 0.0;
    for (int c = 1; c < COLS; c++) {
      const double prior = is_match(rb[r - 1], hb[c - 1]) ? (1.0 - e) : (e / 3.0);
      Mc[c] = prior * (Mp[c - 1] * mm + Xp[c - 1] * gm + Yp[c - 1] * gm);
      Xc[c] = Mp[c] * mx + Xp[c] * xx;
      Yc[c] = Mc[c - 1] * my + Yc[c - 1] * yy;
    }
    double* tmp;
    tmp = Mp; Mp = Mc; Mc = tmp;
    tmp = Xp; Xp = Xc; Xc = tmp;
    tmp = Yp; Yp = Yc; Yc = tmp;
  }
  double s = 0.0;
  for (int c = 1; c < COLS; c++) s += Mp[c] + Xp[c];
  free(pm); free(cm);
  return log10(s) - log10(init_cond);
}

/*
 * Batch of independent pairs over SoA buffers (the layout the C-ABI's device
 * path uses): read k occupies [read_off[k], read_off[k]+read_len[k]) of each of
 * the five byte arrays, hap k occupies [hap_off[k], +hap_len[k]).  Pair p =
 * (pair_read[p], pair_hap[p]).  out_raw_f gets the float-pass raw sum (may be
 * NULL), out_log10 the GKL final value, used_double the rescue flag (may be
 * NULL).  OpenMP over pairs when compiled with -fopenmp (CPU baseline).
 */
void oracle_phmm_batch(const uint8_t* rb, const uint8_t* bq, const uint8_t* iq,
                       const uint8_t* dq, const uint8_t* gq, const int64_t* read_off,
                       const int32_t* read_len, const uint8_t* hb, const int64_t* hap_off,
                       const int32_t* hap_len, const int32_t* pair_read,
                       const int32_t* pair_hap, int64_t n_pairs, float* out_raw_f,
                       double* out_log10, int32_t* used_double, int n_threads) {
  oracle_phmm_init();
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 64) num_threads(n_threads > 0 ? n_threads : 1)
#endif
  for (int64_t p = 0; p < n_pairs; p++) {
    const int ri = pair_read[p], hi = pair_hap[p];
    const int64_t ro = read_off[ri], ho = hap_off[hi];
    const int R = read_len[ri], H = hap_len[hi];
    if (out_raw_f)
      out_raw_f[p] = oracle_phmm_prob_f(rb + ro, bq + ro, iq + ro, dq + ro, gq + ro, R, hb + ho, H);
    int ud = 0;
    double v = oracle_phmm_log10(rb + ro, bq + ro, iq + ro, dq + ro, gq + ro, R, hb + ho, H, &ud);
    if (out_log10) out_log10[p] = v;
    if (used_double) used_double[p] = ud;
  }
}

int oracle_omp_max_threads(void) {
#ifdef _OPENMP
  extern int omp_get_max_threads(void);
  return omp_get_max_threads();
#else
  return 1;
#endif
}

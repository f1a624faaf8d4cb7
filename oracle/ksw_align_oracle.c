/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by, or called
 * from the product library (libfcship.so).  Only tests/, tests/cpu_mock and
 * bench.py's cpu_baseline leg load it, and only as the checker.
 *
 * CPU restatement of bwa's ksw_align2 (lh3/bwa ksw.c, 0.7.x: ksw_qinit,
 * ksw_u8, ksw_i16, ksw_align2), the local Smith-Waterman that bwa mem's mate
 * rescue (bwamem_pair.c mem_matesw) runs inside `bwa-flow mem`, launched by
 * the reference from BWAWorker::setup
 * (/root/reference/src/workers/BWAWorker.cpp:134-166).  bwa is not vendored in
 * /root/reference and no build file pins a version.
 *
 * bwa's kernel is Farrar's striped SSE2 Smith-Waterman, and its results depend
 * on the striping, so this restatement EMULATES THE VECTORS LITERALLY: p lanes
 * (16 x u8 with KSW_XBYTE, else 8 x i16), slen = ceil(qlen / p) segments, query
 * position k in lane k / slen of segment k % slen, the saturating u8/i16
 * arithmetic, the first pass whose F runs only down a lane's own segments,
 * E(i+1, j) taken from that first-pass H, and the lazy-F loop (up to 16 lane
 * shifts, with its early exit).  Then bwa's bookkeeping: imax per column, the
 * b[] list of column maxima >= minsc (KSW_XSUBO) with its append / replace
 * rule, te = first column reaching the best score, qe = the smallest query
 * position holding it in that column (padded positions included), score2 / te2
 * outside te +- ceil(score / max_mat), and with KSW_XSTART the second pass on
 * the reversed query [0, qe] and target [0, te] (the rest of the target in
 * place, bwa's full tlen) stopped at the first score (KSW_XSTOP) giving
 * tb = te - te', qb = qe - qe' when that score is reached again.
 *
 * PARITY UNPINNED: the reference holds no SW fixtures.
 * tests/test_oracle_ksw.py cross-checks score / te / qe against an
 * independent textbook local alignment on cases without insertion-deletion
 * adjacency (the only paths the striping's E rule changes).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define KA_XBYTE 0x10000
#define KA_XSTOP 0x20000
#define KA_XSUBO 0x40000
#define KA_XSTART 0x80000

typedef struct {
  int score, te, qe, score2, te2, tb, qb;
} oracle_kswr_t;

typedef struct {
  int size, p, slen, qlen, shift, max; /* shift: u8 bias (-min(mat)), max: max(mat) */
  int* qp;                             /* m * slen * p profile values, lane-major within a segment */
} ka_q;

static void ka_qinit(ka_q* q, int size, int qlen, const uint8_t* query, int m, const int8_t* mat) {
  q->size = size;
  q->p = size == 1 ? 16 : 8;
  q->slen = (qlen + q->p - 1) / q->p;
  q->qlen = qlen;
  int mn = 127, mx = 0;
  for (int a = 0; a < m * m; a++) {
    if (mat[a] < mn) mn = mat[a];
    if (mat[a] > mx) mx = mat[a];
  }
  q->shift = (256 - (uint8_t)(int8_t)mn) & 0xFF; /* bwa: uint8_t shift = 256 - (uint8_t)min */
  q->max = mx;
  const int nlen = q->slen * q->p;
  q->qp = (int*)malloc(sizeof(int) * (size_t)m * (q->slen > 0 ? q->slen : 1) * q->p);
  int* t = q->qp;
  for (int a = 0; a < m; a++) {
    const int8_t* ma = mat + a * m;
    for (int i = 0; i < q->slen; i++)
      for (int k = i; k < nlen; k += q->slen) {
        const int v = k >= qlen ? 0 : ma[query[k]];
        *t++ = size == 1 ? (int)(uint8_t)(int8_t)(v + q->shift) : v; /* u8: stored as int8, read as uint8 */
      }
  }
}

static inline int sat_u8(int v) { return v < 0 ? 0 : v > 255 ? 255 : v; }
static inline int sat_i16(int v) { return v < -32768 ? -32768 : v > 32767 ? 32767 : v; }
static inline int subs_u(int a, int b) { return a - b < 0 ? 0 : a - b; } /* subs_epu8 / subs_epu16 on values >= 0 */

/* One ksw_u8 / ksw_i16 run.  Vectors are arrays [segment][lane]. */
static oracle_kswr_t ka_run(const ka_q* q, int tlen, const uint8_t* target, int o_del, int e_del, int o_ins,
                            int e_ins, int xtra) {
  const int p = q->p, slen = q->slen, u8 = q->size == 1;
  const int n = slen * p;
  oracle_kswr_t r = {0, -1, -1, -1, -1, -1, -1};
  const int minsc = (xtra & KA_XSUBO) ? xtra & 0xffff : 0x10000;
  const int endsc = (xtra & KA_XSTOP) ? xtra & 0xffff : 0x10000;
  const int oe_del = o_del + e_del, oe_ins = o_ins + e_ins;
  int *H0 = (int*)calloc((size_t)n + 1, sizeof(int)), *H1 = (int*)calloc((size_t)n + 1, sizeof(int));
  int *E = (int*)calloc((size_t)n + 1, sizeof(int)), *Hmax = (int*)calloc((size_t)n + 1, sizeof(int));
  int f[16], h[16], mxv[16], t[16];
  uint64_t* b = NULL;
  int n_b = 0, m_b = 0, gmax = 0, te = -1;
  for (int i = 0; i < tlen; i++) {
    const int* S = q->qp + (size_t)target[i] * slen * p;
    for (int k = 0; k < p; k++) f[k] = 0, mxv[k] = 0;
    /* h = H0[slen - 1] shifted up one lane (lane 0 <- 0): H(i-1, j-1) of each lane's first segment */
    for (int k = p - 1; k > 0; k--) h[k] = slen ? H0[(slen - 1) * p + k - 1] : 0;
    h[0] = 0;
    for (int j = 0; j < slen; j++) {
      for (int k = 0; k < p; k++) {
        int x = h[k];
        if (u8) {
          x = sat_u8(x + S[j * p + k]);
          x = subs_u(x, q->shift);
        } else {
          x = sat_i16(x + S[j * p + k]);
        }
        const int e = E[j * p + k];
        x = x > e ? x : e;
        x = x > f[k] ? x : f[k];
        mxv[k] = mxv[k] > x ? mxv[k] : x;
        H1[j * p + k] = x;
        int en = subs_u(e, e_del), tt = subs_u(x, oe_del);
        E[j * p + k] = en > tt ? en : tt;
        int fn = subs_u(f[k], e_ins);
        tt = subs_u(x, oe_ins);
        f[k] = fn > tt ? fn : tt;
        h[k] = H0[j * p + k];
      }
    }
    /* lazy F: up to 16 lane shifts, early exit when no lane can still raise an H */
    for (int it = 0; it < 16; it++) {
      for (int k = p - 1; k > 0; k--) f[k] = f[k - 1];
      f[0] = 0;
      int done = 0;
      for (int j = 0; j < slen && !done; j++) {
        int all = 1;
        for (int k = 0; k < p; k++) {
          int x = H1[j * p + k];
          x = x > f[k] ? x : f[k];
          H1[j * p + k] = x;
          t[k] = subs_u(x, oe_ins);
          f[k] = subs_u(f[k], e_ins);
          if (u8 ? f[k] > t[k] : f[k] > t[k]) all = 0; /* u8: subs(f, h) == 0 <=> f <= h; i16: !(f > h) */
        }
        if (all) done = 1;
      }
      if (done) break;
    }
    int imax = 0;
    for (int k = 0; k < p; k++) imax = imax > mxv[k] ? imax : mxv[k];
    if (imax >= minsc) {
      if (n_b == 0 || (int32_t)b[n_b - 1] + 1 != i) {
        if (n_b == m_b) {
          m_b = m_b ? m_b << 1 : 8;
          b = (uint64_t*)realloc(b, 8 * (size_t)m_b);
        }
        b[n_b++] = (uint64_t)imax << 32 | (uint32_t)i;
      } else if ((int)(b[n_b - 1] >> 32) < imax) {
        b[n_b - 1] = (uint64_t)imax << 32 | (uint32_t)i;
      }
    }
    if (imax > gmax) {
      gmax = imax;
      te = i;
      memcpy(Hmax, H1, sizeof(int) * (size_t)n);
      if ((u8 && gmax + q->shift >= 255) || gmax >= endsc) break;
    }
    int* sw = H1;
    H1 = H0;
    H0 = sw;
  }
  r.score = u8 ? (gmax + q->shift < 255 ? gmax : 255) : gmax;
  r.te = te;
  if (!u8 || r.score != 255) {
    int max = -1;
    for (int i = 0; i < n; i++) { /* memory order: segment i / p, lane i % p */
      const int pos = i / p + i % p * slen, v = Hmax[i];
      if (v > max) max = v, r.qe = pos;
      else if (v == max && pos < r.qe) r.qe = pos;
    }
    if (b) {
      const int w = (r.score + q->max - 1) / q->max;
      const int low = te - w, high = te + w;
      for (int i = 0; i < n_b; i++) {
        const int e = (int32_t)b[i];
        if ((e < low || e > high) && (int)(b[i] >> 32) > r.score2) r.score2 = (int)(b[i] >> 32), r.te2 = e;
      }
    }
  }
  free(b);
  free(H0), free(H1), free(E), free(Hmax);
  return r;
}

static void ka_rev(int n, uint8_t* s) {
  for (int i = 0; i < n >> 1; i++) {
    const uint8_t t = s[i];
    s[i] = s[n - 1 - i];
    s[n - 1 - i] = t;
  }
}

/*
 * bwa ksw_align2 (qry == NULL).  out[7] = score, te, qe, score2, te2, tb, qb
 * (bwa's kswr_t order).  query / target are copied, never modified.
 */
void oracle_ksw_align2(int qlen, const uint8_t* query, int tlen, const uint8_t* target, int m, const int8_t* mat,
                       int o_del, int e_del, int o_ins, int e_ins, int xtra, int* out) {
  const int size = (xtra & KA_XBYTE) ? 1 : 2;
  uint8_t* qc = (uint8_t*)malloc((size_t)qlen + 1);
  uint8_t* tc = (uint8_t*)malloc((size_t)tlen + 1);
  memcpy(qc, query, (size_t)qlen);
  memcpy(tc, target, (size_t)tlen);
  ka_q q;
  ka_qinit(&q, size, qlen, qc, m, mat);
  oracle_kswr_t r = ka_run(&q, tlen, tc, o_del, e_del, o_ins, e_ins, xtra);
  free(q.qp);
  if ((xtra & KA_XSTART) && !((xtra & KA_XSUBO) && r.score < (xtra & 0xffff))) {
    ka_rev(r.qe + 1, qc);
    ka_rev(r.te + 1, tc);
    ka_q q2;
    ka_qinit(&q2, size, r.qe + 1, qc, m, mat);
    const oracle_kswr_t rr = ka_run(&q2, tlen, tc, o_del, e_del, o_ins, e_ins, KA_XSTOP | r.score);
    free(q2.qp);
    if (r.score == rr.score) r.tb = r.te - rr.te, r.qb = r.qe - rr.qe;
  }
  free(qc);
  free(tc);
  out[0] = r.score, out[1] = r.te, out[2] = r.qe, out[3] = r.score2, out[4] = r.te2, out[5] = r.tb, out[6] = r.qb;
}

/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by, or called
 * from the product library (libfcship.so).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it, and only as the checker.
 *
 * CPU restatement of the BWA-MEM banded Smith-Waterman kernels run under
 * `fcs-genome align`.  The reference launches `bwa-flow mem ... --offload
 * --use_fpga --fpga_path=<root>/fpga/sw.xclbin` from BWAWorker::setup
 * (/root/reference/src/workers/BWAWorker.cpp:134-166, config keys at
 * /root/reference/src/config.cpp:297-300); the SW arithmetic is inside
 * bwa-flow (falcon-bwa v0.4.4-4-gf1dfbc6 per
 * /root/reference/test/resource/bwa2.log:1602), which embeds lh3/bwa's
 * ksw.c.  Neither is vendored in /root/reference and no build file pins a
 * version; the restated algorithm is bwa 0.7.x ksw.c:
 *   - ksw_extend2: banded local extension with end bonus, z-drop, band
 *     shrink/grow driven by zero cells, "E and F open from M" scoring, and
 *     stale eh[] entries beyond the band that are re-read when the band grows
 *     (SURVEY.md Appendix A.2);
 *   - ksw_global2: banded global alignment with a per-cell direction byte
 *     (h in bits 0-1, E-continue bit 2, F-continue bit 5) and the traceback
 *     that produces the CIGAR (op 0=M, 1=I, 2=D, len<<4|op) (Appendix A.3).
 *     One deliberate, documented deviation: bwa mallocs the direction matrix
 *     and, when no alignment fits the band (score ~ MINUS_INF), its traceback
 *     can read cells that were never written (or before the array).  Here the
 *     matrix is zeroed and such reads return 0, so the result is defined and
 *     the GPU kernel reproduces it; for every alignment that fits the band the
 *     traceback never leaves the written cells and the CIGAR is bwa's.
 *
 * PARITY UNPINNED: the reference holds no SW golden vectors, score or CIGAR
 * fixtures.  This restatement is cross-checked by
 * hand-traced known answers and an independent unbanded Python DP in
 * tests/test_oracle_ksw.py.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define KO_MINUS_INF (-0x40000000)

typedef struct { int32_t h, e; } ko_eh;

static int ko_max_mat(const int8_t* mat, int m) {
  int mx = 0;
  for (int i = 0; i < m * m; i++) mx = mx > mat[i] ? mx : mat[i];
  return mx;
}

/*
 * ksw_extend2.  Returns the best score; fills qle/tle/gtle/gscore/max_off.
 * *cells receives the number of (i,j) evaluated inside [beg,end) over all rows
 * actually visited (the unit of the SW GCUPS metric).
 */
int oracle_ksw_extend2(int qlen, const uint8_t* query, int tlen, const uint8_t* target, int m,
                       const int8_t* mat, int o_del, int e_del, int o_ins, int e_ins, int w,
                       int end_bonus, int zdrop, int h0, int* qle_, int* tle_, int* gtle_,
                       int* gscore_, int* max_off_, int64_t* cells) {
  const int oe_del = o_del + e_del, oe_ins = o_ins + e_ins;
  int64_t ncell = 0;
  if (qlen < 0) qlen = 0;
  int8_t* qp = (int8_t*)malloc((size_t)(qlen > 0 ? qlen : 1) * m);
  ko_eh* eh = (ko_eh*)calloc((size_t)qlen + 1, sizeof(ko_eh));
  /* query profile: qp[k*qlen + j] = score of target base k against query[j] */
  for (int k = 0, i = 0; k < m; ++k)
    for (int j = 0; j < qlen; ++j) qp[i++] = mat[k * m + query[j]];
  /* first row: a run of insertions off h0 */
  eh[0].h = h0;
  if (qlen >= 1) eh[1].h = h0 > oe_ins ? h0 - oe_ins : 0;
  for (int j = 2; j <= qlen && eh[j - 1].h > e_ins; ++j) eh[j].h = eh[j - 1].h - e_ins;
  /* cap the band by the longest gap that could still pay off */
  const int mxs = ko_max_mat(mat, m);
  int max_ins = (int)((double)(qlen * mxs + end_bonus - o_ins) / e_ins + 1.);
  max_ins = max_ins > 1 ? max_ins : 1;
  w = w < max_ins ? w : max_ins;
  int max_del = (int)((double)(qlen * mxs + end_bonus - o_del) / e_del + 1.);
  max_del = max_del > 1 ? max_del : 1;
  w = w < max_del ? w : max_del;

  int max = h0, max_i = -1, max_j = -1, max_ie = -1, gscore = -1, max_off = 0;
  int beg = 0, end = qlen;
  for (int i = 0; i < tlen; ++i) {
    int f = 0, h1, mrow = 0, mj = -1, j;
    const int8_t* q = &qp[target[i] * qlen];
    if (beg < i - w) beg = i - w;
    if (end > i + w + 1) end = i + w + 1;
    if (end > qlen) end = qlen;
    if (beg == 0) {
      h1 = h0 - (o_del + e_del * (i + 1));
      if (h1 < 0) h1 = 0;
    } else {
      h1 = 0;
    }
    for (j = beg; j < end; ++j) {
      /* entering: eh[j] = {H(i-1,j-1), E(i,j)}, f = F(i,j), h1 = H(i,j-1) */
      ko_eh* p = &eh[j];
      int M = p->h, e = p->e, h, t;
      p->h = h1;
      M = M ? M + q[j] : 0;
      h = M > e ? M : e;
      h = h > f ? h : f;
      h1 = h;
      mj = mrow > h ? mj : j;
      mrow = mrow > h ? mrow : h;
      t = M - oe_del;
      t = t > 0 ? t : 0;
      e -= e_del;
      e = e > t ? e : t;
      p->e = e;
      t = M - oe_ins;
      t = t > 0 ? t : 0;
      f -= e_ins;
      f = f > t ? f : t;
    }
    ncell += end > beg ? end - beg : 0;
    eh[end].h = h1;
    eh[end].e = 0;
    if (j == qlen) {
      max_ie = gscore > h1 ? max_ie : i;
      gscore = gscore > h1 ? gscore : h1;
    }
    if (mrow == 0) break;
    if (mrow > max) {
      max = mrow, max_i = i, max_j = mj;
      int d = mj - i < 0 ? i - mj : mj - i;
      max_off = max_off > d ? max_off : d;
    } else if (zdrop > 0) {
      if (i - max_i > mj - max_j) {
        if (max - mrow - ((i - max_i) - (mj - max_j)) * e_del > zdrop) break;
      } else {
        if (max - mrow - ((mj - max_j) - (i - max_i)) * e_ins > zdrop) break;
      }
    }
    /* shrink the band to the non-zero span for the next row */
    for (j = beg; j < end && eh[j].h == 0 && eh[j].e == 0; ++j) {}
    beg = j;
    for (j = end; j >= beg && eh[j].h == 0 && eh[j].e == 0; --j) {}
    end = j + 2 < qlen ? j + 2 : qlen;
  }
  free(eh);
  free(qp);
  if (qle_) *qle_ = max_j + 1;
  if (tle_) *tle_ = max_i + 1;
  if (gtle_) *gtle_ = max_ie + 1;
  if (gscore_) *gscore_ = gscore;
  if (max_off_) *max_off_ = max_off;
  if (cells) *cells = ncell;
  return max;
}

static int ko_push_cigar(int* n, int* cap, uint32_t** cig, int op, int len) {
  if (*n == 0 || op != (int)((*cig)[*n - 1] & 0xf)) {
    if (*n == *cap) {
      *cap = *cap ? (*cap) << 1 : 4;
      *cig = (uint32_t*)realloc(*cig, (size_t)(*cap) * 4);
    }
    (*cig)[(*n)++] = (uint32_t)len << 4 | (uint32_t)op;
  } else {
    (*cig)[*n - 1] += (uint32_t)len << 4;
  }
  return 0;
}

/*
 * ksw_global2.  Returns the global score.  If cigar_out != NULL, writes up to
 * cigar_cap ops and sets *n_cigar (the true count, which may exceed the cap).
 */
int oracle_ksw_global2(int qlen, const uint8_t* query, int tlen, const uint8_t* target, int m,
                       const int8_t* mat, int o_del, int e_del, int o_ins, int e_ins, int w,
                       int* n_cigar, uint32_t* cigar_out, int cigar_cap) {
  const int oe_del = o_del + e_del, oe_ins = o_ins + e_ins;
  const int want_cigar = n_cigar != NULL;
  if (n_cigar) *n_cigar = 0;
  if (qlen < 0) qlen = 0;
  int n_col = qlen < 2 * w + 1 ? qlen : 2 * w + 1;
  const long zsize = (long)n_col * (tlen > 0 ? tlen : 0);
  uint8_t* z = want_cigar ? (uint8_t*)calloc((size_t)(zsize > 0 ? zsize : 1), 1) : NULL;
  int8_t* qp = (int8_t*)malloc((size_t)(qlen > 0 ? qlen : 1) * m);
  ko_eh* eh = (ko_eh*)calloc((size_t)qlen + 1, sizeof(ko_eh));
  for (int k = 0, i = 0; k < m; ++k)
    for (int j = 0; j < qlen; ++j) qp[i++] = mat[k * m + query[j]];
  eh[0].h = 0;
  eh[0].e = KO_MINUS_INF;
  int j;
  for (j = 1; j <= qlen && j <= w; ++j) eh[j].h = -(o_ins + e_ins * j), eh[j].e = KO_MINUS_INF;
  for (; j <= qlen; ++j) eh[j].h = eh[j].e = KO_MINUS_INF;
  for (int i = 0; i < tlen; ++i) {
    int32_t f = KO_MINUS_INF, h1, beg, end, t;
    const int8_t* q = &qp[target[i] * qlen];
    beg = i > w ? i - w : 0;
    end = i + w + 1 < qlen ? i + w + 1 : qlen;
    h1 = beg == 0 ? -(o_del + e_del * (i + 1)) : KO_MINUS_INF;
    uint8_t* zi = want_cigar ? &z[(size_t)i * n_col] : NULL;
    for (j = beg; j < end; ++j) {
      ko_eh* p = &eh[j];
      int32_t h, mm = p->h, e = p->e;
      uint8_t d;
      p->h = h1;
      mm += q[j];
      d = mm >= e ? 0 : 1;
      h = mm >= e ? mm : e;
      d = h >= f ? d : 2;
      h = h >= f ? h : f;
      h1 = h;
      t = mm - oe_del;
      e -= e_del;
      d |= e > t ? 1 << 2 : 0;
      e = e > t ? e : t;
      p->e = e;
      t = mm - oe_ins;
      f -= e_ins;
      d |= f > t ? 2 << 4 : 0;
      f = f > t ? f : t;
      if (zi) zi[j - beg] = d;
    }
    eh[end].h = h1;
    eh[end].e = KO_MINUS_INF;
  }
  int score = eh[qlen].h;
  if (want_cigar) {
    int n = 0, cap = 0, which = 0, i = tlen - 1, k;
    uint32_t* cig = NULL;
    k = (i + w + 1 < qlen ? i + w + 1 : qlen) - 1;
    while (i >= 0 && k >= 0) {
      const long zi = (long)i * n_col + (k - (i > w ? i - w : 0));
      which = (zi >= 0 && zi < zsize) ? (z[zi] >> (which << 1) & 3) : 0;
      if (which == 0) ko_push_cigar(&n, &cap, &cig, 0, 1), --i, --k;
      else if (which == 1) ko_push_cigar(&n, &cap, &cig, 2, 1), --i;
      else ko_push_cigar(&n, &cap, &cig, 1, 1), --k;
    }
    if (i >= 0) ko_push_cigar(&n, &cap, &cig, 2, i + 1);
    if (k >= 0) ko_push_cigar(&n, &cap, &cig, 1, k + 1);
    for (int a = 0; a < n >> 1; ++a) {
      uint32_t tmp = cig[a];
      cig[a] = cig[n - 1 - a];
      cig[n - 1 - a] = tmp;
    }
    *n_cigar = n;
    if (cigar_out)
      for (int a = 0; a < n && a < cigar_cap; a++) cigar_out[a] = cig[a];
    free(cig);
  }
  free(eh);
  free(qp);
  free(z);
  return score;
}

/*
 * Batch ksw_extend2 over packed tasks: task k has query bytes at
 * qbuf[qoff[k]..+qlen[k]), target at tbuf[toff[k]..+tlen[k]), its own h0 and w.
 * res is 6 int32 per task: score, qle, tle, gtle, gscore, max_off.
 * cells[k] gets the evaluated cell count.  OpenMP over tasks (CPU baseline).
 */
void oracle_ksw_extend2_batch(const uint8_t* qbuf, const int64_t* qoff, const int32_t* qlen,
                              const uint8_t* tbuf, const int64_t* toff, const int32_t* tlen,
                              const int32_t* h0, const int32_t* w, int64_t n, const int8_t* mat,
                              int o_del, int e_del, int o_ins, int e_ins, int end_bonus,
                              int zdrop, int32_t* res, int64_t* cells, int n_threads) {
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 256) num_threads(n_threads > 0 ? n_threads : 1)
#endif
  for (int64_t k = 0; k < n; k++) {
    int32_t* r = res + 6 * k;
    int64_t c = 0;
    r[0] = oracle_ksw_extend2(qlen[k], qbuf + qoff[k], tlen[k], tbuf + toff[k], 5, mat, o_del,
                              e_del, o_ins, e_ins, w[k], end_bonus, zdrop, h0[k], &r[1], &r[2],
                              &r[3], &r[4], &r[5], &c);
    if (cells) cells[k] = c;
  }
}

/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by, or called
 * from the product library (libfcship.so).  Only tests/, tests/cpu_mock and
 * bench.py's cpu_baseline leg load it.
 *
 * bwa's ksw_align2 (lh3/bwa ksw.c 0.7.x, reached inside `bwa-flow mem`'s mate
 * rescue from /root/reference/src/workers/BWAWorker.cpp:134-166) as the CPU
 * path actually runs it: Farrar's striped Smith-Waterman in SSE2, 16 lanes of
 * u8 (KSW_XBYTE) or 8 lanes of i16, one 128-bit register per segment.  This is
 * the CPU baseline of bench.py's ksw_align2 leg, run over OpenMP threads.
 *
 * It is the vector form of oracle/ksw_align_oracle.c (which emulates the same
 * lanes element by element and is the parity checker): same profile layout
 * (query position k in lane k / slen of segment k % slen), same saturating
 * arithmetic, first pass, lazy-F loop with its early exit and bookkeeping
 * (imax, b[] list, te / qe / score2 / te2, the reversed XSTART pass).
 * tests/test_oracle_ksw.py requires the two to agree on every output.
 * bwa's lane counts (16 / 8) are kept deliberately: the results depend on the
 * striping, so wider vectors (AVX2 / AVX-512) would not be bwa's results.
 *
 * PARITY UNPINNED against bwa itself (not vendored).
 */
#include <emmintrin.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define KS_XBYTE 0x10000
#define KS_XSTOP 0x20000
#define KS_XSUBO 0x40000
#define KS_XSTART 0x80000

typedef struct {
  int score, te, qe, score2, te2, tb, qb;
} ks_r;

typedef struct {
  int u8, p, slen, qlen, shift, max;
  __m128i* qp; /* m * slen vectors: profile of target base a, segment j */
  void* mem;
} ks_q;

static void* ks_alloc16(size_t bytes, void** base) {
  *base = malloc(bytes + 16);
  return (void*)(((uintptr_t)*base + 15) & ~(uintptr_t)15);
}

static void ks_qinit(ks_q* q, int u8, int qlen, const uint8_t* query, int m, const int8_t* mat) {
  q->u8 = u8;
  q->p = u8 ? 16 : 8;
  q->slen = (qlen + q->p - 1) / q->p;
  q->qlen = qlen;
  int mn = 127, mx = 0;
  for (int a = 0; a < m * m; a++) {
    if (mat[a] < mn) mn = mat[a];
    if (mat[a] > mx) mx = mat[a];
  }
  q->shift = (256 - (uint8_t)(int8_t)mn) & 0xFF;
  q->max = mx;
  const int slen = q->slen > 0 ? q->slen : 1;
  q->qp = (__m128i*)ks_alloc16(sizeof(__m128i) * (size_t)m * slen, &q->mem);
  for (int a = 0; a < m; a++)
    for (int j = 0; j < q->slen; j++) {
      __m128i* v = q->qp + (size_t)a * q->slen + j;
      for (int l = 0; l < q->p; l++) {
        const int k = j + l * q->slen;
        const int s = k >= qlen ? 0 : mat[a * m + query[k]];
        if (u8) ((uint8_t*)v)[l] = (uint8_t)(int8_t)(s + q->shift);
        else ((int16_t*)v)[l] = (int16_t)s;
      }
    }
}

static inline int ks_hmax_u8(__m128i v) {
  v = _mm_max_epu8(v, _mm_srli_si128(v, 8));
  v = _mm_max_epu8(v, _mm_srli_si128(v, 4));
  v = _mm_max_epu8(v, _mm_srli_si128(v, 2));
  v = _mm_max_epu8(v, _mm_srli_si128(v, 1));
  return _mm_extract_epi16(v, 0) & 0xFF;
}

static inline int ks_hmax_i16(__m128i v) {
  v = _mm_max_epi16(v, _mm_srli_si128(v, 8));
  v = _mm_max_epi16(v, _mm_srli_si128(v, 4));
  v = _mm_max_epi16(v, _mm_srli_si128(v, 2));
  return (int16_t)_mm_extract_epi16(v, 0);
}

/* b[]: column maxima >= minsc, one entry per run of consecutive columns */
typedef struct {
  uint64_t* a;
  int n, m;
} ks_blist;

static inline void ks_bpush(ks_blist* b, int imax, int i) {
  if (b->n == 0 || (int32_t)b->a[b->n - 1] + 1 != i) {
    if (b->n == b->m) {
      b->m = b->m ? b->m << 1 : 8;
      b->a = (uint64_t*)realloc(b->a, 8 * (size_t)b->m);
    }
    b->a[b->n++] = (uint64_t)imax << 32 | (uint32_t)i;
  } else if ((int)(b->a[b->n - 1] >> 32) < imax) {
    b->a[b->n - 1] = (uint64_t)imax << 32 | (uint32_t)i;
  }
}

static ks_r ks_run(const ks_q* q, int tlen, const uint8_t* target, int o_del, int e_del, int o_ins, int e_ins,
                   int xtra) {
  const int slen = q->slen, u8 = q->u8;
  ks_r r = {0, -1, -1, -1, -1, -1, -1};
  const int minsc = (xtra & KS_XSUBO) ? xtra & 0xffff : 0x10000;
  const int endsc = (xtra & KS_XSTOP) ? xtra & 0xffff : 0x10000;
  const int ns = slen > 0 ? slen : 1;
  void* mem;
  __m128i* H0 = (__m128i*)ks_alloc16(sizeof(__m128i) * 4 * (size_t)ns, &mem);
  __m128i *H1 = H0 + ns, *E = H1 + ns, *Hmax = E + ns;
  memset(H0, 0, sizeof(__m128i) * 4 * (size_t)ns);
  ks_blist b = {NULL, 0, 0};
  int gmax = 0, te = -1;
  const __m128i zero = _mm_setzero_si128();
  if (u8) {
    const __m128i v_oed = _mm_set1_epi8((char)(o_del + e_del)), v_ed = _mm_set1_epi8((char)e_del);
    const __m128i v_oei = _mm_set1_epi8((char)(o_ins + e_ins)), v_ei = _mm_set1_epi8((char)e_ins);
    const __m128i v_sh = _mm_set1_epi8((char)q->shift);
    for (int i = 0; i < tlen; i++) {
      const __m128i* S = q->qp + (size_t)target[i] * slen;
      __m128i f = zero, mx = zero;
      __m128i h = slen ? _mm_slli_si128(H0[slen - 1], 1) : zero;
      for (int j = 0; j < slen; j++) {
        h = _mm_adds_epu8(h, S[j]);
        h = _mm_subs_epu8(h, v_sh);
        __m128i e = E[j];
        h = _mm_max_epu8(h, e);
        h = _mm_max_epu8(h, f);
        mx = _mm_max_epu8(mx, h);
        H1[j] = h;
        e = _mm_max_epu8(_mm_subs_epu8(e, v_ed), _mm_subs_epu8(h, v_oed));
        E[j] = e;
        f = _mm_max_epu8(_mm_subs_epu8(f, v_ei), _mm_subs_epu8(h, v_oei));
        h = H0[j];
      }
      for (int it = 0; it < 16; it++) {
        f = _mm_slli_si128(f, 1);
        int done = 0;
        for (int j = 0; j < slen; j++) {
          h = _mm_max_epu8(H1[j], f);
          H1[j] = h;
          h = _mm_subs_epu8(h, v_oei);
          f = _mm_subs_epu8(f, v_ei);
          if (_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_subs_epu8(f, h), zero)) == 0xffff) {
            done = 1;
            break;
          }
        }
        if (done) break;
      }
      const int imax = ks_hmax_u8(mx);
      if (imax >= minsc) ks_bpush(&b, imax, i);
      if (imax > gmax) {
        gmax = imax;
        te = i;
        memcpy(Hmax, H1, sizeof(__m128i) * (size_t)slen);
        if (gmax + q->shift >= 255 || gmax >= endsc) break;
      }
      __m128i* sw = H1;
      H1 = H0;
      H0 = sw;
    }
  } else {
    const __m128i v_oed = _mm_set1_epi16((short)(o_del + e_del)), v_ed = _mm_set1_epi16((short)e_del);
    const __m128i v_oei = _mm_set1_epi16((short)(o_ins + e_ins)), v_ei = _mm_set1_epi16((short)e_ins);
    for (int i = 0; i < tlen; i++) {
      const __m128i* S = q->qp + (size_t)target[i] * slen;
      __m128i f = zero, mx = zero;
      __m128i h = slen ? _mm_slli_si128(H0[slen - 1], 2) : zero;
      for (int j = 0; j < slen; j++) {
        h = _mm_adds_epi16(h, S[j]);
        __m128i e = E[j];
        h = _mm_max_epi16(h, e);
        h = _mm_max_epi16(h, f);
        mx = _mm_max_epi16(mx, h);
        H1[j] = h;
        e = _mm_max_epi16(_mm_subs_epu16(e, v_ed), _mm_subs_epu16(h, v_oed));
        E[j] = e;
        f = _mm_max_epi16(_mm_subs_epu16(f, v_ei), _mm_subs_epu16(h, v_oei));
        h = H0[j];
      }
      for (int it = 0; it < 16; it++) {
        f = _mm_slli_si128(f, 2);
        int done = 0;
        for (int j = 0; j < slen; j++) {
          h = _mm_max_epi16(H1[j], f);
          H1[j] = h;
          h = _mm_subs_epu16(h, v_oei);
          f = _mm_subs_epu16(f, v_ei);
          if (!_mm_movemask_epi8(_mm_cmpgt_epi16(f, h))) {
            done = 1;
            break;
          }
        }
        if (done) break;
      }
      const int imax = ks_hmax_i16(mx);
      if (imax >= minsc) ks_bpush(&b, imax, i);
      if (imax > gmax) {
        gmax = imax;
        te = i;
        memcpy(Hmax, H1, sizeof(__m128i) * (size_t)slen);
        if (gmax >= endsc) break;
      }
      __m128i* sw = H1;
      H1 = H0;
      H0 = sw;
    }
  }
  r.score = u8 ? (gmax + q->shift < 255 ? gmax : 255) : gmax;
  r.te = te;
  if (!u8 || r.score != 255) {
    const int p = q->p, n = slen * p;
    int max = -1;
    for (int i = 0; i < n; i++) { /* memory order: segment i / p, lane i % p */
      const int pos = i / p + i % p * slen;
      const int v = u8 ? ((const uint8_t*)Hmax)[i] : ((const int16_t*)Hmax)[i];
      if (v > max) max = v, r.qe = pos;
      else if (v == max && pos < r.qe) r.qe = pos;
    }
    if (b.n) {
      const int w = (r.score + q->max - 1) / q->max;
      const int low = te - w, high = te + w;
      for (int i = 0; i < b.n; i++) {
        const int e = (int32_t)b.a[i];
        if ((e < low || e > high) && (int)(b.a[i] >> 32) > r.score2) r.score2 = (int)(b.a[i] >> 32), r.te2 = e;
      }
    }
  }
  free(b.a);
  free(mem);
  return r;
}

static void ks_rev(int n, uint8_t* s) {
  for (int i = 0; i < n >> 1; i++) {
    const uint8_t t = s[i];
    s[i] = s[n - 1 - i];
    s[n - 1 - i] = t;
  }
}

/* bwa ksw_align2 (qry == NULL): out[7] = score, te, qe, score2, te2, tb, qb. */
void oracle_ksw_align2_sse(int qlen, const uint8_t* query, int tlen, const uint8_t* target, int m, const int8_t* mat,
                           int o_del, int e_del, int o_ins, int e_ins, int xtra, int* out) {
  const int u8 = (xtra & KS_XBYTE) != 0;
  uint8_t* qc = (uint8_t*)malloc((size_t)qlen + 1);
  uint8_t* tc = (uint8_t*)malloc((size_t)tlen + 1);
  memcpy(qc, query, (size_t)qlen);
  memcpy(tc, target, (size_t)tlen);
  ks_q q;
  ks_qinit(&q, u8, qlen, qc, m, mat);
  ks_r r = ks_run(&q, tlen, tc, o_del, e_del, o_ins, e_ins, xtra);
  free(q.mem);
  if ((xtra & KS_XSTART) && !((xtra & KS_XSUBO) && r.score < (xtra & 0xffff))) {
    ks_rev(r.qe + 1, qc);
    ks_rev(r.te + 1, tc);
    ks_q q2;
    ks_qinit(&q2, u8, r.qe + 1, qc, m, mat);
    const ks_r rr = ks_run(&q2, tlen, tc, o_del, e_del, o_ins, e_ins, KS_XSTOP | r.score);
    free(q2.mem);
    if (r.score == rr.score) r.tb = r.te - rr.te, r.qb = r.qe - rr.qe;
  }
  free(qc);
  free(tc);
  out[0] = r.score, out[1] = r.te, out[2] = r.qe, out[3] = r.score2, out[4] = r.te2, out[5] = r.tb, out[6] = r.qb;
}

/* A batch over OpenMP threads (bench.py's CPU baseline): task k = query
 * qbuf[qoff[k], + qlen[k]) against target tbuf[toff[k], + tlen[k]), xtra[k];
 * out[7k ..] as above. */
void oracle_ksw_align2_sse_batch(const uint8_t* qbuf, const int64_t* qoff, const int32_t* qlen, const uint8_t* tbuf,
                                 const int64_t* toff, const int32_t* tlen, const int32_t* xtra, int64_t n,
                                 const int8_t* mat, int o_del, int e_del, int o_ins, int e_ins, int32_t* out,
                                 int n_threads) {
#pragma omp parallel for schedule(dynamic, 16) num_threads(n_threads > 0 ? n_threads : 1)
  for (int64_t k = 0; k < n; k++) {
    int r[7];
    oracle_ksw_align2_sse(qlen[k], qbuf + qoff[k], tlen[k], tbuf + toff[k], 5, mat, o_del, e_del, o_ins, e_ins,
                          xtra[k], r);
    for (int i = 0; i < 7; i++) out[7 * k + i] = r[i];
  }
}

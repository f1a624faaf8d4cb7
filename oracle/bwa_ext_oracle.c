/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by, or called
 * from the product (libfcship.so, libfcsgenome.so).  Only tests/ load it, as
 * the checker of falcon-genome_amd/host/seedext.cpp.
 *
 * CPU restatement of bwa's seed-extension protocol for one seed (SURVEY.md §8
 * row a7), as `fcs-genome align` reaches it in the reference through bwa-flow
 * (/root/reference/src/workers/BWAWorker.cpp:134-166).  bwa is [EXT]: not
 * vendored in /root/reference, version unpinned (bwa 0.7.x bwamem.c / bwa.c
 * restated from their published source).  PARITY UNPINNED against bwa itself;
 * the product is checked against this restatement bit for bit.
 *
 *   bwamem.c cal_max_gap, infer_bw (with the equal-length early return);
 *   bwamem.c mem_chain2aln for a chain of one seed: reference window rmax,
 *     left extension (reversed, h0 = len * a, end bonus pen_clip5) and right
 *     extension (h0 = the left score, pen_clip3), each `for (i = 0; i <
 *     MAX_BAND_TRY; ++i) { prev = a->score; aw = w << i; a->score =
 *     ksw_extend2(...); if (a->score == prev || max_off < (aw>>1) + (aw>>2))
 *     break; }` with a->score starting at -1, then the local / to-end choice
 *     and truesc, a->w = max(aw[0], aw[1]) (both start at w);
 *   bwamem.c mem_reg2aln's band and widening loop around bwa.c
 *     bwa_gen_cigar2 (its own band clamp, and the no-DP path for equal
 *     lengths with w_ == 0).
 * ksw_extend2 / ksw_global2 are this directory's restatements (ksw_oracle.c).
 */
#include <limits.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

int oracle_ksw_extend2(int qlen, const uint8_t* query, int tlen, const uint8_t* target, int m, const int8_t* mat,
                       int o_del, int e_del, int o_ins, int e_ins, int w, int end_bonus, int zdrop, int h0, int* qle_,
                       int* tle_, int* gtle_, int* gscore_, int* max_off_, int64_t* cells);
int oracle_ksw_global2(int qlen, const uint8_t* query, int tlen, const uint8_t* target, int m, const int8_t* mat,
                       int o_del, int e_del, int o_ins, int e_ins, int w, int* n_cigar, uint32_t* cigar_out,
                       int cigar_cap);

#define MAX_BAND_TRY 2

typedef struct {
  const int8_t* mat;
  int a, o_del, e_del, o_ins, e_ins, zdrop, w, pen_clip5, pen_clip3;
} ext_opt;

static int cal_max_gap(const ext_opt* o, int qlen) {
  int l_del = (int)((double)(qlen * o->a - o->o_del) / o->e_del + 1.);
  int l_ins = (int)((double)(qlen * o->a - o->o_ins) / o->e_ins + 1.);
  int l = l_del > l_ins ? l_del : l_ins;
  l = l > 1 ? l : 1;
  return l < o->w << 1 ? l : o->w << 1;
}

static int infer_bw(int l1, int l2, int score, int a, int q, int r) {
  int w;
  if (l1 == l2 && l1 * a - score < (q + r - a) << 1) return 0;
  w = (int)((double)((l1 < l2 ? l1 : l2) * a - score - q) / r + 2.);
  if (w < abs(l1 - l2)) w = abs(l1 - l2);
  return w;
}

/* bwa_gen_cigar2's alignment of query[0, l) against ref[0, rlen) with band w_. */
static int gen_cigar(const ext_opt* o, int w_, int l, const uint8_t* query, int64_t rlen, const uint8_t* ref,
                     int* n_cigar, uint32_t* cigar, int cap) {
  int i, score = 0;
  if (l == rlen && w_ == 0) { /* no gap; no need to do DP */
    for (i = 0; i < l; ++i) score += o->mat[query[i] * 5 + ref[i]];
    if (cap < 1) return INT_MIN;
    cigar[0] = (uint32_t)l << 4;
    *n_cigar = 1;
    return score;
  } else {
    int w, max_gap, max_ins, max_del, min_w;
    max_ins = (int)((double)(((l + 1) >> 1) * o->mat[0] - o->o_ins) / o->e_ins + 1.);
    max_del = (int)((double)(((l + 1) >> 1) * o->mat[0] - o->o_del) / o->e_del + 1.);
    max_gap = max_ins > max_del ? max_ins : max_del;
    max_gap = max_gap > 1 ? max_gap : 1;
    w = (max_gap + abs((int)rlen - l) + 1) >> 1;
    w = w < w_ ? w : w_;
    min_w = abs((int)rlen - l) + 3;
    w = w > min_w ? w : min_w;
    return oracle_ksw_global2(l, query, (int)rlen, ref, 5, o->mat, o->o_del, o->e_del, o->o_ins, o->e_ins, w, n_cigar,
                              cigar, cap);
  }
}

/*
 * One seed of a read on one reference sequence.  out_i = {qb, qe, score,
 * truesc, w, gscore, gw} (gw: band of the last ksw_global2, 0 on the no-DP
 * path), out_r = {rb, re}; the CIGAR (ksw ops) in cigar[0 .. *n_cigar).
 * Returns 0, or -1 when the seed lies outside its query or reference.
 */
int oracle_extend_seed_w(int l_query, const uint8_t* query, int64_t l_ref, const uint8_t* rseq_all, int qbeg,
                         int64_t rbeg, int len, int64_t win_lo, int64_t win_hi, const int8_t* mat, int o_del,
                         int e_del, int o_ins, int e_ins, int zdrop, int w, int pen_clip5, int pen_clip3,
                         int32_t* out_i, int64_t* out_r, uint32_t* cigar, int cigar_cap, int* n_cigar) {
  ext_opt o = {mat, mat[0], o_del, e_del, o_ins, e_ins, zdrop, w, pen_clip5, pen_clip3};
  int64_t rmax[2], b, e;
  int aw[2], max_off, i, score, truesc, qb, qe;
  int64_t rb, re;
  const uint8_t* rseq;
  if (len <= 0 || qbeg < 0 || qbeg + len > l_query || rbeg < 0 || rbeg + len > l_ref) return -1;
  /* the chain's window: mem_chain2aln's rmax, min / max over the chain's
     seeds (win_lo, win_hi), or that of this seed alone (-1), clipped to the sequence */
  b = rbeg - (qbeg + cal_max_gap(&o, qbeg));
  e = rbeg + len + ((l_query - qbeg - len) + cal_max_gap(&o, l_query - qbeg - len));
  if (win_lo >= 0 || win_hi >= 0) b = win_lo, e = win_hi;
  rmax[0] = b > 0 ? b : 0;
  rmax[1] = e < l_ref ? e : l_ref;
  rseq = rseq_all + rmax[0];
  aw[0] = aw[1] = w;
  score = truesc = -1;
  if (qbeg) { /* left extension */
    uint8_t *rs, *qs;
    int qle = 0, tle = 0, gtle = 0, gscore = 0;
    int64_t tmp = rbeg - rmax[0];
    qs = (uint8_t*)malloc(qbeg);
    for (i = 0; i < qbeg; ++i) qs[i] = query[qbeg - 1 - i];
    rs = (uint8_t*)malloc(tmp > 0 ? tmp : 1);
    for (i = 0; i < tmp; ++i) rs[i] = rseq[tmp - 1 - i];
    for (i = 0; i < MAX_BAND_TRY; ++i) {
      int prev = score;
      aw[0] = w << i;
      score = oracle_ksw_extend2(qbeg, qs, (int)tmp, rs, 5, mat, o_del, e_del, o_ins, e_ins, aw[0], pen_clip5, zdrop,
                                 len * o.a, &qle, &tle, &gtle, &gscore, &max_off, NULL);
      if (score == prev || max_off < (aw[0] >> 1) + (aw[0] >> 2)) break;
    }
    if (gscore <= 0 || gscore <= score - pen_clip5) { /* local extension */
      qb = qbeg - qle, rb = rbeg - tle;
      truesc = score;
    } else { /* to-end extension */
      qb = 0, rb = rbeg - gtle;
      truesc = gscore;
    }
    free(qs);
    free(rs);
  } else {
    score = truesc = len * o.a, qb = 0, rb = rbeg;
  }
  if (qbeg + len != l_query) { /* right extension */
    int qle = 0, tle = 0, gtle = 0, gscore = 0, sc0 = score;
    int q0 = qbeg + len;
    int64_t r0 = rbeg + len - rmax[0];
    for (i = 0; i < MAX_BAND_TRY; ++i) {
      int prev = score;
      aw[1] = w << i;
      score = oracle_ksw_extend2(l_query - q0, query + q0, (int)(rmax[1] - rmax[0] - r0), rseq + r0, 5, mat, o_del,
                                 e_del, o_ins, e_ins, aw[1], pen_clip3, zdrop, sc0, &qle, &tle, &gtle, &gscore,
                                 &max_off, NULL);
      if (score == prev || max_off < (aw[1] >> 1) + (aw[1] >> 2)) break;
    }
    if (gscore <= 0 || gscore <= score - pen_clip3) { /* local extension */
      qe = q0 + qle, re = rmax[0] + r0 + tle;
      truesc += score - sc0;
    } else { /* to-end extension */
      qe = l_query, re = rmax[0] + r0 + gtle;
      truesc += gscore - sc0;
    }
  } else {
    qe = l_query, re = rbeg + len;
  }
  out_i[0] = qb, out_i[1] = qe, out_i[2] = score, out_i[3] = truesc;
  out_i[4] = aw[0] > aw[1] ? aw[0] : aw[1];
  out_i[5] = 0, out_i[6] = 0;
  out_r[0] = rb, out_r[1] = re;
  *n_cigar = 0;
  if (qe <= qb || re <= rb) return 0;
  { /* mem_reg2aln: band, widening */
    int w2, tmp, last_sc = INT_MIN, gsc = 0, k = 0;
    tmp = infer_bw(qe - qb, (int)(re - rb), truesc, o.a, o_del, e_del);
    w2 = infer_bw(qe - qb, (int)(re - rb), truesc, o.a, o_ins, e_ins);
    w2 = w2 > tmp ? w2 : tmp;
    if (w2 > w) w2 = w2 < out_i[4] ? w2 : out_i[4];
    do {
      int l = qe - qb;
      int64_t rlen = re - rb;
      w2 = w2 < w << 2 ? w2 : w << 2;
      gsc = gen_cigar(&o, w2, l, query + qb, rlen, rseq_all + rb, n_cigar, cigar, cigar_cap);
      if (l == rlen && w2 == 0) {
        out_i[6] = 0;
      } else {
        int mg, mi, md, bw;
        mi = (int)((double)(((l + 1) >> 1) * mat[0] - o_ins) / e_ins + 1.);
        md = (int)((double)(((l + 1) >> 1) * mat[0] - o_del) / e_del + 1.);
        mg = mi > md ? mi : md;
        mg = mg > 1 ? mg : 1;
        bw = (mg + abs((int)rlen - l) + 1) >> 1;
        bw = bw < w2 ? bw : w2;
        out_i[6] = bw > abs((int)rlen - l) + 3 ? bw : abs((int)rlen - l) + 3;
      }
      if (gsc == last_sc || w2 == w << 2) break;
      last_sc = gsc;
      w2 <<= 1;
    } while (++k < 3 && gsc < truesc - o.a);
    out_i[5] = gsc;
  }
  return 0;
}

int oracle_extend_seed(int l_query, const uint8_t* query, int64_t l_ref, const uint8_t* rseq_all, int qbeg,
                       int64_t rbeg, int len, const int8_t* mat, int o_del, int e_del, int o_ins, int e_ins,
                       int zdrop, int w, int pen_clip5, int pen_clip3, int32_t* out_i, int64_t* out_r,
                       uint32_t* cigar, int cigar_cap, int* n_cigar) {
  return oracle_extend_seed_w(l_query, query, l_ref, rseq_all, qbeg, rbeg, len, -1, -1, mat, o_del, e_del, o_ins,
                              e_ins, zdrop, w, pen_clip5, pen_clip3, out_i, out_r, cigar, cigar_cap, n_cigar);
}

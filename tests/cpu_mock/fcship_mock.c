/*
 * TEST INFRASTRUCTURE ONLY — never shipped, never on a product path.
 *
 * A CPU stand-in for libfcship.so's banded Smith-Waterman entry points
 * (fcs_bsw_extend, fcs_bsw_global, fcs_bsw_align), computed by the oracle's
 * ksw_extend2 / ksw_global2 / ksw_align2 restatements (oracle/ksw_oracle.c,
 * oracle/ksw_align_oracle.c), so that the `-m "not gpu"`
 * tests can drive the aligner's host logic (chains, dedup / patch, primary /
 * supplementary marking, pairing, SAM fields) in a container without a GPU.
 * tests/test_align_host_cpu.py compiles it into a temporary directory and
 * puts that directory first on LD_LIBRARY_PATH of the fcs-genome child it
 * starts (ksw_align2 by the SSE2 striped form, oracle/ksw_align_sse.c, which
 * tests/test_oracle_ksw.py holds equal to the element-wise emulation); the PairHMM entry points fail (FCS_ERR_DEVICE), unless
 * FCS_MOCK_PHMM=1 (2) — then every haplotype but the first (last) scores -10
 * (placeholder likelihoods, no PairHMM at all), or FCS_MOCK_PHMM=3 — then
 * the oracle's PairHMM (oracle/pairhmm_oracle.c, slow) computes them, which lets a developer time the caller's
 * host stages (decode, pileup, regions, GVCF output) on a CPU-only machine.
 * The GPU tests run the same commands on the real library.
 *
 * The reference's CPU path for htc (BASELINE.json configs[0], "C1": GATK
 * HaplotypeCaller with the CPU PairHMM, /root/reference/src/workers/
 * HTCWorker.cpp:85,105) is timed by bench.py's cpu_baseline leg through two
 * more modes:
 *   FCS_MOCK_PHMM=java — GATK's Java LoglessPairHMM semantics (double
 *     throughout, oracle_phmm_java_log10), one pair at a time;
 *   FCS_MOCK_PHMM=gkl  — GKL's AVX-512 PairHMM restated (float pass, double
 *     rescue below 1e-28; oracle/pairhmm_simd.c), the region's pairs as one
 *     batch on FCS_MOCK_PHMM_THREADS OpenMP threads (default 1: the caller's
 *     shard threads are the parallelism, as GATK's -nct processes are).
 * Built by tests/cpu_mock/Makefile into tests/cpu_mock/build/ (never into
 * falcon-genome_amd/), and loaded only through LD_LIBRARY_PATH of the one
 * fcs-genome child process that a CPU test or the bench's baseline leg starts.
 */
#include <stdlib.h>
#include <string.h>

#include "fcship.h"

int oracle_ksw_extend2(int qlen, const uint8_t* query, int tlen, const uint8_t* target, int m, const int8_t* mat,
                       int o_del, int e_del, int o_ins, int e_ins, int w, int end_bonus, int zdrop, int h0, int* qle_,
                       int* tle_, int* gtle_, int* gscore_, int* max_off_, int64_t* cells);
double oracle_phmm_java_log10(const uint8_t* rb, const uint8_t* bq, const uint8_t* iq, const uint8_t* dq,
                              const uint8_t* gq, int R, const uint8_t* hb, int H);
int oracle_phmm_simd_batch(const uint8_t* rb, const uint8_t* bq, const uint8_t* iq, const uint8_t* dq,
                           const uint8_t* gq, const int64_t* read_off, const int32_t* read_len, const uint8_t* hb,
                           const int64_t* hap_off, const int32_t* hap_len, const int32_t* pair_read,
                           const int32_t* pair_hap, int64_t n_pairs, float* out_raw_f, double* out_log10,
                           int32_t* used_double, int n_threads);
void oracle_phmm_batch(const uint8_t* rb, const uint8_t* bq, const uint8_t* iq, const uint8_t* dq, const uint8_t* gq,
                       const int64_t* read_off, const int32_t* read_len, const uint8_t* hb, const int64_t* hap_off,
                       const int32_t* hap_len, const int32_t* pair_read, const int32_t* pair_hap, int64_t n_pairs,
                       float* out_raw_f, double* out_log10, int32_t* used_double, int n_threads);
double oracle_phmm_log10(const uint8_t* rb, const uint8_t* bq, const uint8_t* iq, const uint8_t* dq, const uint8_t* gq,
                         int R, const uint8_t* hb, int H, int* used_double);
int oracle_ksw_global2(int qlen, const uint8_t* query, int tlen, const uint8_t* target, int m, const int8_t* mat,
                       int o_del, int e_del, int o_ins, int e_ins, int w, int* n_cigar, uint32_t* cigar_out,
                       int cigar_cap);

void oracle_ksw_align2_sse(int qlen, const uint8_t* query, int tlen, const uint8_t* target, int m, const int8_t* mat,
                           int o_del, int e_del, int o_ins, int e_ins, int xtra, int* out);

/* FCS_MOCK_BSW_THREADS: OpenMP threads of the banded-SW entry points (default
 * 1).  bench.py's align CPU baseline sets it to the command's host threads, so
 * bwa's per-thread extension work runs on as many cores as the GPU run uses. */
static int bsw_threads(void) {
  const char* t = getenv("FCS_MOCK_BSW_THREADS");
  return t && atoi(t) > 0 ? atoi(t) : 1;
}

static __thread const char* g_err = "";

const char* fcs_last_error(void) { return g_err; }
const char* fcs_version(void) { return "cpu-mock"; }
int fcs_device_count(void) { return 1; }
int fcs_device_release(int32_t device) {
  (void)device;
  return FCS_OK;
}
int fcs_device_warmup(int32_t device, int32_t sessions) {
  (void)device;
  (void)sessions;
  return FCS_OK;
}

void fcs_bsw_params_default(fcs_bsw_params* p) {
  memset(p, 0, sizeof *p);
  for (int i = 0; i < 25; ++i) p->mat[i] = (i / 5 == 4 || i % 5 == 4) ? -1 : (i / 5 == i % 5 ? 1 : -4);
  p->o_del = p->o_ins = 6;
  p->e_del = p->e_ins = 1;
  p->end_bonus = 5;
  p->zdrop = 100;
}

int fcs_bsw_extend(const fcs_bsw_task* t, int32_t n, const fcs_bsw_params* p, fcs_bsw_result* r, int32_t device) {
  (void)device;
#pragma omp parallel for schedule(dynamic, 32) num_threads(bsw_threads())
  for (int32_t k = 0; k < n; ++k) {
    fcs_bsw_result* o = &r[k];
    o->score = oracle_ksw_extend2(t[k].qlen, t[k].query, t[k].tlen, t[k].target, 5, p->mat, p->o_del, p->e_del,
                                  p->o_ins, p->e_ins, t[k].w, p->end_bonus, p->zdrop, t[k].h0, &o->qle, &o->tle,
                                  &o->gtle, &o->gscore, &o->max_off, NULL);
  }
  return FCS_OK;
}

int fcs_bsw_global(const fcs_bsw_task* t, int32_t n, const fcs_bsw_params* p, int32_t* scores, uint32_t* arena,
                   const int64_t* off, const int32_t* cap, int32_t* n_cigar, int32_t device) {
  (void)device;
  int rc = FCS_OK;
#pragma omp parallel for schedule(dynamic, 32) num_threads(bsw_threads()) reduction(min : rc)
  for (int32_t k = 0; k < n; ++k) {
    int nc = 0;
    scores[k] = oracle_ksw_global2(t[k].qlen, t[k].query, t[k].tlen, t[k].target, 5, p->mat, p->o_del, p->e_del,
                                   p->o_ins, p->e_ins, t[k].w, arena ? &nc : NULL, arena ? arena + off[k] : NULL,
                                   arena ? cap[k] : 0);
    if (arena) {
      n_cigar[k] = nc;
      if (nc > cap[k]) rc = FCS_ERR_INVALID; /* negative: the min-reduction keeps it */
    }
  }
  if (rc != FCS_OK) g_err = "fcs_bsw_global: CIGAR longer than its cap";
  return rc;
}

int fcs_bsw_align(const fcs_bsw_task* t, int32_t n, const fcs_bsw_params* p, const int32_t* xtra, fcs_kswr* out,
                  int32_t device) {
  (void)device;
#pragma omp parallel for schedule(dynamic, 8) num_threads(bsw_threads())
  for (int32_t k = 0; k < n; ++k) {
    int r[7];
    oracle_ksw_align2_sse(t[k].qlen, t[k].query, t[k].tlen, t[k].target, 5, p->mat, p->o_del, p->e_del, p->o_ins,
                      p->e_ins, xtra[k], r);
    out[k] = (fcs_kswr){r[0], r[1], r[2], r[3], r[4], r[5], r[6]};
  }
  return FCS_OK;
}

void fcs_phmm_opts_default(fcs_phmm_opts* o) { memset(o, 0, sizeof *o); }

static __thread int64_t g_rescued;

/* FCS_MOCK_PHMM=gkl: one region's reads x haps as the oracle's SoA batch. */
static int mock_gkl_region(const fcs_phmm_region* g, int threads) {
  const int32_t nr = g->n_reads, nh = g->n_haps;
  const int64_t np = (int64_t)nr * nh;
  if (np == 0) return FCS_OK;
  int64_t rbytes = 0, hbytes = 0;
  for (int32_t r = 0; r < nr; ++r) rbytes += g->reads[r].len;
  for (int32_t h = 0; h < nh; ++h) hbytes += g->haps[h].len;
  uint8_t* rb = malloc(5 * (size_t)(rbytes + 1) + (size_t)hbytes + 1);
  int64_t* ro = malloc(sizeof(int64_t) * ((size_t)nr + nh));
  int32_t* rl = malloc(sizeof(int32_t) * ((size_t)nr + nh + 4 * (size_t)np));
  if (!rb || !ro || !rl) {
    free(rb), free(ro), free(rl);
    g_err = "CPU mock: out of memory";
    return FCS_ERR_INVALID;
  }
  uint8_t *bq = rb + rbytes + 1, *iq = bq + rbytes + 1, *dq = iq + rbytes + 1, *gq = dq + rbytes + 1;
  uint8_t* hb = gq + rbytes + 1;
  int64_t* ho = ro + nr;
  int32_t *hl = rl + nr, *pr = hl + nh, *ph = pr + np, *ud = ph + np;
  int64_t o = 0;
  for (int32_t r = 0; r < nr; ++r) {
    const fcs_phmm_read* x = &g->reads[r];
    ro[r] = o, rl[r] = x->len;
    memcpy(rb + o, x->bases, x->len), memcpy(bq + o, x->base_q, x->len), memcpy(iq + o, x->ins_q, x->len);
    memcpy(dq + o, x->del_q, x->len), memcpy(gq + o, x->gcp, x->len);
    o += x->len;
  }
  o = 0;
  for (int32_t h = 0; h < nh; ++h) {
    ho[h] = o, hl[h] = g->haps[h].len;
    memcpy(hb + o, g->haps[h].bases, g->haps[h].len);
    o += g->haps[h].len;
  }
  for (int64_t p = 0; p < np; ++p) pr[p] = (int32_t)(p / nh), ph[p] = (int32_t)(p % nh);
  if (oracle_phmm_simd_batch(rb, bq, iq, dq, gq, ro, rl, hb, ho, hl, pr, ph, np, NULL, g->out_log10, ud, threads) < 0)
    oracle_phmm_batch(rb, bq, iq, dq, gq, ro, rl, hb, ho, hl, pr, ph, np, NULL, g->out_log10, ud, threads);
  for (int64_t p = 0; p < np; ++p) g_rescued += ud[p];
  free(rb), free(ro), free(rl);
  return FCS_OK;
}

int fcs_phmm_compute_regions(const fcs_phmm_region* regions, int32_t n_regions, const fcs_phmm_opts* opts) {
  (void)opts;
  const char* e = getenv("FCS_MOCK_PHMM");
  g_rescued = 0;
  if (e && strcmp(e, "gkl") == 0) {
    const char* t = getenv("FCS_MOCK_PHMM_THREADS");
    const int threads = t && atoi(t) > 0 ? atoi(t) : 1;
    for (int32_t k = 0; k < n_regions; ++k) {
      const int rc = mock_gkl_region(&regions[k], threads);
      if (rc != FCS_OK) return rc;
    }
    return FCS_OK;
  }
  if (e && strcmp(e, "java") == 0) {
    for (int32_t k = 0; k < n_regions; ++k)
      for (int32_t r = 0; r < regions[k].n_reads; ++r)
        for (int32_t h = 0; h < regions[k].n_haps; ++h) {
          const fcs_phmm_read* x = &regions[k].reads[r];
          const fcs_phmm_hap* y = &regions[k].haps[h];
          regions[k].out_log10[(int64_t)r * regions[k].n_haps + h] =
              oracle_phmm_java_log10(x->bases, x->base_q, x->ins_q, x->del_q, x->gcp, x->len, y->bases, y->len);
        }
    return FCS_OK;
  }
  if (!e || (strcmp(e, "1") != 0 && strcmp(e, "2") != 0 && strcmp(e, "3") != 0)) {
    g_err = "CPU mock of libfcship: no PairHMM";
    return FCS_ERR_DEVICE;
  }
  if (e[0] == '3') {
    for (int32_t k = 0; k < n_regions; ++k)
      for (int32_t r = 0; r < regions[k].n_reads; ++r)
        for (int32_t h = 0; h < regions[k].n_haps; ++h) {
          const fcs_phmm_read* x = &regions[k].reads[r];
          const fcs_phmm_hap* y = &regions[k].haps[h];
          int ud = 0;
          regions[k].out_log10[(int64_t)r * regions[k].n_haps + h] = oracle_phmm_log10(
              x->bases, x->base_q, x->ins_q, x->del_q, x->gcp, x->len, y->bases, y->len, &ud);
          g_rescued += ud;
        }
    return FCS_OK;
  }
  for (int32_t k = 0; k < n_regions; ++k)
    for (int32_t r = 0; r < regions[k].n_reads; ++r)
      for (int32_t h = 0; h < regions[k].n_haps; ++h)
        regions[k].out_log10[(int64_t)r * regions[k].n_haps + h] = h == (e[0] == '1' ? 0 : regions[k].n_haps - 1) ? -1.0 : -10.0;
  return FCS_OK;
}
int fcs_phmm_last_rescued(int64_t* count) {
  *count = g_rescued;
  return FCS_OK;
}
int fcs_phmm_last_device_ms(double* device_ms, double* rescue_ms) {
  *device_ms = *rescue_ms = 0;
  return FCS_OK;
}

/* BGZF inflate: the member walk restated and zlib's raw inflate per member
 * (the GPU path is checked against this mock and against zlib in the tests). */
#include <zlib.h>

static uint32_t mock_le16(const uint8_t* p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8; }

int fcs_bgzf_index(const uint8_t* comp, int64_t comp_bytes, int64_t* coff, int64_t* uoff, int32_t cap,
                   int32_t* n_members, int64_t* comp_used) {
  if (!n_members || !comp_used || comp_bytes < 0 || cap < 0 || (comp_bytes > 0 && !comp) || !coff || !uoff) {
    g_err = "[E::fcs_bgzf_index] bad arguments";
    return FCS_ERR_INVALID;
  }
  int64_t at = 0, u = 0;
  int32_t k = 0;
  while (k < cap && comp_bytes - at >= 18) {
    const uint8_t* h = comp + at;
    if (h[0] != 31 || h[1] != 139 || h[2] != 8 || !(h[3] & 4)) {
      g_err = "[E::fcs_bgzf_index] no BGZF header";
      return FCS_ERR_INVALID;
    }
    const int64_t xlen = mock_le16(h + 10);
    if (comp_bytes - at < 12 + xlen) break;
    int64_t bsize = -1;
    for (int64_t x = 12; x + 4 <= 12 + xlen;) {
      const int64_t slen = mock_le16(h + x + 2);
      if (h[x] == 'B' && h[x + 1] == 'C' && slen == 2 && x + 6 <= 12 + xlen) bsize = mock_le16(h + x + 4);
      x += 4 + slen;
    }
    if (bsize < 0 || bsize + 1 < 12 + xlen + 8) {
      g_err = "[E::fcs_bgzf_index] no BGZF block size";
      return FCS_ERR_INVALID;
    }
    const int64_t len = bsize + 1;
    if (comp_bytes - at < len) break;
    const int64_t isize = (int64_t)(mock_le16(h + len - 4) | mock_le16(h + len - 2) << 16);
    if (isize > 65536) {
      g_err = "[E::fcs_bgzf_index] member inflates past 64 KiB";
      return FCS_ERR_INVALID;
    }
    coff[k] = at;
    uoff[k] = u;
    at += len;
    u += isize;
    ++k;
  }
  coff[k] = at;
  uoff[k] = u;
  *n_members = k;
  *comp_used = at;
  return FCS_OK;
}

int fcs_bgzf_inflate(const uint8_t* comp, int64_t comp_bytes, uint8_t* out, int64_t out_cap, int64_t* comp_used,
                     int64_t* out_bytes, int32_t device) {
  (void)device;
  if (!comp_used || !out_bytes || comp_bytes < 0 || (comp_bytes > 0 && !comp) || out_cap < 0 || (out_cap > 0 && !out)) {
    g_err = "[E::fcs_bgzf_inflate] bad arguments";
    return FCS_ERR_INVALID;
  }
  *comp_used = *out_bytes = 0;
  const int64_t most = comp_bytes / 20 + 1;
  int64_t* coff = malloc(sizeof(int64_t) * (size_t)(most + 1));
  int64_t* uoff = malloc(sizeof(int64_t) * (size_t)(most + 1));
  int32_t n = 0;
  int64_t used = 0;
  int rc = coff && uoff ? fcs_bgzf_index(comp, comp_bytes, coff, uoff, (int32_t)most, &n, &used) : FCS_ERR_NOMEM;
  if (rc == FCS_OK && uoff[n] > out_cap) {
    g_err = "[E::fcs_bgzf_inflate] output larger than its capacity";
    rc = FCS_ERR_INVALID;
  }
  for (int32_t k = 0; rc == FCS_OK && k < n; ++k) {
    const uint8_t* h = comp + coff[k];
    const int64_t xlen = mock_le16(h + 10), len = coff[k + 1] - coff[k], isize = uoff[k + 1] - uoff[k];
    z_stream zs;
    memset(&zs, 0, sizeof zs);
    inflateInit2(&zs, -15);
    zs.next_in = (Bytef*)(h + 12 + xlen);
    zs.avail_in = (uInt)(len - 12 - xlen - 8);
    zs.next_out = out + uoff[k];
    zs.avail_out = (uInt)isize;
    const int z = inflate(&zs, Z_FINISH);
    const int64_t got = (int64_t)zs.total_out;
    inflateEnd(&zs);
    const uint32_t want = mock_le16(h + len - 8) | mock_le16(h + len - 6) << 16;
    if (z != Z_STREAM_END || got != isize || (uint32_t)crc32(0, out + uoff[k], (uInt)isize) != want) {
      g_err = "[E::fcs_bgzf_inflate] corrupt member";
      rc = FCS_ERR_INVALID;
    }
  }
  if (rc == FCS_OK) {
    *comp_used = used;
    *out_bytes = uoff[n];
  }
  free(coff);
  free(uoff);
  return rc;
}

/* fcs_bgzf_inflate_try: FCS_MOCK_BGZF_BUSY=all makes every call busy,
 * =alternate every other one, so CPU tests cover the reader's host fallback. */
int fcs_bgzf_inflate_try(const uint8_t* comp, int64_t comp_bytes, uint8_t* out, int64_t out_cap, int64_t* comp_used,
                         int64_t* out_bytes, int32_t device) {
  static int calls = 0;
  const char* m = getenv("FCS_MOCK_BGZF_BUSY");
  const int k = __atomic_fetch_add(&calls, 1, __ATOMIC_RELAXED);
  if (m && (!strcmp(m, "all") || (!strcmp(m, "alternate") && (k & 1)))) {
    if (comp_used) *comp_used = 0;
    return FCS_BGZF_BUSY;
  }
  return fcs_bgzf_inflate(comp, comp_bytes, out, out_cap, comp_used, out_bytes, device);
}

int fcs_bgzf_warmup(int32_t device, int32_t sessions, int64_t arena_bytes) {
  (void)device;
  (void)sessions;
  (void)arena_bytes;
  return FCS_OK;
}

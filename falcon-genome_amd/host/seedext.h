// bwa's seed-extension protocol on the GPU ([EXT] bwa
// bwamem.c mem_chain2aln / mem_reg2aln and bwa.c bwa_gen_cigar2, reached in
// the reference through BWAWorker: /root/reference/src/workers/BWAWorker.cpp:134-166).
//
// Per seed (one exact match of a read on a contig), batched over many seeds:
//   * reference window: rmax = [rbeg - (qbeg + max_gap(qbeg)),
//     rbeg + len + (rest + max_gap(rest))] clipped to the contig, max_gap =
//     bwa's cal_max_gap (min(max over ins/del of (l*a - o)/e + 1, 2w), >= 1);
//   * left extension (reversed prefix vs reversed window, h0 = len * a,
//     end_bonus = pen_clip5), right extension (h0 = the left score, pen_clip3),
//     each tried with w, then 2w while the score changed and max_off >=
//     3/4 of the band (MAX_BAND_TRY = 2);
//   * local vs to-end: to the end when gscore > 0 and gscore > score - pen_clip;
//   * truesc and the band a->w = max(left band, right band);
//   * the CIGAR by ksw_global2 over [qb, qe) x [rb, re) with mem_reg2aln's band
//     (infer_bw over ins/del, capped by a->w when above w, <= 4w, widened up to
//     three times while score < truesc - a) and bwa_gen_cigar2's clamp of it.
// Every ksw_extend2 / ksw_global2 of a round runs as one GPU batch.
// oracle/bwa_ext_oracle.c restates the same protocol on the CPU
// (tests/test_seedext_gpu.py compares every field and CIGAR).
#pragma once

#include <cstdint>
#include <vector>

#include "fcship.h"

namespace fcsg {

struct SeedJob {
  const uint8_t* q = nullptr;  // query codes 0..4 (oriented)
  int qlen = 0;
  const uint8_t* ref = nullptr;  // the contig's codes 0..4
  int64_t rlen = 0;
  int seed_q = 0;  // seed: query offset, contig offset, length
  int64_t seed_r = 0;
  int seed_len = 0;
  // reference window [win_lo, win_hi) of the seed's chain (mem_chain2aln's
  // rmax: min / max over ALL the chain's seeds, clipped to the contig); -1:
  // the window of this seed alone
  int64_t win_lo = -1, win_hi = -1;
};

struct SeedAln {
  int qb = 0, qe = 0;
  int64_t rb = 0, re = 0;
  int score = 0, truesc = 0;  // bwa's a->score (last extension's score) and a->truesc
  int w = 0;                  // a->w: the widest band either extension used
  int gscore = 0;             // ksw_global2 score of the final CIGAR
  int gw = 0;                 // band of the final ksw_global2
  std::vector<uint32_t> cigar;  // ksw ops (len << 4 | 0 M, 1 I, 2 D); empty if qe <= qb or re <= rb
};

struct SeedExtOptions {
  int w = 100;        // band width (bwa -w)
  int pen_clip5 = 5;  // end bonus of the left / right extensions (bwa -L)
  int pen_clip3 = 5;
  int gpu = 0;
  bool want_cigar = true;
  int threads = 1;  // host threads for the per-job protocol work around the GPU calls
};

struct SeedExtStats {
  int64_t ext_tasks = 0, global_tasks = 0;
  double gpu_seconds = 0;
};

// bwa's cal_max_gap.
int bwa_cal_max_gap(const fcs_bsw_params& p, int qlen, int w);
// bwa's infer_bw.
int bwa_infer_bw(int l1, int l2, int score, int a, int q, int r);
// bwa_gen_cigar2's band from mem_reg2aln's w_ (query length l, reference length rlen).
int bwa_cigar_band(const fcs_bsw_params& p, int l, int64_t rlen, int w_);

void extend_seeds(const std::vector<SeedJob>& jobs, const fcs_bsw_params& p, const SeedExtOptions& opt,
                  std::vector<SeedAln>& out, SeedExtStats& st);

// mem_reg2aln's CIGAR stage alone, for alignments whose qb, qe, rb, re,
// truesc and w are set (extend_seeds runs it when opt.want_cigar): fills
// cigar, gscore and gw.  Entries with qe <= qb or re <= rb are left empty.
void global_cigars(const std::vector<SeedJob>& jobs, const fcs_bsw_params& p, const SeedExtOptions& opt,
                   std::vector<SeedAln>& alns, SeedExtStats& st);

// ksw_global2 scores (no CIGAR) of query[qb, qe) x ref[rb, re) at bwa_gen_cigar2's
// band for w_ (bwa_cigar_band; the no-gap case scored directly): mem_patch_reg's test.
struct GlobalScoreJob {
  const uint8_t* q = nullptr;
  const uint8_t* ref = nullptr;
  int qb = 0, qe = 0;
  int64_t rb = 0, re = 0;
  int w = 0;
};
void global_scores(const std::vector<GlobalScoreJob>& jobs, const fcs_bsw_params& p, int gpu, std::vector<int>& scores,
                   SeedExtStats& st);

}  // namespace fcsg

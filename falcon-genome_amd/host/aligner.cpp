#include "aligner.h"

#include <zlib.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <fstream>
#include <future>
#include <iostream>
#include <map>
#include <mutex>
#include <queue>
#include <set>
#include <sstream>
#include <thread>
#include <unordered_map>

#include "common.h"
#include "config.h"
#include "executor.h"
#include "fcship.h"
#include "intervals.h"
#include "seedext.h"
#include "workers.h"

namespace fcsg {

namespace {

uint8_t code_of(char c) {
  switch (c) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': return 3;
    default: return 4;
  }
}

std::vector<uint8_t> encode(const std::string& s) {
  std::vector<uint8_t> o(s.size());
  for (size_t i = 0; i < s.size(); ++i) o[i] = code_of(s[i]);
  return o;
}

std::string revcomp(const std::string& s) {
  std::string o(s.rbegin(), s.rend());
  for (char& c : o) c = c == 'A' ? 'T' : c == 'C' ? 'G' : c == 'G' ? 'C' : c == 'T' ? 'A' : 'N';
  return o;
}

// A seed: one exact match of the oriented read on a contig (bwa's mem_seed_t;
// reverse-strand hits use the reverse-complemented read on the forward contig).
struct Seed {
  int contig = -1;
  bool rev = false;
  int qbeg = 0, len = 0;  // on the oriented read
  int64_t rbeg = 0;       // forward-contig offset
};

// A chain of colinear seeds (bwa's mem_chain_t), with mem_chain_flt's marks.
struct Chain {
  int contig = -1;
  bool rev = false;
  std::vector<Seed> s;  // in the order they joined (query start)
  int weight = 0;
  int kept = 0, first = -1;
  int qb = 0, qe = 0;   // query span [first seed start, last seed end) on the ORIGINAL read
};

// One alignment region of a read (bwa's mem_alnreg_t): the extension of one
// seed (or a mate-rescue hit), on the oriented read / forward contig.
struct Cand {
  bool rev = false;
  int contig = -1;
  int seed_q = 0, seed_len = 0;
  int64_t seed_r = 0;
  int64_t win_lo = -1, win_hi = -1;  // the chain's reference window (-1: the seed's own)
  int seedcov = 0;                   // query bases of the chain's seeds inside the region
  SeedAln aln;                       // qb, qe, rb, re, score, truesc, w (+ CIGAR for output regions)
  int sub = 0, sub_n = 0, secondary = -1;
  int csub = 0;         // bwa's csub: ksw_align2's second-best score of a mate-rescue hit
  uint64_t hash = 0;
  double frac_rep = 0;  // the read's repetitive fraction (bwa's frac_rep; 0 for rescued hits)
  bool rescued = false; // a mate-rescue hit (seedcov = half the shorter span)
  std::vector<int> xa;  // output regions: the alternative hits of its XA tag (bwa mem_gen_alt)
  bool done = false;  // extended
  bool ok = false;    // has an alignment (qe > qb, re > rb)
};

// One read: both orientations, chains, regions and the extension cursor.
struct ReadAln {
  std::string seq[2];            // forward, reverse complement
  std::vector<uint8_t> code[2];  // codes of seq[]
  std::vector<Chain> chains;
  std::vector<Cand> cands;
  // mem_chain2aln's loop state: chain ci, its seeds by score (srt), position k
  size_t ci = 0;
  int k = -1;
  std::vector<uint64_t> srt;
  int best = -1;     // primary region
  std::vector<int> supp;  // supplementary regions (non-overlapping parts of a chimeric read)
  int mapq = 0;
  double frac_rep = 0;  // query fraction under SMEMs with more than max_occ hits
  std::vector<std::pair<int, int>> outs;  // output regions and their MAPQ (first: primary)
};

// query span of a region on the ORIGINAL read
int orig_qb(const Cand& c, int L) { return c.rev ? L - c.aln.qe : c.aln.qb; }
int orig_qe(const Cand& c, int L) { return c.rev ? L - c.aln.qb : c.aln.qe; }

uint64_t hash64(uint64_t key) {  // bwa's hash_64 (Thomas Wang)
  key += ~(key << 32);
  key ^= (key >> 22);
  key += ~(key << 13);
  key ^= (key >> 8);
  key += (key << 3);
  key ^= (key >> 15);
  key += ~(key << 27);
  key ^= (key >> 31);
  return key;
}

// bwa raw_mapq.
int raw_mapq(int diff, int a) { return (int)(6.02 * diff / a + .499); }

// bwa mem_approx_mapq_se (MEM_MAPQ_COEF 30, mapQ_coef_len 0); csub is
// ksw_align2's second-best score for mate-rescue hits, 0 otherwise.
int approx_mapq_se(const Cand& c, int min_seed_len, int match, int mismatch) {
  const SeedAln& a = c.aln;
  int sub = c.sub ? c.sub : min_seed_len * match;
  sub = c.csub > sub ? c.csub : sub;
  if (sub >= a.score || a.score <= 0) return 0;
  const int l = std::max(a.qe - a.qb, (int)(a.re - a.rb));
  const double identity = 1. - (double)(l * match - a.score) / (match + mismatch) / l;
  int mapq = (int)(30.0 * (1. - (double)sub / a.score) * std::log((double)std::max(c.seedcov, 1)) + .499);
  if (identity < 0.95) mapq = (int)(mapq * identity * identity + .499);
  if (c.sub_n > 0) mapq -= (int)(4.343 * std::log((double)c.sub_n + 1) + .499);
  mapq = std::max(0, std::min(60, mapq));
  return (int)(mapq * (1. - c.frac_rep) + .499);
}

// Seeds and chains of one read (bwa mem_collect_intv + mem_chain +
// mem_chain_flt): SMEMs of length >= min_seed_len on the FMD-index (both
// strands at once), re-seeds inside long, rare SMEMs and the third-round
// forward seeds; every occurrence (sampled down to max_occ per SMEM) is a seed;
// seeds join a chain of the same contig and strand when they continue it (bwa
// test_and_merge: colinear, diagonal within w, gaps below max_chain_gap);
// chains are weighed by the query bases their seeds cover, then filtered:
// a chain that overlaps a kept heavier one on the query by >= mask_level of
// the shorter and weighs < drop_ratio of it (and 2 min_seed_len less) is
// dropped (the first such shadowed chain is kept for MAPQ, as bwa does).
void seed_read(const KmerIndex& idx, const AlignOptions& opt, ReadAln& R) {
  const std::vector<uint8_t>& q = R.code[0];
  const int L = (int)q.size();
  std::vector<BiInterval> mems;
  idx.fmd().collect(q.data(), L, opt.k, (int)(opt.k * 1.5 + .499), 10, 20, mems);  // bwa -r 1.5, -y 20
  {  // bwa mem_chain's frac_rep: the union of the query spans of SMEMs with > max_occ hits
    std::vector<std::pair<int, int>> rep;
    for (const BiInterval& m : mems)
      if (m.s > opt.max_occ) rep.emplace_back(m.qb, m.qe);
    std::sort(rep.begin(), rep.end());
    int b = 0, e = 0, l_rep = 0;
    for (const auto& [sb, se] : rep) {
      if (sb > e) l_rep += e - b, b = sb, e = se;
      else e = std::max(e, se);
    }
    l_rep += e - b;
    R.frac_rep = L ? (double)l_rep / L : 0.;
  }
  std::vector<Seed> seeds;
  for (const BiInterval& m : mems) {
    const int64_t step = m.s > opt.max_occ ? m.s / opt.max_occ : 1;
    for (int64_t j = 0, kept = 0; j < m.s && kept < opt.max_occ; j += step, ++kept) {
      Seed sd;
      idx.fmd().locate(m, j, sd.contig, sd.rbeg, sd.rev);
      sd.len = m.qe - m.qb;
      sd.qbeg = sd.rev ? L - m.qe : m.qb;  // query offset in the oriented read
      seeds.push_back(sd);
    }
  }
  if (seeds.empty()) return;
  std::stable_sort(seeds.begin(), seeds.end(), [](const Seed& a, const Seed& b) {
    return a.contig != b.contig ? a.contig < b.contig : a.rev != b.rev ? a.rev < b.rev
         : a.qbeg != b.qbeg ? a.qbeg < b.qbeg : a.rbeg < b.rbeg;
  });
  std::vector<Chain> chains;
  size_t group0 = 0;
  for (size_t i = 0; i < seeds.size(); ++i) {
    const Seed& sd = seeds[i];
    if (i > 0 && (sd.contig != seeds[i - 1].contig || sd.rev != seeds[i - 1].rev)) group0 = chains.size();
    bool merged = false;
    for (size_t c = group0; c < chains.size() && !merged; ++c) {
      const Seed& last = chains[c].s.back();
      if (sd.qbeg >= last.qbeg && sd.qbeg + sd.len <= last.qbeg + last.len && sd.rbeg >= last.rbeg &&
          sd.rbeg + sd.len <= last.rbeg + last.len) {
        merged = true;  // contained in the last seed
        break;
      }
      const int64_t x = sd.qbeg - last.qbeg, y = sd.rbeg - last.rbeg;
      if (y >= 0 && x - y <= opt.w && y - x <= opt.w && x - last.len < opt.max_chain_gap &&
          y - last.len < opt.max_chain_gap) {
        chains[c].s.push_back(sd);
        merged = true;
      }
    }
    if (!merged) {
      Chain ch;
      ch.contig = sd.contig;
      ch.rev = sd.rev;
      ch.s.push_back(sd);
      chains.push_back(std::move(ch));
    }
  }
  for (Chain& ch : chains) {  // bwa mem_chain_weight: query bases covered by the seeds (min with the reference's)
    int64_t wq = 0, wr = 0, endq = 0, endr = 0;
    for (const Seed& sd : ch.s) {
      if (sd.qbeg >= endq) wq += sd.len;
      else if (sd.qbeg + sd.len > endq) wq += sd.qbeg + sd.len - endq;
      endq = std::max<int64_t>(endq, sd.qbeg + sd.len);
    }
    std::vector<const Seed*> byr;
    for (const Seed& sd : ch.s) byr.push_back(&sd);
    std::sort(byr.begin(), byr.end(), [](const Seed* a, const Seed* b) { return a->rbeg < b->rbeg; });
    for (const Seed* sd : byr) {
      if (sd->rbeg >= endr) wr += sd->len;
      else if (sd->rbeg + sd->len > endr) wr += sd->rbeg + sd->len - endr;
      endr = std::max<int64_t>(endr, sd->rbeg + sd->len);
    }
    ch.weight = (int)std::min(wq, wr);
    const int b = ch.s.front().qbeg, e = ch.s.back().qbeg + ch.s.back().len;  // oriented
    ch.qb = ch.rev ? L - e : b;
    ch.qe = ch.rev ? L - b : e;
  }
  // ---- bwa mem_chain_flt
  std::stable_sort(chains.begin(), chains.end(), [](const Chain& a, const Chain& b) { return a.weight > b.weight; });
  std::vector<int> kept{0};
  chains[0].kept = 3;
  for (int i = 1; i < (int)chains.size(); ++i) {
    bool large_ovlp = false;
    size_t k = 0;
    for (; k < kept.size(); ++k) {
      Chain& cj = chains[kept[k]];
      const Chain& ci = chains[i];
      const int b_max = std::max(cj.qb, ci.qb), e_min = std::min(cj.qe, ci.qe);
      if (e_min > b_max) {
        const int li = ci.qe - ci.qb, lj = cj.qe - cj.qb, min_l = std::min(li, lj);
        if (e_min - b_max >= min_l * opt.mask_level && min_l < opt.max_chain_gap) {
          large_ovlp = true;
          if (cj.first < 0) cj.first = i;
          if (ci.weight < cj.weight * opt.drop_ratio && cj.weight - ci.weight >= opt.k << 1) break;
        }
      }
    }
    if (k == kept.size()) {
      kept.push_back(i);
      chains[i].kept = large_ovlp ? 2 : 3;
    }
  }
  for (int j : kept)
    if (chains[j].first >= 0) chains[chains[j].first].kept = 1;
  for (Chain& ch : chains)
    if (ch.kept > 0) R.chains.push_back(std::move(ch));
}

// mem_chain2aln's test: is seed s (almost) inside a region already made? (then
// extending it would repeat that alignment)
bool seed_covered(const Seed& s, const std::vector<Cand>& regs, int L, const fcs_bsw_params& P, int w) {
  for (const Cand& p : regs) {
    if (!p.done || p.contig != s.contig || p.rev != s.rev) continue;
    const SeedAln& a = p.aln;
    if (s.rbeg < a.rb || s.rbeg + s.len > a.re || s.qbeg < a.qb || s.qbeg + s.len > a.qe) continue;
    if (s.len - p.seed_len > .1 * L) continue;  // this seed may give a better alignment
    int64_t qd = s.qbeg - a.qb, rd = s.rbeg - a.rb;  // ahead of the seed
    int mg = bwa_cal_max_gap(P, (int)std::min<int64_t>(qd, rd), w);
    int ww = std::min(mg, a.w);
    if (qd - rd < ww && rd - qd < ww) return true;
    qd = a.qe - (s.qbeg + s.len), rd = a.re - (s.rbeg + s.len);  // behind it
    mg = bwa_cal_max_gap(P, (int)std::min<int64_t>(qd, rd), w);
    ww = std::min(mg, a.w);
    if (qd - rd < ww && rd - qd < ww) return true;
  }
  return false;
}

// One GPU extension round per step of mem_chain2aln over every read: each read
// with work left extends its next seed that no earlier region covers (chains
// in mem_chain_flt order, seeds by length, longest first); the extension's
// region joins the read's list before the read's next seed is tested, as in
// bwa's sequential loop.  Regions get the chain's reference window.
void extend_chains(const KmerIndex& idx, const fcs_bsw_params& P, const AlignOptions& opt,
                   std::vector<ReadAln>& reads, AlignStats& st) {
  std::vector<ReadAln*> active;
  for (ReadAln& R : reads) {
    R.ci = 0;
    R.k = -1;
    R.srt.clear();
    if (!R.chains.empty()) active.push_back(&R);
  }
  // the next seed of read R to extend: its region is appended (not yet done);
  // false when the read's chains are exhausted
  auto next_seed = [&](ReadAln& R) {
    const int L = (int)R.code[0].size();
    while (R.ci < R.chains.size()) {
      const Chain& c = R.chains[R.ci];
      if (R.k < 0 && R.srt.empty()) {
        R.srt.resize(c.s.size());
        for (size_t i = 0; i < c.s.size(); ++i) R.srt[i] = (uint64_t)c.s[i].len << 32 | i;
        std::sort(R.srt.begin(), R.srt.end());
        R.k = (int)c.s.size() - 1;
      }
      int pick = -1;
      for (; R.k >= 0; --R.k) {
        const Seed& s = c.s[(uint32_t)R.srt[R.k]];
        if (seed_covered(s, R.cands, L, P, opt.w)) {
          // unless an already extended, long overlapping seed of this chain sits on another diagonal
          size_t i = R.k + 1;
          for (; i < c.s.size(); ++i) {
            if (R.srt[i] == 0) continue;
            const Seed& t = c.s[(uint32_t)R.srt[i]];
            if (t.len < s.len * .95) continue;
            if (s.qbeg <= t.qbeg && s.qbeg + s.len - t.qbeg >= s.len >> 2 && t.qbeg - s.qbeg != t.rbeg - s.rbeg)
              break;
            if (t.qbeg <= s.qbeg && t.qbeg + t.len - s.qbeg >= s.len >> 2 && s.qbeg - t.qbeg != s.rbeg - t.rbeg)
              break;
          }
          if (i == c.s.size()) {
            R.srt[R.k] = 0;  // not extended
            continue;
          }
        }
        pick = (int)(uint32_t)R.srt[R.k];
        --R.k;
        break;
      }
      if (pick < 0) {  // chain done
        ++R.ci;
        R.k = -1;
        R.srt.clear();
        continue;
      }
      // the chain's window: min / max over its seeds (bwa's rmax), clipped to the contig
      int64_t lo = INT64_MAX, hi = INT64_MIN;
      for (const Seed& t : c.s) {
        const int rest = L - t.qbeg - t.len;
        lo = std::min(lo, t.rbeg - (t.qbeg + bwa_cal_max_gap(P, t.qbeg, opt.w)));
        hi = std::max(hi, t.rbeg + t.len + rest + bwa_cal_max_gap(P, rest, opt.w));
      }
      const Seed& s = c.s[pick];
      Cand C;
      C.rev = c.rev;
      C.contig = c.contig;
      C.seed_q = s.qbeg;
      C.seed_len = s.len;
      C.seed_r = s.rbeg;
      C.win_lo = std::max<int64_t>(0, lo);
      C.win_hi = std::min<int64_t>(hi, (int64_t)idx.codes(c.contig).size());
      C.frac_rep = R.frac_rep;
      R.cands.push_back(std::move(C));
      return true;
    }
    return false;
  };
  while (!active.empty()) {
    std::vector<char> has(active.size());
    parallel_for(active.size(), opt.threads, [&](size_t i) { has[i] = next_seed(*active[i]); });
    std::vector<ReadAln*> now;
    for (size_t i = 0; i < active.size(); ++i)
      if (has[i]) now.push_back(active[i]);
    active.swap(now);
    if (active.empty()) break;
    std::vector<SeedJob> jobs(active.size());
    for (size_t i = 0; i < active.size(); ++i) {
      const ReadAln& R = *active[i];
      const Cand& cc = R.cands.back();
      const std::vector<uint8_t>& rc = idx.codes(cc.contig);
      SeedJob& J = jobs[i];
      J.q = R.code[cc.rev].data();
      J.qlen = (int)R.code[0].size();
      J.ref = rc.data();
      J.rlen = (int64_t)rc.size();
      J.seed_q = cc.seed_q;
      J.seed_r = cc.seed_r;
      J.seed_len = cc.seed_len;
      J.win_lo = cc.win_lo;
      J.win_hi = cc.win_hi;
    }
    SeedExtOptions so;
    so.w = opt.w;
    so.pen_clip5 = so.pen_clip3 = P.end_bonus;
    so.gpu = opt.gpu;
    so.threads = opt.threads;
    so.want_cigar = false;
    std::vector<SeedAln> res;
    SeedExtStats xs;
    extend_seeds(jobs, P, so, res, xs);
    st.ext_tasks += xs.ext_tasks;
    st.gpu_seconds += xs.gpu_seconds;
    parallel_for(active.size(), opt.threads, [&](size_t i) {
      ReadAln& R = *active[i];
      Cand& C = R.cands.back();
      C.aln = std::move(res[i]);
      C.done = true;
      C.ok = C.aln.qe > C.aln.qb && C.aln.re > C.aln.rb;
      for (const Seed& t : R.chains[R.ci].s)  // bwa's seedcov over the chain's seeds
        if (t.qbeg >= C.aln.qb && t.qbeg + t.len <= C.aln.qe && t.rbeg >= C.aln.rb && t.rbeg + t.len <= C.aln.re)
          C.seedcov += t.len;
    });
  }
}

// bwa mem_sort_dedup_patch for every read: regions redundant with a
// better one (overlap > mask_level_redun of both the query and the reference
// spans) are dropped; colinear neighbours on one strand whose joint global
// alignment keeps >= 90% of the predicted score are merged into one region
// (mem_patch_reg: the joint ksw_global2 scores run as GPU rounds); then
// identical hits are dropped.  patch false: redundancy and identity only (bwa
// calls it so on the mate-rescue list, mem_matesw).
void dedup_patch(const KmerIndex& idx, const fcs_bsw_params& P, const AlignOptions& opt,
                 const std::vector<ReadAln*>& reads, bool patch, AlignStats& st) {
  // bwa works in its packed 2 x l_pac reference space (a reverse-strand region
  // [rb, re) of contig c is [2 l_pac - (off_c + re), 2 l_pac - (off_c + rb)))
  // and on original-read query coordinates; regions here hold forward
  // reference coordinates and, on the reverse strand, coordinates of the
  // reverse-complemented read.  Every order and comparison below is bwa's,
  // in bwa's space.
  struct Span2 {
    int64_t rb, re;  // packed 2 l_pac space
    int qb, qe;      // original read
  };
  auto to2 = [&](const Cand& c, int Lq) -> Span2 {
    const int64_t o = idx.offset(c.contig), L2 = 2 * idx.l_pac();
    if (!c.rev) return {o + c.aln.rb, o + c.aln.re, c.aln.qb, c.aln.qe};
    return {L2 - (o + c.aln.re), L2 - (o + c.aln.rb), Lq - c.aln.qe, Lq - c.aln.qb};
  };
  // bwa's loop `for i, for j = i - 1 down`, resumable where a patch needs its
  // global score (one GPU batch per round over all reads)
  struct Scan {
    std::vector<int> order;  // region indices by reference end
    size_t i = 1;
    int j = -2;              // -2: p's inner loop not started
    int w = 0;               // band of the pending patch (q = order[j])
    bool done = false;
  };
  std::vector<Scan> sc(reads.size());
  for (size_t r = 0; r < reads.size(); ++r) {
    ReadAln& R = *reads[r];
    const int Lq = (int)R.code[0].size();
    std::vector<Cand> keep;
    for (Cand& c : R.cands)
      if (c.ok) keep.push_back(std::move(c));
    R.cands.swap(keep);
    Scan& S = sc[r];
    for (size_t k = 0; k < R.cands.size(); ++k) S.order.push_back((int)k);
    // bwa sorts by the END position in its packed space (mem_ars2)
    std::stable_sort(S.order.begin(), S.order.end(), [&](int a, int b) {
      return to2(R.cands[a], Lq).re < to2(R.cands[b], Lq).re;
    });
    S.done = R.cands.size() <= 1;
  }
  const double redun = opt.mask_level_redun;
  for (;;) {
    std::vector<GlobalScoreJob> jobs;
    std::vector<size_t> jr;
    for (size_t r = 0; r < reads.size(); ++r) {
      Scan& S = sc[r];
      ReadAln& R = *reads[r];
      const int Lq = (int)R.code[0].size();
      while (!S.done) {
        if (S.i >= S.order.size()) {
          S.done = true;
          break;
        }
        Cand& p = R.cands[S.order[S.i]];
        const Span2 p2 = to2(p, Lq);
        // same rid (bwa's test) and, as the packed space implies, same strand
        auto near = [&](const Cand& q) {
          return q.contig == p.contig && q.rev == p.rev && p2.rb < to2(q, Lq).re + opt.max_chain_gap;
        };
        if (S.j == -2) {
          if (!near(R.cands[S.order[S.i - 1]])) {
            ++S.i;
            continue;
          }
          S.j = (int)S.i - 1;
        }
        bool wait = false;
        for (; S.j >= 0 && near(R.cands[S.order[S.j]]); --S.j) {
          Cand& q = R.cands[S.order[S.j]];
          if (q.aln.qe == q.aln.qb) continue;  // excluded
          const Span2 q2 = to2(q, Lq);
          const int64_t or_ = q2.re - p2.rb;
          const int64_t oq = q2.qb < p2.qb ? q2.qe - p2.qb : p2.qe - q2.qb;
          const int64_t mr = std::min(q2.re - q2.rb, p2.re - p2.rb);
          const int64_t mq = std::min(q2.qe - q2.qb, p2.qe - p2.qb);
          if (or_ > redun * mr && oq > redun * mq) {  // one of the hits is redundant
            if (p.aln.score < q.aln.score) {
              p.aln.qe = p.aln.qb;
              break;
            }
            q.aln.qe = q.aln.qb;
            continue;
          }
          if (!patch || q2.rb >= p2.rb) continue;
          // mem_patch_reg(q, p): colinear, a band within 2w (4w when they overlap) and a
          // relative band below 0.05 (0.10)
          const Span2 &a = q2, &b = p2;
          if (a.qb >= b.qb || a.qe >= b.qe || a.re >= b.re) continue;
          int w = (int)std::llabs((a.re - b.rb) - (int64_t)(a.qe - b.qb));
          const double rr = std::fabs((double)(a.re - b.rb) / (double)(b.re - a.rb) -
                                      (double)(a.qe - b.qb) / (double)(b.qe - a.qb));
          if (a.re < b.rb || a.qe < b.qb) {
            if (w > opt.w << 1 || rr >= 0.05) continue;
          } else if (w > opt.w << 2 || rr >= 0.10) {
            continue;
          }
          S.w = std::min(w + q.aln.w + p.aln.w, opt.w << 2);
          // the joint span [a.rb, b.re) x [a.qb, b.qe) in bwa's space; on the
          // reverse strand the same span of the forward reference against the
          // reverse-complemented read (both sequences reversed and
          // complemented: the same global score)
          GlobalScoreJob J;
          J.q = R.code[p.rev].data();
          J.ref = idx.codes(p.contig).data();
          if (!p.rev) {
            J.qb = q.aln.qb, J.qe = p.aln.qe, J.rb = q.aln.rb, J.re = p.aln.re;
          } else {
            J.qb = p.aln.qb, J.qe = q.aln.qe, J.rb = p.aln.rb, J.re = q.aln.re;
          }
          J.w = S.w;
          jobs.push_back(J);
          jr.push_back(r);
          wait = true;
          break;
        }
        if (wait) break;
        ++S.i;
        S.j = -2;
      }
    }
    if (jobs.empty()) break;
    std::vector<int> scores;
    SeedExtStats xs;
    global_scores(jobs, P, opt.gpu, scores, xs);
    st.global_tasks += xs.global_tasks;
    st.gpu_seconds += xs.gpu_seconds;
    for (size_t k = 0; k < jr.size(); ++k) {
      Scan& S = sc[jr[k]];
      ReadAln& R = *reads[jr[k]];
      const int Lq = (int)R.code[0].size();
      Cand& p = R.cands[S.order[S.i]];
      Cand& q = R.cands[S.order[S.j]];
      const Span2 a = to2(q, Lq), b = to2(p, Lq);
      const int as = q.aln.score, bs = p.aln.score;
      const int score = scores[k];
      // predicted scores from the query and the reference spans; merge at >= 90% of the larger
      const int q_s = (int)((double)(b.qe - a.qb) / ((b.qe - b.qb) + (a.qe - a.qb)) * (bs + as) + .499);
      const int r_s = (int)((double)(b.re - a.rb) / ((b.re - b.rb) + (a.re - a.rb)) * (bs + as) + .499);
      if (score > 0 && (double)score / std::max(q_s, r_s) >= 0.90) {  // merge q into p: p->qb = q->qb, p->rb = q->rb
        p.seedcov = std::max(p.seedcov, q.seedcov);
        if (!p.rev) {
          p.aln.qb = q.aln.qb;
          p.aln.rb = q.aln.rb;
        } else {  // bwa-space starts are the forward / reverse-complement ends here
          p.aln.qe = q.aln.qe;
          p.aln.re = q.aln.re;
        }
        p.aln.truesc = p.aln.score = score;
        p.aln.w = S.w;
        q.aln.qb = q.aln.qe;  // excluded
      }
      --S.j;  // the inner loop goes on below q
    }
  }
  for (ReadAln* Rp : reads) {
    ReadAln& R = *Rp;
    const int Lq = (int)R.code[0].size();
    std::vector<Cand> keep;
    for (Cand& c : R.cands)
      if (c.aln.qe > c.aln.qb) keep.push_back(std::move(c));
    // identical hits: same score and start on the query and the reference, in
    // bwa's order (alnreg_slt: score, then packed-space start, then query start)
    std::stable_sort(keep.begin(), keep.end(), [&](const Cand& x, const Cand& y) {
      if (x.aln.score != y.aln.score) return x.aln.score > y.aln.score;
      const Span2 a = to2(x, Lq), b = to2(y, Lq);
      if (a.rb != b.rb) return a.rb < b.rb;
      return a.qb < b.qb;
    });
    R.cands.clear();
    for (Cand& c : keep) {
      const Cand* prev = R.cands.empty() ? nullptr : &R.cands.back();
      if (prev && prev->aln.score == c.aln.score && to2(*prev, Lq).rb == to2(c, Lq).rb &&
          to2(*prev, Lq).qb == to2(c, Lq).qb)
        continue;
      R.cands.push_back(std::move(c));
    }
  }
}

// Primary = the first non-secondary region scoring >= min_out_score (bwa -T),
// supplementary = the later ones (bwa mem_reg2sam); MAPQ of the primary.
void pick_outputs(ReadAln& R, const AlignOptions& opt, const fcs_bsw_params& P) {
  R.best = -1;
  R.supp.clear();
  R.mapq = 0;
  for (int i = 0; i < (int)R.cands.size(); ++i) {
    const Cand& c = R.cands[i];
    if (c.secondary >= 0 || c.aln.score < opt.min_out_score) continue;
    if (R.best < 0) R.best = i;
    else R.supp.push_back(i);
  }
  if (R.best >= 0) R.mapq = approx_mapq_se(R.cands[R.best], opt.k, P.mat[0], -P.mat[1]);
}

// bwa mem_mark_primary_se: regions by score (ties by a hash of the read id and
// region index); a region whose ORIGINAL-read span overlaps a higher one's by
// >= mask_level of the shorter is its secondary (and sets that one's sub /
// sub_n); then pick_outputs.
void mark_primary(ReadAln& R, const AlignOptions& opt, uint64_t read_id, const fcs_bsw_params& P) {
  const int L = (int)R.code[0].size();
  for (size_t i = 0; i < R.cands.size(); ++i) {
    Cand& c = R.cands[i];
    c.sub = c.sub_n = 0;
    c.secondary = -1;
    c.hash = hash64(read_id + i);
  }
  std::stable_sort(R.cands.begin(), R.cands.end(), [](const Cand& a, const Cand& b) {
    return a.aln.score != b.aln.score ? a.aln.score > b.aln.score : a.hash < b.hash;
  });
  const int tmp = std::max({P.mat[0] - P.mat[1], P.o_del + P.e_del, P.o_ins + P.e_ins});
  std::vector<int> z;
  if (!R.cands.empty()) z.push_back(0);
  for (int i = 1; i < (int)R.cands.size(); ++i) {
    Cand& ci = R.cands[i];
    size_t k = 0;
    for (; k < z.size(); ++k) {
      Cand& cj = R.cands[z[k]];
      const int b_max = std::max(orig_qb(cj, L), orig_qb(ci, L)), e_min = std::min(orig_qe(cj, L), orig_qe(ci, L));
      if (e_min > b_max) {
        const int min_l = std::min(orig_qe(ci, L) - orig_qb(ci, L), orig_qe(cj, L) - orig_qb(cj, L));
        if (e_min - b_max >= min_l * opt.mask_level) {
          if (cj.sub == 0) cj.sub = ci.aln.score;
          if (cj.aln.score - ci.aln.score <= tmp) ++cj.sub_n;
          break;
        }
      }
    }
    if (k == z.size()) z.push_back(i);
    else ci.secondary = z[k];
  }
  pick_outputs(R, opt, P);
}

// bwa's strand-aware coordinates of a region (its 2 x contig-length space:
// the reverse strand runs backwards after the forward one): the start.
int64_t rb2(const KmerIndex& idx, const Cand& c) {
  return c.rev ? 2 * (int64_t)idx.codes(c.contig).size() - c.aln.re : c.aln.rb;
}

// bwa mem_infer_dir: orientation 0 FF, 1 FR, 2 RF, 3 RR of two regions of one
// contig (starts b1, b2 in the 2 x l space) and their distance.
int infer_dir(int64_t l, int64_t b1, int64_t b2, int64_t& dist) {
  const bool r1 = b1 >= l, r2 = b2 >= l;
  const int64_t p2 = r1 == r2 ? b2 : 2 * l - 1 - b2;  // read 2 on read 1's strand
  dist = p2 > b1 ? p2 - b1 : b1 - p2;
  return (r1 == r2 ? 0 : 1) ^ (p2 > b1 ? 0 : 3);
}

// Insert-size distribution per orientation of one batch (bwa mem_pestat).
struct PeStat {
  bool failed = true;
  int low = 0, high = 0;
  double avg = 0, std = 0;
  int n = 0;
};

// bwa cal_sub: score of the best region overlapping the top one by >=
// mask_level on the query, else min_seed_len x match.
int cal_sub(const ReadAln& R, const AlignOptions& opt, int match) {
  const int L = (int)R.code[0].size();
  const Cand& a0 = R.cands[0];
  for (size_t j = 1; j < R.cands.size(); ++j) {
    const Cand& aj = R.cands[j];
    const int b_max = std::max(orig_qb(aj, L), orig_qb(a0, L)), e_min = std::min(orig_qe(aj, L), orig_qe(a0, L));
    if (e_min > b_max) {
      const int min_l = std::min(orig_qe(aj, L) - orig_qb(aj, L), orig_qe(a0, L) - orig_qb(a0, L));
      if (e_min - b_max >= min_l * opt.mask_level) return aj.aln.score;
    }
  }
  return opt.k * match;
}

// bwa mem_pestat over the top regions (score order) of pairs whose both ends
// are unique (cal_sub <= 0.8 x score) on one contig, distances <= 10000;
// an orientation with < 10 pairs, or < 5% of the commonest, fails.  Per
// orientation: quartiles; mean / sd over [p25 - 2 IQR, p75 + 2 IQR]; proper
// pairs within [p25 - 3 IQR, p75 + 3 IQR], at least mean +- 4 sd, low >= 1.
std::array<PeStat, 4> pestat(const KmerIndex& idx, const std::vector<ReadAln>& m1, const std::vector<ReadAln>& m2,
                             const AlignOptions& opt, int match) {
  std::array<std::vector<int64_t>, 4> isize;
  for (size_t i = 0; i < m1.size(); ++i) {
    const ReadAln &a = m1[i], &b = m2[i];
    if (a.cands.empty() || b.cands.empty()) continue;
    if (cal_sub(a, opt, match) > 0.8 * a.cands[0].aln.score) continue;
    if (cal_sub(b, opt, match) > 0.8 * b.cands[0].aln.score) continue;
    if (a.cands[0].contig != b.cands[0].contig) continue;
    int64_t dist;
    const int d = infer_dir((int64_t)idx.codes(a.cands[0].contig).size(), rb2(idx, a.cands[0]), rb2(idx, b.cands[0]), dist);
    if (dist == 0 || dist > 10000) continue;  // bwa: `if (is && is <= max_ins)`
    isize[d].push_back(dist);
  }
  std::array<PeStat, 4> pes;
  size_t most = 0;
  for (int d = 0; d < 4; ++d) {
    std::vector<int64_t>& q = isize[d];
    PeStat& r = pes[d];
    r.n = (int)q.size();
    most = std::max(most, q.size());
    if (q.size() < 10) continue;
    std::sort(q.begin(), q.end());
    const double n = (double)q.size();
    const int64_t p25 = q[(size_t)(.25 * n + .499)], p75 = q[(size_t)(.75 * n + .499)];
    r.low = std::max(1, (int)(p25 - 2. * (p75 - p25) + .499));
    r.high = (int)(p75 + 2. * (p75 - p25) + .499);
    int x = 0;
    for (int64_t v : q)
      if (v >= r.low && v <= r.high) r.avg += (double)v, ++x;
    r.avg /= x;
    for (int64_t v : q)
      if (v >= r.low && v <= r.high) r.std += ((double)v - r.avg) * ((double)v - r.avg);
    r.std = std::sqrt(r.std / x);
    r.low = (int)(p25 - 3. * (p75 - p25) + .499);
    r.high = (int)(p75 + 3. * (p75 - p25) + .499);
    if (r.low > r.avg - 4. * r.std) r.low = (int)(r.avg - 4. * r.std + .499);
    if (r.high < r.avg + 4. * r.std) r.high = (int)(r.avg + 4. * r.std + .499);
    if (r.low < 1) r.low = 1;
    r.failed = false;
  }
  for (int d = 0; d < 4; ++d)
    if (!pes[d].failed && (double)pes[d].n < most * 0.05) pes[d].failed = true;
  return pes;
}

// Mate rescue (bwa mem_matesw): for each orientation whose distribution holds
// and in which no region of the mate already pairs with `anchor`, the window
// where the mate must lie (bwa's arithmetic in the 2 x l space, then clipped to
// the strand half holding its middle, as bns_fetch_seq does), aligned by a
// local Smith-Waterman with bwa's ksw_align2 semantics (the mate reverse-
// complemented when the orientation says so; xtra = KSW_XSUBO | KSW_XSTART |
// KSW_XBYTE for short mates | min_seed_len * a).  One job per window; the
// jobs of the whole batch run as one fcs_bsw_align call.
struct RescueJob {
  ReadAln* mate = nullptr;
  int contig = -1;
  bool is_rev = false;   // the mate reverse-complemented
  int64_t rb = 0, re = 0;  // the window in the contig's 2 x l space
  std::vector<uint8_t> ref;  // its sequence (the reverse strand's is the reverse complement)
};

void rescue_windows(const KmerIndex& idx, const std::array<PeStat, 4>& pes, const Cand& anchor, ReadAln& mate,
                    const AlignOptions& opt, std::vector<RescueJob>& jobs) {
  const std::vector<uint8_t>& rc = idx.codes(anchor.contig);
  const int64_t l = (int64_t)rc.size(), lms = (int64_t)mate.code[0].size();
  bool skip[4];
  for (int r = 0; r < 4; ++r) skip[r] = pes[r].failed;
  for (const Cand& m : mate.cands) {
    if (!m.done || m.contig != anchor.contig) continue;
    int64_t dist;
    const int r = infer_dir(l, rb2(idx, anchor), rb2(idx, m), dist);
    if (dist >= pes[r].low && dist <= pes[r].high) skip[r] = true;
  }
  const int64_t a_rb = rb2(idx, anchor);
  for (int r = 0; r < 4; ++r) {
    if (skip[r]) continue;
    const bool is_rev = (r >> 1) != (r & 1), is_larger = !(r >> 1);
    int64_t rb, re;
    if (!is_rev) {
      rb = is_larger ? a_rb + pes[r].low : a_rb - pes[r].high;
      re = (is_larger ? a_rb + pes[r].high : a_rb - pes[r].low) + lms;
    } else {
      rb = (is_larger ? a_rb + pes[r].low : a_rb - pes[r].high) - lms;
      re = is_larger ? a_rb + pes[r].high : a_rb - pes[r].low;
    }
    rb = std::max<int64_t>(rb, 0);
    re = std::min<int64_t>(re, 2 * l);
    if (rb >= re) continue;
    const bool rhalf = ((rb + re) >> 1) >= l;  // bns_fetch_seq: the half holding the middle
    if (rhalf) rb = std::max(rb, l);
    else re = std::min(re, l);
    // bwa's own cap is 100000; windows or mates past fcs_bsw_align's limits are
    // skipped here so that one long read cannot fail the batch's call
    if (re - rb < opt.k || re - rb > FCS_ALIGN_MAX_TLEN || lms > FCS_ALIGN_MAX_QLEN) continue;
    RescueJob J;
    J.mate = &mate;
    J.contig = anchor.contig;
    J.is_rev = is_rev;
    J.rb = rb;
    J.re = re;
    J.ref.resize((size_t)(re - rb));
    for (int64_t x = rb; x < re; ++x)  // the 2 x l sequence: forward, then the reverse complement
      J.ref[(size_t)(x - rb)] = x < l ? rc[x] : (rc[2 * l - 1 - x] < 4 ? (uint8_t)(3 - rc[2 * l - 1 - x]) : 4);
    jobs.push_back(std::move(J));
  }
}

// The rescue jobs' local alignments (one batch) and bwa's region for each hit
// scoring >= min_seed_len with a start: query / reference spans mapped back
// from the oriented mate and the 2 x l window, score, csub = score2, seedcov =
// half the shorter span.  Returns the reads that gained a region.
std::vector<ReadAln*> rescue_align(const KmerIndex& idx, const fcs_bsw_params& P, const AlignOptions& opt,
                                   std::vector<RescueJob>& jobs, AlignStats& st) {
  std::vector<ReadAln*> out;
  if (jobs.empty()) return out;
  const int a = P.mat[0];
  std::vector<fcs_bsw_task> tasks(jobs.size());
  std::vector<int32_t> xtra(jobs.size());
  for (size_t k = 0; k < jobs.size(); ++k) {
    const RescueJob& J = jobs[k];
    const std::vector<uint8_t>& q = J.mate->code[J.is_rev];
    tasks[k] = fcs_bsw_task{(int32_t)q.size(), (int32_t)J.ref.size(), 0, 0, q.data(), J.ref.data()};
    xtra[k] = FCS_KSW_XSUBO | FCS_KSW_XSTART | ((int)q.size() * a < 250 ? FCS_KSW_XBYTE : 0) | (opt.k * a);
  }
  std::vector<fcs_kswr> res(jobs.size());
  const uint64_t t0 = now_us();
  if (fcs_bsw_align(tasks.data(), (int32_t)tasks.size(), &P, xtra.data(), res.data(), opt.gpu) != FCS_OK)
    throw internalError(std::string("[E::fcsg] fcs_bsw_align: ") + fcs_last_error());
  st.gpu_seconds += (now_us() - t0) / 1e6;
  st.ext_tasks += (int64_t)jobs.size();
  for (size_t k = 0; k < jobs.size(); ++k) {
    const RescueJob& J = jobs[k];
    const fcs_kswr& x = res[k];
    if (x.score < opt.k || x.qb < 0) continue;  // bwa: aln.score >= min_seed_len && aln.qb >= 0
    const int64_t l = (int64_t)idx.codes(J.contig).size();
    const int lms = (int)J.mate->code[0].size();
    // bwa's region in the 2 x l space and on the original mate
    const int qb = J.is_rev ? lms - (x.qe + 1) : x.qb, qe = J.is_rev ? lms - x.qb : x.qe + 1;
    const int64_t rb = J.is_rev ? 2 * l - (J.rb + x.te + 1) : J.rb + x.tb;
    const int64_t re = J.is_rev ? 2 * l - (J.rb + x.tb) : J.rb + x.te + 1;
    Cand C;
    C.contig = J.contig;
    C.rev = rb >= l;
    if (!C.rev) {
      C.aln.rb = rb, C.aln.re = re, C.aln.qb = qb, C.aln.qe = qe;
    } else {  // forward coordinates, query on the reverse-complemented mate
      C.aln.rb = 2 * l - re, C.aln.re = 2 * l - rb, C.aln.qb = lms - qe, C.aln.qe = lms - qb;
    }
    C.aln.score = C.aln.truesc = x.score;
    C.csub = x.score2 > 0 ? x.score2 : 0;
    C.seedcov = (int)(std::min<int64_t>(C.aln.re - C.aln.rb, C.aln.qe - C.aln.qb) >> 1);
    C.rescued = C.done = C.ok = true;
    ReadAln& M = *J.mate;
    // bwa inserts the region into the mate's score-sorted list (after the
    // equal scores)
    size_t at = 0;
    while (at < M.cands.size() && M.cands[at].aln.score >= C.aln.score) ++at;
    M.cands.insert(M.cands.begin() + (std::ptrdiff_t)at, std::move(C));
    if (out.empty() || out.back() != &M) out.push_back(&M);
  }
  std::sort(out.begin(), out.end());
  out.erase(std::unique(out.begin(), out.end()), out.end());
  return out;
}

// bwa mem_pair: every (region of read 1, region of read 2) in a valid
// orientation with distance in [low, high] scores s1 + s2 + the insert-size
// log-likelihood (.721 log(2 erfc(|z| / sqrt 2)) x match, >= 0); ties by a
// hash of the pair and the pair id.  Returns the best score (0: none), the
// second best (sub), how many others lie within the mismatch/gap cost of it
// (n_sub) and the regions z of the best.
int mem_pair(const KmerIndex& idx, const std::array<PeStat, 4>& pes, const ReadAln* a[2], uint64_t id,
             const fcs_bsw_params& P, int& sub, int& n_sub, int z[2]) {
  struct K {
    uint64_t x, y;
  };
  std::vector<K> v;
  for (int r = 0; r < 2; ++r)
    for (size_t i = 0; i < a[r]->cands.size(); ++i) {
      const Cand& e = a[r]->cands[i];
      const uint64_t fpos = e.rev ? (uint64_t)(e.aln.re - 1) : (uint64_t)e.aln.rb;  // forward position of the 5' end
      v.push_back({(uint64_t)e.contig << 32 | fpos, (uint64_t)(uint32_t)e.aln.score << 32 | i << 2 | (uint64_t)e.rev << 1 | r});
    }
  auto lt = [](const K& p, const K& q) { return p.x != q.x ? p.x < q.x : p.y < q.y; };
  std::sort(v.begin(), v.end(), lt);
  std::vector<K> u;
  int y[4] = {-1, -1, -1, -1};
  for (int i = 0; i < (int)v.size(); ++i) {
    for (int r = 0; r < 2; ++r) {
      const int dir = r << 1 | (int)(v[i].y >> 1 & 1);
      if (pes[dir].failed) continue;
      const int which = r << 1 | (int)((v[i].y & 1) ^ 1);
      if (y[which] < 0) continue;
      for (int k = y[which]; k >= 0; --k) {
        if ((int)(v[k].y & 3) != which) continue;
        const int64_t dist = (int64_t)v[i].x - (int64_t)v[k].x;
        if (dist > pes[dir].high) break;
        if (dist < pes[dir].low) continue;
        const double ns = (dist - pes[dir].avg) / pes[dir].std;
        int q = (int)((double)(v[i].y >> 32) + (double)(v[k].y >> 32) +
                      .721 * std::log(2. * std::erfc(std::fabs(ns) * M_SQRT1_2)) * P.mat[0] + .499);
        if (q < 0) q = 0;
        K p;
        p.y = (uint64_t)k << 32 | (uint64_t)i;
        p.x = (uint64_t)q << 32 | (hash64(p.y ^ id << 8) & 0xffffffffu);
        u.push_back(p);
      }
    }
    y[v[i].y & 3] = i;
  }
  sub = n_sub = 0;
  if (u.empty()) return 0;
  const int tmp = std::max({P.mat[0] - P.mat[1], P.o_del + P.e_del, P.o_ins + P.e_ins});
  std::sort(u.begin(), u.end(), lt);
  const int i = (int)(u.back().y >> 32), k = (int)(uint32_t)u.back().y;
  z[v[i].y & 1] = (int)((uint32_t)v[i].y >> 2);
  z[v[k].y & 1] = (int)((uint32_t)v[k].y >> 2);
  const int ret = (int)(u.back().x >> 32);
  sub = u.size() > 1 ? (int)(u[u.size() - 2].x >> 32) : 0;
  for (int j = (int)u.size() - 2; j >= 0; --j)
    if (sub - (int)(u[j].x >> 32) <= tmp) ++n_sub;
  return ret;
}

// bwa mem_gen_alt: the XA hits of each output region k are the regions that
// are secondary to k (get_pri_idx) and score >= XA_drop_ratio (0.80) x k's
// score; a region with more than max_XA_hits (5) of them gets none.  No ALT
// contigs here, so max_XA_hits_alt does not arise.
void xa_hits(ReadAln& R) {
  constexpr double kXaDropRatio = 0.80;
  constexpr int kMaxXaHits = 5;
  for (Cand& c : R.cands) c.xa.clear();
  for (const auto& o : R.outs) {
    Cand& k = R.cands[o.first];
    for (int i = 0; i < (int)R.cands.size(); ++i)
      if (R.cands[i].secondary == o.first && R.cands[i].aln.score >= k.aln.score * kXaDropRatio) k.xa.push_back(i);
    if ((int)k.xa.size() > kMaxXaHits) k.xa.clear();
  }
}

// The CIGARs (mem_reg2aln / bwa_gen_cigar2) of every output region of the
// batch (R.outs of each read) and of their XA hits, in one round of GPU global
// alignments.
void output_cigars(const KmerIndex& idx, const fcs_bsw_params& P, const AlignOptions& opt,
                   const std::vector<ReadAln*>& reads, AlignStats& st) {
  std::vector<SeedJob> jobs;
  std::vector<SeedAln> alns;
  std::vector<Cand*> who;
  for (ReadAln* R : reads) {
    xa_hits(*R);
    std::vector<int> need;
    for (const auto& o : R->outs) {
      need.push_back(o.first);
      for (int i : R->cands[o.first].xa) need.push_back(i);
    }
    for (int ci : need) {
      Cand& C = R->cands[ci];
      const std::vector<uint8_t>& rc = idx.codes(C.contig);
      SeedJob J;
      J.q = R->code[C.rev].data();
      J.qlen = (int)R->code[C.rev].size();
      J.ref = rc.data();
      J.rlen = (int64_t)rc.size();
      jobs.push_back(J);
      alns.push_back(C.aln);
      who.push_back(&C);
    }
  }
  if (jobs.empty()) return;
  SeedExtOptions so;
  so.w = opt.w;
  so.gpu = opt.gpu;
  so.threads = opt.threads;
  SeedExtStats xs;
  global_cigars(jobs, P, so, alns, xs);
  st.global_tasks += xs.global_tasks;
  st.gpu_seconds += xs.gpu_seconds;
  for (size_t i = 0; i < who.size(); ++i) who[i]->aln = std::move(alns[i]);
}

// The single-end outputs of a read (bwa mem_reg2sam): the primary, then the
// supplementaries with MAPQ capped at the primary's.
void se_outputs(ReadAln& R, const AlignOptions& opt, const fcs_bsw_params& P) {
  R.outs.clear();
  if (R.best < 0) return;
  R.outs.emplace_back(R.best, R.mapq);
  for (int i : R.supp)
    R.outs.emplace_back(i, std::min(R.mapq, approx_mapq_se(R.cands[i], opt.k, P.mat[0], -P.mat[1])));
}

// One output alignment of a read: SAM CIGAR with soft clips, NM, MD, MAPQ.
struct OutAln {
  const Cand* c = nullptr;
  std::vector<uint32_t> cig;
  int nm = 0, mapq = 0;
  std::string md;
};

OutAln out_aln(const Reference& ref, const ReadAln& R, int i, int mapq) {
  OutAln o;
  o.c = &R.cands[i];
  o.mapq = mapq;
  const Cand& C = *o.c;
  const SeedAln& A = C.aln;
  const std::vector<uint8_t>& q = R.code[C.rev];
  if (A.qb > 0) o.cig.push_back(cigar_pack((uint32_t)A.qb, kS));
  for (uint32_t c : A.cigar) {
    const uint32_t op = c & 0xf;  // ksw ops: 0 = M, 1 = I, 2 = D
    o.cig.push_back(cigar_pack(c >> 4, op == 0 ? kM : op == 1 ? kI : kD));
  }
  if (A.qe < (int)q.size()) o.cig.push_back(cigar_pack((uint32_t)(q.size() - A.qe), kS));
  const std::string& Rs = ref.contigs[C.contig].seq;
  int run = 0;
  int qi = A.qb;
  int64_t ri = A.rb;
  for (uint32_t c : A.cigar) {
    const uint32_t len = c >> 4, op = c & 0xf;
    if (op == 0) {
      for (uint32_t j = 0; j < len; ++j, ++qi, ++ri) {
        if (q[qi] != code_of(Rs[ri]) || q[qi] > 3) {
          ++o.nm;
          o.md += std::to_string(run);
          o.md += Rs[ri];
          run = 0;
        } else {
          ++run;
        }
      }
    } else if (op == 1) {
      o.nm += (int)len;
      qi += (int)len;
    } else {
      o.nm += (int)len;
      o.md += std::to_string(run) + "^" + Rs.substr(ri, len);
      run = 0;
      ri += len;
    }
  }
  o.md += std::to_string(run);
  return o;
}

// XA:Z of an output region (bwa mem_gen_alt): "rname,[+-]pos,CIGAR,NM;" per
// alternative hit, CIGAR with soft clips.
std::string xa_tag(const Reference& ref, const ReadAln& R, const Cand& C) {
  std::string s;
  for (int i : C.xa) {
    const OutAln o = out_aln(ref, R, i, 0);
    s += ref.contigs[o.c->contig].name + "," + (o.c->rev ? "-" : "+") + std::to_string(o.c->aln.rb + 1) + ",";
    for (uint32_t c : o.cig) s += std::to_string(cigar_len(c)) + "MIDNSHP=X"[cigar_op(c)];
    s += "," + std::to_string(o.nm) + ";";
  }
  return s;
}

// SA:Z of output alignment `self`: the read's other primary / supplementary
// alignments, "rname,pos,strand,CIGAR,mapQ,NM;" (bwa mem_aln2sam; soft clips).
std::string sa_tag(const Reference& ref, const std::vector<OutAln>& v, size_t self) {
  std::string s;
  for (size_t k = 0; k < v.size(); ++k) {
    if (k == self) continue;
    const OutAln& o = v[k];
    s += ref.contigs[o.c->contig].name + "," + std::to_string(o.c->aln.rb + 1) + "," + (o.c->rev ? "-" : "+") + ",";
    for (uint32_t c : o.cig) s += std::to_string(cigar_len(c)) + "MIDNSHP=X"[cigar_op(c)];
    s += "," + std::to_string(o.mapq) + "," + std::to_string(o.nm) + ";";
  }
  return s;
}

// The BAM records of one read (R.outs): the first alignment with soft clips,
// NM / MD / AS / XS, then the supplementary ones (flag 0x800, hard clips: SEQ
// and QUAL of the aligned part only), SA tags when there are several; or one
// unmapped record.
std::vector<BamRecord> make_records(const Reference& ref, const ReadAln& R, const std::string& name,
                                    const std::string& fq_seq, const std::string& fq_qual, const AlignOptions& opt) {
  auto quals = [&](bool rev) {
    std::vector<uint8_t> q(fq_seq.size());
    for (size_t i = 0; i < q.size(); ++i) {
      const size_t j = rev ? q.size() - 1 - i : i;
      q[i] = (uint8_t)(j < fq_qual.size() ? std::max(0, fq_qual[j] - 33) : 30);
    }
    return q;
  };
  std::vector<BamRecord> out;
  if (R.outs.empty()) {
    BamRecord rec;
    rec.name = name;
    rec.set_aux_string("RG", opt.rg);
    rec.flag = kUnmapped;
    rec.seq = fq_seq;
    rec.qual = quals(false);
    out.push_back(std::move(rec));
    return out;
  }
  std::vector<OutAln> v;
  for (const auto& o : R.outs) v.push_back(out_aln(ref, R, o.first, o.second));
  for (size_t k = 0; k < v.size(); ++k) {
    const OutAln& o = v[k];
    const Cand& C = *o.c;
    BamRecord rec;
    rec.name = name;
    rec.set_aux_string("RG", opt.rg);
    rec.ref_id = C.contig;
    rec.pos = (int32_t)C.aln.rb;
    rec.mapq = (uint8_t)o.mapq;
    rec.flag = (C.rev ? kReverse : 0) | (k ? kSupplementary : 0);
    rec.cigar = o.cig;
    rec.seq = R.seq[C.rev];
    rec.qual = quals(C.rev);
    if (k) {  // supplementary: hard-clipped
      for (uint32_t& c : rec.cigar)
        if (cigar_op(c) == kS) c = cigar_pack(cigar_len(c), kH);
      rec.seq = rec.seq.substr(C.aln.qb, C.aln.qe - C.aln.qb);
      rec.qual = std::vector<uint8_t>(rec.qual.begin() + C.aln.qb, rec.qual.begin() + C.aln.qe);
    }
    rec.set_aux_int("NM", o.nm);
    rec.set_aux_string("MD", o.md);
    rec.set_aux_int("AS", C.aln.score);
    rec.set_aux_int("XS", C.sub);
    if (v.size() > 1) rec.set_aux_string("SA", sa_tag(ref, v, k));
    if (!C.xa.empty()) rec.set_aux_string("XA", xa_tag(ref, R, C));
    out.push_back(std::move(rec));
  }
  return out;
}

// Mate fields of a paired read's records (bwa mem_aln2sam): `mate` is the
// other read's first record.  An unmapped record takes its mate's place and
// strand (its SEQ / QUAL then reverse-complemented, as bwa prints them); TLEN
// from the 5' ends, 0 when either is unmapped.
void link_mate(std::vector<BamRecord>& recs, const BamRecord& mate_in, bool read1, bool proper) {
  for (BamRecord& p : recs) {
    BamRecord m;
    m.ref_id = mate_in.ref_id;
    m.pos = mate_in.pos;
    m.flag = mate_in.flag;
    m.cigar = mate_in.cigar;
    const bool p_unmapped = p.flag & kUnmapped, m_unmapped = m.flag & kUnmapped;
    p.flag |= kPaired | (read1 ? kRead1 : kRead2) | (proper ? kProperPair : 0);
    if (m_unmapped) p.flag |= kMateUnmapped;
    if (p_unmapped && !m_unmapped) {
      p.ref_id = m.ref_id;
      p.pos = m.pos;
      if (m.flag & kReverse) {
        p.flag |= kReverse;
        p.seq = revcomp(p.seq);
        std::reverse(p.qual.begin(), p.qual.end());
      }
    }
    if (m_unmapped && !p_unmapped) {
      m.ref_id = p.ref_id;
      m.pos = p.pos;
      m.flag = (uint16_t)((m.flag & ~kReverse) | (p.flag & kReverse));
    }
    if (m.flag & kReverse) p.flag |= kMateReverse;
    p.next_ref_id = m.ref_id;
    p.next_pos = m.ref_id >= 0 ? m.pos : -1;
    p.tlen = 0;
    if (m.ref_id >= 0 && p.ref_id == m.ref_id && !p_unmapped && !m_unmapped) {
      const int64_t p0 = p.pos + ((p.flag & kReverse) ? cigar_ref_len(p.cigar) - 1 : 0);
      const int64_t p1 = m.pos + ((m.flag & kReverse) ? cigar_ref_len(m.cigar) - 1 : 0);
      p.tlen = (int32_t)(-(p0 - p1 + (p0 > p1 ? 1 : p0 < p1 ? -1 : 0)));
    }
  }
}

// Seeds, chains, the GPU extension rounds and dedup / patch for a batch of
// reads; regions sorted by score (mem_sort_dedup_patch's order).
void align_batch(const KmerIndex& idx, const std::vector<std::string>& seqs, const AlignOptions& opt,
                 std::vector<ReadAln>& reads, AlignStats& st) {
  const uint64_t t0 = now_us();
  reads.assign(seqs.size(), ReadAln{});
  parallel_for(seqs.size(), opt.threads, [&](size_t r) {
    ReadAln& R = reads[r];
    R.seq[0] = seqs[r];
    R.seq[1] = revcomp(seqs[r]);
    R.code[0] = encode(R.seq[0]);
    R.code[1] = encode(R.seq[1]);
    seed_read(idx, opt, R);
  });
  const uint64_t t1 = now_us();
  st.seed_seconds += (t1 - t0) / 1e6;
  extend_chains(idx, st.params, opt, reads, st);
  std::vector<ReadAln*> ptr;
  for (ReadAln& R : reads) ptr.push_back(&R);
  dedup_patch(idx, st.params, opt, ptr, true, st);
  for (ReadAln& R : reads) std::vector<Chain>().swap(R.chains);
  st.extend_seconds += (now_us() - t1) / 1e6;
}

}  // namespace

KmerIndex::KmerIndex(const Reference& ref, int k, const std::string& index_path) : k_(k) {
  if (k < 8 || k > 63) throw invalidParam("minimum seed length must be in [8, 63]");
  for (const Contig& c : ref.contigs) {
    codes_.emplace_back(c.seq.size());
    for (size_t p = 0; p < c.seq.size(); ++p) codes_.back()[p] = code_of(c.seq[p]);
    off_.push_back(l_pac_);
    l_pac_ += (int64_t)c.seq.size();
  }
  if (!index_path.empty()) fmd_ = FmdIndex::load(index_path, codes_);
  loaded_ = fmd_ != nullptr;
  if (!fmd_) fmd_ = std::make_unique<FmdIndex>(codes_);
}

std::string fmd_index_path(const std::string& fasta) { return fasta + ".fcsidx"; }

void build_fmd_index(const std::string& fasta, int sa_intv) {
  const Reference ref = load_fasta(fasta);
  std::vector<std::vector<uint8_t>> codes;
  for (const Contig& c : ref.contigs) {
    codes.emplace_back(c.seq.size());
    for (size_t p = 0; p < c.seq.size(); ++p) codes.back()[p] = code_of(c.seq[p]);
  }
  FmdIndex(codes, sa_intv).save(fmd_index_path(fasta));
}

AlignStats align_reads(const Reference& ref, const KmerIndex& idx, const std::vector<std::string>& names,
                       const std::vector<std::string>& seqs, const std::vector<std::string>& quals,
                       const AlignOptions& opt, std::vector<BamRecord>& out) {
  AlignStats st;
  fcs_bsw_params_default(&st.params);
  const uint64_t t0 = now_us();
  std::vector<ReadAln> reads;
  align_batch(idx, seqs, opt, reads, st);
  const uint64_t tp = now_us();
  parallel_for(reads.size(), opt.threads, [&](size_t r) {
    mark_primary(reads[r], opt, opt.read_id0 + r, st.params);
    se_outputs(reads[r], opt, st.params);
  });
  std::vector<ReadAln*> ptr;
  for (ReadAln& R : reads) ptr.push_back(&R);
  const uint64_t tc = now_us();
  st.pair_seconds += (tc - tp) / 1e6;
  output_cigars(idx, st.params, opt, ptr, st);
  const uint64_t tr = now_us();
  st.extend_seconds += (tr - tc) / 1e6;
  st.reads = (int64_t)seqs.size();
  std::vector<std::vector<BamRecord>> recs(reads.size());
  parallel_for(reads.size(), opt.threads,
               [&](size_t i) { recs[i] = make_records(ref, reads[i], names[i], seqs[i], quals[i], opt); });
  for (auto& v : recs)
    for (BamRecord& r : v) out.push_back(std::move(r));
  st.record_seconds += (now_us() - tr) / 1e6;
  for (const ReadAln& R : reads) st.mapped += R.best >= 0, st.supplementary += R.supp.size();
  st.seconds = (now_us() - t0) / 1e6;
  return st;
}

AlignStats align_pairs(const Reference& ref, const KmerIndex& idx, const std::vector<std::string>& names,
                       const std::vector<std::string>& seqs1, const std::vector<std::string>& quals1,
                       const std::vector<std::string>& seqs2, const std::vector<std::string>& quals2,
                       const AlignOptions& opt, std::vector<BamRecord>& out) {
  AlignStats st;
  fcs_bsw_params_default(&st.params);
  const fcs_bsw_params& P = st.params;
  const uint64_t t0 = now_us();
  const size_t n = names.size();
  if (seqs1.size() != n || seqs2.size() != n) throw invalidParam("align_pairs: mate lists differ in length");
  // both mates in one batch: one GPU round per extension step for all
  std::vector<std::string> both(seqs1);
  both.insert(both.end(), seqs2.begin(), seqs2.end());
  std::vector<ReadAln> all;
  align_batch(idx, both, opt, all, st);
  std::vector<ReadAln> m1(std::make_move_iterator(all.begin()), std::make_move_iterator(all.begin() + n));
  std::vector<ReadAln> m2(std::make_move_iterator(all.begin() + n), std::make_move_iterator(all.end()));
  all.clear();
  const uint64_t tp = now_us();
  const std::array<PeStat, 4> pes = pestat(idx, m1, m2, opt, P.mat[0]);
  st.pe_pairs = pes[1].n;
  st.pe_low = pes[1].low;
  st.pe_high = pes[1].high;
  st.pe_avg = pes[1].avg;
  st.pe_std = pes[1].std;
  // mate rescue (bwa mem_sam_pe): every region of a read within pen_unpaired of
  // its best (at most max_matesw) searches the mate's windows
  if (!pes[0].failed || !pes[1].failed || !pes[2].failed || !pes[3].failed) {
    // the anchors are copies taken before any rescue (bwa's b[] lists); bwa
    // runs mem_matesw anchor by anchor, and each call's skip[] sees the
    // regions the earlier anchors of the same read added to the mate.  Here
    // round k runs the k-th anchor of every read as one device batch, so the
    // k-th anchor's windows are chosen after rounds 0 .. k - 1 have landed.
    // (The two ends are independent: end s's anchors only add to end !s,
    // whose own anchors were copied before.)
    std::vector<std::array<std::vector<Cand>, 2>> anchors(n);
    parallel_for(n, opt.threads, [&](size_t i) {
      ReadAln* r[2] = {&m1[i], &m2[i]};
      for (int s = 0; s < 2; ++s)
        for (const Cand& c : r[s]->cands)
          if (c.aln.score >= r[s]->cands[0].aln.score - opt.pen_unpaired && (int)anchors[i][s].size() < opt.max_matesw)
            anchors[i][s].push_back(c);
    });
    size_t rounds = 0;
    for (const auto& a : anchors) rounds = std::max({rounds, a[0].size(), a[1].size()});
    std::vector<ReadAln*> resc;
    for (size_t k = 0; k < rounds; ++k) {
      std::vector<std::vector<RescueJob>> per(n);
      parallel_for(n, opt.threads, [&](size_t i) {
        ReadAln* r[2] = {&m1[i], &m2[i]};
        for (int s = 0; s < 2; ++s)
          if (k < anchors[i][s].size()) rescue_windows(idx, pes, anchors[i][s][k], *r[!s], opt, per[i]);
      });
      std::vector<RescueJob> jobs;
      for (auto& v : per)
        for (RescueJob& J : v) jobs.push_back(std::move(J));
      if (jobs.empty()) continue;
      const uint64_t te = now_us();
      std::vector<ReadAln*> got = rescue_align(idx, P, opt, jobs, st);
      resc.insert(resc.end(), got.begin(), got.end());
      st.extend_seconds += (now_us() - te) / 1e6;
      st.pair_seconds -= (now_us() - te) / 1e6;
    }
    std::sort(resc.begin(), resc.end());
    resc.erase(std::unique(resc.begin(), resc.end()), resc.end());
    const uint64_t te = now_us();
    dedup_patch(idx, P, opt, resc, false, st);
    st.extend_seconds += (now_us() - te) / 1e6;
    st.pair_seconds -= (now_us() - te) / 1e6;
  }
  // pairing (bwa mem_sam_pe after mem_matesw)
  std::vector<char> proper(n, 0);
  parallel_for(n, opt.threads, [&](size_t i) {
    ReadAln* a[2] = {&m1[i], &m2[i]};
    const uint64_t id = opt.read_id0 + i;
    for (int s = 0; s < 2; ++s) mark_primary(*a[s], opt, id << 1 | s, P);
    int z[2] = {0, 0}, sub = 0, n_sub = 0;
    const ReadAln* ca[2] = {a[0], a[1]};
    const int o = !a[0]->cands.empty() && !a[1]->cands.empty() ? mem_pair(idx, pes, ca, id, P, sub, n_sub, z) : 0;
    bool multi = false;
    for (int s = 0; s < 2 && o > 0; ++s)  // an end with more than one hit (a split read): no pairing
      for (size_t j = 1; j < a[s]->cands.size(); ++j)
        if (a[s]->cands[j].secondary < 0 && a[s]->cands[j].aln.score >= opt.min_out_score) multi = true;
    if (o > 0 && !multi) {
      const int score_un = a[0]->cands[0].aln.score + a[1]->cands[0].aln.score - opt.pen_unpaired;
      const int subo = std::max(sub, score_un);
      int q_pe = raw_mapq(o - subo, P.mat[0]);
      if (n_sub > 0) q_pe -= (int)(4.343 * std::log((double)n_sub + 1) + .499);
      q_pe = std::max(0, std::min(60, q_pe));
      q_pe = (int)(q_pe * (1. - .5 * (a[0]->cands[0].frac_rep + a[1]->cands[0].frac_rep)) + .499);
      int q_se[2];
      if (o > score_un) {  // the pair is preferred: its regions are output, re-rooted if secondary
        for (int s = 0; s < 2; ++s) {
          Cand& c = a[s]->cands[z[s]];
          if (c.secondary >= 0) c.sub = a[s]->cands[c.secondary].aln.score, c.secondary = -2;
          q_se[s] = approx_mapq_se(c, opt.k, P.mat[0], -P.mat[1]);
          q_se[s] = q_se[s] > q_pe ? q_se[s] : q_pe < q_se[s] + 40 ? q_pe : q_se[s] + 40;
          q_se[s] = std::min(q_se[s], raw_mapq(c.aln.score - c.csub, P.mat[0]));  // bwa's tandem-repeat cap
        }
        proper[i] = 1;
      } else {
        z[0] = z[1] = 0;
        for (int s = 0; s < 2; ++s) q_se[s] = approx_mapq_se(a[s]->cands[0], opt.k, P.mat[0], -P.mat[1]);
      }
      for (int s = 0; s < 2; ++s) {
        a[s]->outs.clear();
        a[s]->outs.emplace_back(z[s], q_se[s]);
      }
      return;
    }
    // no pairing: single-end outputs; proper if the top hits make a pair
    for (int s = 0; s < 2; ++s) se_outputs(*a[s], opt, P);
    if (a[0]->best >= 0 && a[1]->best >= 0 && a[0]->cands[0].contig == a[1]->cands[0].contig) {
      int64_t dist;
      const int d = infer_dir((int64_t)idx.codes(a[0]->cands[0].contig).size(), rb2(idx, a[0]->cands[0]),
                              rb2(idx, a[1]->cands[0]), dist);
      if (!pes[d].failed && dist >= pes[d].low && dist <= pes[d].high) proper[i] = 1;
    }
  });
  std::vector<ReadAln*> ptr;
  for (size_t i = 0; i < n; ++i) ptr.push_back(&m1[i]), ptr.push_back(&m2[i]);
  const uint64_t tc = now_us();
  st.pair_seconds += (tc - tp) / 1e6;
  output_cigars(idx, P, opt, ptr, st);
  const uint64_t tr = now_us();
  st.extend_seconds += (tr - tc) / 1e6;
  std::vector<std::vector<BamRecord>> recs(n);
  parallel_for(n, opt.threads, [&](size_t i) {
    std::vector<BamRecord> r1 = make_records(ref, m1[i], names[i], seqs1[i], quals1[i], opt);
    std::vector<BamRecord> r2 = make_records(ref, m2[i], names[i], seqs2[i], quals2[i], opt);
    const BamRecord h1 = r1[0], h2 = r2[0];
    link_mate(r1, h2, true, proper[i]);
    link_mate(r2, h1, false, proper[i]);
    recs[i] = std::move(r1);
    for (BamRecord& r : r2) recs[i].push_back(std::move(r));
  });
  for (auto& v : recs)
    for (BamRecord& r : v) out.push_back(std::move(r));
  st.record_seconds += (now_us() - tr) / 1e6;
  for (size_t i = 0; i < n; ++i) {
    st.mapped += !m1[i].outs.empty() + !m2[i].outs.empty();
    st.supplementary += (m1[i].outs.empty() ? 0 : m1[i].outs.size() - 1) + (m2[i].outs.empty() ? 0 : m2[i].outs.size() - 1);
    st.proper += 2 * proper[i];
    for (const ReadAln* R : {&m1[i], &m2[i]})  // placed by the mate rescue
      st.rescued += !R->outs.empty() && R->cands[R->outs[0].first].rescued;
  }
  st.reads = 2 * (int64_t)n;
  st.seconds = (now_us() - t0) / 1e6;
  return st;
}

// ------------------------------------------------------------------ align jobs
namespace {

// FASTQ records from a plain or gzip-compressed file (zlib's gz reader passes
// plain files through), names without '@', comments or /1 /2.
class FastqReader {
 public:
  explicit FastqReader(const std::string& path) : path_(path) {
    f_ = gzopen(path.c_str(), "rb");
    if (!f_) throw fileNotFound(path);
    gzbuffer(f_, 1 << 18);
  }
  ~FastqReader() {
    if (f_) gzclose(f_);
  }
  FastqReader(const FastqReader&) = delete;
  FastqReader& operator=(const FastqReader&) = delete;
  bool next(std::string& name, std::string& seq, std::string& qual) {
    if (!line(name)) return false;
    if (name.empty() || name[0] != '@') throw formatError(path_ + ": FASTQ record does not start with '@'");
    name.erase(0, 1);
    const size_t ws = name.find_first_of(" \t");
    if (ws != std::string::npos) name.resize(ws);
    if (name.size() > 2 && name[name.size() - 2] == '/') name.resize(name.size() - 2);  // /1, /2
    std::string plus;
    if (!line(seq) || !line(plus) || !line(qual)) throw formatError(path_ + ": truncated FASTQ record " + name);
    if (qual.size() != seq.size()) throw formatError(path_ + ": FASTQ quality length differs for " + name);
    return true;
  }

 private:
  bool line(std::string& out) {
    out.clear();
    char buf[4096];
    for (;;) {
      if (!gzgets(f_, buf, sizeof buf)) return !out.empty();
      out += buf;
      if (!out.empty() && out.back() == '\n') {
        out.pop_back();
        if (!out.empty() && out.back() == '\r') out.pop_back();
        return true;
      }
    }
  }
  std::string path_;
  gzFile f_ = nullptr;
};

// The FMD-index of a reference, built once per process and shared by the
// read-group jobs of one run (bwa-flow loads its prebuilt index per run).
std::shared_ptr<const KmerIndex> index_cached(const std::string& path, const Reference& ref, int k) {
  static std::mutex mu;
  static std::map<std::pair<std::string, int>, std::shared_ptr<const KmerIndex>> cache;
  std::lock_guard<std::mutex> g(mu);
  auto& e = cache[{path, k}];
  if (!e) e = std::make_shared<const KmerIndex>(ref, k, fmd_index_path(path));
  return e;
}

void add_stats(AlignStats& tot, const AlignStats& st) {
  tot.reads += st.reads;
  tot.mapped += st.mapped;
  tot.proper += st.proper;
  tot.supplementary += st.supplementary;
  tot.rescued += st.rescued;
  tot.seconds += st.seconds;
  tot.gpu_seconds += st.gpu_seconds;
  tot.seed_seconds += st.seed_seconds;
  tot.extend_seconds += st.extend_seconds;
  tot.pair_seconds += st.pair_seconds;
  tot.record_seconds += st.record_seconds;
  tot.ext_tasks += st.ext_tasks;
  tot.global_tasks += st.global_tasks;
  if (st.pe_pairs) tot.pe_pairs = st.pe_pairs, tot.pe_low = st.pe_low, tot.pe_high = st.pe_high,
                   tot.pe_avg = st.pe_avg, tot.pe_std = st.pe_std;
}

}  // namespace

AlignStats align_fastq(const AlignJob& job, const std::vector<int>& devices, std::string& report) {
  if (devices.empty())
    throw failedCommand("[E::fcs-genome align] no GPU visible (gpu.devices); the GPU path has no CPU fallback");
  // bwa.gpu_slots host threads per device: a chunk's seeding and host protocol
  // work overlap other chunks' GPU rounds (one slot left the GPU idle between
  // its rounds: 4.6 s vs 2.6 s of alignment wall for 795K reads, gpurun_out/r3y).
  // Seeding is host work (~16 us per read), so by default (0) every host
  // thread gets a slot: hardware threads / devices, at least 4.
  std::vector<int> gpus;
  int per = conf().get_int("bwa.gpu_slots");
  if (per <= 0) per = std::max<int>(4, (int)(host_cpus() / devices.size()));
  for (int k = 0; k < per; ++k) gpus.insert(gpus.end(), devices.begin(), devices.end());
  const uint64_t t_start = now_us();
  const auto ref_p = load_reference_cached(job.ref_path);
  const Reference& ref = *ref_p;
  AlignOptions base;
  base.rg = job.rg;
  base.chunk_size = conf().get_int("bwa.chunk_size");
  const int nslot = (int)gpus.size();
  {
    // bwa.nt host threads for the whole job, shared by the device slots
    const int nt = conf().get_int("bwa.nt");
    const int all = nt > 0 ? nt : (int)host_cpus();
    base.threads = std::max(1, all / nslot);
  }
  const uint64_t t_ref = now_us();
  const auto idx_p = index_cached(job.ref_path, ref, base.k);
  const KmerIndex& idx = *idx_p;
  const uint64_t t_idx = now_us();

  // FASTQ chunks: read on one thread into a short queue, aligned by one host
  // thread per device slot as they come; each chunk's records and statistics
  // are kept under its index, so the merged result is the one-slot result.
  struct Chunk {
    std::vector<std::string> names, s1, q1, s2, q2;
  };
  const bool paired = !job.fq2.empty();
  FastqReader in1(job.fq1);
  std::unique_ptr<FastqReader> in2;
  if (paired) in2 = std::make_unique<FastqReader>(job.fq2);
  const size_t per_chunk = (size_t)std::max(1, paired ? base.chunk_size / 2 : base.chunk_size);
  auto read_chunk = [&](Chunk& c) {
    std::string n1, a1, b1, n2, a2, b2;
    while (c.names.size() < per_chunk) {
      const bool g1 = in1.next(n1, a1, b1);
      if (paired) {  // both files in lockstep
        const bool g2 = in2->next(n2, a2, b2);
        if (g1 != g2) throw formatError("paired FASTQ files differ in read count");
        if (g1 && n1 != n2) throw formatError("paired FASTQ names differ: " + n1 + " vs " + n2);
        if (g1) c.s2.push_back(std::move(a2)), c.q2.push_back(std::move(b2));
      }
      if (!g1) break;
      c.names.push_back(std::move(n1));
      c.s1.push_back(std::move(a1));
      c.q1.push_back(std::move(b1));
    }
  };
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::pair<size_t, Chunk>> queue;
  bool eof = false, stop = false;
  std::exception_ptr err;
  std::vector<std::vector<BamRecord>> results;
  std::vector<AlignStats> chunk_stats;
  auto fail = [&](std::exception_ptr e) {
    std::lock_guard<std::mutex> g(mu);
    if (!err) err = e;
    stop = true;
    cv.notify_all();
  };
  std::thread reader([&] {
    try {
      for (size_t k = 0;; ++k) {
        Chunk c;
        read_chunk(c);
        std::unique_lock<std::mutex> lk(mu);
        if (c.names.empty() || stop) break;
        cv.wait(lk, [&] { return stop || queue.size() <= (size_t)nslot; });
        if (stop) break;
        queue.emplace_back(k, std::move(c));
        cv.notify_all();
      }
    } catch (...) {
      fail(std::current_exception());
    }
    std::lock_guard<std::mutex> g(mu);
    eof = true;
    cv.notify_all();
  });
  std::vector<std::thread> slots;
  for (int s = 0; s < nslot; ++s)
    slots.emplace_back([&, s] {
      AlignOptions opt = base;
      opt.gpu = gpus[s];
      for (;;) {
        std::pair<size_t, Chunk> item;
        {
          std::unique_lock<std::mutex> lk(mu);
          cv.wait(lk, [&] { return stop || eof || !queue.empty(); });
          if (stop || queue.empty()) return;
          item = std::move(queue.front());
          queue.pop_front();
          cv.notify_all();
        }
        if (interrupted()) return fail(std::make_exception_ptr(interruptedError()));
        try {
          const Chunk& c = item.second;
          std::vector<BamRecord> recs;
          opt.read_id0 = (int64_t)(item.first * per_chunk);  // bwa's n_processed: the hash seed of ties
          const AlignStats st = paired ? align_pairs(ref, idx, c.names, c.s1, c.q1, c.s2, c.q2, opt, recs)
                                       : align_reads(ref, idx, c.names, c.s1, c.q1, opt, recs);
          std::lock_guard<std::mutex> g(mu);
          if (results.size() <= item.first) results.resize(item.first + 1), chunk_stats.resize(item.first + 1);
          results[item.first] = std::move(recs);
          chunk_stats[item.first] = st;
        } catch (...) {
          return fail(std::current_exception());
        }
      }
    });
  reader.join();
  for (auto& t : slots) t.join();
  if (err) std::rethrow_exception(err);
  AlignStats tot;
  for (const AlignStats& st : chunk_stats) add_stats(tot, st);  // chunk order: the last batch's insert size
  std::vector<BamRecord> recs;
  {
    size_t n = 0;
    for (const auto& v : results) n += v.size();
    recs.reserve(n);
    for (auto& v : results) {
      for (BamRecord& r : v) recs.push_back(std::move(r));
      std::vector<BamRecord>().swap(v);
    }
  }
  const uint64_t t_aln = now_us();
  // coordinate order by packed keys (reference id as unsigned: unmapped last;
  // the position's sign bit flipped; ties by input order, as a stable sort)
  std::vector<std::pair<uint64_t, uint32_t>> order(recs.size());
  for (size_t i = 0; i < recs.size(); ++i)
    order[i] = {((uint64_t)(uint32_t)recs[i].ref_id << 32) | ((uint32_t)recs[i].pos ^ 0x80000000u), (uint32_t)i};
  std::sort(order.begin(), order.end());
  BamHeader h;
  h.text = "@HD\tVN:1.6\tSO:coordinate\n";
  for (const Contig& c : ref.contigs) {
    h.names.push_back(c.name);
    h.lengths.push_back((int64_t)c.seq.size());
    h.text += "@SQ\tSN:" + c.name + "\tLN:" + std::to_string(c.seq.size()) + "\n";
  }
  h.text += "@RG\tID:" + job.rg + "\tSM:" + job.sample + "\tPL:" + job.platform + "\tLB:" + job.library + "\n";
  h.text += "@PG\tID:fcs-genome\tPN:fcs-genome align\n";
  if (!job.disable_merge) {
    BamWriter w(job.output, h);
    w.index_on_close();
    std::vector<const BamRecord*> sorted(order.size());
    for (size_t i = 0; i < order.size(); ++i) sorted[i] = &recs[order[i].second];
    w.write_all(sorted);
    w.close();
  } else {
    // bwa-flow --merge_bams=0 (reference BWAWorker.cpp:140-147, worker-align.cpp:186-195):
    // num_buckets coordinate-sorted bucket BAMs; here the buckets are the
    // init_contig_intv parts of the genome (the region files htc's BamInput
    // pairs them with), a read goes to the bucket of its alignment start,
    // unmapped reads without a placed mate to the last bucket
    const int nb = std::max(1, conf().get_int("bwa.num_buckets"));
    std::vector<std::pair<std::string, int64_t>> dict;
    for (const Contig& c : ref.contigs) dict.emplace_back(c.name, (int64_t)c.seq.size());
    const auto buckets = partition_contigs(dict, nb, false);
    create_dir(job.output);
    std::vector<std::vector<const BamRecord*>> per(nb);
    std::vector<std::vector<std::pair<int64_t, int64_t>>> span(ref.contigs.size());  // per contig: [lb, ub] -> bucket
    std::vector<std::vector<int>> span_b(ref.contigs.size());
    for (int k = 0; k < nb; ++k)
      for (const Interval& iv : buckets[k]) {
        const int c = ref.index(iv.chrom);
        span[c].emplace_back(iv.lb, iv.ub);
        span_b[c].push_back(k);
      }
    for (const auto& o : order) {
      const BamRecord& r = recs[o.second];
      int k = nb - 1;
      if (r.ref_id >= 0) {
        const auto& sp = span[r.ref_id];
        const int64_t p1 = (int64_t)r.pos + 1;
        for (size_t j = 0; j < sp.size(); ++j)
          if (p1 >= sp[j].first && p1 <= sp[j].second) {
            k = span_b[r.ref_id][j];
            break;
          }
      }
      per[k].push_back(&r);
    }
    for (int k = 0; k < nb; ++k) {
      const std::string bam = get_contig_fname(job.output, k, "bam");
      BamWriter w(bam, h);
      w.index_on_close();
      w.write_all(per[k]);
      w.close();
      std::ofstream bed(get_contig_fname(job.output, k, "bed"));
      for (const Interval& iv : buckets[k]) bed << iv.chrom << '\t' << iv.lb - 1 << '\t' << iv.ub << '\n';
    }
  }
  const uint64_t t_end = now_us();
  std::ostringstream rep;
  rep << "[fcs-genome align] " << tot.reads << " reads, " << tot.mapped << " mapped, " << tot.supplementary << " supplementary, " << tot.ext_tasks
      << " extension tasks, " << tot.global_tasks << " global alignments, " << tot.seconds << " s (GPU calls "
      << tot.gpu_seconds << " s)";
  if (paired)
    rep << "; pairs: " << tot.proper << " reads properly paired, " << tot.rescued << " mates rescued, insert "
        << tot.pe_avg << " +- " << tot.pe_std << " [" << tot.pe_low << ", " << tot.pe_high << "] from " << tot.pe_pairs
        << " pairs";
  rep << "\n[fcs-genome align] read group " << job.rg << " on " << nslot << " device slot(s), " << results.size()
      << " chunks; phases: reference " << (t_ref - t_start) / 1e6 << " s, FMD index " << (t_idx - t_ref) / 1e6
      << " s (" << (idx.loaded() ? "mapped " + fmd_index_path(job.ref_path) : std::string("built in memory")) << ", sa_intv "
      << idx.fmd().sa_intv() << "), FASTQ + alignment " << (t_aln - t_idx) / 1e6 << " s (alignment thread-seconds " << tot.seconds
      << ": seeding " << tot.seed_seconds << ", extension " << tot.extend_seconds << ", pairing " << tot.pair_seconds
      << ", records " << tot.record_seconds << "), sort + BAM + index " << (t_end - t_aln) / 1e6 << " s\n";
  report = rep.str();
  return tot;
}

void merge_sorted_bams(const std::vector<std::string>& inputs, const std::string& output) {
  if (inputs.empty()) throw invalidParam("merge_sorted_bams: no input");
  std::vector<std::unique_ptr<BamReader>> rd;
  for (const std::string& p : inputs) rd.push_back(std::make_unique<BamReader>(p));
  BamHeader h = rd[0]->header();
  for (const auto& r : rd)
    if (r->header().names != h.names || r->header().lengths != h.lengths)
      throw formatError("merge: " + output + " inputs have different reference dictionaries");
  // header: the first input's lines with the @RG lines of every input after its @SQ lines
  std::string head, rgs, tail;
  std::set<std::string> seen;
  for (size_t i = 0; i < rd.size(); ++i) {
    std::istringstream ss(rd[i]->header().text);
    for (std::string line; std::getline(ss, line);) {
      if (line.rfind("@RG", 0) == 0) {
        if (seen.insert(line).second) rgs += line + "\n";
      } else if (i == 0) {
        (line.rfind("@HD", 0) == 0 || line.rfind("@SQ", 0) == 0 ? head : tail) += line + "\n";
      }
    }
  }
  h.text = head + rgs + tail;
  BamWriter w(output, h);
  w.index_on_close();
  // k-way merge by (reference as unsigned: unmapped last, position), ties by input order
  auto key = [](const BamRecord& r) { return ((uint64_t)(uint32_t)r.ref_id << 32) | ((uint32_t)r.pos ^ 0x80000000u); };
  std::vector<BamRecord> cur(rd.size());
  typedef std::pair<uint64_t, size_t> Item;
  std::priority_queue<Item, std::vector<Item>, std::greater<Item>> pq;
  for (size_t i = 0; i < rd.size(); ++i)
    if (rd[i]->next(cur[i])) pq.push({key(cur[i]), i});
  while (!pq.empty()) {
    const size_t i = pq.top().second;
    pq.pop();
    w.write(cur[i]);
    if (rd[i]->next(cur[i])) pq.push({key(cur[i]), i});
  }
  w.close();
}

}  // namespace fcsg

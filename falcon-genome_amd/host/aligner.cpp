#include "aligner.h"

#include <zlib.h>

#include <algorithm>
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

// One candidate placement of a read: a chain's seed (a maximal exact match)
// and, after the GPU extension round, its alignment.
struct Cand {
  bool rev = false;
  int contig = -1;
  int hits = 0;  // k-mer hits of the chain
  int seed_q = 0, seed_len = 0;
  int64_t seed_r = 0;
  SeedAln aln;
  bool done = false;  // extended
  bool ok = false;    // extension produced an alignment with a CIGAR
};

// One read: both orientations and its candidates.
struct ReadAln {
  std::string seq[2];            // forward, reverse complement
  std::vector<uint8_t> code[2];  // codes of seq[]
  std::vector<Cand> cands;
  int best = -1;      // index into cands of the primary alignment
  int sub = 0;        // best score of another locus (bwa's a->sub), 0 if none
  int sub_n = 0;      // other loci scoring close to the best
  int mapq = 0;
};

// bwa mem_approx_mapq_se (MEM_MAPQ_COEF 30, mapQ_coef_len 0): the primary's
// score against the best other locus, scaled by the seed coverage and identity.
int approx_mapq_se(const SeedAln& a, int sub, int sub_n, int seedcov, int min_seed_len, int match, int mismatch) {
  sub = sub ? sub : min_seed_len * match;
  if (sub >= a.truesc || a.truesc <= 0) return 0;
  const int l = std::max(a.qe - a.qb, (int)(a.re - a.rb));
  const double identity = 1. - (double)(l * match - a.truesc) / (match + mismatch) / l;
  int mapq = (int)(30.0 * (1. - (double)sub / a.truesc) * std::log((double)std::max(seedcov, 1)) + .499);
  if (identity < 0.95) mapq = (int)(mapq * identity * identity + .499);
  if (sub_n > 0) mapq -= (int)(4.343 * std::log((double)sub_n + 1) + .499);
  return std::max(0, std::min(60, mapq));
}

int64_t aln_pos(const Cand& c) { return c.aln.rb; }
int64_t aln_end(const Cand& c) { return c.aln.re; }

// Seeds and chains of one read (bwa mem_collect_intv + mem_chain): SMEMs of
// length >= min_seed_len on the FMD-index (both strands at once), re-seeds
// inside long, rare SMEMs and the third-round forward seeds; every occurrence (sampled down to max_occ per
// SMEM) is a seed; seeds join a chain of the same contig and strand when they
// continue it (bwa test_and_merge: colinear, diagonal within w, gaps below
// max_chain_gap); chains weighed by the query bases their seeds cover; up to
// max_chains chains with at least drop_ratio x the best weight become
// candidates, each extended from its longest seed.
void seed_read(const Reference& ref, const KmerIndex& idx, const AlignOptions& opt, ReadAln& R) {
  const std::vector<uint8_t>& q = R.code[0];
  const int L = (int)q.size();
  std::vector<BiInterval> mems;
  idx.fmd().collect(q.data(), L, opt.k, (int)(opt.k * 1.5 + .499), 10, 20, mems);  // bwa -r 1.5, -y 20
  struct Seed {
    int contig;
    bool rev;
    int qbeg, len;
    int64_t rbeg;
  };
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
  struct Chain {
    int contig;
    bool rev;
    std::vector<Seed> s;
    int weight = 0;
  };
  std::vector<Chain> chains;
  const int max_chain_gap = 10000;
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
      if (y >= 0 && x - y <= opt.w && y - x <= opt.w && x - last.len < max_chain_gap && y - last.len < max_chain_gap) {
        chains[c].s.push_back(sd);
        merged = true;
      }
    }
    if (!merged) chains.push_back({sd.contig, sd.rev, {sd}, 0});
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
    endr = 0;
    for (const Seed* sd : byr) {
      if (sd->rbeg >= endr) wr += sd->len;
      else if (sd->rbeg + sd->len > endr) wr += sd->rbeg + sd->len - endr;
      endr = std::max<int64_t>(endr, sd->rbeg + sd->len);
    }
    ch.weight = (int)std::min(wq, wr);
  }
  std::stable_sort(chains.begin(), chains.end(), [](const Chain& a, const Chain& b) { return a.weight > b.weight; });
  const int best_w = chains[0].weight;
  for (const Chain& ch : chains) {
    if ((int)R.cands.size() >= opt.max_chains || ch.weight < opt.drop_ratio * best_w) break;
    const Seed* top = &ch.s[0];
    for (const Seed& sd : ch.s)
      if (sd.len > top->len) top = &sd;
    Cand C;
    C.rev = ch.rev;
    C.contig = ch.contig;
    C.hits = ch.weight;
    C.seed_q = top->qbeg;
    C.seed_len = top->len;
    C.seed_r = top->rbeg;
    R.cands.push_back(std::move(C));
  }
}

// One GPU extension round over every pending candidate of `reads`.
void extend_cands(const KmerIndex& idx, const fcs_bsw_params& P, const AlignOptions& opt, std::vector<ReadAln*>& reads,
                  bool only_new, AlignStats& st) {
  std::vector<SeedJob> jobs;
  std::vector<Cand*> who;
  for (ReadAln* R : reads)
    for (Cand& C : R->cands) {
      if (only_new && C.done) continue;
      const std::vector<uint8_t>& rc = idx.codes(C.contig);
      SeedJob J;
      J.q = R->code[C.rev].data();
      J.qlen = (int)R->code[C.rev].size();
      J.ref = rc.data();
      J.rlen = (int64_t)rc.size();
      J.seed_q = C.seed_q;
      J.seed_r = C.seed_r;
      J.seed_len = C.seed_len;
      jobs.push_back(J);
      who.push_back(&C);
    }
  if (jobs.empty()) return;
  SeedExtOptions so;
  so.w = opt.w;
  so.pen_clip5 = so.pen_clip3 = P.end_bonus;
  so.gpu = opt.gpu;
  so.threads = opt.threads;
  std::vector<SeedAln> res;
  SeedExtStats xs;
  extend_seeds(jobs, P, so, res, xs);
  st.ext_tasks += xs.ext_tasks;
  st.global_tasks += xs.global_tasks;
  st.gpu_seconds += xs.gpu_seconds;
  for (size_t i = 0; i < who.size(); ++i) {
    Cand& C = *who[i];
    C.aln = std::move(res[i]);
    C.done = true;
    C.ok = C.aln.qe > C.aln.qb && C.aln.re > C.aln.rb && !C.aln.cigar.empty();
  }
}

// Primary alignment, the best other locus (bwa's sub) and the single-end MAPQ.
void pick_primary(ReadAln& R, const AlignOptions& opt) {
  R.best = -1;
  for (int i = 0; i < (int)R.cands.size(); ++i) {
    const Cand& C = R.cands[i];
    if (!C.ok) continue;
    if (R.best < 0 || C.aln.truesc > R.cands[R.best].aln.truesc ||
        (C.aln.truesc == R.cands[R.best].aln.truesc && C.hits > R.cands[R.best].hits))
      R.best = i;
  }
  R.sub = 0;
  R.sub_n = 0;
  R.mapq = 0;
  if (R.best < 0) return;
  const Cand& B = R.cands[R.best];
  const int L = (int)R.code[0].size();
  for (int i = 0; i < (int)R.cands.size(); ++i) {
    const Cand& C = R.cands[i];
    if (i == R.best || !C.ok) continue;
    const bool same_locus = C.contig == B.contig && C.rev == B.rev && std::llabs(C.aln.rb - B.aln.rb) < L / 2;
    if (same_locus) continue;
    R.sub = std::max(R.sub, C.aln.truesc);
    if (C.aln.truesc >= B.aln.truesc - 5) ++R.sub_n;  // bwa: other hits within the mapQ_coef window
  }
  R.mapq = approx_mapq_se(B.aln, R.sub, R.sub_n, std::max(B.hits, B.seed_len), opt.k, 1, 4);
}

// Insert-size distribution of one batch (bwa mem_pestat, FR orientation):
// quartiles of the fragment lengths of confidently placed pairs; proper pairs
// lie in [p25 - 3 IQR, p75 + 3 IQR] (at least mean +- 4 sd), mean / sd over the
// values within [p25 - 2 IQR, p75 + 2 IQR].
struct PeStat {
  bool ok = false;
  int low = 0, high = 0;
  double avg = 0, std = 1;
  int n = 0;
};

int64_t frag_len(const Cand& a, const Cand& b) {
  return std::max(aln_end(a), aln_end(b)) - std::min(aln_pos(a), aln_pos(b));
}

bool fr_pair(const Cand& a, const Cand& b) {
  if (a.contig != b.contig || a.rev == b.rev) return false;
  const Cand& f = a.rev ? b : a;  // forward mate starts at the left
  const Cand& r = a.rev ? a : b;
  return aln_pos(f) <= aln_pos(r) && aln_end(f) <= aln_end(r) + 16;
}

PeStat pestat(const std::vector<ReadAln>& m1, const std::vector<ReadAln>& m2) {
  PeStat ps;
  std::vector<int64_t> v;
  for (size_t i = 0; i < m1.size(); ++i) {
    const ReadAln &a = m1[i], &b = m2[i];
    if (a.best < 0 || b.best < 0 || a.mapq < 20 || b.mapq < 20) continue;
    const Cand &x = a.cands[a.best], &y = b.cands[b.best];
    if (!fr_pair(x, y)) continue;
    const int64_t f = frag_len(x, y);
    if (f > 0 && f < 10000) v.push_back(f);
  }
  ps.n = (int)v.size();
  if (v.size() < 25) return ps;  // bwa: too few pairs to estimate
  std::sort(v.begin(), v.end());
  const double p25 = (double)v[(size_t)(.25 * v.size() + .499)], p75 = (double)v[(size_t)(.75 * v.size() + .499)];
  const double iqr = p75 - p25;
  const double lo2 = p25 - 2. * iqr, hi2 = p75 + 2. * iqr;
  double s = 0, s2 = 0;
  int n = 0;
  for (int64_t x : v)
    if (x >= lo2 && x <= hi2) s += (double)x, s2 += (double)x * (double)x, ++n;
  ps.avg = s / n;
  ps.std = std::sqrt(std::max(1e-9, s2 / n - ps.avg * ps.avg));
  ps.low = (int)(p25 - 3. * iqr + .499);
  ps.high = (int)(p75 + 3. * iqr + .499);
  if (ps.low > ps.avg - 4. * ps.std) ps.low = (int)(ps.avg - 4. * ps.std + .499);
  if (ps.high < ps.avg + 4. * ps.std) ps.high = (int)(ps.avg + 4. * ps.std + .499);
  ps.low = std::max(ps.low, 1);
  ps.ok = true;
  return ps;
}

// bwa mem_pair's insert-size log-likelihood term in score units.
int pair_penalty(const PeStat& ps, int64_t dist, int match) {
  const double ns = ((double)dist - ps.avg) / ps.std;
  return (int)(.721 * std::log(2. * std::erfc(std::fabs(ns) * M_SQRT1_2)) * match + .499);
}

// Mate rescue (bwa mem_matesw's role): the mate is searched in the window the
// insert-size distribution allows opposite `anchor`, on the other strand, by
// 12-mer exact hits of the window; the best-supported diagonal becomes a seed
// for the regular extension round.  Returns false when nothing seeds.
bool rescue_seed(const KmerIndex& idx, const PeStat& ps, const Cand& anchor, ReadAln& mate) {
  const int kk = 12;
  const std::vector<uint8_t>& rc = idx.codes(anchor.contig);
  const int64_t L = (int64_t)mate.code[0].size();
  const bool rev = !anchor.rev;
  int64_t wb, we;
  if (!anchor.rev) {  // anchor forward at the left: the mate ends within [pos + low, pos + high]
    wb = aln_pos(anchor) + ps.low - L;
    we = aln_pos(anchor) + ps.high;
  } else {  // anchor reverse at the right: the mate starts within [end - high, end - low]
    wb = aln_end(anchor) - ps.high;
    we = aln_end(anchor) - ps.low + L;
  }
  wb = std::max<int64_t>(0, wb);
  we = std::min<int64_t>((int64_t)rc.size(), we);
  if (we - wb < kk || we - wb > 100000) return false;
  std::unordered_multimap<uint32_t, int64_t> win;
  win.reserve((size_t)(we - wb));
  uint32_t key = 0;
  int valid = 0;
  const uint32_t mask = (1u << (2 * kk)) - 1;
  for (int64_t p = wb; p < we; ++p) {
    if (rc[p] > 3) {
      valid = 0;
      continue;
    }
    key = ((key << 2) | rc[p]) & mask;
    if (++valid >= kk) win.emplace(key, p - kk + 1);
  }
  const std::vector<uint8_t>& q = mate.code[rev];
  std::map<int64_t, std::pair<int, int>> diag;  // diagonal -> (hits, first query pos)
  key = 0;
  valid = 0;
  for (int i = 0; i < (int)q.size(); ++i) {
    if (q[i] > 3) {
      valid = 0;
      continue;
    }
    key = ((key << 2) | q[i]) & mask;
    if (++valid < kk) continue;
    const int qp = i - kk + 1;
    auto range = win.equal_range(key);
    for (auto it = range.first; it != range.second; ++it) {
      auto& d = diag[it->second - qp];
      if (d.first++ == 0) d.second = qp;
    }
  }
  int best = 0;
  int64_t bd = 0;
  int bq = 0;
  for (const auto& [d, h] : diag)
    if (h.first > best) best = h.first, bd = d, bq = h.second;
  if (best < 2) return false;
  Cand C;
  C.rev = rev;
  C.contig = anchor.contig;
  C.hits = best;
  int qs = bq, qe = bq + kk;
  int64_t rs = bd + bq;
  while (qs > 0 && rs > 0 && q[qs - 1] < 4 && q[qs - 1] == rc[rs - 1]) --qs, --rs;
  while (qe < (int)q.size() && rs + (qe - qs) < (int64_t)rc.size() && q[qe] < 4 && q[qe] == rc[rs + (qe - qs)]) ++qe;
  C.seed_q = qs;
  C.seed_len = qe - qs;
  C.seed_r = rs;
  mate.cands.push_back(std::move(C));
  return true;
}

// The BAM record of one read: its primary alignment (soft clips, NM / MD /
// AS) or an unmapped record.
BamRecord make_record(const Reference& ref, const ReadAln& R, const std::string& name, const std::string& fq_seq,
                      const std::string& fq_qual, const AlignOptions& opt) {
  BamRecord rec;
  rec.name = name;
  rec.set_aux_string("RG", opt.rg);
  auto quals = [&](bool rev) {
    std::vector<uint8_t> q(fq_seq.size());
    for (size_t i = 0; i < q.size(); ++i) {
      const size_t j = rev ? q.size() - 1 - i : i;
      q[i] = (uint8_t)(j < fq_qual.size() ? std::max(0, fq_qual[j] - 33) : 30);
    }
    return q;
  };
  if (R.best < 0) {
    rec.flag = kUnmapped;
    rec.seq = fq_seq;
    rec.qual = quals(false);
    return rec;
  }
  const Cand& C = R.cands[R.best];
  const SeedAln& A = C.aln;
  const std::vector<uint8_t>& q = R.code[C.rev];
  std::vector<uint32_t> cig;
  if (A.qb > 0) cig.push_back(cigar_pack((uint32_t)A.qb, kS));
  for (uint32_t c : A.cigar) {
    const uint32_t op = c & 0xf;  // ksw ops: 0 = M, 1 = I, 2 = D
    cig.push_back(cigar_pack(c >> 4, op == 0 ? kM : op == 1 ? kI : kD));
  }
  if (A.qe < (int)q.size()) cig.push_back(cigar_pack((uint32_t)(q.size() - A.qe), kS));
  const std::string& Rs = ref.contigs[C.contig].seq;
  int nm = 0, run = 0;
  std::string md;
  int qi = A.qb;
  int64_t ri = A.rb;
  for (uint32_t c : A.cigar) {
    const uint32_t len = c >> 4, op = c & 0xf;
    if (op == 0) {
      for (uint32_t j = 0; j < len; ++j, ++qi, ++ri) {
        if (q[qi] != code_of(Rs[ri]) || q[qi] > 3) {
          ++nm;
          md += std::to_string(run);
          md += Rs[ri];
          run = 0;
        } else {
          ++run;
        }
      }
    } else if (op == 1) {
      nm += (int)len;
      qi += (int)len;
    } else {
      nm += (int)len;
      md += std::to_string(run) + "^" + Rs.substr(ri, len);
      run = 0;
      ri += len;
    }
  }
  md += std::to_string(run);
  rec.ref_id = C.contig;
  rec.pos = (int32_t)A.rb;
  rec.mapq = (uint8_t)R.mapq;
  rec.flag = C.rev ? kReverse : 0;
  rec.cigar = cig;
  rec.seq = R.seq[C.rev];
  rec.qual = quals(C.rev);
  rec.set_aux_int("NM", nm);
  rec.set_aux_string("MD", md);
  rec.set_aux_int("AS", A.truesc);
  return rec;
}

// Seeds, chains and the GPU extension round for a batch of reads.
void align_batch(const Reference& ref, const KmerIndex& idx, const std::vector<std::string>& seqs,
                 const AlignOptions& opt, std::vector<ReadAln>& reads, AlignStats& st) {
  const uint64_t t0 = now_us();
  reads.assign(seqs.size(), ReadAln{});
  parallel_for(seqs.size(), opt.threads, [&](size_t r) {
    ReadAln& R = reads[r];
    R.seq[0] = seqs[r];
    R.seq[1] = revcomp(seqs[r]);
    R.code[0] = encode(R.seq[0]);
    R.code[1] = encode(R.seq[1]);
    seed_read(ref, idx, opt, R);
  });
  const uint64_t t1 = now_us();
  st.seed_seconds += (t1 - t0) / 1e6;
  std::vector<ReadAln*> ptr;
  for (ReadAln& R : reads) ptr.push_back(&R);
  extend_cands(idx, st.params, opt, ptr, false, st);
  const uint64_t t2 = now_us();
  st.extend_seconds += (t2 - t1) / 1e6;
  parallel_for(reads.size(), opt.threads, [&](size_t r) { pick_primary(reads[r], opt); });
  st.pair_seconds += (now_us() - t2) / 1e6;
}

}  // namespace

KmerIndex::KmerIndex(const Reference& ref, int k, const std::string& index_path) : k_(k) {
  if (k < 8 || k > 63) throw invalidParam("minimum seed length must be in [8, 63]");
  for (const Contig& c : ref.contigs) {
    codes_.emplace_back(c.seq.size());
    for (size_t p = 0; p < c.seq.size(); ++p) codes_.back()[p] = code_of(c.seq[p]);
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
  align_batch(ref, idx, seqs, opt, reads, st);
  st.reads = (int64_t)seqs.size();
  const size_t base = out.size();
  out.resize(base + reads.size());
  const uint64_t tr = now_us();
  parallel_for(reads.size(), opt.threads,
               [&](size_t i) { out[base + i] = make_record(ref, reads[i], names[i], seqs[i], quals[i], opt); });
  st.record_seconds += (now_us() - tr) / 1e6;
  for (const ReadAln& R : reads) st.mapped += R.best >= 0;
  st.seconds = (now_us() - t0) / 1e6;
  return st;
}

AlignStats align_pairs(const Reference& ref, const KmerIndex& idx, const std::vector<std::string>& names,
                       const std::vector<std::string>& seqs1, const std::vector<std::string>& quals1,
                       const std::vector<std::string>& seqs2, const std::vector<std::string>& quals2,
                       const AlignOptions& opt, std::vector<BamRecord>& out) {
  AlignStats st;
  fcs_bsw_params_default(&st.params);
  const uint64_t t0 = now_us();
  const size_t n = names.size();
  if (seqs1.size() != n || seqs2.size() != n) throw invalidParam("align_pairs: mate lists differ in length");
  // both mates in one batch: one GPU extension round for all
  std::vector<std::string> both(seqs1);
  both.insert(both.end(), seqs2.begin(), seqs2.end());
  std::vector<ReadAln> all;
  align_batch(ref, idx, both, opt, all, st);
  std::vector<ReadAln> m1(std::make_move_iterator(all.begin()), std::make_move_iterator(all.begin() + n));
  std::vector<ReadAln> m2(std::make_move_iterator(all.begin() + n), std::make_move_iterator(all.end()));
  all.clear();
  const uint64_t tp = now_us();
  const PeStat ps = pestat(m1, m2);
  st.pe_pairs = ps.n;
  st.pe_low = ps.low;
  st.pe_high = ps.high;
  st.pe_avg = ps.avg;
  st.pe_std = ps.std;
  // mate rescue: a confidently placed mate whose partner has no alignment in the
  // allowed window gets the window searched for the partner
  if (ps.ok) {
    std::vector<ReadAln*> resc;
    for (size_t i = 0; i < n; ++i)
      for (int side = 0; side < 2; ++side) {
        ReadAln& a = side ? m2[i] : m1[i];
        ReadAln& b = side ? m1[i] : m2[i];
        if (a.best < 0 || a.mapq < 20) continue;
        const Cand& A = a.cands[a.best];
        bool have = false;
        for (const Cand& C : b.cands)
          if (C.ok && fr_pair(A, C) && frag_len(A, C) >= ps.low && frag_len(A, C) <= ps.high) have = true;
        if (have) continue;
        if (rescue_seed(idx, ps, A, b)) resc.push_back(&b);
      }
    std::sort(resc.begin(), resc.end());
    resc.erase(std::unique(resc.begin(), resc.end()), resc.end());
    st.rescued = (int64_t)resc.size();
    const uint64_t te = now_us();
    extend_cands(idx, st.params, opt, resc, true, st);
    st.extend_seconds += (now_us() - te) / 1e6;
    st.pair_seconds -= (now_us() - te) / 1e6;
  }
  // pairing (bwa mem_pair): the best FR combination within [low, high] by
  // score + insert-size log-likelihood, against the unpaired best - pen_unpaired
  const int pen_unpaired = 17;
  std::vector<char> proper(n, 0);
  for (size_t i = 0; i < n; ++i) {
    ReadAln &a = m1[i], &b = m2[i];
    pick_primary(a, opt);
    pick_primary(b, opt);
    if (!ps.ok) continue;
    int bi = -1, bj = -1, best = INT32_MIN, second = INT32_MIN;
    for (int x = 0; x < (int)a.cands.size(); ++x)
      for (int y = 0; y < (int)b.cands.size(); ++y) {
        const Cand &A = a.cands[x], &B = b.cands[y];
        if (!A.ok || !B.ok || !fr_pair(A, B)) continue;
        const int64_t f = frag_len(A, B);
        if (f < ps.low || f > ps.high) continue;
        const int s = A.aln.truesc + B.aln.truesc + pair_penalty(ps, f, 1);
        if (s > best) second = best, best = s, bi = x, bj = y;
        else if (s > second) second = s;
      }
    if (bi < 0) continue;
    const int unpaired = (a.best >= 0 ? a.cands[a.best].aln.truesc : 0) +
                         (b.best >= 0 ? b.cands[b.best].aln.truesc : 0) - pen_unpaired;
    if (best < unpaired) continue;
    proper[i] = 1;
    const int q_pe = second == INT32_MIN ? 60 : std::min(60, (int)(6.02 * (best - second) + .499));
    for (int side = 0; side < 2; ++side) {
      ReadAln& r = side ? b : a;
      const int pick = side ? bj : bi;
      const int q_se = pick == r.best ? r.mapq : 0;
      r.best = pick;
      r.mapq = std::max(q_se, std::min(q_pe, q_se + 40));
    }
  }
  const uint64_t tr = now_us();
  st.pair_seconds += (tr - tp) / 1e6;
  const size_t base = out.size();
  out.resize(base + 2 * n);
  parallel_for(n, opt.threads, [&](size_t i) {
    BamRecord r1 = make_record(ref, m1[i], names[i], seqs1[i], quals1[i], opt);
    BamRecord r2 = make_record(ref, m2[i], names[i], seqs2[i], quals2[i], opt);
    r1.flag |= kPaired | kRead1;
    r2.flag |= kPaired | kRead2;
    const bool u1 = r1.flag & kUnmapped, u2 = r2.flag & kUnmapped;
    if (!u1 && u2) r2.ref_id = r1.ref_id, r2.pos = r1.pos;  // SAM: an unmapped mate takes its partner's place
    if (u1 && !u2) r1.ref_id = r2.ref_id, r1.pos = r2.pos;
    auto link = [](BamRecord& x, const BamRecord& y) {
      x.next_ref_id = y.ref_id;
      x.next_pos = y.pos;
      if (y.flag & kUnmapped) x.flag |= kMateUnmapped;
      if (y.flag & kReverse) x.flag |= kMateReverse;
    };
    link(r1, r2);
    link(r2, r1);
    if (proper[i]) {
      r1.flag |= kProperPair;
      r2.flag |= kProperPair;
    }
    if (!u1 && !u2 && r1.ref_id == r2.ref_id) {  // TLEN: leftmost to rightmost mapped base, signed
      const int64_t b = std::min<int64_t>(r1.pos, r2.pos), e = std::max(r1.end(), r2.end());
      const int32_t t = (int32_t)(e - b);
      const bool first = r1.pos < r2.pos || (r1.pos == r2.pos && !(r1.flag & kReverse));
      r1.tlen = first ? t : -t;
      r2.tlen = first ? -t : t;
    }
    out[base + 2 * i] = std::move(r1);
    out[base + 2 * i + 1] = std::move(r2);
  });
  st.record_seconds += (now_us() - tr) / 1e6;
  for (size_t i = 0; i < n; ++i) st.mapped += (m1[i].best >= 0) + (m2[i].best >= 0);
  for (size_t i = 0; i < n; ++i) st.proper += 2 * proper[i];
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

AlignStats align_fastq(const AlignJob& job, const std::vector<int>& gpus, std::string& report) {
  if (gpus.empty()) throw failedCommand("[E::fcs-genome align] no GPU visible (gpu.devices); the GPU path has no CPU fallback");
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
    const int all = nt > 0 ? nt : (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
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
    for (const auto& o : order) w.write(recs[o.second]);
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
      for (const BamRecord* r : per[k]) w.write(*r);
      w.close();
      std::ofstream bed(get_contig_fname(job.output, k, "bed"));
      for (const Interval& iv : buckets[k]) bed << iv.chrom << '\t' << iv.lb - 1 << '\t' << iv.ub << '\n';
    }
  }
  const uint64_t t_end = now_us();
  std::ostringstream rep;
  rep << "[fcs-genome align] " << tot.reads << " reads, " << tot.mapped << " mapped, " << tot.ext_tasks
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

#include "aligner.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <iostream>
#include <map>
#include <thread>

#include "common.h"
#include "config.h"
#include "executor.h"
#include "fcship.h"
#include "seedext.h"

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

// Static split of [0, n) over up to `threads` std::threads.
template <typename F>
void parallel_for(size_t n, int threads, F&& fn) {
  const size_t nt = std::max<size_t>(1, std::min<size_t>((size_t)std::max(threads, 1), n / 256 + 1));
  if (nt == 1) {
    for (size_t i = 0; i < n; ++i) fn(i);
    return;
  }
  std::vector<std::thread> th;
  for (size_t t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      for (size_t i = n * t / nt; i < n * (t + 1) / nt; ++i) fn(i);
    });
  for (auto& x : th) x.join();
}

// One read's alignment in progress.
struct Aln {
  int read = -1;
  bool rev = false, mapped = false;
  int contig = -1;
  int mapq = 0;
  std::string seq;            // oriented query bases (revcomp for reverse)
  std::vector<uint8_t> q;     // codes of seq
  std::vector<uint8_t> qual;  // oriented quals
  int64_t seed_r = 0;         // contig offset of the seed start
  int seed_q = 0, seed_len = 0;
  int score = 0, truesc = 0;
  int qb = 0, qe = 0;
  int64_t rb = 0, re = 0;
  std::vector<uint32_t> cigar;
  int nm = 0;
  std::string md;
};

}  // namespace

KmerIndex::KmerIndex(const Reference& ref, int k) : k_(k) {
  if (k < 8 || k > 31) throw invalidParam("seed length must be in [8, 31]");
  uint64_t g = 0;
  std::vector<std::pair<uint64_t, uint64_t>> kv;
  for (const Contig& c : ref.contigs) {
    starts_.push_back(g);
    const int64_t L = (int64_t)c.seq.size();
    codes_.emplace_back(L);
    for (int64_t p = 0; p < L; ++p) codes_.back()[p] = code_of(c.seq[p]);
    uint64_t key = 0;
    int valid = 0;
    const uint64_t mask = (k == 32) ? ~0ull : ((1ull << (2 * k)) - 1);
    for (int64_t p = 0; p < L; ++p) {
      const uint8_t b = code_of(c.seq[p]);
      if (b > 3) {
        valid = 0;
        key = 0;
        continue;
      }
      key = ((key << 2) | b) & mask;
      if (++valid >= k) kv.emplace_back(key, g + (uint64_t)(p - k + 1));
    }
    g += (uint64_t)L;
  }
  starts_.push_back(g);
  std::sort(kv.begin(), kv.end());
  keys_.resize(kv.size());
  pos_.resize(kv.size());
  for (size_t i = 0; i < kv.size(); ++i) {
    keys_[i] = kv[i].first;
    pos_[i] = kv[i].second;
  }
}

std::pair<const uint64_t*, const uint64_t*> KmerIndex::lookup(uint64_t key) const {
  auto lo = std::lower_bound(keys_.begin(), keys_.end(), key);
  auto hi = std::upper_bound(lo, keys_.end(), key);
  return {pos_.data() + (lo - keys_.begin()), pos_.data() + (hi - keys_.begin())};
}

int KmerIndex::contig_of(uint64_t g, int64_t& off) const {
  const auto it = std::upper_bound(starts_.begin(), starts_.end(), g);
  const int c = (int)(it - starts_.begin()) - 1;
  off = (int64_t)(g - starts_[c]);
  return c;
}

AlignStats align_reads(const Reference& ref, const KmerIndex& idx, const std::vector<std::string>& names,
                       const std::vector<std::string>& seqs, const std::vector<std::string>& quals,
                       const AlignOptions& opt, std::vector<BamRecord>& out) {
  AlignStats st;
  const uint64_t t0 = now_us();
  fcs_bsw_params P;
  fcs_bsw_params_default(&P);
  const int k = idx.k();
  const uint64_t kmask = (1ull << (2 * k)) - 1;
  std::vector<Aln> alns(seqs.size());

  // ---- seeds and the best chain per read (host threads over reads)
  st.reads = (int64_t)seqs.size();
  auto seed_read = [&](size_t r) {
    Aln& A = alns[r];
    A.read = (int)r;
    struct Hit {
      int64_t d;
      int qp;
      uint64_t g;
    };
    std::vector<Hit> hits;
    int best_hits = 0, second_hits = 0, best_qp = 0;
    uint64_t best_g = 0;
    bool best_rev = false;
    for (int strand = 0; strand < 2; ++strand) {
      const std::string s = strand ? revcomp(seqs[r]) : seqs[r];
      const std::vector<uint8_t> c = encode(s);
      hits.clear();
      for (int qp = 0; qp + k <= (int)c.size(); qp += opt.seed_step) {
        uint64_t key = 0;
        bool ok = true;
        for (int i = 0; i < k && ok; ++i) {
          if (c[qp + i] > 3) ok = false;
          key = ((key << 2) | c[qp + i]) & kmask;
        }
        if (!ok) continue;
        const auto [b, e] = idx.lookup(key);
        if (e - b == 0 || e - b > opt.max_occ) continue;
        for (const uint64_t* p = b; p != e; ++p) hits.push_back({(int64_t)*p - qp, qp, *p});
      }
      // chains: diagonals within 8 of the previous one (indels shift them);
      // a chain's seed is its earliest hit on its most supported diagonal
      std::sort(hits.begin(), hits.end(), [](const Hit& x, const Hit& y) { return x.d != y.d ? x.d < y.d : x.qp < y.qp; });
      size_t i = 0;
      while (i < hits.size()) {
        size_t j = i;
        int n = 0, dn_best = 0;
        const Hit* seed = &hits[i];
        while (j < hits.size() && (j == i || hits[j].d - hits[j - 1].d <= 8)) {
          size_t e = j;
          while (e < hits.size() && hits[e].d == hits[j].d) ++e;  // one diagonal
          if ((int)(e - j) > dn_best) {
            dn_best = (int)(e - j);
            seed = &hits[j];
          }
          n += (int)(e - j);
          j = e;
        }
        if (n > best_hits) {
          second_hits = best_hits;
          best_hits = n;
          best_rev = strand;
          best_qp = seed->qp;
          best_g = seed->g;
        } else if (n > second_hits) {
          second_hits = n;
        }
        i = j;
      }
    }
    if (best_hits == 0) return;
    A.rev = best_rev;
    A.seq = best_rev ? revcomp(seqs[r]) : seqs[r];
    A.q = encode(A.seq);
    A.qual.resize(A.seq.size());
    for (size_t i = 0; i < A.seq.size(); ++i) {
      const size_t j = best_rev ? A.seq.size() - 1 - i : i;
      A.qual[i] = (uint8_t)(j < quals[r].size() ? std::max(0, quals[r][j] - 33) : 30);
    }
    int64_t off = 0;
    A.contig = idx.contig_of(best_g, off);
    const std::string& R = ref.contigs[A.contig].seq;
    // grow the k-mer hit to a maximal exact match
    int qs = best_qp, qe = best_qp + k;
    int64_t rs = off;
    while (qs > 0 && rs > 0 && A.q[qs - 1] < 4 && A.q[qs - 1] == code_of(R[rs - 1])) --qs, --rs;
    while (qe < (int)A.q.size() && rs + (qe - qs) < (int64_t)R.size() && A.q[qe] < 4 &&
           A.q[qe] == code_of(R[rs + (qe - qs)]))
      ++qe;
    A.seed_q = qs;
    A.seed_len = qe - qs;
    A.seed_r = rs;
    A.mapped = true;
    A.mapq = second_hits >= best_hits ? 0 : std::min(60, (int)std::lround(60.0 * (best_hits - second_hits) / best_hits));
  };
  parallel_for(seqs.size(), opt.threads, seed_read);

  // ---- bwa's extension protocol on the GPU (host/seedext.cpp): left and right
  // extensions with band retry, local vs to-end, CIGARs by banded global alignment
  {
    std::vector<SeedJob> jobs;
    std::vector<int> who;
    for (Aln& A : alns) {
      if (!A.mapped) continue;
      const std::vector<uint8_t>& R = idx.codes(A.contig);
      SeedJob J;
      J.q = A.q.data();
      J.qlen = (int)A.q.size();
      J.ref = R.data();
      J.rlen = (int64_t)R.size();
      J.seed_q = A.seed_q;
      J.seed_r = A.seed_r;
      J.seed_len = A.seed_len;
      jobs.push_back(J);
      who.push_back(A.read);
    }
    SeedExtOptions so;
    so.w = opt.w;
    so.pen_clip5 = so.pen_clip3 = P.end_bonus;
    so.gpu = opt.gpu;
    std::vector<SeedAln> res;
    SeedExtStats xs;
    extend_seeds(jobs, P, so, res, xs);
    st.ext_tasks += xs.ext_tasks;
    st.global_tasks += xs.global_tasks;
    st.gpu_seconds += xs.gpu_seconds;
    for (size_t i = 0; i < who.size(); ++i) {
      Aln& A = alns[who[i]];
      SeedAln& x = res[i];
      A.qb = x.qb;
      A.qe = x.qe;
      A.rb = x.rb;
      A.re = x.re;
      A.score = x.score;
      A.truesc = x.truesc;
      A.cigar.swap(x.cigar);
      if (A.qe <= A.qb || A.re <= A.rb) A.mapped = false;
    }
  }

  // ---- records (host threads; one slot per read keeps the input order)
  const size_t base = out.size();
  out.resize(base + alns.size());
  std::vector<char> mapped_flag(alns.size(), 0);
  parallel_for(alns.size(), opt.threads, [&](size_t ai) {
    Aln& A = alns[ai];
    BamRecord& rec = out[base + ai];
    rec.name = names[A.read];
    rec.set_aux_string("RG", opt.rg);
    if (!A.mapped || A.cigar.empty()) {
      rec.flag = kUnmapped;
      rec.seq = seqs[A.read];
      rec.qual.resize(rec.seq.size());
      for (size_t i = 0; i < rec.seq.size(); ++i)
        rec.qual[i] = (uint8_t)(i < quals[A.read].size() ? std::max(0, quals[A.read][i] - 33) : 30);
      return;
    }
    mapped_flag[ai] = 1;
    std::vector<uint32_t> cig;
    if (A.qb > 0) cig.push_back(cigar_pack((uint32_t)A.qb, kS));
    for (uint32_t c : A.cigar) {
      // ksw ops: 0 = M, 1 = I, 2 = D
      const uint32_t op = c & 0xf;
      cig.push_back(cigar_pack(c >> 4, op == 0 ? kM : op == 1 ? kI : kD));
    }
    if (A.qe < (int)A.q.size()) cig.push_back(cigar_pack((uint32_t)(A.q.size() - A.qe), kS));
    // NM / MD over the aligned part
    const std::string& R = ref.contigs[A.contig].seq;
    int nm = 0, run = 0;
    std::string md;
    int qi = A.qb;
    int64_t ri = A.rb;
    for (uint32_t c : A.cigar) {
      const uint32_t len = c >> 4, op = c & 0xf;
      if (op == 0) {
        for (uint32_t j = 0; j < len; ++j, ++qi, ++ri) {
          if (A.q[qi] != code_of(R[ri]) || A.q[qi] > 3) {
            ++nm;
            md += std::to_string(run);
            md += R[ri];
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
        md += std::to_string(run) + "^" + R.substr(ri, len);
        run = 0;
        ri += len;
      }
    }
    md += std::to_string(run);
    rec.ref_id = A.contig;
    rec.pos = (int32_t)A.rb;
    rec.mapq = (uint8_t)A.mapq;
    rec.flag = A.rev ? kReverse : 0;
    rec.cigar = cig;
    rec.seq = A.seq;
    rec.qual = A.qual;
    rec.set_aux_int("NM", nm);
    rec.set_aux_string("MD", md);
    rec.set_aux_int("AS", A.truesc);
  });
  for (char m : mapped_flag) st.mapped += m;
  st.seconds = (now_us() - t0) / 1e6;
  return st;
}

// ------------------------------------------------------------------ align command
namespace {

bool read_fastq(std::ifstream& in, std::string& name, std::string& seq, std::string& qual) {
  std::string plus;
  if (!std::getline(in, name)) return false;
  if (name.empty() || name[0] != '@') throw formatError("FASTQ record does not start with '@'");
  name = name.substr(1);
  const size_t ws = name.find_first_of(" \t");
  if (ws != std::string::npos) name.resize(ws);
  if (name.size() > 2 && name[name.size() - 2] == '/') name.resize(name.size() - 2);  // /1, /2
  if (!std::getline(in, seq) || !std::getline(in, plus) || !std::getline(in, qual))
    throw formatError("truncated FASTQ record " + name);
  if (qual.size() != seq.size()) throw formatError("FASTQ quality length differs for " + name);
  return true;
}

}  // namespace

int align_main(int argc, char** argv) {
  std::string ref_path, fq1, fq2, output, rg = "sample", sp = "sample", pl = "illumina", lb = "sample";
  bool force = false;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto val = [&]() -> std::string {
      if (i + 1 >= argc) throw invalidParam(a + " needs a value");
      return argv[++i];
    };
    if (a == "-h" || a == "--help") {
      std::cerr << "'fcs-genome align' options:\n  -r, --ref arg\n  -1, --fastq1 arg\n  -2, --fastq2 arg\n"
                   "  -o, --output arg\n  -R, --rg arg\n  -S, --sp arg\n  -P, --pl arg\n  -L, --lb arg\n"
                   "  -l, --align-only\n  -f, --force\n";
      throw helpRequest();
    } else if (a == "-r" || a == "--ref") ref_path = val();
    else if (a == "-1" || a == "--fastq1") fq1 = val();
    else if (a == "-2" || a == "--fastq2") fq2 = val();
    else if (a == "-o" || a == "--output") output = val();
    else if (a == "-R" || a == "--rg") rg = val();
    else if (a == "-S" || a == "--sp") sp = val();
    else if (a == "-P" || a == "--pl") pl = val();
    else if (a == "-L" || a == "--lb") lb = val();
    else if (a == "-f" || a == "--force") force = true;
    else if (a == "-l" || a == "--align-only" || a == "--disable-merge") continue;
    else throw invalidParam(a);
  }
  if (ref_path.empty()) throw invalidParam("--ref is required");
  if (fq1.empty()) throw invalidParam("--fastq1 is required");
  if (output.empty()) throw invalidParam("--output is required");
  if (!is_regular_file(ref_path)) throw fileNotFound(ref_path);
  if (!is_regular_file(fq1)) throw fileNotFound(fq1);
  if (!fq2.empty() && !is_regular_file(fq2)) throw fileNotFound(fq2);
  if (!force && path_exists(output)) throw invalidParam("output " + output + " exists (use -f)");
  const std::vector<int> gpus = conf().gpu_devices();
  if (gpus.empty()) throw failedCommand("[E::fcs-genome] no GPU visible (gpu.devices); the GPU path has no CPU fallback");

  const Reference ref = load_fasta(ref_path);
  AlignOptions opt;
  opt.gpu = gpus[0];
  opt.rg = rg;
  opt.chunk_size = conf().get_int("bwa.chunk_size");
  {
    const int nt = conf().get_int("bwa.nt");
    opt.threads = nt > 0 ? nt : (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
  }
  const KmerIndex idx(ref, opt.k);
  std::vector<BamRecord> recs;
  AlignStats tot;
  for (int mate = 0; mate < (fq2.empty() ? 1 : 2); ++mate) {
    std::ifstream in(mate ? fq2 : fq1);
    std::vector<std::string> names, seqs, quals;
    std::string n, s, q;
    auto flush = [&] {
      if (names.empty()) return;
      const size_t first = recs.size();
      const AlignStats st = align_reads(ref, idx, names, seqs, quals, opt, recs);
      if (!fq2.empty())
        for (size_t i = first; i < recs.size(); ++i) recs[i].flag |= kPaired | (mate ? kRead2 : kRead1);
      tot.reads += st.reads;
      tot.mapped += st.mapped;
      tot.seconds += st.seconds;
      tot.gpu_seconds += st.gpu_seconds;
      tot.ext_tasks += st.ext_tasks;
      tot.global_tasks += st.global_tasks;
      names.clear();
      seqs.clear();
      quals.clear();
    };
    while (read_fastq(in, n, s, q)) {
      names.push_back(n);
      seqs.push_back(s);
      quals.push_back(q);
      if ((int)names.size() >= opt.chunk_size) flush();
    }
    flush();
  }
  std::stable_sort(recs.begin(), recs.end(), [](const BamRecord& x, const BamRecord& y) {
    const uint32_t a = (uint32_t)x.ref_id, b = (uint32_t)y.ref_id;  // unmapped (-1) last
    return a != b ? a < b : x.pos < y.pos;
  });
  BamHeader h;
  h.text = "@HD\tVN:1.6\tSO:coordinate\n";
  for (const Contig& c : ref.contigs) {
    h.names.push_back(c.name);
    h.lengths.push_back((int64_t)c.seq.size());
    h.text += "@SQ\tSN:" + c.name + "\tLN:" + std::to_string(c.seq.size()) + "\n";
  }
  h.text += "@RG\tID:" + rg + "\tSM:" + sp + "\tPL:" + pl + "\tLB:" + lb + "\n";
  h.text += "@PG\tID:fcs-genome\tPN:fcs-genome align\n";
  {
    BamWriter w(output, h);
    for (const BamRecord& r : recs) w.write(r);
    w.close();
  }
  bam_index_build(output);
  std::cerr << "[fcs-genome align] " << tot.reads << " reads, " << tot.mapped << " mapped, " << tot.ext_tasks
            << " extension tasks, " << tot.global_tasks << " global alignments, " << tot.seconds << " s (GPU calls "
            << tot.gpu_seconds << " s)" << std::endl;
  return 0;
}

}  // namespace fcsg

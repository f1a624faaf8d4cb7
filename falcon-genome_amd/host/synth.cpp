#include "synth.h"

#include "intervals.h"

#include <algorithm>
#include <array>
#include <atomic>
#include <cstdio>
#include <thread>
#include <tuple>
#include <cmath>
#include <fstream>
#include <map>

#include "bam.h"
#include "common.h"
#include "vcf.h"

namespace fcsg {

namespace {

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed, uint64_t stream) : s(seed * 0x9E3779B97F4A7C15ull ^ (stream + 0x632BE59BD9B4E019ull)) {}
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  double uniform() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
  uint64_t below(uint64_t n) { return n ? next() % n : 0; }
};

const char kBases[] = "ACGT";

char other_base(Rng& r, char b) {
  for (;;) {
    const char c = kBases[r.below(4)];
    if (c != b) return c;
  }
}

// One haplotype of a contig: sequence and, per base, its reference position (-1 = inserted).
struct Hap {
  std::string seq;
  std::vector<int64_t> ref_pos;
};

Hap build_hap(const std::string& ref, const std::vector<const SynthVariant*>& vars) {
  Hap h;
  h.seq.reserve(ref.size() + 1024);
  h.ref_pos.reserve(ref.size() + 1024);
  int64_t p = 0;
  for (const SynthVariant* v : vars) {  // sorted, non-overlapping, left-anchored
    for (; p < v->pos; ++p) {
      h.seq += ref[p];
      h.ref_pos.push_back(p);
    }
    // anchor / substituted base at v->pos
    h.seq += v->alt[0];
    h.ref_pos.push_back(v->pos);
    for (size_t k = 1; k < v->alt.size(); ++k) {  // inserted bases
      h.seq += v->alt[k];
      h.ref_pos.push_back(-1);
    }
    p = v->pos + (int64_t)v->ref.size();  // deleted bases are skipped
  }
  for (; p < (int64_t)ref.size(); ++p) {
    h.seq += ref[p];
    h.ref_pos.push_back(p);
  }
  return h;
}

struct SimRead {
  int64_t pos;
  BamRecord rec;
};

// Reads are drawn in fixed chunks of kChunk draws, each chunk from its own
// RNG stream and named by its draw index, so the data set does not depend on
// how many threads generate it.
constexpr int64_t kChunk = 1 << 15;

Rng chunk_rng(uint64_t seed, uint64_t stream, int64_t chunk) {
  return Rng(seed, stream ^ ((uint64_t)(chunk + 1) << 32));
}

int synth_threads() { return (int)host_cpus(); }

// parallel_for whose bodies may be interrupted: the workers stop at the next
// item and the caller raises interruptedError (an exception must not leave a
// worker thread).
template <typename F>
void parallel_items(size_t n, F&& fn) {
  std::atomic<bool> stop{false};
  parallel_tasks(n, synth_threads(), [&](size_t i) {
    if (stop.load(std::memory_order_relaxed)) return;
    if (interrupted()) {
      stop = true;
      return;
    }
    fn(i);
  });
  if (stop) throw interruptedError();
}

// FASTQ text of a read as sequenced (a reverse-strand read is reverse-complemented).
void append_fastq(std::string& o, const std::string& name, const std::string& seq, const std::vector<uint8_t>& qual,
                  bool rev) {
  o += '@';
  o += name;
  o += '\n';
  const size_t n = seq.size();
  if (!rev) {
    o += seq;
  } else {
    for (size_t i = n; i-- > 0;) {
      const char c = seq[i];
      o += c == 'A' ? 'T' : c == 'C' ? 'G' : c == 'G' ? 'C' : c == 'T' ? 'A' : 'N';
    }
  }
  o += "\n+\n";
  for (size_t i = 0; i < n; ++i) o += (char)(33 + qual[rev ? n - 1 - i : i]);
  o += '\n';
}

// Formats items [0, n) into text blocks on worker threads and writes the
// blocks in order (a bounded window of blocks is held at a time).
template <typename F>
void write_text_parallel(const std::string& path, size_t n, F&& fmt) {
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) throw std::runtime_error("cannot write " + path);
  constexpr size_t kBlock = 1 << 14;
  const size_t nblk = (n + kBlock - 1) / kBlock, win = (size_t)synth_threads() * 4;
  std::vector<std::string> text(win);
  for (size_t b0 = 0; b0 < nblk; b0 += win) {
    const size_t nb = std::min(win, nblk - b0);
    parallel_items(nb, [&](size_t k) {
      std::string& s = text[k];
      s.clear();
      for (size_t i = (b0 + k) * kBlock; i < std::min(n, (b0 + k + 1) * kBlock); ++i) fmt(i, s);
    });
    for (size_t k = 0; k < nb; ++k) std::fwrite(text[k].data(), 1, text[k].size(), f);
  }
  if (std::fclose(f) != 0) throw std::runtime_error("cannot write " + path);
}

// Coordinate order of the reads (reference, position, then draw order: a stable sort).
std::vector<uint32_t> coordinate_order(const std::vector<SimRead>& reads) {
  struct Key {
    uint64_t k;
    uint32_t i;
  };
  std::vector<Key> keys(reads.size());
  for (size_t i = 0; i < reads.size(); ++i)
    keys[i] = {((uint64_t)(uint32_t)reads[i].rec.ref_id << 40) | (uint64_t)reads[i].pos, (uint32_t)i};
  std::sort(keys.begin(), keys.end(), [](const Key& a, const Key& b) { return a.k != b.k ? a.k < b.k : a.i < b.i; });
  std::vector<uint32_t> o(reads.size());
  for (size_t i = 0; i < o.size(); ++i) o[i] = keys[i].i;
  return o;
}

// Read covering hap[s, s + L): CIGAR from the haplotype's reference map.
bool make_read(const Hap& h, int64_t s, int L, Rng& r, double err, SimRead& out) {
  std::string seq = h.seq.substr(s, L);
  std::vector<uint8_t> q(L);
  for (int i = 0; i < L; ++i) {
    q[i] = (uint8_t)(25 + r.below(16));
    if (r.uniform() < err) {
      seq[i] = other_base(r, seq[i]);
      q[i] = (uint8_t)(8 + r.below(13));
    }
  }
  std::vector<uint32_t> cig;
  auto push = [&](CigarOp op, uint32_t n) {
    if (!n) return;
    if (!cig.empty() && cigar_op(cig.back()) == op) cig.back() += n << 4;
    else cig.push_back(cigar_pack(n, op));
  };
  int64_t first = -1, prev = -1;
  int lead = 0;
  for (int i = 0; i < L; ++i) {
    const int64_t rp = h.ref_pos[s + i];
    if (rp < 0) {
      if (first < 0) ++lead;
      else push(kI, 1);
      continue;
    }
    if (first < 0) {
      first = rp;
      push(kS, (uint32_t)lead);
    } else if (rp > prev + 1) {
      push(kD, (uint32_t)(rp - prev - 1));
    }
    push(kM, 1);
    prev = rp;
  }
  if (first < 0) return false;  // read entirely inside an insertion
  // trailing insertion → soft clip
  if (cigar_op(cig.back()) == kI) cig.back() = cigar_pack(cigar_len(cig.back()), kS);
  out.pos = first;
  out.rec.pos = (int32_t)first;
  out.rec.cigar = cig;
  out.rec.seq = seq;
  out.rec.qual = q;
  out.rec.mapq = 60;
  return true;
}

void write_reads(const std::vector<SimRead>& reads, const std::vector<uint32_t>& order, const BamHeader& hdr,
                 const std::string& bam, const std::string& fastq) {
  {
    BamWriter w(bam, hdr, 1);  // synthetic inputs: fastest deflate level
    w.index_on_close();
    // records encode on worker threads, a window at a time, and are written in order
    constexpr size_t kBlock = 1 << 12;
    const size_t win = (size_t)synth_threads() * 4 * kBlock;
    std::vector<std::string> body(std::min(win, order.size()));
    for (size_t i0 = 0; i0 < order.size(); i0 += win) {
      const size_t n = std::min(win, order.size() - i0);
      parallel_items((n + kBlock - 1) / kBlock, [&](size_t b) {
        for (size_t k = b * kBlock; k < std::min(n, (b + 1) * kBlock); ++k)
          encode_bam_record(reads[order[i0 + k]].rec, body[k]);
      });
      for (size_t k = 0; k < n; ++k) w.write_encoded(reads[order[i0 + k]].rec, body[k]);
    }
    w.close();
  }
  if (!fastq.empty())
    write_text_parallel(fastq, order.size(), [&](size_t k, std::string& s) {
      const BamRecord& r = reads[order[k]].rec;
      append_fastq(s, r.name, r.seq, r.qual, r.flag & kReverse);
    });
}

}  // namespace

SynthOutputs synth_dataset(const SynthSpec& spec, const std::string& dir) {
  create_dir(dir);
  SynthOutputs out;
  Reference ref;
  for (size_t c = 0; c < spec.contigs.size(); ++c) {
    Rng r(spec.seed, 0x1000 + c);
    Contig ct{spec.contigs[c].first, std::string((size_t)spec.contigs[c].second, 'A')};
    for (char& b : ct.seq) b = kBases[r.below(4)];
    ref.contigs.push_back(std::move(ct));
  }
  out.ref_fasta = dir + "/ref.fasta";
  write_fasta(out.ref_fasta, ref);
  write_fai(out.ref_fasta, ref);
  write_dict(dict_path_for(out.ref_fasta), ref);

  // ---- truth set: left-normalised, unambiguous (no shiftable indels), >= 30 bp apart
  std::vector<std::vector<SynthVariant>> per(ref.contigs.size());
  for (size_t c = 0; c < ref.contigs.size(); ++c) {
    Rng r(spec.seed, 0x2000 + c);
    const std::string& s = ref.contigs[c].seq;
    const double rate = spec.snp_rate + spec.indel_rate + spec.somatic_rate;
    int64_t p = 200;
    while (rate > 0) {
      p += 30 + (int64_t)(-std::log(1.0 - r.uniform()) / rate);
      if (p >= (int64_t)s.size() - 200) break;
      SynthVariant v;
      v.chrom = ref.contigs[c].name;
      v.pos = p;
      const double u = r.uniform() * rate;
      const bool somatic = u >= spec.snp_rate + spec.indel_rate;
      const bool indel = !somatic ? u >= spec.snp_rate : r.uniform() < 0.2;
      if (!indel) {
        v.ref = std::string(1, s[p]);
        v.alt = std::string(1, other_base(r, s[p]));
      } else {
        const int k = 1 + (int)r.below(5);
        if (r.uniform() < 0.5) {  // deletion of s[p+1 .. p+k]
          const std::string D = s.substr(p + 1, k);
          if (s[p] == D.back() || s[p + k + 1] == D[0]) continue;  // shiftable: skip
          v.ref = s.substr(p, k + 1);
          v.alt = std::string(1, s[p]);
        } else {  // insertion after s[p]
          std::string I;
          for (int i = 0; i < k; ++i) I += kBases[r.below(4)];
          if (I.back() == s[p] || I[0] == s[p + 1]) continue;
          v.ref = std::string(1, s[p]);
          v.alt = s[p] + I;
        }
      }
      if (somatic) {
        v.somatic = true;
        v.gt = 1;
        v.af = spec.somatic_af;
      } else {
        v.gt = r.uniform() < spec.hom_frac ? 2 : 1;
      }
      v.af = somatic ? spec.somatic_af : (v.gt == 2 ? 1.0 : 0.5);
      p += (int64_t)v.ref.size();
      per[c].push_back(v);
    }
  }

  for (const auto& [chrom, centre] : spec.spikes) {
    const int c = ref.index(chrom);
    if (c < 0 || centre < 200 || centre + 200 >= (int64_t)ref.contigs[c].seq.size())
      throw invalidParam("--spike " + chrom + ":" + std::to_string(centre) + " is not inside a contig");
    auto& vs = per[c];
    vs.erase(std::remove_if(vs.begin(), vs.end(),
                            [&](const SynthVariant& v) { return v.pos + 100 >= centre && v.pos <= centre + 100; }),
             vs.end());
    Rng r(spec.seed, 0x3000 + (uint64_t)centre);
    for (int64_t d : {-30, 0, 30}) {
      SynthVariant v;
      v.chrom = chrom;
      v.pos = centre + d;
      v.ref = std::string(1, ref.contigs[c].seq[v.pos]);
      v.alt = std::string(1, other_base(r, ref.contigs[c].seq[v.pos]));
      v.gt = 1;
      v.af = 0.5;
      vs.push_back(v);
    }
    std::sort(vs.begin(), vs.end(), [](const SynthVariant& a, const SynthVariant& b) { return a.pos < b.pos; });
  }

  // ---- reads
  BamHeader hdr;
  hdr.text = "@HD\tVN:1.6\tSO:coordinate\n";
  for (const Contig& c : ref.contigs) {
    hdr.names.push_back(c.name);
    hdr.lengths.push_back((int64_t)c.seq.size());
    hdr.text += "@SQ\tSN:" + c.name + "\tLN:" + std::to_string(c.seq.size()) + "\n";
  }
  // haplotypes of contig c: [copy][somatic?] (germline variants only unless `som`)
  auto contig_haps = [&](size_t c, bool tumor, Hap (&haps)[2][2]) {
    for (int copy = 0; copy < 2; ++copy)
      for (int som = 0; som < (tumor ? 2 : 1); ++som) {
        std::vector<const SynthVariant*> vs;
        for (const SynthVariant& v : per[c]) {
          if (v.somatic && !som) continue;
          // het germline and somatic variants sit on copy 0 or 1 by a per-site coin
          const bool on = v.gt == 2 || ((v.pos * 2654435761u) >> 7 & 1) == (uint64_t)copy;
          if (on) vs.push_back(&v);
        }
        haps[copy][som] = build_hap(ref.contigs[c].seq, vs);
      }
  };
  const int L = spec.read_len;
  // chunks of the n draws of one contig, and the draws of the contigs before c
  // (the first global draw index of contig c: read names)
  struct Chunk {
    int64_t chunk, k0, k1;
  };
  auto chunks_of = [](int64_t n) {
    std::vector<Chunk> v;
    for (int64_t k0 = 0; k0 < n; k0 += kChunk) v.push_back({k0 / kChunk, k0, std::min(n, k0 + kChunk)});
    return v;
  };
  auto draws = [&](size_t c, double cov) { return (int64_t)(cov * (double)ref.contigs[c].seq.size() / L); };
  auto draws_before = [&](size_t c, double cov) {
    int64_t b = 0;
    for (size_t k = 0; k < c; ++k) b += draws(k, cov);
    return b;
  };
  auto sample_reads = [&](const std::string& sample, bool tumor, double coverage, uint64_t stream) {
    std::string h = hdr.text + "@RG\tID:" + sample + "\tSM:" + sample + "\n";
    std::vector<SimRead> reads;
    for (size_t c = 0; c < ref.contigs.size(); ++c) {
      Hap haps[2][2];
      contig_haps(c, tumor, haps);
      const auto chunks = chunks_of(draws(c, coverage));
      const int64_t base = draws_before(c, coverage);
      std::vector<std::vector<SimRead>> part(chunks.size());
      parallel_items(chunks.size(), [&](size_t t) {
        const Chunk& ch = chunks[t];
        Rng hr = chunk_rng(spec.seed, stream + 0x10 * c, ch.chunk);
        std::vector<SimRead>& o = part[t];
        o.reserve((size_t)(ch.k1 - ch.k0));
        for (int64_t k = ch.k0; k < ch.k1; ++k) {
          const int copy = (int)hr.below(2);
          const int som = tumor && hr.uniform() < 2 * spec.somatic_af ? 1 : 0;  // somatic on one copy → AF = somatic_af
          const Hap& hp = haps[copy][som];
          if ((int64_t)hp.seq.size() <= L) continue;
          const int64_t s = (int64_t)hr.below(hp.seq.size() - L);
          SimRead sr;
          if (!make_read(hp, s, L, hr, spec.err_rate, sr)) continue;
          if (spec.noisy_frac > 0 && hr.uniform() < spec.noisy_frac)
            for (size_t i = 0; i < sr.rec.seq.size(); ++i)
              if (hr.uniform() < 0.2) {
                sr.rec.seq[i] = other_base(hr, sr.rec.seq[i]);
                sr.rec.qual[i] = (uint8_t)(35 + hr.below(6));
              }
          sr.rec.ref_id = (int32_t)c;
          sr.rec.name = sample + ":" + std::to_string(base + k);
          sr.rec.flag = hr.uniform() < 0.5 ? kReverse : 0;
          sr.rec.set_aux_string("RG", sample);
          o.push_back(std::move(sr));
        }
      });
      size_t tot = reads.size();
      for (const auto& v : part) tot += v.size();
      reads.reserve(tot);
      for (auto& v : part) {
        for (SimRead& r : v) reads.push_back(std::move(r));
        std::vector<SimRead>().swap(v);
      }
    }
    std::vector<uint32_t> order = coordinate_order(reads);
    if (spec.max_reads >= 0 && (int64_t)order.size() > spec.max_reads) order.resize(spec.max_reads);
    BamHeader hh = hdr;
    hh.text = h;
    return std::make_tuple(std::move(reads), std::move(order), hh);
  };
  {
    auto [reads, order, hh] = sample_reads("sample", false, spec.coverage, 0x3000);
    out.bam = dir + "/sample.bam";
    out.fastq = spec.single_fastq ? dir + "/sample.fastq" : "";
    out.n_reads = (int64_t)order.size();
    write_reads(reads, order, hh, out.bam, out.fastq);
    if (spec.parts > 0) {
      std::vector<std::pair<std::string, int64_t>> dict;
      for (const Contig& c : ref.contigs) dict.emplace_back(c.name, (int64_t)c.seq.size());
      const auto buckets = partition_contigs(dict, spec.parts, false);
      out.parts_dir = dir + "/parts";
      create_dir(out.parts_dir);
      for (int k = 0; k < spec.parts; ++k) {
        std::vector<uint32_t> part;
        for (uint32_t i : order) {
          const SimRead& sr = reads[i];
          const std::string& chrom = ref.contigs[sr.rec.ref_id].name;
          for (const Interval& iv : buckets[k])
            if (iv.chrom == chrom && sr.pos + 1 >= iv.lb && sr.pos + 1 <= iv.ub) {
              part.push_back(i);
              break;
            }
        }
        write_reads(reads, part, hh, get_contig_fname(out.parts_dir, k, "bam"), "");
        std::ofstream bed(get_contig_fname(out.parts_dir, k, "bed"));
        for (const Interval& iv : buckets[k]) bed << iv.chrom << '\t' << iv.lb - 1 << '\t' << iv.ub << '\n';
      }
    }
  }
  if (spec.paired_insert > 0) {  // FR pairs of germline fragments
    out.fastq1 = dir + "/sample_1.fastq";
    out.fastq2 = dir + "/sample_2.fastq";
    out.pairs_truth = dir + "/pairs_truth.tsv";
    FILE* fo[3] = {std::fopen(out.fastq1.c_str(), "wb"), std::fopen(out.fastq2.c_str(), "wb"),
                   std::fopen(out.pairs_truth.c_str(), "wb")};
    for (FILE* f : fo)
      if (!f) throw std::runtime_error("cannot write the paired FASTQ files in " + dir);
    for (size_t c = 0; c < ref.contigs.size(); ++c) {
      Hap haps[2][2];
      contig_haps(c, false, haps);
      const auto chunks = chunks_of(draws(c, spec.coverage / 2));
      const int64_t base = draws_before(c, spec.coverage / 2);
      const size_t win = (size_t)synth_threads() * 2;
      std::vector<std::array<std::string, 3>> text(win);
      for (size_t t0 = 0; t0 < chunks.size(); t0 += win) {
        const size_t nt = std::min(win, chunks.size() - t0);
        parallel_items(nt, [&](size_t t) {
          const Chunk& ch = chunks[t0 + t];
          Rng hr = chunk_rng(spec.seed, 0x5000 + 0x10 * c, ch.chunk);
          auto& [s1, s2, st] = text[t];
          s1.clear();
          s2.clear();
          st.clear();
          for (int64_t k = ch.k0; k < ch.k1; ++k) {
            const Hap& hp = haps[hr.below(2)][0];
            const double u1 = std::max(hr.uniform(), 1e-12), u2 = hr.uniform();
            const double z = std::sqrt(-2. * std::log(u1)) * std::cos(6.283185307179586 * u2);
            const int64_t ins = std::max<int64_t>(L, (int64_t)std::llround(spec.paired_insert + spec.paired_sd * z));
            if ((int64_t)hp.seq.size() <= ins) continue;
            const int64_t s0 = (int64_t)hr.below(hp.seq.size() - ins);
            SimRead fw, rv;
            if (!make_read(hp, s0, L, hr, spec.err_rate, fw) || !make_read(hp, s0 + ins - L, L, hr, spec.err_rate, rv))
              continue;
            const bool flip = hr.uniform() < 0.5;  // read 1 from the reverse strand
            const std::string name = "pair:" + std::to_string(base + k);
            const SimRead& m1 = flip ? rv : fw;
            const SimRead& m2 = flip ? fw : rv;
            append_fastq(s1, name + "/1", m1.rec.seq, m1.rec.qual, flip);
            append_fastq(s2, name + "/2", m2.rec.seq, m2.rec.qual, !flip);
            st += name + "\t1\t" + std::to_string(c) + '\t' + std::to_string(m1.pos) + '\t' + (flip ? "1" : "0") + '\n';
            st += name + "\t2\t" + std::to_string(c) + '\t' + std::to_string(m2.pos) + '\t' + (flip ? "0" : "1") + '\n';
          }
        });
        for (size_t t = 0; t < nt; ++t)
          for (int j = 0; j < 3; ++j) std::fwrite(text[t][j].data(), 1, text[t][j].size(), fo[j]);
      }
    }
    for (FILE* f : fo)
      if (std::fclose(f) != 0) throw std::runtime_error("cannot write the paired FASTQ files in " + dir);
  }
  if (spec.somatic_rate > 0) {
    auto [reads, order, hh] = sample_reads("tumor", true, spec.tumor_coverage, 0x4000);
    out.tumor_bam = dir + "/tumor.bam";
    out.n_tumor_reads = (int64_t)order.size();
    write_reads(reads, order, hh, out.tumor_bam, "");
  }

  // ---- truth VCF (1-based, VCF alleles)
  VcfHeader vh;
  for (const Contig& c : ref.contigs) vh.contigs.emplace_back(c.name, (int64_t)c.seq.size());
  vh.samples = {"sample"};
  vh.meta = {"##INFO=<ID=SOMATIC,Number=0,Type=Flag,Description=\"Somatic variant (tumor only)\">",
             "##FORMAT=<ID=GT,Number=1,Type=String,Description=\"Genotype\">"};
  vh.source = "fcs-genome synth";
  out.truth_vcf = dir + "/truth.vcf";
  VcfWriter vw(out.truth_vcf, vh);
  for (const auto& vs : per)
    for (const SynthVariant& v : vs) {
      VcfRecord rec;
      rec.chrom = v.chrom;
      rec.pos = v.pos + 1;
      rec.ref = v.ref;
      rec.alts = {v.alt};
      rec.info = v.somatic ? "SOMATIC" : ".";
      rec.format = "GT";
      const bool copy0 = ((v.pos * 2654435761u) >> 7 & 1) == 0;
      rec.samples = {v.somatic ? "0|0" : v.gt == 2 ? "1|1" : copy0 ? "1|0" : "0|1"};
      vw.write(rec);
      out.variants.push_back(v);
    }
  vw.close();
  return out;
}

}  // namespace fcsg

#include "synth.h"

#include "intervals.h"

#include <algorithm>
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

std::string revcomp(const std::string& s) {
  std::string o(s.rbegin(), s.rend());
  for (char& c : o) c = c == 'A' ? 'T' : c == 'C' ? 'G' : c == 'G' ? 'C' : c == 'T' ? 'A' : 'N';
  return o;
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
  std::string fq_seq, fq_qual;
};

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

void write_reads(std::vector<SimRead>& reads, const BamHeader& hdr, const std::string& bam, const std::string& fastq) {
  std::stable_sort(reads.begin(), reads.end(), [](const SimRead& a, const SimRead& b) {
    return a.rec.ref_id != b.rec.ref_id ? a.rec.ref_id < b.rec.ref_id : a.pos < b.pos;
  });
  {
    BamWriter w(bam, hdr);
    w.index_on_close();
    for (const SimRead& sr : reads) w.write(sr.rec);
    w.close();
  }
  if (!fastq.empty()) {
    std::ofstream fq(fastq);
    for (const SimRead& sr : reads) fq << '@' << sr.rec.name << '\n' << sr.fq_seq << "\n+\n" << sr.fq_qual << '\n';
  }
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
  auto sample_reads = [&](const std::string& sample, bool tumor, double coverage, uint64_t stream) {
    std::string h = hdr.text + "@RG\tID:" + sample + "\tSM:" + sample + "\n";
    std::vector<SimRead> reads;
    int64_t idx = 0;
    for (size_t c = 0; c < ref.contigs.size(); ++c) {
      Rng hr(spec.seed, stream + 0x10 * c);
      // haplotypes: [copy][somatic?]
      Hap haps[2][2];
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
      const int L = spec.read_len;
      const int64_t n = (int64_t)(coverage * (double)ref.contigs[c].seq.size() / L);
      for (int64_t k = 0; k < n; ++k) {
        if ((k & 0xFFFF) == 0 && interrupted()) throw interruptedError();
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
        sr.rec.name = sample + ":" + std::to_string(idx++);
        const bool rev = hr.uniform() < 0.5;
        sr.rec.flag = rev ? kReverse : 0;
        sr.rec.set_aux_string("RG", sample);
        std::string qs(sr.rec.qual.size(), '!');
        for (size_t i = 0; i < qs.size(); ++i) qs[i] = (char)(33 + sr.rec.qual[i]);
        sr.fq_seq = rev ? revcomp(sr.rec.seq) : sr.rec.seq;
        sr.fq_qual = rev ? std::string(qs.rbegin(), qs.rend()) : qs;
        reads.push_back(std::move(sr));
      }
    }
    if (spec.max_reads >= 0 && (int64_t)reads.size() > spec.max_reads) {
      std::stable_sort(reads.begin(), reads.end(), [](const SimRead& a, const SimRead& b) {
        return a.rec.ref_id != b.rec.ref_id ? a.rec.ref_id < b.rec.ref_id : a.pos < b.pos;
      });
      reads.resize(spec.max_reads);
    }
    BamHeader hh = hdr;
    hh.text = h;
    return std::make_pair(std::move(reads), hh);
  };
  {
    auto rs = sample_reads("sample", false, spec.coverage, 0x3000);
    out.bam = dir + "/sample.bam";
    out.fastq = dir + "/sample.fastq";
    out.n_reads = (int64_t)rs.first.size();
    write_reads(rs.first, rs.second, out.bam, out.fastq);
    if (spec.parts > 0) {
      std::vector<std::pair<std::string, int64_t>> dict;
      for (const Contig& c : ref.contigs) dict.emplace_back(c.name, (int64_t)c.seq.size());
      const auto buckets = partition_contigs(dict, spec.parts, false);
      out.parts_dir = dir + "/parts";
      create_dir(out.parts_dir);
      for (int k = 0; k < spec.parts; ++k) {
        std::vector<SimRead> part;
        for (const SimRead& sr : rs.first) {
          const std::string& chrom = ref.contigs[sr.rec.ref_id].name;
          for (const Interval& iv : buckets[k])
            if (iv.chrom == chrom && sr.pos + 1 >= iv.lb && sr.pos + 1 <= iv.ub) {
              part.push_back(sr);
              break;
            }
        }
        write_reads(part, rs.second, get_contig_fname(out.parts_dir, k, "bam"), "");
        std::ofstream bed(get_contig_fname(out.parts_dir, k, "bed"));
        for (const Interval& iv : buckets[k]) bed << iv.chrom << '\t' << iv.lb - 1 << '\t' << iv.ub << '\n';
      }
    }
  }
  if (spec.paired_insert > 0) {  // FR pairs of germline fragments
    out.fastq1 = dir + "/sample_1.fastq";
    out.fastq2 = dir + "/sample_2.fastq";
    out.pairs_truth = dir + "/pairs_truth.tsv";
    std::ofstream f1(out.fastq1), f2(out.fastq2), tt(out.pairs_truth);
    int64_t idx = 0;
    const int L = spec.read_len;
    for (size_t c = 0; c < ref.contigs.size(); ++c) {
      Rng hr(spec.seed, 0x5000 + 0x10 * c);
      Hap haps[2];
      for (int copy = 0; copy < 2; ++copy) {
        std::vector<const SynthVariant*> vs;
        for (const SynthVariant& v : per[c])
          if (!v.somatic && (v.gt == 2 || ((v.pos * 2654435761u) >> 7 & 1) == (uint64_t)copy)) vs.push_back(&v);
        haps[copy] = build_hap(ref.contigs[c].seq, vs);
      }
      const int64_t n = (int64_t)(spec.coverage / 2 * (double)ref.contigs[c].seq.size() / L);
      for (int64_t k = 0; k < n; ++k) {
        if ((k & 0xFFFF) == 0 && interrupted()) throw interruptedError();
        const Hap& hp = haps[hr.below(2)];
        const double u1 = std::max(hr.uniform(), 1e-12), u2 = hr.uniform();
        const double z = std::sqrt(-2. * std::log(u1)) * std::cos(6.283185307179586 * u2);
        const int64_t ins = std::max<int64_t>(L, (int64_t)std::llround(spec.paired_insert + spec.paired_sd * z));
        if ((int64_t)hp.seq.size() <= ins) continue;
        const int64_t s0 = (int64_t)hr.below(hp.seq.size() - ins);
        SimRead fw, rv;
        if (!make_read(hp, s0, L, hr, spec.err_rate, fw) || !make_read(hp, s0 + ins - L, L, hr, spec.err_rate, rv))
          continue;
        const bool flip = hr.uniform() < 0.5;  // read 1 from the reverse strand
        const std::string name = "pair:" + std::to_string(idx++);
        auto fq = [](const SimRead& r, bool rev) {
          std::string qs(r.rec.qual.size(), '!');
          for (size_t i = 0; i < qs.size(); ++i) qs[i] = (char)(33 + r.rec.qual[i]);
          return rev ? std::make_pair(revcomp(r.rec.seq), std::string(qs.rbegin(), qs.rend()))
                     : std::make_pair(r.rec.seq, qs);
        };
        const SimRead& m1 = flip ? rv : fw;
        const SimRead& m2 = flip ? fw : rv;
        const auto a = fq(m1, flip), b = fq(m2, !flip);
        f1 << '@' << name << "/1\n" << a.first << "\n+\n" << a.second << '\n';
        f2 << '@' << name << "/2\n" << b.first << "\n+\n" << b.second << '\n';
        tt << name << "\t1\t" << c << '\t' << m1.pos << '\t' << (flip ? 1 : 0) << '\n';
        tt << name << "\t2\t" << c << '\t' << m2.pos << '\t' << (flip ? 0 : 1) << '\n';
      }
    }
  }
  if (spec.somatic_rate > 0) {
    auto rs = sample_reads("tumor", true, spec.tumor_coverage, 0x4000);
    out.tumor_bam = dir + "/tumor.bam";
    out.n_tumor_reads = (int64_t)rs.first.size();
    write_reads(rs.first, rs.second, out.tumor_bam, "");
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

// extern "C" hooks of libfcsgenome.so for the Python tests (tests/test_host_*.py):
// the host pieces with exact expected outputs — GATK read preparation,
// interval partitioning, BGZF, BAM record coding, BAI/TBI building, the
// executor's stage/error semantics.  Not part of the hot-path ABI (include/fcship.h).
#include <cstring>
#include <functional>
#include <memory>
#include <string>

#include "bam.h"
#include "bam_input.h"
#include "caller.h"
#include "bgzf.h"
#include "common.h"
#include "config.h"
#include "executor.h"
#include "fasta.h"
#include "fmindex.h"
#include "gatk_prep.h"
#include "seedext.h"
#include "aligner.h"
#include "intervals.h"
#include "sample_sheet.h"
#include "vcf.h"

using namespace fcsg;

namespace {
thread_local std::string g_err;
int guard(const std::function<void()>& fn) {
  try {
    fn();
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}
int copy_out(const std::string& s, char* buf, int cap) {
  if ((int)s.size() + 1 > cap) return -(int)s.size() - 1;
  std::memcpy(buf, s.c_str(), s.size() + 1);
  return (int)s.size();
}
}  // namespace

extern "C" {

const char* fcsg_last_error() { return g_err.c_str(); }

int fcsg_prepare_read(const char* bases, const uint8_t* quals, int len, const char* bi, const char* bd, int mapq,
                      int threshold, int pcr_model, uint8_t* bq, uint8_t* iq, uint8_t* dq, uint8_t* gcp) {
  return guard([&] {
    PreparedRead pr;
    gatk_prepare_read(std::string(bases, len), std::vector<uint8_t>(quals, quals + len), bi ? std::string(bi) : "",
                      bd ? std::string(bd) : "", mapq, pr, threshold, (PcrIndelModel)pcr_model);
    std::memcpy(bq, pr.base_q.data(), len);
    std::memcpy(iq, pr.ins_q.data(), len);
    std::memcpy(dq, pr.del_q.data(), len);
    std::memcpy(gcp, pr.gcp.data(), len);
  });
}

// "sample\tfastq1\tfastq2\trg\tplatform\tlibrary\n" lines of a sample sheet
// (file or FASTQ folder), samples in name order, read groups in sheet order.
int fcsg_sample_sheet(const char* path, char* buf, int cap) {
  int rc = 0;
  const int g = guard([&] {
    std::string s;
    for (const auto& [sample, list] : read_sample_sheet(path))
      for (const SampleDetails& d : list)
        s += sample + "\t" + d.fastqR1 + "\t" + d.fastqR2 + "\t" + d.ReadGroup + "\t" + d.Platform + "\t" +
             d.LibraryID + "\n";
    rc = copy_out(s, buf, cap);
  });
  return g ? g : rc;
}

// merge_sorted_bams (align's per-sample merge of read-group BAMs).
int fcsg_merge_bams(const char* const* inputs, int n, const char* output) {
  return guard([&] { merge_sorted_bams(std::vector<std::string>(inputs, inputs + n), output); });
}

// "shard\tchrom\tlb\tub\n" lines of the init_contig_intv partition of a .dict.
int fcsg_partition_dict(const char* dict_path, int ncontigs, int skip_pseudo, char* buf, int cap) {
  int rc = 0;
  const int g = guard([&] {
    const auto parts = partition_contigs(read_dict(dict_path), ncontigs, skip_pseudo != 0);
    std::string s;
    for (size_t k = 0; k < parts.size(); ++k)
      for (const Interval& iv : parts[k])
        s += std::to_string(k) + "\t" + iv.chrom + "\t" + std::to_string(iv.lb) + "\t" + std::to_string(iv.ub) + "\n";
    rc = copy_out(s, buf, cap);
  });
  return g ? g : rc;
}

// BamInput::merge_region: "bam1,bam2,...\n<region file>\n" of shard `contig`.
int fcsg_bam_input_shard(const char* path, int contig, int ncontigs, const char* temp_dir, char* buf, int cap) {
  int rc = 0;
  const int g = guard([&] {
    const BamShard sh = BamInput(path).merge_region(contig, ncontigs, temp_dir);
    std::string s;
    for (size_t i = 0; i < sh.bams.size(); ++i) s += (i ? "," : "") + sh.bams[i];
    s += "\n" + sh.region + "\n";
    rc = copy_out(s, buf, cap);
  });
  return g ? g : rc;
}

// read_regions of each path, intersected when several: "chrom\tlb\tub\n" lines.
int fcsg_intersect_regions(const char* const* paths, int n, char* buf, int cap) {
  int rc = 0;
  const int g = guard([&] {
    std::vector<std::vector<Interval>> sets;
    for (int i = 0; i < n; ++i) sets.push_back(read_regions(paths[i]));
    const auto out = sets.size() == 1 ? sets[0] : intersect_interval_sets(sets);
    std::string s;
    for (const Interval& iv : out) s += iv.chrom + "\t" + std::to_string(iv.lb) + "\t" + std::to_string(iv.ub) + "\n";
    rc = copy_out(s, buf, cap);
  });
  return g ? g : rc;
}

int fcsg_gvcf_band(int gq) { return gvcf_band(gq); }

// SMEM seeding on an FMD-index of the given contigs (codes 0..4): seeds of q
// (bwa mem_collect_intv; max_mem_intv 0 skips its third round), out = {qb, qe, occurrences} per SMEM and
// loc = {contig, offset, reverse} of every occurrence (at most loc_cap rows,
// SMEM by SMEM, each SMEM's occurrences in suffix-array order).  Returns the
// SMEM count, or < 0 on error.
// sa_intv: the index's SA sampling; index_path non-empty: the index is saved
// there and the query runs on the file mapped back (FmdIndex::load).
int fcsg_fmd_smems(const uint8_t* ref, const int64_t* clen, int ncontig, const uint8_t* q, int qlen, int min_len,
                   int split_len, int split_width, int max_mem_intv, int32_t* out, int cap, int64_t* loc,
                   int loc_cap, int sa_intv, const char* index_path) {
  int n = -1;
  const int rc = guard([&] {
    std::vector<std::vector<uint8_t>> cs;
    int64_t o = 0;
    for (int i = 0; i < ncontig; ++i) {
      cs.emplace_back(ref + o, ref + o + clen[i]);
      o += clen[i];
    }
    std::unique_ptr<FmdIndex> built = std::make_unique<FmdIndex>(cs, sa_intv), mapped;
    if (index_path && *index_path) {
      built->save(index_path);
      built.reset();
      mapped = FmdIndex::load(index_path, cs);
      if (!mapped) throw internalError("saved FMD-index did not load");
    }
    const FmdIndex& fmd = mapped ? *mapped : *built;
    std::vector<BiInterval> v;
    fmd.collect(q, qlen, min_len, split_len, split_width, max_mem_intv, v);
    if ((int)v.size() > cap) throw invalidParam("fcsg_fmd_smems: capacity");
    int64_t nl = 0;
    for (size_t i = 0; i < v.size(); ++i) {
      out[3 * i] = v[i].qb, out[3 * i + 1] = v[i].qe, out[3 * i + 2] = (int32_t)v[i].s;
      for (int64_t j = 0; j < v[i].s && nl < loc_cap; ++j, ++nl) {
        int c;
        int64_t off;
        bool rev;
        fmd.locate(v[i], j, c, off, rev);
        loc[3 * nl] = c, loc[3 * nl + 1] = off, loc[3 * nl + 2] = rev;
      }
    }
    n = (int)v.size();
  });
  return rc < 0 ? rc : n;
}

// bwa's seed-extension protocol (host/seedext.h) over n seeds on one reference
// sequence (codes 0..4), each with its chain's window (win_lo / win_hi, or
// null / -1 for the seed's own); per job out_i = {qb, qe, score, truesc, w, gscore, gw},
// out_r = {rb, re}, the CIGAR (ksw ops) in cig[cig_off[i] ...] (ncig[i] ops).
int fcsg_extend_seeds(int n, const uint8_t* qbuf, const int64_t* qoff, const int32_t* qlen, const uint8_t* ref,
                      int64_t rlen, const int32_t* seed_q, const int64_t* seed_r, const int32_t* seed_len, int w,
                      int pen_clip5, int pen_clip3, int gpu, int32_t* out_i, int64_t* out_r, uint32_t* cig,
                      const int64_t* cig_off, const int32_t* cig_cap, int32_t* ncig, const int64_t* win_lo,
                      const int64_t* win_hi) {
  return guard([&] {
    std::vector<SeedJob> jobs(n);
    for (int i = 0; i < n; ++i) {
      if (win_lo) jobs[i].win_lo = win_lo[i];
      if (win_hi) jobs[i].win_hi = win_hi[i];
      jobs[i].q = qbuf + qoff[i];
      jobs[i].qlen = qlen[i];
      jobs[i].ref = ref;
      jobs[i].rlen = rlen;
      jobs[i].seed_q = seed_q[i];
      jobs[i].seed_r = seed_r[i];
      jobs[i].seed_len = seed_len[i];
    }
    fcs_bsw_params P;
    fcs_bsw_params_default(&P);
    SeedExtOptions so;
    so.w = w;
    so.pen_clip5 = pen_clip5;
    so.pen_clip3 = pen_clip3;
    so.gpu = gpu;
    std::vector<SeedAln> res;
    SeedExtStats st;
    extend_seeds(jobs, P, so, res, st);
    for (int i = 0; i < n; ++i) {
      const SeedAln& x = res[i];
      int32_t* o = out_i + 7 * (int64_t)i;
      o[0] = x.qb, o[1] = x.qe, o[2] = x.score, o[3] = x.truesc, o[4] = x.w, o[5] = x.gscore, o[6] = x.gw;
      out_r[2 * i] = x.rb;
      out_r[2 * i + 1] = x.re;
      if ((int64_t)x.cigar.size() > cig_cap[i]) throw invalidParam("fcsg_extend_seeds: CIGAR capacity");
      std::copy(x.cigar.begin(), x.cigar.end(), cig + cig_off[i]);
      ncig[i] = (int32_t)x.cigar.size();
    }
  });
}
int fcsg_tandem_repeat_units(const char* bases, int offset) { return tandem_repeat_units(bases, offset); }
void fcsg_tandem_repeat_runs(const char* bases, int n, uint8_t* out) { tandem_repeat_runs(bases, n, out); }
int fcsg_pcr_indel_cap(int repeat_len, int model) { return pcr_indel_cap(repeat_len, (PcrIndelModel)model); }

int fcsg_bgzf_compress_file(const char* in, const char* out) {
  return guard([&] { bgzip_file(in, out); });
}

// Decompress a BGZF file with the library's reader (tests compare with Python's gzip).
int fcsg_bgzf_decompress_file(const char* in, const char* out) {
  return guard([&] {
    BgzfReader r(in);
    std::string all;
    char buf[1 << 16];
    for (size_t n; (n = r.read(buf, sizeof buf)) > 0;) all.append(buf, n);
    write_file(out, all);
  });
}

// BAM → SAM-like text (one line per record) with the library's reader.
int fcsg_bam_to_text(const char* bam, const char* out) {
  return guard([&] {
    BamReader r(bam);
    std::string s;
    for (size_t i = 0; i < r.header().names.size(); ++i)
      s += "@SQ\t" + r.header().names[i] + "\t" + std::to_string(r.header().lengths[i]) + "\n";
    BamRecord rec;
    while (r.next(rec)) {
      std::string q;
      for (uint8_t x : rec.qual) q += (char)(x + 33);
      std::string md;
      int64_t nm = -1;
      rec.get_aux_string("MD", md);
      rec.get_aux_int("NM", nm);
      s += rec.name + "\t" + std::to_string(rec.flag) + "\t" + std::to_string(rec.ref_id) + "\t" +
           std::to_string(rec.pos) + "\t" + std::to_string(rec.mapq) + "\t" + cigar_string(rec.cigar) + "\t" + rec.seq +
           "\t" + (q.empty() ? "*" : q) + "\t" + md + "\t" + std::to_string(nm) + "\n";
    }
    write_file(out, s);
  });
}

// SAM-like text (name flag ref_id pos mapq cigar seq qual; leading '@' lines
// are header lines) → BAM with the library's writer.
int fcsg_text_to_bam(const char* text, const char* bam, const char* names_csv, const char* lengths_csv) {
  return guard([&] {
    BamHeader h;
    std::string nm = names_csv, ln = lengths_csv;
    for (size_t p = 0; p < nm.size();) {
      const size_t e = std::min(nm.find(',', p), nm.size());
      h.names.push_back(nm.substr(p, e - p));
      p = e + 1;
    }
    for (size_t p = 0; p < ln.size();) {
      const size_t e = std::min(ln.find(',', p), ln.size());
      h.lengths.push_back(std::stoll(ln.substr(p, e - p)));
      p = e + 1;
    }
    for (size_t i = 0; i < h.names.size(); ++i)
      h.text += "@SQ\tSN:" + h.names[i] + "\tLN:" + std::to_string(h.lengths[i]) + "\n";
    std::string body = read_file(text);
    while (!body.empty() && body[0] == '@') {  // leading header lines (@RG, @PG) join the header
      const size_t e = std::min(body.find('\n'), body.size());
      h.text += body.substr(0, e) + "\n";
      body.erase(0, e + 1);
    }
    BamWriter w(bam, h);
    size_t p = 0;
    while (p < body.size()) {
      const size_t e = std::min(body.find('\n', p), body.size());
      const std::string line = body.substr(p, e - p);
      p = e + 1;
      if (line.empty()) continue;
      std::vector<std::string> f;
      for (size_t a = 0; a <= line.size();) {
        const size_t b = std::min(line.find('\t', a), line.size());
        f.push_back(line.substr(a, b - a));
        a = b + 1;
      }
      if (f.size() < 8) throw formatError("text record needs 8 fields");
      BamRecord r;
      r.name = f[0];
      r.flag = (uint16_t)std::stoi(f[1]);
      r.ref_id = std::stoi(f[2]);
      r.pos = std::stoi(f[3]);
      r.mapq = (uint8_t)std::stoi(f[4]);
      r.cigar = parse_cigar(f[5]);
      r.seq = f[6];
      if (f[7] != "*")
        for (char c : f[7]) r.qual.push_back((uint8_t)(c - 33));
      w.write(r);
    }
    w.close();
  });
}

int fcsg_bam_index(const char* bam) {
  return guard([&] { bam_index_build(bam); });
}

int fcsg_bam_seek_offset(const char* bai, int tid, long long beg, unsigned long long* off) {
  return guard([&] { *off = BamIndex(bai).seek_offset(tid, beg); });
}

int fcsg_vcf_concat(const char* const* inputs, int n, const char* output) {
  return guard([&] { vcf_concat(std::vector<std::string>(inputs, inputs + n), output); });
}

int fcsg_vcf_concat_bgzip_tabix(const char* const* inputs, int n, const char* plain, const char* gz) {
  return guard([&] { vcf_concat_bgzip_tabix(std::vector<std::string>(inputs, inputs + n), plain, gz); });
}

int fcsg_bgzip_tabix(const char* in, const char* out) {
  return guard([&] { bgzip_tabix_file(in, out); });
}
int fcsg_tabix(const char* vcf_gz) {
  return guard([&] { tabix_index_vcf(vcf_gz); });
}

unsigned fcsg_reg2bin(long long beg, long long end) { return reg2bin(beg, end); }

// Runs an executor with n_tasks shell-command workers (cmd per task, %d = task
// index) over n_threads threads and GPU slots gpus_csv; writes the per-task
// FCS_GPU_DEVICE seen by each command into its own output.  Returns the
// exception class on failure: 0 ok, 4 failedCommand, 1 other; findError text in buf.
int fcsg_run_stage(const char* cmd_fmt, int n_tasks, int n_threads, const char* gpus_csv, const char* log_dir,
                   char* buf, int cap) {
  try {
    conf().init("");
    conf().set("log_dir", log_dir);
    std::vector<int> gpus;
    std::string g = gpus_csv;
    for (size_t p = 0; p < g.size();) {
      const size_t e = std::min(g.find(',', p), g.size());
      if (e > p) gpus.push_back(std::stoi(g.substr(p, e - p)));
      p = e + 1;
    }
    class Cmd : public Worker {
     public:
      explicit Cmd(std::string c) : Worker(1, 1, {}, "test stage") { cmd_ = std::move(c); }
    };
    Executor ex("test", n_threads, gpus);
    for (int i = 0; i < n_tasks; ++i) {
      char c[4096];
      std::snprintf(c, sizeof c, cmd_fmt, i);
      ex.addTask(std::make_shared<Cmd>(c), "");
    }
    ex.run();
    copy_out("", buf, cap);
    return 0;
  } catch (const failedCommand&) {
    copy_out(g_err, buf, cap);
    return 4;
  } catch (const std::exception& e) {
    g_err = e.what();
    copy_out(g_err, buf, cap);
    return 1;
  }
}

int fcsg_find_error(const char* const* logs, int n, char* buf, int cap) {
  return copy_out(LogUtils::findError(std::vector<std::string>(logs, logs + n)), buf, cap);
}

}  // extern "C"

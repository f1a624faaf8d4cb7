// fcs-genome command line: the reference's CLI surface
// for the GPU-backed commands — `htc`, `mutect2`, `align` — with its option
// names (src/worker-htc.cpp:25-33, src/worker-mutect2.cpp:26-40,
// src/worker-align.cpp:29-42), config keys (`conf`) and exit codes
// (src/main.cpp:165-240: help 0, bad option 1/2, missing file 3, failed
// stage 4, other error -1), plus `synth` for the synthetic C1/C4/C5 inputs.
#include <algorithm>
#include <malloc.h>
#include <sys/resource.h>
#include <unistd.h>

#include <cerrno>

#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <thread>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "common.h"
#include "config.h"
#include "executor.h"
#include "fcship.h"
#include "aligner.h"
#include "intervals.h"
#include "sample_sheet.h"
#include "synth.h"
#include "workers.h"

namespace fcsg {

namespace {

// Minimal boost::program_options stand-in: long/short options with values or flags.
class Args {
 public:
  struct Opt {
    std::string lng, shrt, help;
    bool flag, required;
  };
  void add(const std::string& lng, const std::string& shrt, bool flag, bool required, const std::string& help) {
    opts_.push_back({lng, shrt, help, flag, required});
  }
  void parse(int argc, char** argv) {
    for (int i = 1; i < argc; ++i) {
      std::string a = argv[i];
      if (a == "-h" || a == "--help") throw helpRequest();
      const Opt* o = nullptr;
      std::string val;
      bool has_val = false;
      for (const Opt& x : opts_) {
        if (a == "--" + x.lng || (!x.shrt.empty() && a == "-" + x.shrt)) o = &x;
        else if (a.rfind("--" + x.lng + "=", 0) == 0) {
          o = &x;
          val = a.substr(x.lng.size() + 3);
          has_val = true;
        }
        if (o) break;
      }
      if (!o) throw invalidParam(a);
      if (o->flag) {
        vals_[o->lng].push_back("1");
        continue;
      }
      if (!has_val) {
        if (i + 1 >= argc) throw invalidParam(a + " needs a value");
        val = argv[++i];
      }
      vals_[o->lng].push_back(val);
    }
    for (const Opt& x : opts_)
      if (x.required && !vals_.count(x.lng)) throw invalidParam("--" + x.lng + " is required");
  }
  bool has(const std::string& k) const { return vals_.count(k) > 0; }
  std::string get(const std::string& k, const std::string& def = "") const {
    auto it = vals_.find(k);
    if (it == vals_.end()) return def;
    if (it->second.back().empty()) throw pathEmpty(k);
    return it->second.back();
  }
  std::vector<std::string> all(const std::string& k) const {
    auto it = vals_.find(k);
    return it == vals_.end() ? std::vector<std::string>{} : it->second;
  }
  std::string help() const {
    std::string s;
    for (const Opt& x : opts_)
      s += "  " + (x.shrt.empty() ? std::string("    ") : "-" + x.shrt + ", ") + "--" + x.lng +
           (x.flag ? "" : " arg") + "\t" + x.help + "\n";
    return s;
  }

 private:
  std::vector<Opt> opts_;
  std::map<std::string, std::vector<std::string>> vals_;
};

void common_opts(Args& a) {
  a.add("force", "f", true, false, "overwrite output files if they exist");
  a.add("extra-options", "O", false, false, "extra options for the command");
}

std::vector<int> slots() {
  std::vector<int> g = conf().gpu_devices();
  if (g.empty()) throw failedCommand("[E::fcs-genome] no GPU visible (gpu.devices); the GPU path has no CPU fallback");
  return g;
}

// Shards of the run: -L list (one file for all shards) or the reference's 32 interval parts.
std::vector<std::vector<std::string>> shard_intervals(const std::string& ref, const std::string& intv_list) {
  const int n = conf().get_int("gatk.ncontigs");
  std::vector<std::vector<std::string>> out(n);
  if (!intv_list.empty()) {
    // split the user's list into n shard files, contig order preserved
    const auto iv = read_interval_list(intv_list);
    std::vector<std::pair<std::string, int64_t>> pseudo;  // (name, length) of each listed interval
    for (const Interval& i : iv) pseudo.emplace_back(i.chrom, i.ub - i.lb + 1);
    const auto parts = partition_contigs(pseudo, n, false);
    const std::string dir = conf().temp_dir() + "/intv_user";
    create_dir(dir);
    for (int k = 0; k < n; ++k) {
      std::vector<Interval> shifted;
      for (const Interval& p : parts[k]) {
        // map back: pseudo-contig i starts at iv[i].lb
        for (const Interval& src : iv)
          if (src.chrom == p.chrom && p.lb - 1 + src.lb <= src.ub) {
            shifted.push_back({src.chrom, src.lb + p.lb - 1, src.lb + p.ub - 1});
            break;
          }
      }
      const std::string path = get_contig_fname(dir, k, "list", "part-");
      write_interval_list(path, shifted);
      out[k].push_back(path);
    }
    return out;
  }
  const auto paths = init_contig_intv(ref, n, conf().temp_dir(), conf().get_bool("gatk.skip_pseudo_chr"));
  for (int k = 0; k < n; ++k) out[k].push_back(paths[k]);
  return out;
}

// Shards of a directory input (BamInput): the parts' region files give the
// intervals, so only the user's -L (if any) goes to every shard
// (src/worker-htc.cpp:88-97: init_contig_intv only for a regular-file input).
std::vector<std::vector<std::string>> dir_shards(const std::string& intv_list) {
  std::vector<std::vector<std::string>> out(conf().get_int("gatk.ncontigs"));
  if (!intv_list.empty())
    for (auto& v : out) v.push_back(intv_list);
  return out;
}

// FCS_TIMELINE=1: seconds since the process started at named points
// (where a command's wall time goes outside its stages)
void timeline(const char* what) {
  static const bool on = [] {
    const char* e = std::getenv("FCS_TIMELINE");
    return e && *e && *e != '0';
  }();
  if (!on) return;
  double up = 0, start = 0;
  if (std::FILE* f = std::fopen("/proc/uptime", "r")) {
    if (std::fscanf(f, "%lf", &up) != 1) up = 0;
    std::fclose(f);
  }
  if (std::FILE* f = std::fopen("/proc/self/stat", "r")) {
    char buf[1024];
    const size_t n = std::fread(buf, 1, sizeof buf - 1, f);
    std::fclose(f);
    buf[n] = 0;
    const char* p = std::strrchr(buf, ')');  // fields after the command name; starttime is field 22
    unsigned long long ticks = 0;
    for (int field = 3; p && *p && field <= 22; ++field) {
      p = std::strchr(p + 1, ' ');
      if (p && field == 22) ticks = std::strtoull(p + 1, nullptr, 10);
    }
    start = (double)ticks / (double)sysconf(_SC_CLK_TCK);
  }
  struct rusage ru {};
  getrusage(RUSAGE_SELF, &ru);
  char line[256];
  std::snprintf(line, sizeof line, "[fcs-genome timeline] %s %.2f s (user %.2f s, sys %.2f s, minor faults %ld, csw %ld/%ld)",
                what, up - start, ru.ru_utime.tv_sec + ru.ru_utime.tv_usec / 1e6,
                ru.ru_stime.tv_sec + ru.ru_stime.tv_usec / 1e6, ru.ru_minflt, ru.ru_nvcsw, ru.ru_nivcsw);
  std::cerr << line << std::endl;
}

int htc_main(int argc, char** argv) {
  Args a;
  common_opts(a);
  a.add("ref", "r", false, true, "reference genome path");
  a.add("input", "i", false, true, "input BAM file or directory of part-XXXXXX.bam + .bed/.list");
  a.add("output", "o", false, true, "output GVCF/VCF file (<output>.gz + .tbi are written too)");
  a.add("produce-vcf", "v", true, false, "produce VCF instead of GVCF (reference-confidence blocks)");
  a.add("intervalList", "L", false, false, "interval list file");
  a.add("sample-id", "", false, false, "sample id for log files");
  a.add("skip-concat", "s", true, false, "(deprecated) produce a set of VCF files instead of one");
  a.add("gatk4", "g", true, false, "accepted for compatibility");
  a.add("dump-regions", "", false, false, "debug: write every region's PairHMM inputs/outputs to <path>.<shard>");
  try {
    a.parse(argc, argv);
  } catch (helpRequest&) {
    std::cerr << "'fcs-genome htc' options:\n" << a.help();
    throw;
  }
  const std::string ref = a.get("ref"), input = a.get("input"), output = a.get("output");
  const bool force = a.has("force");
  const std::string sample_id = a.get("sample-id");
  std::vector<std::string> extra = a.all("extra-options");
  if (a.has("dump-regions")) extra.push_back("--dump-regions " + a.get("dump-regions"));
  const std::vector<int> gpus = slots();
  const std::string out_dir = conf().temp_dir() + "/htc";
  create_dir(out_dir);
  const bool flag_vcf = a.has("produce-vcf");
  timeline("options parsed");
  const auto shards = is_directory(input) ? dir_shards(a.get("intervalList")) : shard_intervals(ref, a.get("intervalList"));
  timeline("shards");
  // the GPU runtime and tables come up in the background while the first
  // shards decode and pile up their reads (the reference's BackgroundExecutor
  // NAM daemon runs beside its Executor the same way)
  BackgroundExecutor warm("gpu-warmup", std::make_shared<DeviceWarmupWorker>(gpus));
  Executor ex("Haplotype Caller", conf().get_int("gatk.htc.nprocs", "gatk.nprocs"), gpus);
  std::vector<std::string> parts;
  for (size_t k = 0; k < shards.size(); ++k) {
    const std::string part = get_contig_fname(out_dir, (int)k, flag_vcf ? "vcf" : "g.vcf");
    parts.push_back(part);
    ex.addTask(std::make_shared<HTCWorker>(ref, shards[k], input, part, extra, (int)k, flag_vcf, true), sample_id);
  }
  const std::string plain = output;
  if (!a.has("skip-concat")) {
    if (!force && path_exists(plain + ".gz")) throw invalidParam("output " + plain + ".gz exists (use -f)");
    // concat -> bgzip -> tabix as one pass over the parts
    ex.addTask(std::make_shared<VCFConcatWorker>(parts, plain, plain + ".gz", /*consume=*/true), sample_id, true);
  } else {
    ex.addTask(std::make_shared<VCFConcatWorker>(parts, plain), sample_id, true);
  }
  if (conf().get_bool("gpu.release_early")) ex.addTask(std::make_shared<GpuReleaseWorker>(gpus, &warm), sample_id);
  timeline("stages queued");
  ex.run();
  timeline("stages done");
  warm.wait();
  timeline("warm-up joined");
  if (warm.status() != 0) throw failedCommand(std::string("[E::fcs-genome] GPU warm-up failed: ") + fcs_last_error());
  return 0;
}

int mutect2_main(int argc, char** argv) {
  Args a;
  common_opts(a);
  a.add("ref", "r", false, true, "reference genome path");
  a.add("normal", "n", false, true, "input normal BAM file or directory");
  a.add("tumor", "t", false, true, "input tumor BAM file or directory");
  a.add("output", "o", false, true, "output VCF file");
  a.add("intervalList", "L", false, false, "interval list file");
  a.add("normal_name", "a", false, false, "normal sample name");
  a.add("tumor_name", "b", false, false, "tumor sample name");
  a.add("sample-id", "", false, false, "sample id for log file");
  for (const char* k : {"dbsnp", "cosmic", "germline", "panels_of_normals", "contamination_table", "filtered_vcf"})
    a.add(k, "", false, false, "accepted for compatibility (not used by the GPU caller)");
  a.add("dump-regions", "", false, false, "debug: write every region's PairHMM inputs/outputs to <path>.<shard>");
  try {
    a.parse(argc, argv);
  } catch (helpRequest&) {
    std::cerr << "'fcs-genome mutect2' options:\n" << a.help();
    throw;
  }
  const std::string ref = a.get("ref"), output = a.get("output");
  const std::vector<int> gpus = slots();
  const std::string out_dir = conf().temp_dir() + "/mutect2";
  create_dir(out_dir);
  // reference intervals only when both inputs are plain BAM files (src/worker-mutect2.cpp:146-150)
  const auto shards = (is_regular_file(a.get("normal")) && is_regular_file(a.get("tumor")))
                          ? shard_intervals(ref, a.get("intervalList"))
                          : dir_shards(a.get("intervalList"));
  BackgroundExecutor warm("gpu-warmup", std::make_shared<DeviceWarmupWorker>(gpus));
  Executor ex("Mutect2", conf().get_int("gatk.mutect2.nprocs", "gatk.nprocs"), gpus);
  std::vector<std::string> parts;
  const std::string sample_id = a.get("sample-id");
  std::vector<std::string> extra = a.all("extra-options");
  if (a.has("dump-regions")) extra.push_back("--dump-regions " + a.get("dump-regions"));
  for (size_t k = 0; k < shards.size(); ++k) {
    const std::string part = get_contig_fname(out_dir, (int)k, "vcf");
    parts.push_back(part);
    ex.addTask(std::make_shared<Mutect2Worker>(ref, shards[k], a.get("normal"), a.get("tumor"), part, extra, (int)k,
                                               true),
               sample_id);
  }
  ex.addTask(std::make_shared<VCFConcatWorker>(parts, output, output + ".gz", /*consume=*/true), sample_id, true);
  if (conf().get_bool("gpu.release_early")) ex.addTask(std::make_shared<GpuReleaseWorker>(gpus, &warm), sample_id);
  ex.run();
  warm.wait();
  if (warm.status() != 0) throw failedCommand(std::string("[E::fcs-genome] GPU warm-up failed: ") + fcs_last_error());
  return 0;
}

// `fcs-genome align` (reference src/worker-align.cpp:19-256): a single read
// group (-1/-2, -R/-S/-P/-L) or a sample sheet (-F; file or FASTQ folder).
// One BWAWorker per (sample, read group), each in its own stage and on every
// GPU slot; a sample with several read groups gets a merge stage.  The
// reference's sambamba INDEX stage is not needed: BAMs are written with their
// index.  Without -F a single-end run (-1 only) is accepted as well.
int align_main(int argc, char** argv) {
  Args a;
  common_opts(a);
  a.add("ref", "r", false, true, "reference genome path");
  a.add("fastq1", "1", false, false, "input pair-end fastq file (plain or .gz)");
  a.add("fastq2", "2", false, false, "input pair-end fastq file (plain or .gz)");
  a.add("output", "o", false, true,
        "output BAM file (with --disable-merge a directory of bucket BAMs; with --sample_sheet the folder of the "
        "samples' outputs)");
  a.add("sample_sheet", "F", false, false, "sample sheet (#sample_id,fastq1,fastq2,rg,platform_id,library_id) or "
        "folder of *_1.fastq.gz / *_2.fastq.gz");
  a.add("rg", "R", false, false, "read group id ('ID' in BAM header)");
  a.add("sp", "S", false, false, "sample id ('SM' in BAM header)");
  a.add("pl", "P", false, false, "platform id ('PL' in BAM header)");
  a.add("lb", "L", false, false, "library id ('LB' in BAM header)");
  a.add("align-only", "l", true, false, "skip mark duplicates");
  a.add("disable-merge", "", true, false, "give bucket bams instead of the whole bam");
  try {
    a.parse(argc, argv);
  } catch (helpRequest&) {
    std::cerr << "'fcs-genome align' options:\n" << a.help();
    throw;
  }
  const std::string ref = a.get("ref"), sheet = a.get("sample_sheet"), fq1 = a.get("fastq1"), fq2 = a.get("fastq2");
  const std::string output = a.get("output");
  const bool force = a.has("force"), disable_merge = a.has("disable-merge");
  const std::vector<std::string> extra = a.all("extra-options");
  SampleSheetMap samples;
  if (sheet.empty()) {
    if (fq1.empty()) throw invalidParam("Either --sample_sheet or --fastq1,fastq2 needs to be specified");
    SampleDetails d;
    d.fastqR1 = fq1;
    d.fastqR2 = fq2;
    d.ReadGroup = a.get("rg", "sample");
    d.Platform = a.get("pl", "illumina");
    d.LibraryID = a.get("lb", "sample");
    samples[a.get("sp", "sample")].push_back(d);
  } else {
    if (!fq1.empty() || !fq2.empty())
      throw invalidParam("--sample_sheet and --fastq1,fastq2 cannot be specified at the same time");
    samples = read_sample_sheet(sheet);
  }
  if (!is_regular_file(ref)) throw fileNotFound(ref);
  if (sheet.empty() && !disable_merge) {
    if (!force && path_exists(output)) throw invalidParam("output " + output + " exists (use -f)");
  } else {
    if (path_exists(output) && !is_directory(output))
      throw fileNotFound("Output path " + output + " is not a directory");
    create_dir(output);
  }
  const std::vector<int> gpus = slots();
  const std::string temp_dir = conf().temp_dir() + "/align";
  create_dir(temp_dir);
  for (const auto& [sample_id, list] : samples) {
    // one Executor per sample (the reference runs it inside the sample loop);
    // one task at a time, each task on every GPU slot
    Executor ex("align", 1, gpus);
    const std::string merge_dir = temp_dir + "/" + sample_id + "merge";
    create_dir(merge_dir);
    const std::string merged = sheet.empty() ? output : output + "/" + sample_id + ".bam";
    std::vector<std::string> rg_out;
    for (const SampleDetails& d : list) {
      const std::string out_rg = list.size() == 1 ? merged : merge_dir + "/" + sample_id + "_" + d.ReadGroup + ".bam";
      // two read groups of one sample writing one BAM would lose one lane and
      // merge the other twice, silently
      if (std::find(rg_out.begin(), rg_out.end(), out_rg) != rg_out.end())
        throw invalidParam("sample " + sample_id + " lists read group " + d.ReadGroup +
                           " more than once (each read group is aligned to its own BAM)");
      rg_out.push_back(out_rg);
      ex.addTask(std::make_shared<BWAWorker>(ref, d.fastqR1, d.fastqR2, out_rg, extra, sample_id, d.ReadGroup,
                                             d.Platform, d.LibraryID, !disable_merge, force || list.size() > 1, gpus),
                 sample_id, true);
    }
    if (list.size() > 1) {
      if (!disable_merge) {
        ex.addTask(std::make_shared<MergeBamWorker>(rg_out, merged, force), sample_id, true);
      } else {  // bucket i of every read group -> bucket i of the sample (worker-align.cpp:226-246)
        create_dir(merged);
        const int nb = std::max(1, conf().get_int("bwa.num_buckets"));
        for (int i = 0; i < nb; ++i) {
          std::vector<std::string> in;
          for (const std::string& r : rg_out) in.push_back(get_contig_fname(r, i, "bam"));
          ex.addTask(std::make_shared<MergeBamWorker>(in, get_contig_fname(merged, i, "bam"), true), sample_id,
                     i == 0);
        }
      }
    }
    ex.run();
  }
  return 0;
}

// `fcs-genome index -r ref.fasta`: the aligner's FMD-index, saved next to the
// FASTA (<ref>.fcsidx) so that align maps it instead of building one per run
// (bwa-flow reads the prebuilt bwa index; the reference expects it beside the
// FASTA, src/workers/BWAWorker.cpp:134-147).
int index_main(int argc, char** argv) {
  Args a;
  a.add("ref", "r", false, true, "reference genome path");
  a.add("sa-intv", "", false, false, "suffix-array sampling interval (default: automatic, <= 8 GiB of samples)");
  try {
    a.parse(argc, argv);
  } catch (helpRequest&) {
    std::cerr << "'fcs-genome index' options:\n" << a.help();
    throw;
  }
  const std::string ref = a.get("ref");
  if (!is_regular_file(ref)) throw fileNotFound(ref);
  const uint64_t t0 = now_us();
  build_fmd_index(ref, a.has("sa-intv") ? std::stoi(a.get("sa-intv")) : 0);
  std::cerr << "[fcs-genome index] " << fmd_index_path(ref) << " written in " << (now_us() - t0) / 1e6 << " s"
            << std::endl;
  return 0;
}

int synth_main(int argc, char** argv) {
  Args a;
  a.add("output", "o", false, true, "output directory");
  a.add("contigs", "c", false, false, "name:length[,name:length...] (default chr20:1000000)");
  a.add("coverage", "x", false, false, "sample coverage (default 30)");
  a.add("seed", "s", false, false, "seed (default 20261015)");
  a.add("max-reads", "n", false, false, "keep only the first N reads by position (C1: 1000)");
  a.add("tumor", "T", true, false, "also write tumor.bam with somatic variants (C5)");
  a.add("tumor-coverage", "", false, false, "tumor coverage (default 40)");
  a.add("somatic-af", "", false, false, "somatic allele fraction (default 0.3)");
  a.add("noisy-frac", "", false, false, "fraction of reads drawn with 20% high-quality mismatches (mis-mapped-like)");
  a.add("spike", "", false, false, "chr:pos[,chr:pos...] plant three het SNVs at pos-30, pos, pos+30 (1-based)");
  a.add("parts", "", false, false, "also split the sample into parts/part-XXXXXX.bam + .bed (N buckets)");
  a.add("paired", "", false, false, "also write sample_1/2.fastq: FR pairs with fragment length ~ N(ARG, 50)");
  a.add("no-fastq", "", true, false, "do not write sample.fastq (the single-end FASTQ of the sample's reads)");
  a.parse(argc, argv);
  SynthSpec sp;
  if (a.has("contigs")) {
    sp.contigs.clear();
    std::string s = a.get("contigs");
    size_t p = 0;
    while (p < s.size()) {
      const size_t e = std::min(s.find(',', p), s.size());
      const std::string tok = s.substr(p, e - p);
      const size_t c = tok.find(':');
      if (c == std::string::npos) throw invalidParam("--contigs " + s);
      sp.contigs.emplace_back(tok.substr(0, c), std::stoll(tok.substr(c + 1)));
      p = e + 1;
    }
  }
  if (a.has("spike")) {
    std::string s = a.get("spike");
    for (size_t p = 0; p < s.size();) {
      const size_t e = std::min(s.find(',', p), s.size());
      const std::string tok = s.substr(p, e - p);
      const size_t c = tok.rfind(':');
      if (c == std::string::npos) throw invalidParam("--spike " + s);
      sp.spikes.emplace_back(tok.substr(0, c), std::stoll(tok.substr(c + 1)) - 1);
      p = e + 1;
    }
  }
  if (a.has("no-fastq")) sp.single_fastq = false;
  if (a.has("noisy-frac")) sp.noisy_frac = std::stod(a.get("noisy-frac"));
  if (a.has("parts")) sp.parts = std::stoi(a.get("parts"));
  if (a.has("paired")) sp.paired_insert = std::stoi(a.get("paired"));
  if (a.has("coverage")) sp.coverage = std::stod(a.get("coverage"));
  if (a.has("seed")) sp.seed = std::stoull(a.get("seed"));
  if (a.has("max-reads")) sp.max_reads = std::stoll(a.get("max-reads"));
  if (a.has("tumor")) sp.somatic_rate = 1e-4;
  if (a.has("tumor-coverage")) sp.tumor_coverage = std::stod(a.get("tumor-coverage"));
  if (a.has("somatic-af")) sp.somatic_af = std::stod(a.get("somatic-af"));
  const SynthOutputs o = synth_dataset(sp, a.get("output"));
  std::cout << "{\"ref\": \"" << o.ref_fasta << "\", \"bam\": \"" << o.bam << "\", \"fastq\": \"" << o.fastq
            << "\", \"truth\": \"" << o.truth_vcf << "\", \"tumor_bam\": \"" << o.tumor_bam
            << "\", \"parts\": \"" << o.parts_dir << "\", \"fastq1\": \"" << o.fastq1 << "\", \"fastq2\": \""
            << o.fastq2 << "\", \"pairs_truth\": \"" << o.pairs_truth
            << "\", \"reads\": " << o.n_reads << ", \"tumor_reads\": " << o.n_tumor_reads
            << ", \"variants\": " << o.variants.size() << "}" << std::endl;
  return 0;
}

// SIGINT / SIGTERM / SIGHUP (the reference's sigint_handler, src/main.cpp:43-54):
// an async-signal-safe handler writes the signal number to a pipe, and a
// watcher thread announces the interrupt and sets the flag the Executor and
// the workers poll; the run then unwinds, removes its temp dir and exits
// 128 + signal.  A second signal exits at once.  No signal is blocked, so the
// threads of the HIP runtime and of a profiler (rocprofv3) see the process's
// signals as they would without fcs-genome's handling (round 2 blocked the
// three signals in every thread, and a profiled run hung at exit).
int g_sig_pipe[2] = {-1, -1};
volatile sig_atomic_t g_sig_seen = 0;

extern "C" void on_signal(int sig) {
  if (g_sig_seen) _exit(128 + sig);
  g_sig_seen = sig;
  const unsigned char b = (unsigned char)sig;
  if (write(g_sig_pipe[1], &b, 1) < 0) _exit(128 + sig);
}

void start_signal_thread() {
  if (pipe(g_sig_pipe) != 0) return;
  std::thread([] {
    unsigned char b = 0;
    for (;;) {
      const ssize_t n = read(g_sig_pipe[0], &b, 1);
      if (n == 1) break;
      if (n < 0 && errno == EINTR) continue;
      return;
    }
    std::cerr << "[fcs-genome] Caught interrupt, cleaning up..." << std::endl;
    set_interrupted((int)b);
  }).detach();
  struct sigaction sa;
  std::memset(&sa, 0, sizeof sa);
  sa.sa_handler = on_signal;
  sigemptyset(&sa.sa_mask);
  sa.sa_flags = SA_RESTART;
  for (int sig : {SIGINT, SIGTERM, SIGHUP}) sigaction(sig, &sa, nullptr);
}

int print_help() {
  std::cout << "Falcon Genome Analysis Toolkit (MI355X / gfx950 build)\n"
               "Usage: fcs-genome [command] <options>\n\nCommands:\n"
               "  align           align FASTQ reads into a sorted BAM (GPU banded SW)\n"
               "  htc             variant calling, HaplotypeCaller-style (GPU PairHMM)\n"
               "  mutect2         somatic variant calling, tumor/normal (GPU PairHMM)\n"
               "  conf            print configuration keys\n"
               "  index           build the aligner's FMD-index of a reference (<ref>.fcsidx)\n"
               "  synth           write synthetic reference/BAM/FASTQ/truth inputs\n";
  return 0;
}

}  // namespace
}  // namespace fcsg

int main(int argc, char** argv) {
  using namespace fcsg;
  if (argc < 2) {
    print_help();
    return 1;
  }
  std::string cmd = argv[1];
  for (char& c : cmd) c = (char)std::tolower((unsigned char)c);
  int ret = 0;
  std::string root;
  {
    std::string self = argv[0];
    const size_t k = self.find_last_of('/');
    root = k == std::string::npos ? "." : self.substr(0, k) + "/..";
  }
  timeline("main");
  // Shard threads allocate and free large blocks in batches (PairHMM region
  // batches, per-window vectors): keep freed memory in the allocator instead
  // of returning it (munmap / heap trim) only to fault it back in — with 32
  // threads in one process those faults serialize on the memory-map lock.
  mallopt(M_MMAP_THRESHOLD, 256 << 20);
  mallopt(M_TRIM_THRESHOLD, 1 << 30);
  start_signal_thread();
  try {
    conf().init(root);
    if (cmd == "htc") ret = htc_main(argc - 1, argv + 1);
    else if (cmd == "mutect2") ret = mutect2_main(argc - 1, argv + 1);
    else if (cmd == "align" || cmd == "al") ret = align_main(argc - 1, argv + 1);
    else if (cmd == "synth") ret = synth_main(argc - 1, argv + 1);
    else if (cmd == "index") ret = index_main(argc - 1, argv + 1);
    else if (cmd == "conf") {
      std::cerr << "fcs-genome configuration options:\n" << conf().dump();
      ret = 1;  // the reference exits through silentExit here
    } else if (cmd == "--version") {
      std::cout << "fcs-genome (gfx950) / " << fcs_version() << std::endl;
    } else {
      print_help();
      ret = 1;
    }
    remove_path(conf().temp_dir());
    timeline("temp removed");
  } catch (helpRequest&) {
    ret = 0;
  } catch (invalidParam& e) {
    std::cerr << "[fcs-genome] ERROR: Failed to parse arguments: invalid option " << e.what() << std::endl;
    ret = 1;
  } catch (pathEmpty& e) {
    std::cerr << "[fcs-genome] ERROR: Failed to parse arguments: option " << e.what() << " cannot be empty" << std::endl;
    ret = 1;
  } catch (fileNotFound& e) {
    std::cerr << "[fcs-genome] ERROR: " << e.what() << std::endl;
    ret = 3;
  } catch (silentExit&) {
    ret = 1;
  } catch (interruptedError&) {
    remove_path(conf().temp_dir());
    ret = 128 + interrupt_signal();
  } catch (failedCommand& e) {
    if (*e.what()) std::cerr << e.what() << std::endl;
    ret = 4;
  } catch (std::runtime_error& e) {
    std::cerr << "[fcs-genome] ERROR: Encountered an error: " << e.what() << std::endl;
    ret = -1;
  }
  timeline("exit");
  // Every output is closed; flush the streams and leave without running static
  // destructors or the GPU runtime's teardown (≈ 0.3 s of unloading and
  // freeing after the last output on the bench box); the kernel reclaims the
  // process's memory and devices as it does for any exit.
  std::cout.flush();
  std::cerr.flush();
  std::fflush(nullptr);
#if defined(__SANITIZE_ADDRESS__) || defined(__SANITIZE_THREAD__)
  return ret;  // sanitizer builds keep the normal exit (leak and race reports run at exit)
#else
  if (std::getenv("FCS_NORMAL_EXIT")) return ret;  // profilers that report from atexit handlers
  std::_Exit(ret);
#endif
}

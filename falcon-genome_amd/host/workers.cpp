#include "workers.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <map>
#include <mutex>

#include "aligner.h"

#include "common.h"
#include "config.h"
#include "fcship.h"
#include "gatk_prep.h"
#include "intervals.h"
#include "vcf.h"

namespace fcsg {

std::shared_ptr<const Reference> load_reference_cached(const std::string& path) {
  static std::mutex mu;
  static std::map<std::string, std::shared_ptr<const Reference>> cache;
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(path);
  if (it != cache.end()) return it->second;
  auto ref = std::make_shared<const Reference>(load_fasta(path));
  cache[path] = ref;
  return ref;
}

CallerOptions caller_options_from_config(int gpu) {
  const Config& c = conf();
  CallerOptions o;
  o.gpu = gpu < 0 ? 0 : gpu;
  o.min_base_quality = c.get_int("htc.min_base_quality");
  o.base_quality_threshold = c.get_int("htc.base_quality_threshold");
  o.pcr_indel_model = (int)parse_pcr_indel_model(c.get_string("htc.pcr_indel_model"));
  o.min_mapq = c.get_int("htc.min_mapq");
  o.active_fraction = std::stod(c.get_string("htc.active_fraction"));
  o.somatic_active_fraction = std::stod(c.get_string("mutect2.active_fraction"));
  o.padding = c.get_int("htc.padding");
  o.max_region = c.get_int("htc.max_region");
  o.max_reads_per_region = c.get_int("htc.max_reads_per_region");
  o.batch_regions = c.get_int("gpu.phmm.batch_regions");
  o.combine_ms = c.get_int("gpu.phmm.combine_ms");
  o.fp64_rescue = c.get_bool("gpu.phmm.rescue");
  o.gpu_inflate = c.get_bool("gpu.bam_inflate");
  // (merged passes wait for every active shard's pass: a shard run inside
  // another's flush would hold that pass back, so no help then)
  if (c.get_bool("gpu.warmup_help") && o.combine_ms == 0)
    o.help_while_cold = [] { return !devices_warm() && executor_help_once(); };
  o.tlod = std::stod(c.get_string("mutect2.tlod"));
  o.nlod = std::stod(c.get_string("mutect2.nlod"));
  if (o.padding < 0 || o.max_region < 1 || o.batch_regions < 1 || o.max_reads_per_region < 1 || o.combine_ms < 0)
    throw invalidParam(
        "htc.padding / htc.max_region / gpu.phmm.batch_regions / htc.max_reads_per_region / gpu.phmm.combine_ms");
  return o;
}

// The shard's intervals: the intersection of every -L set (GATK -isr
// INTERSECTION); no set at all means the whole reference (GATK without -L).
static std::vector<Interval> read_all(const Reference& ref, const std::vector<std::string>& paths,
                                      const std::string& region = "", const std::string& region2 = "") {
  std::vector<std::vector<Interval>> sets;
  for (const std::string& p : paths) sets.push_back(read_regions(p));
  for (const std::string* r : {&region, &region2})
    if (!r->empty()) sets.push_back(read_regions(*r));
  if (sets.empty()) {
    std::vector<Interval> all;
    for (const Contig& c : ref.contigs) all.push_back({c.name, 1, (int64_t)c.seq.size()});
    return all;
  }
  if (sets.size() == 1) return sets[0];
  return intersect_interval_sets(sets);
}

static std::string shard_temp_dir(const char* tool) { return conf().temp_dir() + "/" + tool + "_regions"; }

// ------------------------------------------------------------------ HTC
HTCWorker::HTCWorker(std::string ref_path, std::vector<std::string> intv_paths, std::string input_path,
                     std::string output_path, std::vector<std::string> extra_opts, int contig, bool flag_vcf,
                     bool flag_f, bool /*flag_gatk*/)
    : Worker(1, 1, std::move(extra_opts), "Haplotype Caller"),
      ref_path_(std::move(ref_path)),
      input_path_(std::move(input_path)),
      output_path_(std::move(output_path)),
      intv_paths_(std::move(intv_paths)),
      contig_(contig),
      flag_vcf_(flag_vcf),
      flag_f_(flag_f) {}

void HTCWorker::check() {
  if (!is_regular_file(ref_path_)) throw fileNotFound(ref_path_);
  for (const std::string& p : intv_paths_)
    if (!is_regular_file(p)) throw fileNotFound(p);
  shard_ = BamInput(input_path_).merge_region(contig_, conf().get_int("gatk.ncontigs"), shard_temp_dir("htc"));
  for (const std::string& b : shard_.bams)
    if (!is_regular_file(b)) throw fileNotFound(b);
  if (!flag_f_ && path_exists(output_path_)) throw invalidParam("output " + output_path_ + " exists (use -f)");
}

int HTCWorker::run(TaskContext& ctx) {
  auto ref = load_reference_cached(ref_path_);
  CallerOptions opt = caller_options_from_config(ctx.gpu);
  auto it = extra_opts_.find("--dump-regions");
  if (it != extra_opts_.end() && !it->second.empty()) opt.dump_path = it->second[0] + "." + std::to_string(contig_);
  opt.gvcf = !flag_vcf_;  // the reference's default: --emitRefConfidence GVCF unless -v (HTCWorker.cpp:83-97)
  const VcfHeader h = caller_vcf_header(*ref, {"sample"}, false, ref_path_, opt.gvcf);
  VcfWriter out(output_path_, h);
  stats_ = call_intervals(*ref, shard_.bams, {}, read_all(*ref, intv_paths_, shard_.region), opt, out);
  out.close();
  if (ctx.log)
    std::fprintf(ctx.log,
                 "[fcs-genome htc] shard %d gpu %d: %lld reads, %lld regions, %lld pairs, %lld cells, %lld rescued, "
                 "%lld calls, %.3f s (PairHMM %.3f s, device %.4f s, rescue %.4f s, %lld device passes; decode %.3f s "
                 "(%lld passes, inflate %lld gpu / %lld host chunks), pileup %.3f s, regions %.3f s, genotype %.3f s, output %.3f s; thread cpu %.3f s, "
                 "minor faults %lld/%lld/%lld/%lld; ran %lld queued shards in %.3f s while the device came up)\n",
                 contig_, ctx.gpu, (long long)stats_.reads, (long long)stats_.regions, (long long)stats_.pairs,
                 (long long)stats_.cells, (long long)stats_.rescued, (long long)stats_.calls, stats_.seconds,
                 stats_.phmm_seconds, stats_.phmm_device_seconds, stats_.rescue_device_seconds,
                 (long long)stats_.device_passes, stats_.decode_seconds, (long long)stats_.decode_passes,
                 (long long)stats_.inflate_gpu_chunks, (long long)stats_.inflate_host_chunks, stats_.pileup_seconds,
                 stats_.region_seconds, stats_.genotype_seconds, stats_.output_seconds, stats_.cpu_seconds,
                 (long long)stats_.faults[0], (long long)stats_.faults[1], (long long)stats_.faults[2],
                 (long long)stats_.faults[3], (long long)stats_.helped_tasks, stats_.helped_seconds);
  return 0;
}

// ------------------------------------------------------------------ Mutect2
Mutect2Worker::Mutect2Worker(std::string ref_path, std::vector<std::string> intv_paths, std::string normal_path,
                             std::string tumor_path, std::string output_path, std::vector<std::string> extra_opts,
                             int contig, bool flag_f)
    : Worker(1, 1, std::move(extra_opts), "Mutect2"),
      ref_path_(std::move(ref_path)),
      normal_path_(std::move(normal_path)),
      tumor_path_(std::move(tumor_path)),
      output_path_(std::move(output_path)),
      intv_paths_(std::move(intv_paths)),
      contig_(contig),
      flag_f_(flag_f) {}

void Mutect2Worker::check() {
  if (!is_regular_file(ref_path_)) throw fileNotFound(ref_path_);
  for (const std::string& p : intv_paths_)
    if (!is_regular_file(p)) throw fileNotFound(p);
  const int n = conf().get_int("gatk.ncontigs");
  normal_ = BamInput(normal_path_).merge_region(contig_, n, shard_temp_dir("mutect2_normal"));
  tumor_ = BamInput(tumor_path_).merge_region(contig_, n, shard_temp_dir("mutect2_tumor"));
  for (const BamShard* sh : {&normal_, &tumor_})
    for (const std::string& b : sh->bams)
      if (!is_regular_file(b)) throw fileNotFound(b);
  if (!flag_f_ && path_exists(output_path_)) throw invalidParam("output " + output_path_ + " exists (use -f)");
}

int Mutect2Worker::run(TaskContext& ctx) {
  auto ref = load_reference_cached(ref_path_);
  CallerOptions opt = caller_options_from_config(ctx.gpu);
  opt.somatic = true;
  auto it = extra_opts_.find("--dump-regions");
  if (it != extra_opts_.end() && !it->second.empty()) opt.dump_path = it->second[0] + "." + std::to_string(contig_);
  const VcfHeader h = caller_vcf_header(*ref, {"TUMOR", "NORMAL"}, true, ref_path_);
  VcfWriter out(output_path_, h);
  stats_ = call_intervals(*ref, tumor_.bams, normal_.bams, read_all(*ref, intv_paths_, normal_.region, tumor_.region), opt,
                          out);
  out.close();
  if (ctx.log)
    std::fprintf(ctx.log,
                 "[fcs-genome mutect2] shard %d gpu %d: %lld reads, %lld regions, %lld pairs, %lld cells, %lld rescued, "
                 "%lld calls, %.3f s (PairHMM %.3f s, device %.4f s, rescue %.4f s, %lld device passes; decode %.3f s "
                 "(%lld passes, inflate %lld gpu / %lld host chunks), pileup %.3f s, regions %.3f s, genotype %.3f s, output %.3f s; thread cpu %.3f s, "
                 "minor faults %lld/%lld/%lld/%lld)\n",
                 contig_, ctx.gpu, (long long)stats_.reads, (long long)stats_.regions, (long long)stats_.pairs,
                 (long long)stats_.cells, (long long)stats_.rescued, (long long)stats_.calls, stats_.seconds,
                 stats_.phmm_seconds, stats_.phmm_device_seconds, stats_.rescue_device_seconds,
                 (long long)stats_.device_passes, stats_.decode_seconds, (long long)stats_.decode_passes,
                 (long long)stats_.inflate_gpu_chunks, (long long)stats_.inflate_host_chunks, stats_.pileup_seconds,
                 stats_.region_seconds, stats_.genotype_seconds, stats_.output_seconds, stats_.cpu_seconds,
                 (long long)stats_.faults[0], (long long)stats_.faults[1], (long long)stats_.faults[2],
                 (long long)stats_.faults[3]);
  return 0;
}

// ------------------------------------------------------------------ VCF tail
VCFConcatWorker::VCFConcatWorker(std::vector<std::string> inputs, std::string output, std::string gz, bool consume)
    : Worker(1, 1, {}, gz.empty() ? "VCF concat" : "VCF concat + bgzip + tabix"),
      inputs_(std::move(inputs)),
      output_(std::move(output)),
      gz_(std::move(gz)),
      consume_(consume) {}

void VCFConcatWorker::check() {
  if (inputs_.empty()) throw invalidParam("no VCF to concatenate");
}

int VCFConcatWorker::run(TaskContext&) {
  if (gz_.empty()) vcf_concat(inputs_, output_);
  else vcf_concat_bgzip_tabix(inputs_, output_, gz_, consume_);
  return 0;
}

ZIPWorker::ZIPWorker(std::string input, std::string output, bool, bool index)
    : Worker(1, 1, {}, index ? "bgzip + tabix" : "bgzip"), input_(std::move(input)), output_(std::move(output)),
      index_(index) {}

void ZIPWorker::check() {}

int ZIPWorker::run(TaskContext&) {
  if (index_) bgzip_tabix_file(input_, output_);
  else bgzip_file(input_, output_);
  return 0;
}

TabixWorker::TabixWorker(std::string path) : Worker(1, 1, {}, "tabix"), path_(std::move(path)) {}

int TabixWorker::run(TaskContext&) {
  tabix_index_vcf(path_);
  return 0;
}

// ------------------------------------------------------------------ align
BWAWorker::BWAWorker(std::string ref_path, std::string fq1_path, std::string fq2_path, std::string output_path,
                     std::vector<std::string> extra_opts, std::string sample_id, std::string read_group,
                     std::string platform_id, std::string library_id, bool flag_merge_bams, bool flag_f,
                     std::vector<int> gpus)
    : Worker(1, 1, std::move(extra_opts), "bwa mem"),
      ref_path_(std::move(ref_path)),
      fq1_path_(std::move(fq1_path)),
      fq2_path_(std::move(fq2_path)),
      output_path_(std::move(output_path)),
      sample_id_(std::move(sample_id)),
      read_group_(std::move(read_group)),
      platform_id_(std::move(platform_id)),
      library_id_(std::move(library_id)),
      flag_merge_bams_(flag_merge_bams),
      flag_f_(flag_f),
      gpus_(std::move(gpus)) {}

void BWAWorker::check() {
  if (flag_merge_bams_ && !flag_f_ && path_exists(output_path_))
    throw invalidParam("output " + output_path_ + " exists (use -f)");
  if (sample_id_.empty() || read_group_.empty() || platform_id_.empty() || library_id_.empty())
    throw invalidParam("Invalid @RG info");
  for (const std::string* p : {&ref_path_, &fq1_path_})
    if (!is_regular_file(*p)) throw fileNotFound(*p);
  if (!fq2_path_.empty() && !is_regular_file(fq2_path_)) throw fileNotFound(fq2_path_);
  // temporary storage >= 3x the FASTQ input (BWAWorker.cpp:70-91)
  const uint64_t need = 3 * (file_size(fq1_path_) + (fq2_path_.empty() ? 0 : file_size(fq2_path_)));
  const std::string tmp = conf().temp_dir();
  const size_t k = tmp.find_last_of('/');
  const uint64_t avail = available_space(k == std::string::npos ? "." : k == 0 ? "/" : tmp.substr(0, k));
  if (avail < need) {
    std::cerr << "[fcs-genome] ERROR: Not enough space in temporary storage. The size of the temporary folder "
                 "should be at least 3 times the size of input FASTQ files"
              << std::endl;
    throw silentExit();
  }
}

int BWAWorker::run(TaskContext& ctx) {
  AlignJob job;
  job.ref_path = ref_path_;
  job.fq1 = fq1_path_;
  job.fq2 = fq2_path_;
  job.output = output_path_;
  job.rg = read_group_;
  job.sample = sample_id_;
  job.platform = platform_id_;
  job.library = library_id_;
  job.disable_merge = !flag_merge_bams_;
  std::string report;
  align_fastq(job, gpus_, report);
  if (ctx.log) std::fputs(report.c_str(), ctx.log);
  std::cerr << report << std::flush;
  return 0;
}

MergeBamWorker::MergeBamWorker(std::vector<std::string> inputs, std::string output, bool flag_f)
    : Worker(1, 1, {}, "Merge BAM"), inputs_(std::move(inputs)), output_(std::move(output)), flag_f_(flag_f) {}

void MergeBamWorker::check() {
  if (inputs_.empty()) throw invalidParam("no BAM to merge into " + output_);
  if (!flag_f_ && path_exists(output_)) throw invalidParam("output " + output_ + " exists (use -f)");
}

int MergeBamWorker::run(TaskContext&) {
  for (const std::string& p : inputs_)
    if (!is_regular_file(p)) throw fileNotFound(p);
  merge_sorted_bams(inputs_, output_);
  const std::string bed_in = inputs_[0].substr(0, inputs_[0].size() - 4) + ".bed";
  if (inputs_[0].size() > 4 && is_regular_file(bed_in))
    write_file(output_.substr(0, output_.size() - 4) + ".bed", read_file(bed_in));
  return 0;
}

DeviceWarmupWorker::DeviceWarmupWorker(std::vector<int> gpus) : Worker(1, 1, {}, "GPU warm-up"), gpus_(std::move(gpus)) {}

int DeviceWarmupWorker::run(TaskContext&) {
  // runtime, code objects, GKL tables and the pooled call sessions of each
  // device, while the shards decode their first reads; then, with
  // gpu.bam_inflate, warm inflate sessions (the windows decoded before they
  // are ready inflate on their own threads)
  for (int d : gpus_)
    if (fcs_device_warmup(d, 0) != FCS_OK) return 1;
  // FCS_TEST_COLD_DEVICE=1 (tests): the devices never count as warm, so every
  // shard's pass first runs the queued shards (tests/test_c1_cpu.py)
  if (!std::getenv("FCS_TEST_COLD_DEVICE")) set_devices_warm(true);
  if (conf().get_bool("gpu.bam_inflate"))
    for (int d : gpus_)
      if (fcs_bgzf_warmup(d, 8, (int64_t)112 << 20) != FCS_OK) return 1;
  return 0;
}

GpuReleaseWorker::GpuReleaseWorker(std::vector<int> gpus, BackgroundExecutor* warm)
    : Worker(1, 1, {}, "GPU release"), gpus_(std::move(gpus)), warm_(warm) {
  std::sort(gpus_.begin(), gpus_.end());
  gpus_.erase(std::unique(gpus_.begin(), gpus_.end()), gpus_.end());
}

int GpuReleaseWorker::run(TaskContext&) {
  if (warm_) warm_->wait();
  // a failure only means the teardown happens at exit as before
  for (int d : gpus_)
    if (d >= 0 && fcs_device_release(d) != FCS_OK) std::fprintf(stderr, "[W::fcs-genome] %s\n", fcs_last_error());
  return 0;
}

}  // namespace fcsg

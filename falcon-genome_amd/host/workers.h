// Workers of the GPU-backed commands (reference: include/fcs-genome/workers/*.h).
// HTCWorker / Mutect2Worker keep the reference's constructor arguments
// (src/workers/HTCWorker.cpp:17-47, Mutect2Worker.cpp:17-107) but run the
// caller in-process on the task's GPU slot instead of launching GATK.  Their
// input is a BamInput (one indexed BAM, or a directory of part BAMs whose
// shard `contig` check() resolves with merge_region, as HTCWorker::check does
// at src/workers/HTCWorker.cpp:36-46); the shard's intervals are the
// intersection of every -L set (GATK -isr INTERSECTION, HTCWorker.cpp:68):
// user list, init_contig_intv part, part-BAM region file;
// VCFConcatWorker / ZIPWorker / TabixWorker are the same tail as
// src/worker-htc.cpp:153-176, done natively instead of via bcftools/bgzip/tabix.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "bam_input.h"
#include "caller.h"
#include "executor.h"
#include "fasta.h"

namespace fcsg {

// Process-wide reference cache (shard tasks of one run share the genome).
std::shared_ptr<const Reference> load_reference_cached(const std::string& path);

class HTCWorker : public Worker {
 public:
  HTCWorker(std::string ref_path, std::vector<std::string> intv_paths, std::string input_path,
            std::string output_path, std::vector<std::string> extra_opts, int contig, bool flag_vcf, bool flag_f,
            bool flag_gatk = false);
  void check() override;
  int run(TaskContext& ctx) override;
  CallerStats stats() const { return stats_; }

 private:
  std::string ref_path_, input_path_, output_path_;
  std::vector<std::string> intv_paths_;
  int contig_;
  bool flag_vcf_, flag_f_;
  BamShard shard_;
  CallerStats stats_;
};

class Mutect2Worker : public Worker {
 public:
  Mutect2Worker(std::string ref_path, std::vector<std::string> intv_paths, std::string normal_path,
                std::string tumor_path, std::string output_path, std::vector<std::string> extra_opts, int contig,
                bool flag_f);
  void check() override;
  int run(TaskContext& ctx) override;
  CallerStats stats() const { return stats_; }

 private:
  std::string ref_path_, normal_path_, tumor_path_, output_path_;
  std::vector<std::string> intv_paths_;
  int contig_;
  bool flag_f_;
  BamShard normal_, tumor_;
  CallerStats stats_;
};

class VCFConcatWorker : public Worker {
 public:
  // gz non-empty: also gz + gz.tbi from the same pass (concat + bgzip + tabix as one stage);
  // consume: the inputs are temporary parts, removed as soon as they are read
  VCFConcatWorker(std::vector<std::string> inputs, std::string output, std::string gz = "", bool consume = false);
  void check() override;
  int run(TaskContext& ctx) override;

 private:
  std::vector<std::string> inputs_;
  std::string output_, gz_;
  bool consume_;
};

class ZIPWorker : public Worker {
 public:
  // index: also write output.tbi from the same pass (bgzip + tabix as one stage)
  ZIPWorker(std::string input, std::string output, bool flag_f = true, bool index = false);
  void check() override;
  int run(TaskContext& ctx) override;

 private:
  std::string input_, output_;
  bool index_;
};

class TabixWorker : public Worker {
 public:
  explicit TabixWorker(std::string path);
  int run(TaskContext& ctx) override;

 private:
  std::string path_;
};

// One read group of `fcs-genome align` (reference BWAWorker,
// src/workers/BWAWorker.cpp:17-186, run per (sample, RG) by
// src/worker-align.cpp:168-183).  check(): @RG fields non-empty, inputs
// present, the output free (unless -f) and temp space >= 3x the FASTQ
// (BWAWorker.cpp:48-92); run(): align_fastq on every GPU slot of the run
// instead of bwa-flow on the FPGA.
class BWAWorker : public Worker {
 public:
  BWAWorker(std::string ref_path, std::string fq1_path, std::string fq2_path, std::string output_path,
            std::vector<std::string> extra_opts, std::string sample_id, std::string read_group,
            std::string platform_id, std::string library_id, bool flag_merge_bams, bool flag_f,
            std::vector<int> gpus);
  void check() override;
  int run(TaskContext& ctx) override;

 private:
  std::string ref_path_, fq1_path_, fq2_path_, output_path_, sample_id_, read_group_, platform_id_, library_id_;
  bool flag_merge_bams_, flag_f_;
  std::vector<int> gpus_;
};

// Merges coordinate-sorted BAMs into one sorted, indexed BAM (the reference's
// SambambaWorker MERGE action, src/workers/SambambaWorker.cpp, used by
// src/worker-align.cpp:218-246 for samples with several read groups); a
// bucket's .bed region file is carried over when the inputs have one.
class MergeBamWorker : public Worker {
 public:
  MergeBamWorker(std::vector<std::string> inputs, std::string output, bool flag_f);
  void check() override;
  int run(TaskContext& ctx) override;

 private:
  std::vector<std::string> inputs_;
  std::string output_;
  bool flag_f_;
};

// Loads libfcship's per-device tables on every GPU slot before the shard
// tasks start (the role the Blaze NAM daemon plays for the FPGA:
// src/worker-htc.cpp:100-112).  Run by a BackgroundExecutor.
class DeviceWarmupWorker : public Worker {
 public:
  explicit DeviceWarmupWorker(std::vector<int> gpus);
  int run(TaskContext& ctx) override;

 private:
  std::vector<int> gpus_;
};

// Releases the devices the job's callers used (fcs_device_release) once the
// caller stage is done, beside the VCF tail, so the GPU context's teardown
// does not follow the last output (gpu.release_early).  Waits for the warm-up
// first: nothing else uses the devices by then.
class GpuReleaseWorker : public Worker {
 public:
  GpuReleaseWorker(std::vector<int> gpus, BackgroundExecutor* warm);
  int run(TaskContext& ctx) override;

 private:
  std::vector<int> gpus_;
  BackgroundExecutor* warm_;
};

// Applies the caller's config keys (htc.*, mutect2.*, gpu.*) to options.
CallerOptions caller_options_from_config(int gpu);

}  // namespace fcsg

// Caller side of the PairHMM for `fcs-genome htc` / `mutect2` (SURVEY.md §8f
// row f2): per interval shard, find active regions from the pileup, build
// candidate haplotypes, prepare reads the GATK way (gatk_prep.h), send many
// regions per device pass through fcs_phmm_compute_regions (the hot path,
// include/fcship.h), scatter the read-major likelihood matrices back and
// genotype from them.
//
// What stands in for GATK here [EXT, not in /root/reference]: haplotypes come
// from the candidate alleles seen in the reads (every combination of up to
// kMaxCandidates alleles per region) instead of GATK's local de-Bruijn
// assembly, genotypes from the standard diploid read-likelihood model
// (GATK's GenotypingEngine with the default heterozygosity prior), and the
// Mutect2 mode from the tumor/normal LOD test (TLOD >= 6.3, NLOD >= 2.2).  The
// likelihoods themselves are GKL's PairHMM, bit-for-bit the hot-path kernels.
#pragma once

#include <cstdint>
#include <functional>
#include <string>
#include <vector>

#include "fasta.h"
#include "intervals.h"
#include "vcf.h"

namespace fcsg {

constexpr int kMaxCandidates = 4;  // haplotypes = all 2^k allele combinations

struct CallerOptions {
  int gpu = 0;
  bool somatic = false;  // Mutect2 mode (tumor BAM + normal BAM)
  int min_base_quality = 10;
  int base_quality_threshold = 18;
  int pcr_indel_model = 3;  // PcrIndelModel (gatk_prep.h): GATK's default CONSERVATIVE
  int min_mapq = 20;
  double active_fraction = 0.15;
  double somatic_active_fraction = 0.10;  // Mutect2 mode: of the tumor's depth
  int padding = 50;
  int max_region = 300;
  int max_reads_per_region = 250;
  int batch_regions = 4096;
  // concurrent shards' passes merged per device (caller.cpp PassCombiner): the
  // leader's wait window in ms (0, the default: every flush is its own pass;
  // at the C4 shape merging gives 4-9 passes instead of 32 but costs mutect2
  // ~10% of its wall time) and the pass cap
  int combine_ms = 0;
  int64_t combine_max_pairs = 4000000;
  bool fp64_rescue = true;
  // window BAM blocks through fcs_bgzf_inflate (BgzfReader::use_device); off by
  // default: at the htc shard shape the host's libdeflate is faster
  bool gpu_inflate = false;
  // called before each PairHMM pass until it returns false: while the device
  // is still coming up it runs another queued shard on this thread
  // (gpu.warmup_help; set by the shard workers, empty elsewhere)
  std::function<bool()> help_while_cold;
  double min_qual = 30.0;  // stand_call_conf
  double tlod = 6.3, nlod = 2.2;
  std::string dump_path;  // if set: append every region's PairHMM inputs/outputs here (tests)
  bool gvcf = false;      // htc without -v: reference-confidence blocks + <NON_REF> (GATK --emitRefConfidence GVCF)
};

struct CallerStats {
  int64_t reads = 0, regions = 0, pairs = 0, cells = 0, calls = 0, device_passes = 0, decode_passes = 0;
  int64_t inflate_gpu_chunks = 0, inflate_host_chunks = 0;  // gpu.bam_inflate: window chunks by where they inflated
  int64_t rescued = 0;  // pairs the fp64 rescue recomputed (fp32 sum < 1e-28)
  double seconds = 0, phmm_seconds = 0;
  // wall-time breakdown of `seconds`: BAM decode, pileup + active sites,
  // regions (candidates, haplotypes, read preparation), genotyping, GVCF
  // blocks + record sort + VCF write; phmm_seconds = the PairHMM calls
  double decode_seconds = 0, pileup_seconds = 0, region_seconds = 0, genotype_seconds = 0, output_seconds = 0;
  // the calling thread's CPU seconds and minor page faults (decode, pileup,
  // regions + PairHMM + genotyping, output): where host time goes
  double cpu_seconds = 0;
  int64_t faults[4] = {0, 0, 0, 0};
  // device time of the PairHMM calls (HIP events: schedule + forward + rescue) and of the fp64 rescue alone
  double phmm_device_seconds = 0, rescue_device_seconds = 0;
  // other shards run on this thread while the device came up (help_while_cold):
  // their wall and CPU time, left out of this shard's figures above
  int64_t helped_tasks = 0;
  double helped_seconds = 0, helped_cpu_seconds = 0;
  void add(const CallerStats& o);
};

// Calls variants of `bams` (the parts of one sample, read as one; the tumor in
// Mutect2 mode, with `normal_bams`) on the intervals; records with POS inside an
// interval are written to `out` in coordinate order.  In GVCF mode every
// position of the intervals is covered once: by a call or by a hom-ref block.
CallerStats call_intervals(const Reference& ref, const std::vector<std::string>& bams,
                           const std::vector<std::string>& normal_bams, const std::vector<Interval>& intervals,
                           const CallerOptions& opt, VcfWriter& out);

// Header of the caller's VCF (FORMAT/INFO definitions, contigs, samples).
VcfHeader caller_vcf_header(const Reference& ref, const std::vector<std::string>& samples, bool somatic,
                            const std::string& ref_path, bool gvcf = false);

// GATK's default GVCF GQ bands (--GVCFGQBands 1..60, 70, 80, 90, 99): the
// band index of a GQ value; a block holds consecutive positions of one band.
int gvcf_band(int gq);

}  // namespace fcsg

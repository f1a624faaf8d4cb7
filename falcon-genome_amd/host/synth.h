// Synthetic inputs of the end-to-end configs (C1 1k reads,
// C4 30x, C5 tumor/normal with spiked variants; GRCh38 is not available
// offline).  A random reference, a diploid truth set of SNVs and indels, reads
// sampled from the two haplotypes with sequencing errors, aligned by
// construction (CIGAR from the haplotype-to-reference map), written as a
// coordinate-sorted BAM + BAI, the FASTQ of the same reads (input of `align`)
// and the truth VCF.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "fasta.h"

namespace fcsg {

struct SynthVariant {
  std::string chrom;
  int64_t pos = 0;  // 0-based on the reference
  std::string ref, alt;
  int gt = 1;       // 1 = het (first haplotype), 2 = hom alt
  bool somatic = false;
  double af = 1.0;  // somatic allele fraction in the tumor
};

struct SynthSpec {
  uint64_t seed = 20261015;
  std::vector<std::pair<std::string, int64_t>> contigs{{"chr20", 1000000}};
  double coverage = 30.0;
  int read_len = 151;
  double snp_rate = 1e-3, indel_rate = 1.5e-4, hom_frac = 0.35;
  double err_rate = 0.004;
  int64_t max_reads = -1;   // C1: stop after this many reads (sorted by position)
  double somatic_rate = 0;  // > 0: also write a tumor BAM with somatic variants at somatic_af
  double somatic_af = 0.3;
  double tumor_coverage = 40.0;
  // reads drawn as if mis-mapped from a paralog: 20% mismatches at Q35-40
  // (their PairHMM likelihoods underflow the fp32 pass: C5's fp64 rescue)
  double noisy_frac = 0;
  // planted clusters: three het SNVs at centre - 30, centre, centre + 30
  // (0-based), replacing random variants within 100 bp (shard-boundary tests)
  std::vector<std::pair<std::string, int64_t>> spikes;
  // > 0: also write <dir>/parts/part-XXXXXX.bam (+ .bai, .bed) — the sample's
  // reads split by alignment start into `parts` genome buckets (init_contig_intv
  // arithmetic), the layout `fcs-genome align --disable-merge` leaves for htc
  int parts = 0;
  // > 0: also write <dir>/sample_1.fastq + sample_2.fastq, FR read pairs of
  // fragments with length ~ N(paired_insert, paired_sd) (coverage / 2 of
  // fragments), and <dir>/pairs_truth.tsv (name, mate, contig, pos, reverse)
  int paired_insert = 0;
  int paired_sd = 50;
  // write <dir>/sample.fastq (the sample's reads as sequenced, BAM order)
  bool single_fastq = true;
};

struct SynthOutputs {
  std::string ref_fasta, bam, tumor_bam, fastq, truth_vcf, parts_dir, fastq1, fastq2, pairs_truth;
  int64_t n_reads = 0, n_tumor_reads = 0;
  std::vector<SynthVariant> variants;
};

// Writes <dir>/ref.fasta(+.fai,.dict), <dir>/sample.bam(+.bai), <dir>/sample.fastq,
// <dir>/truth.vcf and, with somatic_rate > 0, <dir>/tumor.bam(+.bai).
SynthOutputs synth_dataset(const SynthSpec& spec, const std::string& dir);

}  // namespace fcsg

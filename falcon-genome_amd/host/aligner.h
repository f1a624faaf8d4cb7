// Seed-extension driver of `fcs-genome align` ([EXT]
// bwa bwamem.c mem_chain2aln / mem_reg2aln and bwa.c bwa_gen_cigar2, reached
// in the reference through BWAWorker: /root/reference/src/workers/BWAWorker.cpp:94-186).
//
// Per chunk of reads (bwa.chunk_size), bwa mem's steps:
//   * seeds: SMEMs on an FMD-index of the reference (host/fmindex.h), re-seeds
//     and third-round seeds (mem_collect_intv), every hit (max_occ sampled);
//   * chains (mem_chain's colinearity test) weighed by covered query bases,
//     filtered by mem_chain_flt (shadowed lighter chains dropped, the first
//     shadowed one kept for MAPQ);
//   * mem_chain2aln: seeds of each chain longest first, a seed (almost)
//     inside an earlier region skipped; each extension (left / right
//     ksw_extend2 with band retry, inside the chain's reference window) is a
//     GPU task, one GPU round per step over the whole chunk (host/seedext.h);
//   * mem_sort_dedup_patch: redundant regions dropped, colinear neighbours
//     merged when their joint ksw_global2 score (GPU) keeps >= 90%;
//   * mem_mark_primary_se: secondary by query overlap, sub / sub_n, MAPQ
//     (mem_approx_mapq_se with frac_rep); supplementary = further
//     non-overlapping regions (split reads: flag 0x800, hard clips, SA tags);
//   * paired ends (mem_sam_pe): mem_pestat per orientation, mate rescue in
//     mem_matesw's windows by bwa's ksw_align2 (GPU, fcs_bsw_align: score,
//     score2 as csub, start by the reverse pass), mem_pair's best pair by score + insert-size
//     likelihood, secondary regions re-rooted when they make the pair, paired
//     MAPQ; split reads and unpaired best hits go out single-end style;
//   * CIGARs by mem_reg2aln / bwa_gen_cigar2 (GPU ksw_global2); NM / MD / AS /
//     XS tags; sorted BAM + BAI.
// [EXT] bwa is not vendored, so this is a restatement (parity unpinned against
// bwa itself).  Known differences: reverse-strand regions are extended
// right-first where bwa extends its reverse-complement space left-first
// (tie-breaking only), mem_flt_chained_seeds (long reads only) is not applied,
// a rescued region's truesc is its score (bwa leaves it 0, which would give
// its CIGAR a zero band), and the rescue list is deduplicated once after all
// anchors rather than after each.  Rescue windows follow bwa's anchor order:
// anchor k of every read runs in device round k, after the regions that
// anchors 0 .. k - 1 added to the mate (mem_matesw's skip[] sees them).
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "bam.h"
#include "fasta.h"
#include "fmindex.h"
#include "fcship.h"

namespace fcsg {

struct AlignOptions {
  int gpu = 0;
  int k = 19;            // minimum SMEM length (bwa -k min_seed_len)
  int max_occ = 500;     // occurrences kept per SMEM (bwa -c max_occ; sampled beyond)
  int w = 100;           // band width
  int chunk_size = 100000;
  int threads = 16;        // host threads for seeding / task building (bwa.nt)
  double drop_ratio = 0.5;   // mem_chain_flt: a shadowed chain lighter than this x the heavier is dropped (bwa -D)
  double mask_level = 0.5;   // query overlap that makes a region secondary / a chain shadowed (bwa mask_level)
  double mask_level_redun = 0.95;  // mem_sort_dedup_patch's redundancy overlap
  int max_chain_gap = 10000; // bwa max_chain_gap
  int min_out_score = 30;    // bwa -T: regions scoring below are not output
  int pen_unpaired = 17;     // bwa -U
  int max_matesw = 50;       // bwa max_matesw: rescue anchors per read
  int64_t read_id0 = 0;      // index of the batch's first read (pair) in the input: bwa's hash seed for ties
  std::string rg = "sample", sample = "sample", platform = "illumina", library = "sample";
};

struct AlignStats {
  int64_t reads = 0, mapped = 0, ext_tasks = 0, ext_cells = 0, global_tasks = 0;
  int64_t proper = 0, rescued = 0;  // paired: reads flagged proper pair, reads placed by the mate rescue
  int64_t supplementary = 0;        // supplementary records (split reads)
  double seconds = 0, gpu_seconds = 0;
  // wall seconds of the phases: seeding + chaining, extension (host protocol +
  // GPU calls), pairing / primary choice, record building
  double seed_seconds = 0, extend_seconds = 0, pair_seconds = 0, record_seconds = 0;
  // paired: the insert-size estimate of the (last) batch
  int pe_pairs = 0, pe_low = 0, pe_high = 0;
  double pe_avg = 0, pe_std = 0;
  fcs_bsw_params params{};  // scoring of the batch (bwa defaults)
};

// The aligner's reference index: contigs as codes and their FMD-index
// (host/fmindex.h) for SMEM seeding.
class KmerIndex {
 public:
  // index_path: a saved FMD-index of `ref` (fcs-genome index) to map instead
  // of building one; empty or unusable: built in memory
  KmerIndex(const Reference& ref, int k, const std::string& index_path = "");
  bool loaded() const { return loaded_; }  // the saved index was used
  int k() const { return k_; }  // minimum seed length (bwa -k)
  // the contig's bases as codes 0..4 (A, C, G, T, other)
  const std::vector<uint8_t>& codes(int contig) const { return codes_[contig]; }
  const FmdIndex& fmd() const { return *fmd_; }
  // bwa's packed-reference coordinates: the contig's start in the
  // concatenated forward strand, and its total length l_pac (the reverse
  // strand occupies [l_pac, 2 l_pac))
  int64_t offset(int contig) const { return off_[contig]; }
  int64_t l_pac() const { return l_pac_; }

 private:
  int k_;
  bool loaded_ = false;
  std::vector<std::vector<uint8_t>> codes_;
  std::vector<int64_t> off_;
  int64_t l_pac_ = 0;
  std::unique_ptr<FmdIndex> fmd_;
};

// The saved FMD-index of a FASTA (fcs-genome index): <fasta>.fcsidx.
std::string fmd_index_path(const std::string& fasta);
// Builds and saves it (bwa index's role); sa_intv 0: automatic.
void build_fmd_index(const std::string& fasta, int sa_intv);

// Aligns FASTQ reads single-end; records (primary, supplementary ones or an
// unmapped one per read) appended to `out` (unsorted).
AlignStats align_reads(const Reference& ref, const KmerIndex& idx, const std::vector<std::string>& names,
                       const std::vector<std::string>& seqs, const std::vector<std::string>& quals,
                       const AlignOptions& opt, std::vector<BamRecord>& out);

// Paired-end batch (bwa mem_sam_pe's role): both mates seeded and extended in
// the same GPU rounds, the insert-size distribution estimated from the batch,
// mates rescued, the best pair chosen against the unpaired best - pen_unpaired,
// then proper-pair / mate flags, RNEXT / PNEXT / TLEN (bwa's 5'-end rule) and
// paired MAPQ.  Records (read 1's, then read 2's per pair) appended to `out`.
AlignStats align_pairs(const Reference& ref, const KmerIndex& idx, const std::vector<std::string>& names,
                       const std::vector<std::string>& seqs1, const std::vector<std::string>& quals1,
                       const std::vector<std::string>& seqs2, const std::vector<std::string>& quals2,
                       const AlignOptions& opt, std::vector<BamRecord>& out);

// One read group of `fcs-genome align` (the work of one reference
// BWAWorker: /root/reference/src/workers/BWAWorker.cpp:94-186).
struct AlignJob {
  std::string ref_path, fq1, fq2, output;  // fq2 empty: single-end
  std::string rg = "sample", sample = "sample", platform = "illumina", library = "sample";
  bool disable_merge = false;  // bwa.num_buckets sorted bucket BAMs (+ .bai, .bed) in the directory `output`
};

// Aligns one read group on the device slots `gpus`: FASTQ chunks
// (bwa.chunk_size reads) go to the slots as they free up, one host thread per
// slot; every chunk's records are kept under the chunk's index and merged in
// chunk order, so the output is the same for any slot list.  Writes the
// sorted BAM + BAI (or the bucket directory) and returns the statistics;
// `report` receives the summary lines.
AlignStats align_fastq(const AlignJob& job, const std::vector<int>& gpus, std::string& report);

// k-way merge of coordinate-sorted BAMs with the same reference dictionary
// into one sorted BAM + BAI; the header keeps the first input's lines and the
// @RG lines of every input (the reference's sambamba merge step,
// src/worker-align.cpp:218-246).
void merge_sorted_bams(const std::vector<std::string>& inputs, const std::string& output);

}  // namespace fcsg

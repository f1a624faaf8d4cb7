// Seed-extension driver of `fcs-genome align` ([EXT]
// bwa bwamem.c mem_chain2aln / mem_reg2aln and bwa.c bwa_gen_cigar2, reached
// in the reference through BWAWorker: /root/reference/src/workers/BWAWorker.cpp:94-186).
//
// Per chunk of reads (bwa.chunk_size): SMEM seeds, up to max_chains chains
// per read, then bwa's extension protocol on the GPU (host/seedext.h: mem_chain2aln's windows, left / right extensions with
// band retry, local vs to-end, mem_reg2aln / bwa_gen_cigar2's global
// alignment for the CIGAR).  NM / MD / AS tags, soft clips, sorted BAM + BAI.
// Seeds are bwa's SMEMs on an FMD-index of the reference (host/fmindex.h),
// chained as bwa's mem_chain does; [EXT] bwa is not vendored, so this is a
// restatement (parity unpinned against bwa itself).
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
  int max_chains = 3;      // candidate chains extended per read
  double drop_ratio = 0.5; // ... with at least this fraction of the best chain's hits (bwa -D)
  std::string rg = "sample", sample = "sample", platform = "illumina", library = "sample";
};

struct AlignStats {
  int64_t reads = 0, mapped = 0, ext_tasks = 0, ext_cells = 0, global_tasks = 0;
  int64_t proper = 0, rescued = 0;  // paired: reads flagged proper pair, mates rescued
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

 private:
  int k_;
  bool loaded_ = false;
  std::vector<std::vector<uint8_t>> codes_;
  std::unique_ptr<FmdIndex> fmd_;
};

// The saved FMD-index of a FASTA (fcs-genome index): <fasta>.fcsidx.
std::string fmd_index_path(const std::string& fasta);
// Builds and saves it (bwa index's role); sa_intv 0: automatic.
void build_fmd_index(const std::string& fasta, int sa_intv);

// Aligns FASTQ reads; records appended to `out` (unsorted).  Up to
// max_chains candidate chains per read are extended; the best by truesc is
// primary, the best other locus sets bwa's single-end MAPQ.
AlignStats align_reads(const Reference& ref, const KmerIndex& idx, const std::vector<std::string>& names,
                       const std::vector<std::string>& seqs, const std::vector<std::string>& quals,
                       const AlignOptions& opt, std::vector<BamRecord>& out);

// Paired-end batch (bwa mem_sam_pe's role): both mates seeded and extended in
// one GPU round, the insert-size distribution estimated from the batch (FR
// pairs, bwa mem_pestat's quartile bounds), mates rescued in the window the
// distribution allows, the best pair chosen by score + insert-size likelihood
// against the unpaired best - 17, then proper-pair / mate flags, RNEXT / PNEXT
// / TLEN and paired MAPQ.  Records (read 1, read 2 per pair) appended to `out`.
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

// Seed-extension driver of `fcs-genome align` ([EXT]
// bwa bwamem.c mem_chain2aln / mem_reg2aln and bwa.c bwa_gen_cigar2, reached
// in the reference through BWAWorker: /root/reference/src/workers/BWAWorker.cpp:94-186).
//
// Per chunk of reads (bwa.chunk_size): exact-match seeds from a k-mer index of
// the reference, the best chain per read, then bwa's extension protocol on the
// GPU (host/seedext.h: mem_chain2aln's windows, left / right extensions with
// band retry, local vs to-end, mem_reg2aln / bwa_gen_cigar2's global
// alignment for the CIGAR).  NM / MD / AS tags, soft clips, sorted BAM + BAI.
// What stands in for bwa [EXT]: seeds are k-mer hits grown to maximal exact
// matches instead of SMEMs from an FM-index, and chaining keeps the diagonal
// with the most hits.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "bam.h"
#include "fasta.h"

namespace fcsg {

struct AlignOptions {
  int gpu = 0;
  int k = 19;            // seed k-mer length (bwa min_seed_len)
  int seed_step = 4;     // query positions sampled for seeds
  int max_occ = 64;      // ignore k-mers with more hits
  int w = 100;           // band width
  int chunk_size = 100000;
  int threads = 16;        // host threads for seeding / task building (bwa.nt)
  std::string rg = "sample", sample = "sample", platform = "illumina", library = "sample";
};

struct AlignStats {
  int64_t reads = 0, mapped = 0, ext_tasks = 0, ext_cells = 0, global_tasks = 0;
  double seconds = 0, gpu_seconds = 0;
};

class KmerIndex {
 public:
  KmerIndex(const Reference& ref, int k);
  // hits of the k-mer starting at codes[0] (2-bit codes, no N): global positions
  std::pair<const uint64_t*, const uint64_t*> lookup(uint64_t key) const;
  int k() const { return k_; }
  // global coordinate ↔ (contig, offset)
  int contig_of(uint64_t g, int64_t& off) const;
  uint64_t global(int contig) const { return starts_[contig]; }
  // the contig's bases as codes 0..4 (A, C, G, T, other)
  const std::vector<uint8_t>& codes(int contig) const { return codes_[contig]; }

 private:
  int k_;
  std::vector<std::vector<uint8_t>> codes_;
  std::vector<uint64_t> keys_, pos_;  // sorted by key
  std::vector<uint64_t> starts_;
};

// Aligns FASTQ reads; records appended to `out` (unsorted).
AlignStats align_reads(const Reference& ref, const KmerIndex& idx, const std::vector<std::string>& names,
                       const std::vector<std::string>& seqs, const std::vector<std::string>& quals,
                       const AlignOptions& opt, std::vector<BamRecord>& out);

}  // namespace fcsg

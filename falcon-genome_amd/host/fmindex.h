// FMD-index of a reference and bwa's super-maximal exact match (SMEM) seeding
// ([EXT] bwa bwt.c bwt_extend / bwt_smem1 and bwamem.c
// mem_collect_intv, reached in the reference through bwa-flow:
// /root/reference/src/workers/BWAWorker.cpp:134-166).
//
// Text T = F . revcomp(F) . $ with F = 5 C_1 5 C_2 ... 5 C_n 5 over the
// alphabet $ = 0, A = 1, C = 2, G = 3, T = 4, 5 = separator / N (a match never
// runs through a 5, and revcomp(F) also starts and ends with 5).  The suffix
// array comes from SA-IS; Occ from 64-position blocks of per-base bit vectors
// plus block counts, interleaved so that one occurrence query reads one cache line.  A bi-interval (k, l, s) holds the SA interval of P
// (k, s) and of revcomp(P) (l, s), so P extends in both directions (bwa's
// bwt_extend); bwt_smem1 finds, for a query position x, the SMEMs overlapping
// x, and mem_collect_intv's three rounds (all SMEMs of length >= min_len,
// re-seeding inside long SMEMs with few occurrences, and the LAST-like forward
// seeds of bwt_seed_strategy1) give the seeds.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "fasta.h"

namespace fcsg {

struct BiInterval {
  int64_t k = 0, l = 0, s = 0;
  int qb = 0, qe = 0;  // query range [qb, qe) of the match
};

class FmdIndex {
 public:
  // contigs as codes 0..4 (A, C, G, T, other).  sa_intv: keep SA[i] for rows
  // i % sa_intv == 0 (bwa's sa_intv; rows in between are located by LF-mapping
  // walks); 0 picks the smallest power of two whose sample fits 8 GiB.
  explicit FmdIndex(const std::vector<std::vector<uint8_t>>& contigs, int sa_intv = 0);
  ~FmdIndex();
  FmdIndex(const FmdIndex&) = delete;
  FmdIndex& operator=(const FmdIndex&) = delete;
  // Writes the index (bwa-index's role: built once, loaded by every align run).
  void save(const std::string& path) const;
  // Memory-maps an index written by save(); null if the file is absent, from
  // another version, or was built from contigs of other lengths or content.
  static std::unique_ptr<FmdIndex> load(const std::string& path, const std::vector<std::vector<uint8_t>>& contigs);
  int64_t size() const { return n_; }
  int sa_intv() const { return intv_; }
  // bwt_smem1: SMEMs of q (codes 0..4) overlapping position x with at least
  // min_intv occurrences; returns the next start position (bwa's return value).
  int smem1(const uint8_t* q, int len, int x, int64_t min_intv, std::vector<BiInterval>& out) const;
  // mem_collect_intv: SMEMs of length >= min_len; re-seeds inside SMEMs longer
  // than split_len with <= split_width occurrences; when max_mem_intv > 0, the
  // third round (bwt_seed_strategy1: from each x, the first forward match of
  // length >= min_len with fewer than max_mem_intv occurrences).  Sorted by
  // query start.
  void collect(const uint8_t* q, int len, int min_len, int split_len, int split_width, int64_t max_mem_intv,
               std::vector<BiInterval>& out) const;
  // Occurrence j (< s) of interval iv: contig, forward-strand offset of the
  // match start, and whether the match is on the reverse strand (then the
  // reverse complement of the query matches the contig at that offset).
  void locate(const BiInterval& iv, int64_t j, int& contig, int64_t& off, bool& rev) const;

 private:
  FmdIndex() = default;
  void extend(const BiInterval& ik, BiInterval ok[5], bool is_back) const;
  void occ4(int64_t i, int64_t o[4]) const;  // occurrences of A, C, G, T in BWT[0, i)
  void set_intv(int c, BiInterval& iv) const;
  int64_t sa_at(int64_t row) const;          // SA[row]: sampled, special, or by LF walk
  static uint64_t text_digest(const std::vector<std::vector<uint8_t>>& contigs);
  int64_t n_ = 0, flen_ = 0;
  int intv_ = 1;
  uint64_t digest_ = 0;
  std::vector<int64_t> C_;               // C_[c] = symbols < c
  // per 64-position block, one 64-byte line: the counts of A, C, G, T before
  // the block, then their bit vectors in it; one extra block holds the totals
  const uint64_t* occ_ = nullptr;
  int64_t nocc_ = 0;                     // uint64 words of occ_
  const uint64_t* sa_ = nullptr;         // SA of rows 0, intv, 2 intv, ...
  int64_t nsa_ = 0;
  // rows whose BWT symbol is $ or a separator (no LF step): (row, SA) sorted by row
  const std::pair<int64_t, int64_t>* special_ = nullptr;
  int64_t nspecial_ = 0;
  std::vector<int64_t> cstart_;          // forward-text start of each contig
  std::vector<int64_t> clen_;
  // storage: built in memory, or the mapped file
  std::vector<uint64_t> occ_store_, sa_store_;
  std::vector<std::pair<int64_t, int64_t>> special_store_;
  void* map_ = nullptr;
  size_t map_len_ = 0;
};

// SA-IS suffix array of s[0, n) over the alphabet [0, K) with s[n-1] == 0
// unique and smallest (64-bit positions: whole human references fit).
void sais(const uint8_t* s, uint64_t* sa, int64_t n, int K);

}  // namespace fcsg

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
#include <string>
#include <vector>

#include "fasta.h"

namespace fcsg {

struct BiInterval {
  int64_t k = 0, l = 0, s = 0;
  int qb = 0, qe = 0;  // query range [qb, qe) of the match
};

class FmdIndex {
 public:
  // contigs as codes 0..4 (A, C, G, T, other)
  explicit FmdIndex(const std::vector<std::vector<uint8_t>>& contigs);
  FmdIndex(const FmdIndex&) = delete;
  FmdIndex& operator=(const FmdIndex&) = delete;
  int64_t size() const { return n_; }
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
  void extend(const BiInterval& ik, BiInterval ok[5], bool is_back) const;
  void occ4(int64_t i, int64_t o[4]) const;  // occurrences of A, C, G, T in BWT[0, i)
  void set_intv(int c, BiInterval& iv) const;
  int64_t n_ = 0, flen_ = 0;
  std::vector<int64_t> C_;               // C_[c] = symbols < c
  std::vector<uint64_t> sa_;             // suffix array
  // per 64-position block, one 64-byte line: the counts of A, C, G, T before
  // the block, then their bit vectors in it; one extra block holds the totals
  std::vector<uint64_t> occ_store_;
  const uint64_t* occ_ = nullptr;        // occ_store_ aligned to 64 bytes
  std::vector<int64_t> cstart_;          // forward-text start of each contig
  std::vector<int64_t> clen_;
};

// SA-IS suffix array of s[0, n) over the alphabet [0, K) with s[n-1] == 0
// unique and smallest (64-bit positions: whole human references fit).
void sais(const uint8_t* s, uint64_t* sa, int64_t n, int K);

}  // namespace fcsg

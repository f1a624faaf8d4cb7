// BAM records and files (SAM/BAM spec §4.2) over BGZF — the read input of
// `fcs-genome htc/mutect2` (the reference hands a BAM path to GATK:
// /root/reference/src/workers/HTCWorker.cpp:51-85) and the output of `align`.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "bgzf.h"

namespace fcsg {

enum CigarOp : uint8_t { kM = 0, kI = 1, kD = 2, kN = 3, kS = 4, kH = 5, kP = 6, kEq = 7, kX = 8 };
inline uint32_t cigar_pack(uint32_t len, CigarOp op) { return (len << 4) | op; }
inline uint32_t cigar_len(uint32_t c) { return c >> 4; }
inline CigarOp cigar_op(uint32_t c) { return (CigarOp)(c & 0xf); }
// Reference bases consumed (M, D, N, =, X).
int64_t cigar_ref_len(const std::vector<uint32_t>& cigar);
std::string cigar_string(const std::vector<uint32_t>& cigar);
std::vector<uint32_t> parse_cigar(const std::string& s);

enum BamFlag : uint16_t {
  kPaired = 0x1, kProperPair = 0x2, kUnmapped = 0x4, kMateUnmapped = 0x8, kReverse = 0x10,
  kMateReverse = 0x20, kRead1 = 0x40, kRead2 = 0x80, kSecondary = 0x100, kQcFail = 0x200,
  kDuplicate = 0x400, kSupplementary = 0x800
};

struct BamRecord {
  int32_t ref_id = -1;
  int32_t pos = -1;  // 0-based leftmost
  uint8_t mapq = 0;
  uint16_t flag = 0;
  int32_t next_ref_id = -1, next_pos = -1, tlen = 0;
  std::string name;
  std::vector<uint32_t> cigar;
  std::string seq;           // ASCII bases (=ACMGRSVTWYHKDBN)
  std::vector<uint8_t> qual; // phred, no +33; empty = absent (0xff in BAM)
  std::string aux;           // raw BAM aux bytes

  int64_t end() const { return pos + cigar_ref_len(cigar); }  // exclusive
  // Aux access.  get_aux_* return false when the tag is absent.
  bool get_aux_string(const char tag[2], std::string& out) const;
  bool get_aux_int(const char tag[2], int64_t& out) const;
  void set_aux_string(const char tag[2], const std::string& v);
  void set_aux_int(const char tag[2], int32_t v);
};

struct BamHeader {
  std::string text;  // SAM header text
  std::vector<std::string> names;
  std::vector<int64_t> lengths;
  int ref_index(const std::string& name) const;
};

// UCSC binning scheme (SAM spec §5.3) for [beg, end).
uint16_t reg2bin(int64_t beg, int64_t end);

class BamWriter {
 public:
  BamWriter(const std::string& path, const BamHeader& h, int level = kBgzfLevel);
  void write(const BamRecord& r);
  // write(r) with the record body already encoded by encode_bam_record(r, body)
  // (callers encode many records on worker threads and write them in order).
  void write_encoded(const BamRecord& r, const std::string& body);
  // write() of every record in order, the encoding spread over the host pool.
  void write_all(const std::vector<const BamRecord*>& recs);
  // Also write <path>.bai at close(), from the records as they are written
  // (coordinate order required): the index bam_index_build would compute,
  // without reading the file back.
  void index_on_close() { index_ = true; }
  void close();
  uint64_t tell() { return bgzf_.tell(); }

 private:
  struct Span {
    int32_t ref_id;
    int64_t beg, end;
    uint64_t u0, u1;
  };
  std::string path_;
  size_t nref_ = 0;
  BgzfWriter bgzf_;
  std::string rec_;
  bool index_ = false, closed_ = false;
  std::vector<Span> spans_;
};

class BamReader {
 public:
  explicit BamReader(const std::string& path);
  const BamHeader& header() const { return hdr_; }
  bool next(BamRecord& r);  // false at end
  // The next record's raw body (after block_size), valid until the next call;
  // false at end.  For readers that decode only the fields they use.
  bool next_raw(const uint8_t*& body, size_t& n);
  uint64_t tell() const { return bgzf_.tell(); }
  void seek(uint64_t voff) { bgzf_.seek(voff); }
  // BgzfReader::use_device: later blocks inflated on GPU `device`; `span` =
  // the estimated compressed bytes of the range read from the next seek
  void use_device(int device, size_t span) { bgzf_.use_device(device, span); }
  int device_chunks() const { return bgzf_.device_chunks(); }
  int host_chunks() const { return bgzf_.host_chunks(); }

 private:
  BgzfReader bgzf_;
  BamHeader hdr_;
  std::vector<uint8_t> buf_;
};

// Serialisation of one record body (after block_size), exposed for tests.
void encode_bam_record(const BamRecord& r, std::string& out);
void decode_bam_record(const uint8_t* p, size_t n, BamRecord& r);
// The l_seq bases of a packed 4-bit BAM SEQ field as ASCII (=ACMGRSVTWYHKDBN).
void decode_bam_seq(const uint8_t* packed, int32_t l_seq, char* out);
// A 'Z' aux value of tag in the raw aux bytes aux[0, n); false when absent.
bool bam_aux_string(const uint8_t* aux, size_t n, const char tag[2], std::string& out);

}  // namespace fcsg

namespace fcsg {

// BAI index of a coordinate-sorted BAM (SAM spec §5.2: UCSC bins + 16 kb
// linear index), so an interval shard seeks straight to its first read.
void bam_index_build(const std::string& bam_path);  // writes <bam>.bai

class BamIndex {
 public:
  explicit BamIndex(const std::string& bai_path);
  // Virtual offset at or before the first record overlapping [beg, ...) on
  // reference tid (0-based beg); 0 if unknown (scan from the start).
  uint64_t seek_offset(int tid, int64_t beg) const;

 private:
  std::vector<std::vector<uint64_t>> linear_;
};

}  // namespace fcsg

// VCF output tail of htc/mutect2: per-shard VCF
// writing, concatenation in shard order, bgzip and a tabix (.tbi) index —
// what the reference runs as VCFConcatWorker → ZIPWorker → TabixWorker
// (/root/reference/src/worker-htc.cpp:153-176).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace fcsg {

struct VcfRecord {
  std::string chrom;
  int64_t pos = 0;  // 1-based
  std::string id = ".";
  std::string ref;
  std::vector<std::string> alts;
  double qual = -1;  // < 0 → "."
  std::string filter = "PASS";
  std::string info = ".";
  std::string format;                // e.g. "GT:AD:DP:GQ:PL"
  std::vector<std::string> samples;  // one formatted column per sample
  std::string to_line() const;
  void append_line(std::string& out) const;  // to_line() appended to out
};

struct VcfHeader {
  std::vector<std::pair<std::string, int64_t>> contigs;
  std::vector<std::string> samples;
  std::vector<std::string> meta;  // extra "##..." lines (INFO/FORMAT/FILTER definitions)
  std::string source = "fcs-genome";
  std::string reference;
  std::string to_text() const;
};

class VcfWriter {
 public:
  VcfWriter(const std::string& path, const VcfHeader& h);
  ~VcfWriter();
  void write(const VcfRecord& r);
  // whole, already formatted record lines
  void write_text(const std::string& lines);
  void close();

 private:
  struct Impl;
  Impl* impl_;
};

// Concatenate shard VCFs (plain text) in order: header of the first, records of all.
void vcf_concat(const std::vector<std::string>& inputs, const std::string& output);
// bgzip a text file.
void bgzip_file(const std::string& input, const std::string& output);
// Build <bgzipped VCF>.tbi (tabix spec: VCF preset, 14-bit binning, 16 kb linear index).
void tabix_index_vcf(const std::string& vcf_gz);
// bgzip_file + tabix_index_vcf in one pass over the plain VCF (the index from
// the plain lines and the writer's block offsets; same files as the two calls).
void bgzip_tabix_file(const std::string& input, const std::string& output);
// vcf_concat(inputs, plain) + bgzip_tabix_file(plain, gz) in one pass over
// the parts (HTC's concat → bgzip → tabix tail as one stage).
// consume_inputs: each input file is removed once it has been read (temporary
// shard parts; their pages leave the page cache inside this pass instead of in
// a separate removal afterwards).
void vcf_concat_bgzip_tabix(const std::vector<std::string>& inputs, const std::string& plain, const std::string& gz,
                            bool consume_inputs = false);

}  // namespace fcsg

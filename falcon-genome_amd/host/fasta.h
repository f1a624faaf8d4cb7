// Reference genome: FASTA in memory plus the .fai and .dict side files the
// reference's tools expect next to ref.fasta (init_contig_intv reads the
// .dict: /root/reference/src/config.cpp:430-470).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace fcsg {

struct Contig {
  std::string name;
  std::string seq;  // upper-case A/C/G/T/N
};

struct Reference {
  std::vector<Contig> contigs;
  int index(const std::string& name) const;
  int64_t total_length() const;
};

Reference load_fasta(const std::string& path);
void write_fasta(const std::string& path, const Reference& ref, int line_width = 60);
// samtools-faidx layout: name, length, offset, line bases, line bytes.
void write_fai(const std::string& fasta_path, const Reference& ref, int line_width = 60);
// Picard CreateSequenceDictionary layout: @HD + one @SQ SN:<name> LN:<len> per contig.
void write_dict(const std::string& dict_path, const Reference& ref);
// <ref>.dict path the way the reference derives it (replace the extension).
std::string dict_path_for(const std::string& ref_path);
// Contig (name, length) list from a .dict file.
std::vector<std::pair<std::string, int64_t>> read_dict(const std::string& dict_path);

}  // namespace fcsg

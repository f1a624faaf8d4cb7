#include "sample_sheet.h"

#include <algorithm>
#include <fstream>

#include "common.h"

namespace fcsg {

namespace {

std::vector<std::string> split_commas(const std::string& s) {
  std::vector<std::string> out;
  size_t p = 0;
  for (;;) {
    const size_t e = s.find(',', p);
    out.push_back(s.substr(p, e == std::string::npos ? std::string::npos : e - p));
    if (e == std::string::npos) return out;
    p = e + 1;
  }
}

bool ends_with(const std::string& s, const std::string& suf) {
  return s.size() >= suf.size() && s.compare(s.size() - suf.size(), suf.size(), suf) == 0;
}

// A header field names a column when it ends with the column's key
// (the reference matches "(.*)(key)", so "#sample_id" names sample_id).
std::string column_of(const std::string& f) {
  for (const char* k : {"sample_id", "fastq1", "fastq2", "platform_id", "library_id", "rg"})
    if (ends_with(f, k)) return k;
  return "";
}

SampleSheetMap from_file(const std::string& path) {
  std::ifstream in(path);
  std::string header;
  if (!std::getline(in, header) || header.empty() || header[0] != '#')
    throw formatError("The header of Sample Sheet : " + path + " is malformatted");
  if (!header.empty() && header.back() == '\r') header.pop_back();
  std::vector<std::string> cols;
  for (const std::string& f : split_commas(header)) cols.push_back(column_of(f));
  SampleSheetMap out;
  std::string line;
  while (std::getline(in, line)) {
    if (!line.empty() && line.back() == '\r') line.pop_back();
    if (line.empty()) continue;
    const std::vector<std::string> v = split_commas(line);
    if (v.size() != cols.size())
      throw formatError("Check PATH : " + path +
                        " :  Number of Fields in Data Block is inconsistent with that of in Header");
    std::string sample;
    SampleDetails d;
    for (size_t k = 0; k < v.size(); ++k) {
      if (cols[k] == "sample_id") sample = v[k];
      else if (cols[k] == "fastq1") d.fastqR1 = v[k];
      else if (cols[k] == "fastq2") d.fastqR2 = v[k];
      else if (cols[k] == "rg") d.ReadGroup = v[k];
      else if (cols[k] == "platform_id") d.Platform = v[k];
      else if (cols[k] == "library_id") d.LibraryID = v[k];
    }
    out[sample].push_back(d);
  }
  if (out.empty()) throw formatError("Sample Sheet " + path + " lists no sample");
  return out;
}

// <dir>/<sample>_<anything>1.fastq.gz with its ...2.fastq.gz mate; read groups
// RG-<sample>_<NN><NN> and libraries LIB<sample>_<NN>, the reference's name
// pattern (src/SampleSheet.cpp:146-200).  The reference restarts NN at 00 and
// 01 only, so a sample's third pair would share the second's read group; the
// per-read-group BAM path comes from that name (align_main: <s>_<RG>.bam), so
// here NN is the pair's index within the sample (00, 01, 02, ...).
SampleSheetMap from_folder(const std::string& dir) {
  std::vector<std::string> r1;
  for (const std::string& f : list_dir(dir, "1.fastq.gz")) r1.push_back(basename_of(f));
  if (r1.empty())
    throw fileNotFound("FASTQ files (fastq.gz) in " + dir + " . Folder maybe empty or no FASTQ files");
  std::sort(r1.begin(), r1.end());
  SampleSheetMap out;
  for (const std::string& f : r1) {
    const size_t us = f.find('_');
    const std::string sample = f.substr(0, us);
    std::string f2 = f;
    f2.replace(f2.rfind("1.fastq.gz"), std::string("1.fastq.gz").size(), "2.fastq.gz");
    const size_t idx = out.count(sample) ? out[sample].size() : 0;
    const std::string nn = (idx < 10 ? "0" : "") + std::to_string(idx);
    SampleDetails d;
    d.fastqR1 = dir + "/" + f;
    d.fastqR2 = dir + "/" + f2;
    d.ReadGroup = "RG-" + sample + "_" + nn + nn;
    d.Platform = "Illumina";
    d.LibraryID = "LIB" + sample + "_" + nn;
    out[sample].push_back(d);
  }
  return out;
}

}  // namespace

SampleSheetMap read_sample_sheet(const std::string& path) {
  if (is_directory(path)) return from_folder(path);
  if (is_regular_file(path)) return from_file(path);
  throw fileNotFound("Input " + path + " is neither a file nor directory");
}

}  // namespace fcsg

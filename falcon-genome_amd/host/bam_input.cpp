#include "bam_input.h"

#include <fstream>
#include <iomanip>
#include <sstream>
#include <stdexcept>

#include "common.h"

namespace fcsg {

namespace {

// <dir>/part-XXXXXX.bam (reference common.cpp:226 get_bucket_fname)
std::string bucket_fname(const std::string& dir, int i) {
  std::ostringstream ss;
  ss << dir << "/part-" << std::setw(6) << std::setfill('0') << i << ".bam";
  return ss.str();
}

// same stem, other extension (reference common.cpp:216 get_fname_by_ext)
std::string with_ext(const std::string& path, const std::string& ext) {
  const size_t slash = path.find_last_of('/');
  const size_t dot = path.find_last_of('.');
  const std::string stem = (dot == std::string::npos || (slash != std::string::npos && dot < slash)) ? path
                                                                                                      : path.substr(0, dot);
  return stem + "." + ext;
}

}  // namespace

std::string bam_index_path(const std::string& bam) {
  if (is_regular_file(bam + ".bai")) return bam + ".bai";
  const std::string b = with_ext(bam, "bai");
  return is_regular_file(b) ? b : "";
}

BamInput::BamInput(const std::string& path) : path_(path) {
  if (!path_exists(path)) throw fileNotFound("input " + path);
  if (is_directory(path)) {
    is_dir_ = true;
    n_bam_ = (int)list_dir(path, ".bam").size();
    n_bai_ = (int)list_dir(path, ".bai").size();
    n_bed_ = (int)list_dir(path, ".bed").size();
    n_list_ = (int)list_dir(path, ".list").size();
  } else {
    n_bam_ = 1;
    if (bam_index_path(path).empty())
      throw fileNotFound("index of input BAM " + path + " (" + with_ext(path, "bai") + " or " + path + ".bai)");
    n_bai_ = 1;
  }
}

BamShard BamInput::merge_region(int contig, int ncontigs, const std::string& temp_dir) const {
  BamShard s;
  if (!is_dir_) {
    s.bams.push_back(path_);
    return s;
  }
  int n_region;
  std::string ext;
  if (n_bed_ == 0) {
    if (n_list_ == 0) throw std::runtime_error("No BED or list files in " + path_);
    if (n_list_ < ncontigs) throw std::runtime_error("Number of List Files less than ncontig");
    n_region = n_list_;
    ext = "list";
  } else {
    if (n_bed_ < ncontigs) throw std::runtime_error("Number of BED Files less than ncontig");
    n_region = n_bed_;
    ext = "bed";
  }
  const int per = n_region / ncontigs;
  const int first = contig * per;
  int last = (contig + 1) * per;
  // reference quirk kept (BamInput.cpp:104-111): when the region files outnumber
  // the BAMs, an odd BAM count drops its last part
  if (last > n_bam_) last = (n_bam_ % 2 == 0) ? n_bam_ : n_bam_ - 1;
  std::vector<std::string> regions;
  for (int i = first; i < last; ++i) {
    const std::string bam = bucket_fname(path_, i);
    const std::string reg = with_ext(bam, ext);
    if (is_regular_file(reg)) regions.push_back(reg);
    s.bams.push_back(bam);
  }
  if (last - first == 1) {
    if (!regions.empty()) s.region = regions[0];
  } else if (last - first > 1) {
    // several parts per shard: their region files concatenated into one (the
    // reference names it .bed whatever the kind; here it keeps the kind's extension)
    create_dir(temp_dir);
    s.region = temp_dir + "/part-" + std::to_string(first) + "_" + std::to_string(last - 1) + "." + ext;
    std::ofstream out(s.region, std::ios::trunc);
    if (!out) throw fileNotFound(s.region + " (cannot write)");
    for (const std::string& r : regions) {
      std::ifstream in(r);
      out << in.rdbuf();
    }
  }
  return s;
}

}  // namespace fcsg

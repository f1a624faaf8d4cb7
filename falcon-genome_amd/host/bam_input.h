// BAM input of htc / mutect2: one indexed BAM file, or a directory of
// part-XXXXXX.bam (+ .bai) files with per-part region files (.bed or GATK
// .list) as `fcs-genome align --disable-merge` leaves them — the reference's
// BamInput (/root/reference/src/BamInput.cpp:27-149,
// include/fcs-genome/BamInput.h).  Shard `contig` of gatk.ncontigs takes the
// parts [contig * n, (contig + 1) * n), n = region files / ncontigs, and the
// union of their region files (merged into one file when there are several).
#pragma once

#include <string>
#include <vector>

namespace fcsg {

struct BamShard {
  std::vector<std::string> bams;  // BAM files of the shard (each indexed)
  std::string region;             // region file of the shard ("" = none: the reference runs without -L)
};

class BamInput {
 public:
  // Throws fileNotFound if the path does not exist or a single BAM has no
  // index (<x>.bai or <x>.bam.bai; the reference logs and exits 1).
  explicit BamInput(const std::string& path);
  bool is_dir() const { return is_dir_; }
  const std::string& path() const { return path_; }
  int bam_files() const { return n_bam_; }
  int bed_files() const { return n_bed_; }
  int list_files() const { return n_list_; }
  // The BAMs and region file of shard `contig`; merged region files are
  // written under temp_dir.  Errors as the reference: no BED/list files, or
  // fewer region files than shards (std::runtime_error).
  BamShard merge_region(int contig, int ncontigs, const std::string& temp_dir) const;

 private:
  std::string path_;
  bool is_dir_ = false;
  int n_bam_ = 0, n_bai_ = 0, n_bed_ = 0, n_list_ = 0;
};

// <path>.bai or <path without .bam>.bai, whichever exists ("" if neither).
std::string bam_index_path(const std::string& bam);

}  // namespace fcsg

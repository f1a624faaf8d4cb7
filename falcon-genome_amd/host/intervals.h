// Interval shards of htc/mutect2: the reference's init_contig_intv
// (/root/reference/src/config.cpp:420-511) splits the genome from ref.dict
// into gatk.ncontigs pieces of ceil(total/ncontigs) positions and writes one
// part-XXXXXX.list per shard ("chr:lb-ub" per line, 1-based inclusive); the
// shards are then the unit of work dealt to executors (and here to GPUs).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace fcsg {

struct Interval {
  std::string chrom;
  int64_t lb = 0, ub = 0;  // 1-based, inclusive
};

// In-memory partition (same arithmetic as init_contig_intv).  Contigs after
// the 25th are dropped when skip_pseudo_chr (gatk.skip_pseudo_chr).
std::vector<std::vector<Interval>> partition_contigs(const std::vector<std::pair<std::string, int64_t>>& dict,
                                                    int ncontigs, bool skip_pseudo_chr = true);
// Writes <temp_dir>/intv_<n>/part-XXXXXX.list and returns their paths.
std::vector<std::string> init_contig_intv(const std::string& ref_path, int ncontigs, const std::string& temp_dir,
                                          bool skip_pseudo_chr = true);
std::vector<Interval> read_interval_list(const std::string& path);
void write_interval_list(const std::string& path, const std::vector<Interval>& iv);
// BED (chrom, 0-based start, end; half-open) as 1-based inclusive intervals;
// "track"/"browser"/"#" lines skipped.
std::vector<Interval> read_bed(const std::string& path);
// A region file by extension: .bed as BED, anything else as a GATK interval list.
std::vector<Interval> read_regions(const std::string& path);
// GATK's -isr INTERSECTION of several -L sets: the positions every set holds,
// as sorted, merged intervals (contig order = first appearance in sets[0]).
std::vector<Interval> intersect_interval_sets(const std::vector<std::vector<Interval>>& sets);

}  // namespace fcsg

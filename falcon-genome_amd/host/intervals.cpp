#include "intervals.h"

#include <algorithm>
#include <fstream>
#include <map>
#include <sstream>

#include "common.h"
#include "fasta.h"

namespace fcsg {

std::vector<std::vector<Interval>> partition_contigs(const std::vector<std::pair<std::string, int64_t>>& dict_in,
                                                    int ncontigs, bool skip_pseudo_chr) {
  if (ncontigs <= 0) throw invalidParam("gatk.ncontigs must be positive");
  std::vector<std::pair<std::string, int64_t>> dict;
  int64_t total = 0;
  for (size_t i = 0; i < dict_in.size(); ++i) {
    if (skip_pseudo_chr && i >= 25) break;
    dict.push_back(dict_in[i]);
    total += dict_in[i].second;
  }
  std::vector<std::vector<Interval>> parts(ncontigs);
  // positions per part, the remaining budget of the current part, 1-based bounds
  const int64_t per = (total + ncontigs - 1) / ncontigs;
  int64_t remain = per, lb = 1;
  int part = 0;
  for (const auto& c : dict) {
    int64_t npos = c.second;
    while (npos > remain) {  // the contig spills over the current part
      const int64_t ub = remain + lb - 1;
      parts[part].push_back({c.first, lb, ub});
      lb = ub + 1;
      npos -= remain;
      remain = per;
      ++part;
      if (part >= ncontigs) throw internalError("interval partition overflow");
    }
    if (npos > 0) {
      parts[part].push_back({c.first, lb, c.second});
      remain -= npos;
      lb = 1;
    }
  }
  return parts;
}

std::vector<std::string> init_contig_intv(const std::string& ref_path, int ncontigs, const std::string& temp_dir,
                                          bool skip_pseudo_chr) {
  const std::string dir = temp_dir + "/intv_" + std::to_string(ncontigs);
  create_dir(dir);
  const std::string dict = dict_path_for(ref_path);
  if (!path_exists(dict)) throw fileNotFound(dict);
  const auto parts = partition_contigs(read_dict(dict), ncontigs, skip_pseudo_chr);
  std::vector<std::string> paths(ncontigs);
  for (int i = 0; i < ncontigs; ++i) {
    paths[i] = get_contig_fname(dir, i, "list", "part-");
    write_interval_list(paths[i], parts[i]);
  }
  return paths;
}

std::vector<Interval> read_interval_list(const std::string& path) {
  std::ifstream in(path);
  if (!in) throw fileNotFound(path);
  std::vector<Interval> out;
  std::string line;
  while (std::getline(in, line)) {
    if (line.empty() || line[0] == '@' || line[0] == '#') continue;
    const size_t colon = line.rfind(':');
    const size_t dash = line.rfind('-');
    Interval iv;
    if (colon == std::string::npos) {  // bare contig name: the whole contig
      iv.chrom = line;
      iv.lb = 1;
      iv.ub = INT64_MAX;
    } else {
      if (dash == std::string::npos || dash < colon) throw invalidParam("interval '" + line + "' in " + path);
      iv.chrom = line.substr(0, colon);
      iv.lb = std::stoll(line.substr(colon + 1, dash - colon - 1));
      iv.ub = std::stoll(line.substr(dash + 1));
    }
    out.push_back(iv);
  }
  return out;
}

void write_interval_list(const std::string& path, const std::vector<Interval>& iv) {
  std::ofstream out(path);
  if (!out) throw fileNotFound(path + " (cannot write)");
  for (const Interval& i : iv) out << i.chrom << ':' << i.lb << '-' << i.ub << '\n';
}

std::vector<Interval> read_bed(const std::string& path) {
  std::ifstream in(path);
  if (!in) throw fileNotFound(path);
  std::vector<Interval> out;
  std::string line;
  while (std::getline(in, line)) {
    if (line.empty() || line[0] == '#' || line.rfind("track", 0) == 0 || line.rfind("browser", 0) == 0) continue;
    std::istringstream ss(line);
    Interval iv;
    int64_t b0 = 0, e0 = 0;
    if (!(ss >> iv.chrom >> b0 >> e0) || b0 < 0 || e0 < b0) throw invalidParam("BED line '" + line + "' in " + path);
    if (e0 == b0) continue;  // empty
    iv.lb = b0 + 1;
    iv.ub = e0;
    out.push_back(iv);
  }
  return out;
}

std::vector<Interval> read_regions(const std::string& path) {
  const size_t n = path.size();
  if (n >= 4 && path.compare(n - 4, 4, ".bed") == 0) return read_bed(path);
  return read_interval_list(path);
}

namespace {

// sorted, merged (overlapping or adjacent) intervals per contig
std::map<std::string, std::vector<std::pair<int64_t, int64_t>>> normalise(const std::vector<Interval>& iv) {
  std::map<std::string, std::vector<std::pair<int64_t, int64_t>>> m;
  for (const Interval& i : iv) m[i.chrom].emplace_back(i.lb, i.ub);
  for (auto& [c, v] : m) {
    std::sort(v.begin(), v.end());
    std::vector<std::pair<int64_t, int64_t>> o;
    for (const auto& x : v) {
      if (!o.empty() && x.first <= o.back().second + 1) o.back().second = std::max(o.back().second, x.second);
      else o.push_back(x);
    }
    v = std::move(o);
  }
  return m;
}

}  // namespace

std::vector<Interval> intersect_interval_sets(const std::vector<std::vector<Interval>>& sets) {
  if (sets.empty()) return {};
  std::vector<std::string> order;
  for (const Interval& i : sets[0])
    if (std::find(order.begin(), order.end(), i.chrom) == order.end()) order.push_back(i.chrom);
  auto acc = normalise(sets[0]);
  for (size_t k = 1; k < sets.size(); ++k) {
    auto other = normalise(sets[k]);
    for (auto& [c, v] : acc) {
      const auto it = other.find(c);
      std::vector<std::pair<int64_t, int64_t>> o;
      if (it != other.end()) {
        const auto& w = it->second;
        size_t a = 0, b = 0;
        while (a < v.size() && b < w.size()) {
          const int64_t lo = std::max(v[a].first, w[b].first), hi = std::min(v[a].second, w[b].second);
          if (lo <= hi) o.emplace_back(lo, hi);
          if (v[a].second < w[b].second) ++a;
          else ++b;
        }
      }
      v = std::move(o);
    }
  }
  std::vector<Interval> out;
  for (const std::string& c : order)
    for (const auto& x : acc[c]) out.push_back({c, x.first, x.second});
  return out;
}

}  // namespace fcsg

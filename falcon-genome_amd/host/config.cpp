#include "config.h"

#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <thread>

#include "common.h"
#include "fcship.h"

namespace fcsg {

Config& Config::global() {
  static Config c;
  return c;
}

void Config::declare(const std::string& key, const std::string& def, const std::string& help) {
  kv_[key] = Entry{def, help, false};
}

void Config::init(const std::string& root_dir) {
  kv_.clear();
  const unsigned ncpu = host_cpus();
  // common (config.cpp:274-296)
  declare("temp_dir", "/tmp", "temp dir for fast access");
  declare("log_dir", "./log", "log dir");
  declare("hosts", "", "host list for scale-out mode");
  declare("latency_mode", "false", "enable latency mode");
  // tools (config.cpp:298-353), the GATK/BWA knobs that still mean something here
  declare("bwa.verbose", "0", "verbose level of the aligner");
  declare("bwa.nt", "-1", "host threads of the aligner (-1: all)");
  declare("bwa.num_buckets", "1024", "number of BAM buckets");
  declare("bwa.chunk_size", "100000", "reads per SW batch handed to the GPU");
  declare("bwa.gpu_slots", "0", "aligner host threads (chunks in flight) per GPU; 0: host threads / GPUs, at least 4");
  declare("gatk.intv.path", "", "default path to existing contig intervals");
  declare("gatk.ncontigs", "32", "contig partition num in htc/mutect2");
  declare("gatk.nprocs", std::to_string(std::min(32u, ncpu)), "default concurrent shard tasks");
  declare("gatk.htc.nprocs", "", "concurrent shard tasks in htc (default gatk.nprocs)");
  declare("gatk.mutect2.nprocs", "", "concurrent shard tasks in mutect2 (default gatk.nprocs)");
  declare("gatk.skip_pseudo_chr", "true", "skip pseudo chromosome intervals (contigs after the 25th)");
  // accelerator (replaces bwa.use_fpga / bwa.fpga.bit_path / blaze.nam_path)
  declare("gpu.devices", "all", "GPU ordinals for shard tasks: all | comma list");
  declare("gpu.phmm.batch_regions", "4096", "active regions per PairHMM device pass");
  declare("gpu.phmm.combine_ms", "0", "ms a shard's PairHMM pass waits to merge with other shards' (0: no merging)");
  declare("gpu.phmm.rescue", "true", "fp64 rescue of pairs whose fp32 likelihood underflows (GKL)");
  declare("gpu.release_early", "true",
          "release the GPUs beside the VCF tail once the callers are done (their teardown off the critical path)");
  declare("gpu.warmup_help", "false",
          "a shard whose PairHMM pass finds the GPU runtime still coming up runs a queued shard meanwhile");
  declare("gpu.bam_inflate", "false",
          "inflate a calling window's BAM blocks on the GPU (fcs_bgzf_inflate) instead of host libdeflate");
  // caller knobs (GATK HaplotypeCaller / Mutect2 argument defaults)
  declare("htc.min_base_quality", "10", "min base quality counted as evidence of activity");
  declare("htc.base_quality_threshold", "18", "PairHMM: base quals below this become 6");
  declare("htc.pcr_indel_model", "CONSERVATIVE",
          "GATK --pcr-indel-model: NONE, HOSTILE, AGGRESSIVE, CONSERVATIVE (gap-open caps in tandem repeats)");
  declare("htc.min_mapq", "20", "reads below this mapping quality are ignored");
  declare("htc.active_fraction", "0.15", "mismatch/indel fraction that makes a site active");
  declare("mutect2.active_fraction", "0.10", "tumor mismatch/indel fraction that makes a site active (mutect2)");
  declare("htc.padding", "50", "bases added either side of an active site");
  declare("htc.max_region", "300", "max active region length");
  declare("htc.max_reads_per_region", "250", "downsampling cap per region");
  declare("mutect2.tlod", "6.3", "tumor LOD threshold");
  declare("mutect2.nlod", "2.2", "normal LOD threshold");
  declare("root_dir", root_dir, "install root");

  if (!root_dir.empty()) load_file(root_dir + "/fcs-genome.conf", false);  // 3rd priority
  load_file("fcs-genome.conf", true);                                       // 2nd priority
  load_env();                                                               // 1st priority

  const char* user = std::getenv("USER");
  temp_dir_ = get_string("temp_dir") + "/fcs-genome-" + (user ? user : "root") + "-" + std::to_string(getpid());
}

void Config::load_file(const std::string& path, bool override_existing) {
  std::ifstream in(path);
  if (!in) return;
  std::string line, section;
  while (std::getline(in, line)) {
    const size_t hash = line.find('#');
    if (hash != std::string::npos) line.resize(hash);
    auto trim = [](std::string s) {
      s.erase(0, s.find_first_not_of(" \t\r"));
      s.erase(s.find_last_not_of(" \t\r") + 1);
      return s;
    };
    line = trim(line);
    if (line.empty()) continue;
    if (line.front() == '[' && line.back() == ']') {
      section = trim(line.substr(1, line.size() - 2));
      continue;
    }
    const size_t eq = line.find('=');
    if (eq == std::string::npos) throw invalidParam("config line '" + line + "' in " + path);
    std::string key = trim(line.substr(0, eq));
    if (!section.empty()) key = section + "." + key;
    if (!kv_.count(key)) throw invalidParam("unknown config key '" + key + "' in " + path);
    Entry& e = kv_[key];
    if (e.set_explicitly && !override_existing) continue;
    e.value = trim(line.substr(eq + 1));
    e.set_explicitly = true;
  }
}

void Config::load_env() {
  for (auto& kv : kv_) {
    std::string env = "FCS_" + kv.first;
    std::transform(env.begin(), env.end(), env.begin(), [](char c) { return c == '.' ? '_' : (char)std::toupper(c); });
    const char* v = std::getenv(env.c_str());
    if (v) {
      kv.second.value = v;
      kv.second.set_explicitly = true;
    }
  }
}

bool Config::has(const std::string& key) const {
  auto it = kv_.find(key);
  return it != kv_.end() && !it->second.value.empty();
}

std::string Config::get_string(const std::string& key) const {
  auto it = kv_.find(key);
  if (it == kv_.end()) throw invalidParam("unknown config key " + key);
  return it->second.value;
}

int Config::get_int(const std::string& key) const {
  const std::string v = get_string(key);
  try {
    return std::stoi(v);
  } catch (...) {
    throw invalidParam(key + " = '" + v + "' is not an integer");
  }
}

int Config::get_int(const std::string& key, const std::string& fallback) const {
  return has(key) ? get_int(key) : get_int(fallback);
}

bool Config::get_bool(const std::string& key) const {
  std::string v = get_string(key);
  std::transform(v.begin(), v.end(), v.begin(), ::tolower);
  if (v == "true" || v == "1" || v == "yes" || v == "on") return true;
  if (v == "false" || v == "0" || v == "no" || v == "off" || v.empty()) return false;
  throw invalidParam(key + " = '" + v + "' is not a boolean");
}

void Config::set(const std::string& key, const std::string& value) {
  if (!kv_.count(key)) throw invalidParam("unknown config key " + key);
  kv_[key].value = value;
  kv_[key].set_explicitly = true;
}

std::string Config::dump() const {
  std::ostringstream ss;
  for (const auto& kv : kv_)
    ss << "  " << kv.first << " = " << kv.second.value << (kv.second.help.empty() ? "" : "    # " + kv.second.help)
       << '\n';
  return ss.str();
}

std::vector<int> Config::gpu_devices() const {
  const std::string v = get_string("gpu.devices");
  std::vector<int> out;
  if (v.empty() || v == "all") {
    const int n = fcs_device_count();
    for (int i = 0; i < n; ++i) out.push_back(i);
    return out;
  }
  std::stringstream ss(v);
  std::string tok;
  while (std::getline(ss, tok, ',')) {
    if (tok.empty()) continue;
    try {
      out.push_back(std::stoi(tok));
    } catch (...) {
      throw invalidParam("gpu.devices = '" + v + "'");
    }
  }
  return out;
}

}  // namespace fcsg

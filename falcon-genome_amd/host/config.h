// fcs-genome configuration keys (reference:
// /root/reference/src/config.cpp:239-353).  Same key names and precedence as
// the reference — environment FCS_<key> first, then ./fcs-genome.conf, then
// <install root>/fcs-genome.conf, then built-in defaults — with
// `gatk.<tool>.nprocs` falling back to `gatk.nprocs` as in set_config
// (config.cpp:155-180).  The accelerator keys are gpu.* (the reference's
// bwa.use_fpga / blaze.* select the FPGA; here the GPU is the only backend).
#pragma once

#include <map>
#include <string>
#include <vector>

namespace fcsg {

class Config {
 public:
  // Built-in defaults + files + environment, in the reference's order.
  static Config& global();
  void init(const std::string& root_dir);
  void load_file(const std::string& path, bool override_existing);
  void load_env();

  bool has(const std::string& key) const;
  std::string get_string(const std::string& key) const;
  int get_int(const std::string& key) const;
  bool get_bool(const std::string& key) const;
  // `key` if set explicitly, else `fallback` (the reference's get_config<T>(arg, def_arg)).
  int get_int(const std::string& key, const std::string& fallback) const;
  void set(const std::string& key, const std::string& value);
  std::string dump() const;  // `fcs-genome conf`
  // GPU ordinals from gpu.devices ("all" = every visible device, else "0,2,3").
  std::vector<int> gpu_devices() const;
  std::string temp_dir() const { return temp_dir_; }

 private:
  struct Entry {
    std::string value, help;
    bool set_explicitly = false;
  };
  void declare(const std::string& key, const std::string& def, const std::string& help);
  std::map<std::string, Entry> kv_;
  std::string temp_dir_;
};

inline Config& conf() { return Config::global(); }

}  // namespace fcsg

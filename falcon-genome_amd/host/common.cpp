#include "common.h"

#include <dirent.h>
#include <sched.h>
#include <sys/stat.h>
#include <sys/statvfs.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <thread>

namespace fcsg {

namespace {
std::atomic<int> g_interrupt{0};
}
bool interrupted() { return g_interrupt.load(std::memory_order_relaxed) != 0; }
int interrupt_signal() { return g_interrupt.load(); }
void set_interrupted(int sig) { g_interrupt.store(sig); }

bool path_exists(const std::string& p) {
  struct stat st;
  return ::stat(p.c_str(), &st) == 0;
}

bool is_regular_file(const std::string& p) {
  struct stat st;
  return ::stat(p.c_str(), &st) == 0 && S_ISREG(st.st_mode);
}

bool is_directory(const std::string& p) {
  struct stat st;
  return ::stat(p.c_str(), &st) == 0 && S_ISDIR(st.st_mode);
}

void create_dir(const std::string& p) {
  if (p.empty()) return;
  std::string cur;
  std::stringstream ss(p);
  std::string part;
  if (p[0] == '/') cur = "/";
  while (std::getline(ss, part, '/')) {
    if (part.empty()) continue;
    cur += part + "/";
    if (::mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST)
      throw internalError("[E::fcsg] cannot create directory " + cur + ": " + std::strerror(errno));
  }
}

void remove_path(const std::string& p) {
  if (is_directory(p)) {
    if (DIR* d = ::opendir(p.c_str())) {
      while (dirent* e = ::readdir(d)) {
        const std::string n = e->d_name;
        if (n == "." || n == "..") continue;
        remove_path(p + "/" + n);
      }
      ::closedir(d);
    }
    ::rmdir(p.c_str());
  } else {
    ::unlink(p.c_str());
  }
}

std::vector<std::string> list_dir(const std::string& p, const std::string& suffix) {
  std::vector<std::string> out;
  if (DIR* d = ::opendir(p.c_str())) {
    while (dirent* e = ::readdir(d)) {
      const std::string n = e->d_name;
      if (n == "." || n == "..") continue;
      if (!suffix.empty() && (n.size() < suffix.size() || n.compare(n.size() - suffix.size(), suffix.size(), suffix)))
        continue;
      out.push_back(p + "/" + n);
    }
    ::closedir(d);
  }
  std::sort(out.begin(), out.end());
  return out;
}

uint64_t file_size(const std::string& p) {
  struct stat st;
  return ::stat(p.c_str(), &st) == 0 ? (uint64_t)st.st_size : 0;
}

uint64_t available_space(const std::string& dir) {
  struct statvfs v;
  if (::statvfs(dir.c_str(), &v) != 0) return UINT64_MAX;  // unknown: do not block the run
  return (uint64_t)v.f_bavail * v.f_frsize;
}

std::string read_file(const std::string& p) {
  std::ifstream in(p, std::ios::binary);
  if (!in) throw fileNotFound(p);
  std::ostringstream ss;
  ss << in.rdbuf();
  return ss.str();
}

void write_file(const std::string& p, const std::string& data) {
  std::ofstream out(p, std::ios::binary);
  if (!out) throw fileNotFound(p + " (cannot write)");
  out << data;
}

unsigned host_cpus() {
  static const unsigned n = [] {
    // FCS_HOST_THREADS: an explicit share (several GPU ranks on one node)
    if (const char* e = std::getenv("FCS_HOST_THREADS"); e && std::atoi(e) > 0) return (unsigned)std::atoi(e);
    unsigned c = std::max(1u, std::thread::hardware_concurrency());
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) c = std::min(c, (unsigned)std::max(1, CPU_COUNT(&set)));
    // cgroup v2 "quota period" (or "max period"); v1 cfs_quota_us / cfs_period_us
    long long quota = -1, period = 0;
    if (std::FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
      char q[32] = {0};
      if (std::fscanf(f, "%31s %lld", q, &period) == 2 && std::strcmp(q, "max") != 0) quota = std::atoll(q);
      std::fclose(f);
    } else if (std::FILE* g = std::fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r")) {
      if (std::fscanf(g, "%lld", &quota) != 1) quota = -1;
      std::fclose(g);
      if (std::FILE* h = std::fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r")) {
        if (std::fscanf(h, "%lld", &period) != 1) period = 0;
        std::fclose(h);
      }
    }
    if (quota > 0 && period > 0) c = std::min(c, (unsigned)std::max(1LL, (quota + period - 1) / period));
    return c;
  }();
  return n;
}

}  // namespace fcsg

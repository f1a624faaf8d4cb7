// Shared host-side definitions of the fcs-genome orchestrator (SURVEY.md §8f
// row f1): the error types the reference's drivers throw and catch
// (/root/reference/include/fcs-genome/common.h:27-67), file-name helpers
// (get_contig_fname, :232-245) and timing.
#pragma once

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <iomanip>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace fcsg {

// Static split of [0, n) over up to `threads` std::threads (one thread for
// fewer than 256 items per extra thread).
template <typename F>
void parallel_for(size_t n, int threads, F&& fn) {
  const size_t nt = std::max<size_t>(1, std::min<size_t>((size_t)std::max(threads, 1), n / 256 + 1));
  if (nt == 1) {
    for (size_t i = 0; i < n; ++i) fn(i);
    return;
  }
  std::vector<std::thread> th;
  for (size_t t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      for (size_t i = n * t / nt; i < n * (t + 1) / nt; ++i) fn(i);
    });
  for (auto& x : th) x.join();
}

// Dynamic split of [0, n) over up to `threads` std::threads: each thread takes
// the next item from a shared counter (for a few coarse items of uneven cost).
template <typename F>
void parallel_tasks(size_t n, int threads, F&& fn) {
  const size_t nt = std::min<size_t>((size_t)std::max(threads, 1), n);
  if (nt <= 1) {
    for (size_t i = 0; i < n; ++i) fn(i);
    return;
  }
  std::atomic<size_t> next{0};
  std::vector<std::thread> th;
  for (size_t t = 0; t < nt; ++t)
    th.emplace_back([&] {
      for (size_t i; (i = next.fetch_add(1, std::memory_order_relaxed)) < n;) fn(i);
    });
  for (auto& x : th) x.join();
}

// Exit codes of `fcs-genome` (reference main.cpp: helpRequest → 0 after help,
// invalidParam/pathEmpty/fileNotFound → 1, failedCommand → 4, internal → 3).
class helpRequest : public std::runtime_error {
 public:
  helpRequest() : std::runtime_error("") {}
};
class silentExit : public std::runtime_error {
 public:
  silentExit() : std::runtime_error("") {}
};
class invalidParam : public std::runtime_error {
 public:
  explicit invalidParam(const std::string& what) : std::runtime_error("Invalid parameter: " + what) {}
};
class fileNotFound : public std::runtime_error {
 public:
  explicit fileNotFound(const std::string& what) : std::runtime_error("Cannot find " + what) {}
};
class failedCommand : public std::runtime_error {
 public:
  explicit failedCommand(const std::string& what) : std::runtime_error(what) {}
};
class internalError : public std::runtime_error {
 public:
  explicit internalError(const std::string& what) : std::runtime_error(what) {}
};
class pathEmpty : public std::runtime_error {
 public:
  explicit pathEmpty(const std::string& what) : std::runtime_error("Path of " + what + " is empty") {}
};
// Raised where work notices that SIGINT/SIGTERM/SIGHUP arrived (interrupted());
// fcs-genome then removes its temp dir and exits 130.
class interruptedError : public failedCommand {
 public:
  interruptedError() : failedCommand("[E::fcs-genome] interrupted") {}
};
class formatError : public std::runtime_error {
 public:
  explicit formatError(const std::string& what) : std::runtime_error("[E::fcsg] " + what) {}
};

// CPUs this process may use: the hardware threads, narrowed by the affinity
// mask and by a cgroup CPU quota (a GPU box grants 16 of its many cores;
// hardware_concurrency alone reports them all).  FCS_HOST_THREADS > 0 sets it
// (ranks sharing a node each take their share).
unsigned host_cpus();

inline uint64_t now_us() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::microseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// <base>/<prefix><contig as 6 digits>.<ext> — the reference's per-shard file naming.
inline std::string get_contig_fname(const std::string& base, int contig, const std::string& ext = "bam",
                                    const std::string& prefix = "part-") {
  std::ostringstream ss;
  ss << base << "/" << prefix << std::setw(6) << std::setfill('0') << contig << "." << ext;
  return ss.str();
}

inline std::string basename_of(const std::string& path) {
  const size_t k = path.find_last_of('/');
  return k == std::string::npos ? path : path.substr(k + 1);
}

// Interrupt state (the reference's sigint_handler, src/main.cpp:43-54): set by
// the signal thread of main(), polled by the Executor before it starts a task
// and by the in-process workers between device passes.
bool interrupted();
int interrupt_signal();
void set_interrupted(int sig);

bool path_exists(const std::string& p);
bool is_regular_file(const std::string& p);
bool is_directory(const std::string& p);
void create_dir(const std::string& p);   // mkdir -p
void remove_path(const std::string& p);  // rm -rf
std::vector<std::string> list_dir(const std::string& p, const std::string& suffix = "");
std::string read_file(const std::string& p);
uint64_t file_size(const std::string& p);         // 0 if absent
uint64_t available_space(const std::string& dir);  // bytes free to this user (statvfs)
void write_file(const std::string& p, const std::string& data);

}  // namespace fcsg

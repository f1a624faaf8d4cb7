// Python-free driver for the ThreadSanitizer build of the host orchestrator
// (tools/sanitize.sh).  TSAN cannot run under the Python test suite (torch and
// the HIP runtime deadlock under its interposition), so this exercises the
// host's threaded code through the same C hooks the CPU tests use
// (falcon-genome_amd/host/capi.cpp):
//   * Executor stages: many tasks over a slot pool, repeated, plus a failing
//     stage (failedCommand path, findError over the part logs);
//   * concurrent format work from several threads (BGZF round trips, read
//     preparation with the PCR indel model) beside the stages.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

extern "C" {
int fcsg_run_stage(const char* cmd_fmt, int n_tasks, int n_threads, const char* gpus_csv, const char* log_dir,
                   char* buf, int cap);
int fcsg_bgzf_compress_file(const char* in, const char* out);
int fcsg_bgzf_decompress_file(const char* in, const char* out);
int fcsg_prepare_read(const char* bases, const uint8_t* quals, int len, const char* bi, const char* bd, int mapq,
                      int threshold, int pcr_model, uint8_t* bq, uint8_t* iq, uint8_t* dq, uint8_t* gcp);
}

static int fails = 0;

static void check(bool ok, const char* what) {
  if (!ok) {
    std::fprintf(stderr, "FAIL: %s\n", what);
    __atomic_add_fetch(&fails, 1, __ATOMIC_RELAXED);
  }
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp/fcs_host_race";
  std::vector<std::thread> side;
  for (int t = 0; t < 4; ++t)
    side.emplace_back([t, &dir] {
      const std::string a = dir + "/in" + std::to_string(t), z = a + ".gz", b = a + ".out";
      FILE* f = std::fopen(a.c_str(), "w");
      for (int i = 0; i < 20000; ++i) std::fprintf(f, "line %d of thread %d\n", i, t);
      std::fclose(f);
      for (int r = 0; r < 5; ++r) {
        check(fcsg_bgzf_compress_file(a.c_str(), z.c_str()) == 0, "bgzf compress");
        check(fcsg_bgzf_decompress_file(z.c_str(), b.c_str()) == 0, "bgzf decompress");
      }
      const char* bases = "GATTTTTTTTCAGACACACACACGT";
      const int n = (int)std::strlen(bases);
      std::vector<uint8_t> q(n, 30), o[4];
      for (auto& v : o) v.assign(n, 0);
      for (int r = 0; r < 200; ++r)
        check(fcsg_prepare_read(bases, q.data(), n, nullptr, nullptr, 60, 18, 3, o[0].data(), o[1].data(),
                                o[2].data(), o[3].data()) == 0,
              "prepare_read");
    });
  char buf[1 << 14];
  for (int r = 0; r < 4; ++r) {
    const std::string logs = dir + "/stage" + std::to_string(r);
    check(fcsg_run_stage("true %d", 96, 12, "0,1,2,3", logs.c_str(), buf, sizeof buf) == 0, "stage");
  }
  const std::string logs = dir + "/fail";
  check(fcsg_run_stage("sh -c 'if [ %d -eq 7 ]; then echo \"[E::x] boom\"; exit 2; fi'", 32, 8, "", logs.c_str(), buf,
                       sizeof buf) == 4,
        "failing stage returns 4");
  for (auto& t : side) t.join();
  std::printf("host_race: %s\n", fails ? "FAILED" : "ok");
  return fails ? 1 : 0;
}

// Worker / Stage / Executor / BackgroundExecutor — the reference's task
// runtime (/root/reference/include/fcs-genome/{Worker,Executor,BackgroundExecutor}.h,
// src/Executor.cpp, src/BackgroundExecutor.cpp) re-done on std::thread with
// GPU slots.
//
// Same contract: a Worker is check()ed on the caller thread when its Stage
// starts (a throw aborts the run), then setup() + run + teardown() on a pool
// thread with a per-task log file; Stages run in order, the tasks of one
// Stage concurrently on `num_executors` threads; any failed task makes the
// Stage collect its "[E::" / "##### ERROR" log lines (LogUtils::findError) and
// throw failedCommand.  Differences: a Worker may run in-process (run()) instead of
// a shell command (cmd_), and every task gets a GPU slot — the device
// ordinal gpu.devices[job_id % n], the rule the reference applies to hosts
// (Executor.cpp:262).
#pragma once

#include <atomic>
#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <queue>
#include <string>
#include <thread>
#include <vector>

namespace fcsg {

struct TaskContext {
  int job_id = 0;
  int gpu = -1;          // device ordinal, -1 when no GPU is configured
  std::string log_path;  // the task's log file
  std::FILE* log = nullptr;
};

class Worker {
 public:
  Worker(int num_proc = 1, int num_t = 1, std::vector<std::string> extra_opts = {}, std::string task_name = "");
  virtual ~Worker() = default;
  virtual void check() {}
  virtual void setup() {}
  virtual void teardown() {}
  // Default: run cmd_ through the shell with the log as stdout/stderr and
  // FCS_GPU_DEVICE set to the slot.  In-process workers override this.
  virtual int run(TaskContext& ctx);
  std::string getCommand() const { return cmd_; }
  std::string getTaskName() const { return task_name_; }

 protected:
  std::string cmd_;
  std::map<std::string, std::vector<std::string>> extra_opts_;  // "--key value" pairs, as the reference parses them
  int num_process_, num_thread_;
  std::string task_name_;
};
typedef std::shared_ptr<Worker> Worker_ptr;

class Executor;

class Stage {
 public:
  Stage(Executor* ex, std::string label);
  void add(Worker_ptr w);
  void run();
  const std::string& label() const { return label_; }

 private:
  Executor* ex_;
  std::vector<Worker_ptr> tasks_;
  std::vector<std::string> logs_;
  std::string label_;
  std::map<int, int> status_;
  std::mutex mu_;
};
typedef std::shared_ptr<Stage> Stage_ptr;

// Runs one task still queued on the running Executor on the calling thread;
// false when none is queued (or no Executor runs).  A shard that would block
// for a device still coming up does other shards' host work meanwhile.
bool executor_help_once();
// Set by the device warm-up once the GPU runtime and sessions are up.
void set_devices_warm(bool warm);
bool devices_warm();

class Executor {
 public:
  Executor(std::string job_name, int num_executors = 1, std::vector<int> gpus = {});
  ~Executor();
  void addTask(Worker_ptr w, const std::string& sample_id = "", bool wait_for_prev = false);
  void run();
  int execute(Worker_ptr w, const std::string& log);
  void post(std::function<void()> fn);
  bool try_run_one();
  std::string get_log_name(const std::string& label, int idx = -1);
  const std::string& job_name() const { return job_name_; }
  int num_executors() const { return num_executors_; }

 private:
  void stop();
  std::string job_name_;
  int num_executors_;
  std::vector<int> gpus_;
  std::string log_dir_;
  std::queue<Stage_ptr> stages_;
  std::atomic<int> job_id_{0};
  std::vector<std::thread> pool_;
  std::queue<std::function<void()>> q_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool stopping_ = false;
};

// A worker kept alive in a background thread for the life of the object (the
// reference runs the FPGA NAM daemon this way: src/BackgroundExecutor.cpp:13-74).
class BackgroundExecutor {
 public:
  BackgroundExecutor(std::string job_name, Worker_ptr w, int gpu = -1);
  ~BackgroundExecutor();
  int status() const { return status_.load(); }  // -1 running, else the worker's return code
  void wait();

 private:
  std::string job_name_;
  Worker_ptr worker_;
  std::thread th_;
  std::atomic<int> status_{-1};
};

namespace LogUtils {
// "##### ERROR" and "[E::" lines of the logs; the message shared by all
// logs, else the last line of the first failing log (src/LogUtils.cpp:10-40).
std::string findError(const std::vector<std::string>& logs);
}

}  // namespace fcsg

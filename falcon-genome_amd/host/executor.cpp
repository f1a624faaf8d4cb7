#include "executor.h"

#include <sys/wait.h>

#include <cctype>
#include <cstdio>
#include <ctime>
#include <fstream>
#include <future>
#include <iostream>
#include <sstream>

#include "common.h"
#include "config.h"

namespace fcsg {

// ------------------------------------------------------------------ Worker
Worker::Worker(int num_proc, int num_t, std::vector<std::string> extra_opts, std::string task_name)
    : num_process_(num_proc), num_thread_(num_t), task_name_(std::move(task_name)) {
  // "--key value" / "--flag" tokens (reference Worker.h:28-51); -nct is dropped as there
  for (const std::string& opt : extra_opts) {
    std::istringstream ss(opt);
    std::vector<std::string> toks;
    for (std::string t; ss >> t;) toks.push_back(t);
    for (size_t i = 0; i < toks.size(); ++i) {
      const std::string& key = toks[i];
      if (key.empty() || key[0] != '-') continue;
      std::string value;
      if (i + 1 < toks.size() && toks[i + 1][0] != '-') value = toks[++i];
      if (key != "-nct") extra_opts_[key].push_back(value);
    }
  }
}

int Worker::run(TaskContext& ctx) {
  if (cmd_.empty()) return 0;
  std::string cmd = "{ ";
  if (ctx.gpu >= 0) cmd += "export FCS_GPU_DEVICE=" + std::to_string(ctx.gpu) + "; ";
  cmd += cmd_ + "; } >> '" + ctx.log_path + "' 2>&1";
  const int rc = std::system(cmd.c_str());
  if (rc == -1) return 1;
  return WIFEXITED(rc) ? WEXITSTATUS(rc) : 128 + (WIFSIGNALED(rc) ? WTERMSIG(rc) : 0);
}

// ------------------------------------------------------------------ Stage
Stage::Stage(Executor* ex, std::string label) : ex_(ex), label_(std::move(label)) {}

void Stage::add(Worker_ptr w) {
  logs_.push_back(ex_->get_log_name(label_, (int)logs_.size()));
  tasks_.push_back(std::move(w));
}

void Stage::run() {
  const uint64_t t0 = now_us();
  std::cerr << "[fcs-genome] Start doing " << label_ << std::endl;
  std::vector<std::future<void>> pending;
  for (size_t i = 0; i < tasks_.size(); ++i) {
    if (interrupted()) break;
    tasks_[i]->check();  // caller thread, like the reference: a bad argument aborts before anything runs
    auto done = std::make_shared<std::promise<void>>();
    pending.push_back(done->get_future());
    ex_->post([this, i, done] {
      const int rc = ex_->execute(tasks_[i], logs_[i]);
      if (rc) {
        std::lock_guard<std::mutex> g(mu_);
        status_[(int)i] = rc;
      }
      done->set_value();
    });
  }
  for (auto& f : pending) f.wait();
  if (interrupted()) throw interruptedError();
  const std::string stage_log = ex_->get_log_name(label_);
  {
    std::ofstream out(stage_log, std::ios::app);
    for (const std::string& l : logs_) {
      std::ifstream in(l);
      if (in) out << in.rdbuf();
    }
  }
  if (!status_.empty()) {
    const std::string match = LogUtils::findError(logs_);
    std::cerr << "[fcs-genome] ERROR: " << label_ << " failed, please check log: " << stage_log << " for details."
              << std::endl;
    if (!match.empty()) std::cerr << "Potential errors:\n" << match;
    throw failedCommand(label_ + " failed");
  }
  std::cerr << "[fcs-genome] " << label_ << " finishes in " << (now_us() - t0) / 1e6 << " seconds" << std::endl;
  for (const std::string& l : logs_) std::remove(l.c_str());
}

// ------------------------------------------------------------------ Executor
Executor::Executor(std::string job_name, int num_executors, std::vector<int> gpus)
    : job_name_(std::move(job_name)), num_executors_(std::max(1, num_executors)), gpus_(std::move(gpus)) {
  log_dir_ = conf().has("log_dir") ? conf().get_string("log_dir") : "./log";
  create_dir(log_dir_);
  for (int i = 0; i < num_executors_; ++i)
    pool_.emplace_back([this] {
      for (;;) {
        std::function<void()> fn;
        {
          std::unique_lock<std::mutex> lk(mu_);
          cv_.wait(lk, [this] { return stopping_ || !q_.empty(); });
          if (q_.empty()) return;
          fn = std::move(q_.front());
          q_.pop();
        }
        fn();
      }
    });
}

Executor::~Executor() { stop(); }

void Executor::stop() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stopping_ = true;
  }
  cv_.notify_all();
  for (auto& t : pool_)
    if (t.joinable()) t.join();
  pool_.clear();
}

namespace {
std::atomic<Executor*> g_running{nullptr};
std::atomic<bool> g_devices_warm{false};
}  // namespace

bool executor_help_once() {
  Executor* ex = g_running.load();
  return ex && ex->try_run_one();
}
void set_devices_warm(bool warm) { g_devices_warm.store(warm); }
bool devices_warm() { return g_devices_warm.load(); }

bool Executor::try_run_one() {
  std::function<void()> fn;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (stopping_ || q_.empty()) return false;
    fn = std::move(q_.front());
    q_.pop();
  }
  fn();
  return true;
}

void Executor::post(std::function<void()> fn) {
  {
    std::lock_guard<std::mutex> g(mu_);
    q_.push(std::move(fn));
  }
  cv_.notify_one();
}

void Executor::addTask(Worker_ptr w, const std::string& sample_id, bool wait_for_prev) {
  if (stages_.empty() || wait_for_prev) {
    std::string label = w->getTaskName();
    if (!sample_id.empty()) label += " " + sample_id;
    stages_.push(std::make_shared<Stage>(this, label));
  }
  stages_.back()->add(std::move(w));
}

void Executor::run() {
  struct Running {
    Executor* self;
    explicit Running(Executor* e) : self(e) { g_running.store(e); }
    ~Running() {
      Executor* e = self;
      g_running.compare_exchange_strong(e, nullptr);
    }
  } running(this);
  while (!stages_.empty()) {
    stages_.front()->run();
    stages_.pop();
  }
}

int Executor::execute(Worker_ptr w, const std::string& log) {
  if (interrupted()) return 128 + interrupt_signal();  // queued but not started
  TaskContext ctx;
  ctx.job_id = job_id_.fetch_add(1);
  ctx.gpu = gpus_.empty() ? -1 : gpus_[ctx.job_id % gpus_.size()];
  ctx.log_path = log;
  ctx.log = std::fopen(log.c_str(), "a");
  int rc = 0;
  try {
    w->setup();
    rc = w->run(ctx);
    w->teardown();
  } catch (const std::exception& e) {
    if (ctx.log) std::fprintf(ctx.log, "[E::%s] %s\n", w->getTaskName().c_str(), e.what());
    rc = 1;
  }
  if (ctx.log) std::fclose(ctx.log);
  return rc;
}

std::string Executor::get_log_name(const std::string& label, int idx) {
  std::string name;
  for (char c : label) name += (c == ' ') ? '-' : (char)std::tolower((unsigned char)c);
  const std::time_t ts = std::time(nullptr);
  std::tm tm{};
  localtime_r(&ts, &tm);
  char buf[32];
  std::strftime(buf, sizeof buf, "%Y%m%d-%H%M%S", &tm);
  std::string p = log_dir_ + "/" + name + "-" + buf;
  if (idx >= 0) p += ".part-" + std::to_string(idx);
  return p + ".log";
}

// ------------------------------------------------------------------ BackgroundExecutor
BackgroundExecutor::BackgroundExecutor(std::string job_name, Worker_ptr w, int gpu)
    : job_name_(std::move(job_name)), worker_(std::move(w)) {
  th_ = std::thread([this, gpu] {
    TaskContext ctx;
    ctx.gpu = gpu;
    ctx.log_path = "/dev/null";
    int rc = 1;
    try {
      worker_->setup();
      rc = worker_->run(ctx);
      worker_->teardown();
    } catch (const std::exception& e) {
      std::cerr << "[E::" << job_name_ << "] " << e.what() << std::endl;
    }
    status_.store(rc);
  });
}

void BackgroundExecutor::wait() {
  if (th_.joinable()) th_.join();
}

BackgroundExecutor::~BackgroundExecutor() { wait(); }

// ------------------------------------------------------------------ LogUtils
std::string LogUtils::findError(const std::vector<std::string>& logs) {
  std::string message;
  for (const std::string& path : logs) {
    std::ifstream in(path);
    std::string match, last, line;
    while (std::getline(in, line)) {
      if (line.find("##### ERROR") != std::string::npos || line.find("[E::") != std::string::npos)
        match += line + "\n";
      else if (!line.empty())
        last = line + "\n";
    }
    if (message.empty()) message = match.empty() ? last : match;
    else if (message != match) return match;
  }
  return message;
}

}  // namespace fcsg

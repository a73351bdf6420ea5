// mipipe native runtime (module ``mipipe._runtime``): process-group supervisor, DAG scheduler
// core and multi-threaded record loader.  Host C++ only (no GPU code), bound in bindings.cpp.
#pragma once
#include <sys/types.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

namespace mipipe_rt {

// ---------------------------------------------------------------- process supervisor
class ProcessGroup {
 public:
  explicit ProcessGroup(bool echo) : echo_(echo) {}
  ~ProcessGroup();
  // argv[0] is looked up on PATH; env as "K=V" strings (empty: inherit); returns child index
  int spawn(const std::vector<std::string>& argv, const std::vector<std::string>& env,
            const std::string& cwd, const std::string& log_path, const std::string& prefix);
  int wait(double timeout, double grace);
  void signal_all(int sig);
  void interrupt() { interrupted_ = true; }
  std::vector<int> exit_codes() const;
  std::vector<int> pids() const;
  int failed_rank() const { return failed_rank_; }

 private:
  struct Child {
    pid_t pid = -1;
    int out_fd = -1;
    FILE* log = nullptr;
    std::string prefix;
    bool exited = false;
    int code = -1;
  };
  void pump_loop();
  bool reap_nonblocking();
  void reap_all_blocking();
  bool echo_;
  std::vector<Child> children_;
  std::mutex mu_;
  std::thread pump_;
  std::atomic<bool> stop_pump_{false}, all_spawned_{false}, interrupted_{false};
  bool finished_ = false;
  int failed_rank_ = -1;
};

// ---------------------------------------------------------------- DAG scheduler core
class DagScheduler {
 public:
  enum State { kPending = 0, kRunning = 1, kSucceeded = 2, kCached = 3, kSkipped = 4,
               kFailed = 5, kCancelled = 6 };
  DagScheduler(int n, const std::vector<std::vector<int>>& deps,
               const std::vector<bool>& always_run, bool fail_fast);
  std::vector<int> next_ready();
  void complete(int i, int state);
  std::vector<int> take_cancelled();
  // a failure outside this DAG (fail-fast across sub-DAGs): cancel pending non-exit tasks
  void mark_external_failure() { any_failed_ = true; }
  bool finished() const;
  bool deadlocked() const;
  const std::vector<int>& states() const { return state_; }
  const std::vector<int>& topo_order() const { return topo_; }

 private:
  int n_;
  std::vector<std::vector<int>> deps_;
  std::vector<bool> always_;
  bool fail_fast_;
  std::vector<int> state_;
  std::vector<std::vector<int>> children_;
  std::vector<int> topo_, cancelled_;
  int running_ = 0;
  bool any_failed_ = false;
};

// ---------------------------------------------------------------- record loader
struct LoaderConfig {
  std::vector<std::string> files;
  int header_bytes = 0;
  int label_bytes = 1;
  int C = 3, H = 32, W = 32;
  int batch = 128;
  bool train = true;
  int pad = 4;
  bool flip = true;
  std::vector<float> mean, stdv;
  uint64_t seed = 0;
  int workers = 8;
  int prefetch = 4;
  bool drop_last = false;
};

class RecordLoader {
 public:
  explicit RecordLoader(const LoaderConfig& cfg);
  ~RecordLoader();
  int64_t size() const { return total_; }
  void start_epoch(const std::vector<int64_t>& indices, int64_t epoch);
  // copies the next batch to x [n,C,H,W] f32 / y [n] i64; returns n (0 = epoch exhausted)
  int next(float* x, int64_t* y);
  int64_t batches_per_epoch() const;
  const uint8_t* record(int64_t i) const;

 private:
  void worker();
  void fill(int slot, int64_t b, const std::vector<int64_t>& idx, int64_t epoch);
  LoaderConfig cfg_;
  size_t rec_bytes_ = 0;
  std::vector<std::pair<const uint8_t*, size_t>> maps_;
  std::vector<int64_t> file_start_;
  int64_t total_ = 0;
  std::vector<std::vector<float>> slot_x_;
  std::vector<std::vector<int64_t>> slot_y_;
  std::vector<int> slot_n_;
  std::vector<int64_t> slot_batch_;
  std::vector<int64_t> indices_;
  int64_t epoch_ = 0, nbatches_ = 0, next_produce_ = 0, next_consume_ = 0;
  uint64_t gen_ = 0;
  int busy_ = 0;
  bool shutdown_ = false;
  std::mutex mu_;
  std::condition_variable cv_work_, cv_slot_;
  std::vector<std::thread> threads_;
};

}  // namespace mipipe_rt

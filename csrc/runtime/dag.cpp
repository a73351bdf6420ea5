// Native DAG scheduler core of the local pipeline orchestrator (mipipe.orchestrator).
//
// The reference submits its compiled kfp-v2 job spec to Vertex AI Pipelines, whose backend
// executes the DAG in dependency order and reports per-step state (SURVEY.md §2.1 O9,
// pytorch-pipeline.ipynb:253-258).  This is the state machine of that executor:
//   PENDING -> RUNNING -> {SUCCEEDED, CACHED, SKIPPED, FAILED}, or PENDING -> CANCELLED
// with kfp semantics: a task whose upstream FAILED/was CANCELLED is CANCELLED unless its
// trigger policy is ALL_UPSTREAM_TASKS_COMPLETED (exit handlers); with fail-fast, the first
// failure cancels every task not yet started (same exception for exit handlers).
// Cycles are rejected at construction.  The Python runner asks for ready tasks, runs them on
// its worker pool and reports completions.
#include "runtime.hpp"

#include <stdexcept>

namespace mipipe_rt {

DagScheduler::DagScheduler(int n, const std::vector<std::vector<int>>& deps,
                           const std::vector<bool>& always_run, bool fail_fast)
    : n_(n), deps_(deps), always_(always_run), fail_fast_(fail_fast), state_(n, kPending),
      children_(n) {
  if ((int)deps_.size() != n || (int)always_.size() != n)
    throw std::invalid_argument("deps/always_run must have one entry per task");
  for (int i = 0; i < n; ++i)
    for (int d : deps_[i]) {
      if (d < 0 || d >= n) throw std::invalid_argument("dependency index out of range");
      children_[d].push_back(i);
    }
  // Kahn's algorithm: reject cycles, record a topological order
  std::vector<int> indeg(n, 0);
  for (int i = 0; i < n; ++i) indeg[i] = (int)deps_[i].size();
  std::vector<int> q;
  for (int i = 0; i < n; ++i)
    if (indeg[i] == 0) q.push_back(i);
  for (size_t h = 0; h < q.size(); ++h)
    for (int c : children_[q[h]])
      if (--indeg[c] == 0) q.push_back(c);
  if ((int)q.size() != n) throw std::invalid_argument("pipeline DAG has a cycle");
  topo_ = q;
}

static bool terminal(int s) { return s >= DagScheduler::kSucceeded; }

std::vector<int> DagScheduler::next_ready() {
  std::vector<int> out;
  bool changed = true;
  while (changed) {  // cancellations can unblock further cancellations
    changed = false;
    for (int i : topo_) {
      if (state_[i] != kPending) continue;
      bool ready = true, up_failed = false;
      for (int d : deps_[i]) {
        if (!terminal(state_[d])) ready = false;
        if (state_[d] == kFailed || state_[d] == kCancelled) up_failed = true;
      }
      if (!ready) continue;
      if (!always_[i] && (up_failed || (fail_fast_ && any_failed_))) {
        state_[i] = kCancelled;
        cancelled_.push_back(i);
        changed = true;
        continue;
      }
      state_[i] = kRunning;
      ++running_;
      out.push_back(i);
    }
  }
  return out;
}

void DagScheduler::complete(int i, int st) {
  if (i < 0 || i >= n_) throw std::invalid_argument("task index out of range");
  if (state_[i] != kRunning) throw std::logic_error("complete() on a task that is not running");
  if (st < kSucceeded || st == kCancelled) throw std::invalid_argument("bad completion state");
  state_[i] = st;
  --running_;
  if (st == kFailed) any_failed_ = true;
}

std::vector<int> DagScheduler::take_cancelled() {
  std::vector<int> r;
  r.swap(cancelled_);
  return r;
}

bool DagScheduler::finished() const {
  for (int s : state_)
    if (!terminal(s)) return false;
  return true;
}

bool DagScheduler::deadlocked() const {
  // nothing running, nothing dispatchable, not finished  (cannot happen for a DAG; guards bugs)
  if (running_ > 0 || finished()) return false;
  for (int i = 0; i < n_; ++i) {
    if (state_[i] != kPending) continue;
    bool ready = true;
    for (int d : deps_[i]) ready &= terminal(state_[d]);
    if (ready) return false;
  }
  return true;
}

}  // namespace mipipe_rt

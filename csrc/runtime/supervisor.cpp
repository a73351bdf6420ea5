// Native process-group supervisor for the local job launcher (mipipe.launch).
//
// Replaces what the reference gets from Vertex AI's CustomTrainingJob (pytorch-pipeline.ipynb
// :167-196: replica_count=3 VMs, each running task.py) and from torch.multiprocessing.spawn
// (task.py:124): start every rank of a job, stream each rank's stdout/stderr to its log file
// (and optionally to ours, prefixed), and enforce fail-fast semantics — the first rank that
// exits non-zero (or the job timeout) tears the whole group down with SIGTERM, then SIGKILL
// after a grace period, like torchrun's elastic agent.
//
// Children are started with posix_spawnp (no fork of a possibly GPU-initialised parent
// image) in their own session, so a signal to the process group also reaches grandchildren
// (e.g. torchrun's workers).
#include "runtime.hpp"

#include <errno.h>
#include <fcntl.h>
#include <poll.h>
#include <signal.h>
#include <spawn.h>
#include <string.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <stdexcept>
#include <thread>

extern char** environ;

namespace mipipe_rt {

static double now_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

ProcessGroup::~ProcessGroup() {
  if (!finished_) {
    signal_all(SIGKILL);
    reap_all_blocking();
  }
  stop_pump_ = true;
  if (pump_.joinable()) pump_.join();
  for (auto& c : children_) {
    if (c.out_fd >= 0) close(c.out_fd);
    if (c.log != nullptr) fclose(c.log);
  }
}

int ProcessGroup::spawn(const std::vector<std::string>& argv, const std::vector<std::string>& env,
                        const std::string& cwd, const std::string& log_path,
                        const std::string& prefix) {
  if (argv.empty()) throw std::invalid_argument("empty argv");
  int fds[2];
  if (pipe2(fds, O_CLOEXEC) != 0) throw std::runtime_error(std::string("pipe: ") + strerror(errno));
  posix_spawn_file_actions_t fa;
  posix_spawn_file_actions_init(&fa);
  posix_spawn_file_actions_adddup2(&fa, fds[1], 1);
  posix_spawn_file_actions_adddup2(&fa, fds[1], 2);
  posix_spawn_file_actions_addclose(&fa, fds[0]);
  if (!cwd.empty()) {
#if defined(__GLIBC__) && (__GLIBC__ > 2 || (__GLIBC__ == 2 && __GLIBC_MINOR__ >= 29))
    posix_spawn_file_actions_addchdir_np(&fa, cwd.c_str());
#endif
  }
  posix_spawnattr_t at;
  posix_spawnattr_init(&at);
  short flags = POSIX_SPAWN_SETSID | POSIX_SPAWN_SETSIGMASK | POSIX_SPAWN_SETSIGDEF;
  posix_spawnattr_setflags(&at, flags);
  sigset_t empty, all;
  sigemptyset(&empty);
  sigfillset(&all);
  posix_spawnattr_setsigmask(&at, &empty);
  posix_spawnattr_setsigdefault(&at, &all);

  std::vector<char*> av, ev;
  for (auto& s : argv) av.push_back(const_cast<char*>(s.c_str()));
  av.push_back(nullptr);
  for (auto& s : env) ev.push_back(const_cast<char*>(s.c_str()));
  ev.push_back(nullptr);
  pid_t pid = -1;
  int rc = posix_spawnp(&pid, av[0], &fa, &at, av.data(), env.empty() ? environ : ev.data());
  posix_spawn_file_actions_destroy(&fa);
  posix_spawnattr_destroy(&at);
  close(fds[1]);
  if (rc != 0) {
    close(fds[0]);
    throw std::runtime_error("spawn " + argv[0] + ": " + strerror(rc));
  }
  Child c;
  c.pid = pid;
  c.out_fd = fds[0];
  fcntl(c.out_fd, F_SETFL, O_NONBLOCK);
  c.prefix = prefix;
  if (!log_path.empty()) c.log = fopen(log_path.c_str(), "a");
  {
    std::lock_guard<std::mutex> g(mu_);
    children_.push_back(c);
  }
  if (!pump_.joinable()) pump_ = std::thread([this] { pump_loop(); });
  return (int)children_.size() - 1;
}

// Drain every child's pipe into its log (+ our stdout, line-prefixed) until all are closed.
void ProcessGroup::pump_loop() {
  std::vector<std::string> partial;
  while (!stop_pump_) {
    std::vector<pollfd> pfds;
    std::vector<int> idx;
    {
      std::lock_guard<std::mutex> g(mu_);
      partial.resize(children_.size());
      for (size_t i = 0; i < children_.size(); ++i)
        if (children_[i].out_fd >= 0) {
          pfds.push_back({children_[i].out_fd, POLLIN, 0});
          idx.push_back((int)i);
        }
    }
    if (pfds.empty()) {
      if (all_spawned_) break;
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
      continue;
    }
    int n = poll(pfds.data(), pfds.size(), 50);
    if (n <= 0) continue;
    for (size_t k = 0; k < pfds.size(); ++k) {
      if (!(pfds[k].revents & (POLLIN | POLLHUP | POLLERR))) continue;
      Child& c = children_[idx[k]];
      char buf[8192];
      ssize_t r = read(c.out_fd, buf, sizeof(buf));
      if (r > 0) {
        if (c.log) {
          fwrite(buf, 1, r, c.log);
          fflush(c.log);
        }
        if (echo_) {
          std::string& p = partial[idx[k]];
          p.append(buf, r);
          size_t pos;
          while ((pos = p.find('\n')) != std::string::npos) {
            std::string line = c.prefix + p.substr(0, pos + 1);
            fwrite(line.data(), 1, line.size(), stdout);
            p.erase(0, pos + 1);
          }
          fflush(stdout);
        }
      } else if (r == 0 || (r < 0 && errno != EAGAIN && errno != EINTR)) {
        std::lock_guard<std::mutex> g(mu_);
        if (echo_ && !partial[idx[k]].empty()) {
          std::string line = c.prefix + partial[idx[k]] + "\n";
          fwrite(line.data(), 1, line.size(), stdout);
          fflush(stdout);
          partial[idx[k]].clear();
        }
        close(c.out_fd);
        c.out_fd = -1;
      }
    }
  }
}

void ProcessGroup::signal_all(int sig) {
  for (auto& c : children_)
    if (!c.exited) {
      if (killpg(c.pid, sig) != 0) kill(c.pid, sig);
    }
}

static int decode_status(int st) {
  if (WIFEXITED(st)) return WEXITSTATUS(st);
  if (WIFSIGNALED(st)) return 128 + WTERMSIG(st);
  return 255;
}

bool ProcessGroup::reap_nonblocking() {
  bool all = true;
  for (auto& c : children_) {
    if (c.exited) continue;
    int st = 0;
    pid_t r = waitpid(c.pid, &st, WNOHANG);
    if (r == c.pid) {
      c.exited = true;
      c.code = decode_status(st);
    } else {
      all = false;
    }
  }
  return all;
}

void ProcessGroup::reap_all_blocking() {
  for (auto& c : children_) {
    if (c.exited) continue;
    int st = 0;
    if (waitpid(c.pid, &st, 0) == c.pid) c.code = decode_status(st);
    c.exited = true;
  }
}

// Wait for the group.  Returns 0 when every child exited 0; otherwise the exit code of the
// first failing child (128+signal for signalled children), 124 on timeout.  On failure the
// remaining children are SIGTERMed, then SIGKILLed after `grace` seconds.
int ProcessGroup::wait(double timeout, double grace) {
  all_spawned_ = true;
  const double t0 = now_s();
  int first_fail = 0;
  while (true) {
    bool all = reap_nonblocking();
    for (auto& c : children_)
      if (c.exited && c.code != 0 && first_fail == 0) {
        first_fail = c.code;
        failed_rank_ = (int)(&c - &children_[0]);
      }
    if (first_fail != 0 || all) break;
    if (timeout > 0 && now_s() - t0 > timeout) {
      first_fail = 124;
      break;
    }
    if (interrupted_) {
      first_fail = 130;
      break;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
  if (first_fail != 0) {
    signal_all(SIGTERM);
    const double d = now_s() + grace;
    while (now_s() < d && !reap_nonblocking()) std::this_thread::sleep_for(std::chrono::milliseconds(20));
    signal_all(SIGKILL);
    reap_all_blocking();
  }
  finished_ = true;
  // let the pump drain what the children wrote before they exited
  const double d = now_s() + 5.0;
  while (now_s() < d) {
    bool open = false;
    {
      std::lock_guard<std::mutex> g(mu_);
      for (auto& c : children_) open |= c.out_fd >= 0;
    }
    if (!open) break;
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  }
  return first_fail;
}

std::vector<int> ProcessGroup::exit_codes() const {
  std::vector<int> r;
  for (auto& c : children_) r.push_back(c.exited ? c.code : -1);
  return r;
}

std::vector<int> ProcessGroup::pids() const {
  std::vector<int> r;
  for (auto& c : children_) r.push_back((int)c.pid);
  return r;
}

}  // namespace mipipe_rt

#include "sync/transport.h"

#include <fcntl.h>
#include <poll.h>
#include <signal.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cstring>
#include <chrono>
#include <thread>

#include "core/strutil.h"
#include "platform/platform.h"

namespace ds {
namespace sync {

static long mono_us() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1000000L + ts.tv_nsec / 1000;
}

// ------------------------------------------------------------------ local shell

namespace {
class LocalShell : public Shell {
 public:
  std::unique_ptr<Process> p;
  int in() override { return p->stdin_fd(); }
  int out() override { return p->stdout_fd(); }
  int err() override { return p->stderr_fd(); }
  bool alive() override { return p && p->running(); }
  void terminate() override {
    if (p) p->kill(SIGKILL);
  }
  void close() override {
    if (!p) return;
    if (p->stdin_fd() >= 0) {
      write_all(p->stdin_fd(), "exit\n");
      p->close_stdin();
    }
    if (p->wait(500) < 0) {
      p->kill(SIGKILL);
      p->wait(2000);
    }
    p->close_stdout();
    p->close_stderr();
  }
  ~LocalShell() override { close(); }
};
}  // namespace

LocalShellTransport::LocalShellTransport(std::string cwd, std::string root_prefix,
                                         std::map<std::string, std::string> env)
    : cwd_(std::move(cwd)), root_(std::move(root_prefix)), env_(std::move(env)) {}

std::unique_ptr<Shell> LocalShellTransport::open(const std::vector<std::string>& argv) {
  auto s = std::make_unique<LocalShell>();
  s->p = std::make_unique<Process>();
  ProcOptions o;
  o.cwd = cwd_;
  o.env = env_;
  if (!s->p->start(argv, o)) throw std::runtime_error("start " + join(argv, " ") + ": " + s->p->error());
  // 1 MiB pipes (the Linux default for unprivileged processes' maximum) instead of 64 KiB:
  // bulk transfers cross the pipe in 16x fewer wake-ups
  for (int fd : {s->p->stdin_fd(), s->p->stdout_fd()}) plat::grow_pipe(fd, 1 << 20);
  return s;
}

// ------------------------------------------------------------------ fault injection

namespace {
class FaultShell : public Shell {
 public:
  std::unique_ptr<Shell> inner;
  FaultPlan plan;
  Fd in_r, in_w, out_r, out_w, err_r, err_w;
  std::thread t_in, t_out, t_err;
  std::atomic<bool> dead{false};

  void start() {
    make_pipe(&in_r, &in_w);
    make_pipe(&out_r, &out_w);
    make_pipe(&err_r, &err_w);
    t_in = std::thread([this] {
      size_t total = 0;
      char buf[4096];
      while (true) {
        ssize_t n = read_some(in_r.get(), buf, sizeof(buf));
        if (n <= 0) break;
        if (plan.kill_after_stdin_bytes && total + (size_t)n >= plan.kill_after_stdin_bytes) {
          size_t take = plan.kill_after_stdin_bytes - total;
          if (take) write_all(inner->in(), buf, take);
          kill_all();
          break;
        }
        total += (size_t)n;
        if (!write_all(inner->in(), buf, (size_t)n)) break;
      }
      in_r.reset();  // the stream is gone: writers get EPIPE instead of blocking on a full pipe
    });
    t_out = std::thread([this] {
      char buf[4096];
      bool corrupted = plan.corrupt_from.empty();
      std::string pending;
      size_t total = 0;
      while (true) {
        ssize_t n = read_some(inner->out(), buf, sizeof(buf));
        if (n <= 0) break;
        if (plan.kill_after_stdout_bytes && total + (size_t)n >= plan.kill_after_stdout_bytes) {
          size_t take = plan.kill_after_stdout_bytes - total;
          if (take) write_all(out_w.get(), buf, take);
          kill_all();
          break;
        }
        total += (size_t)n;
        if (plan.stall_stdout_ms) std::this_thread::sleep_for(std::chrono::milliseconds(plan.stall_stdout_ms));
        std::string chunk(buf, (size_t)n);
        if (!corrupted) {
          size_t pos = chunk.find(plan.corrupt_from);
          if (pos != std::string::npos) {
            chunk.replace(pos, plan.corrupt_from.size(), plan.corrupt_to);
            corrupted = true;
          }
        }
        if (!write_all(out_w.get(), chunk)) break;
      }
      out_w.reset();
    });
    t_err = std::thread([this] {
      char buf[4096];
      while (true) {
        ssize_t n = read_some(inner->err(), buf, sizeof(buf));
        if (n <= 0) break;
        if (!write_all(err_w.get(), buf, (size_t)n)) break;
      }
      err_w.reset();
    });
  }
  void kill_all() {
    if (dead.exchange(true)) return;
    inner->terminate();
  }
  int in() override { return in_w.get(); }
  int out() override { return out_r.get(); }
  int err() override { return err_r.get(); }
  bool alive() override { return !dead && inner->alive(); }
  void terminate() override { kill_all(); }
  void close() override {
    kill_all();
    in_w.reset();
    if (t_in.joinable()) t_in.join();
    if (t_out.joinable()) t_out.join();
    if (t_err.joinable()) t_err.join();
    inner->close();
  }
  ~FaultShell() override { close(); }
};
}  // namespace

std::unique_ptr<Shell> FaultInjectingTransport::open(const std::vector<std::string>& argv) {
  ++opened_;
  auto inner = inner_->open(argv);
  if (plan_.only_shell && plan_.only_shell != opened_) return inner;
  auto s = std::make_unique<FaultShell>();
  s->inner = std::move(inner);
  s->plan = plan_;
  s->start();
  return s;
}

// ------------------------------------------------------------------ line reader

void LineReader::reset(int fd) {
  fd_ = fd;
  buf_.clear();
  eof_ = false;
  last_us_ = mono_us();
}

bool LineReader::fill(int timeout_ms) {
  if (eof_) return false;
  char buf[65536];
  ssize_t n = ds::read_some(fd_, buf, sizeof(buf), timeout_ms);
  if (n == -2) return false;  // timeout
  if (n <= 0) {
    eof_ = true;
    return false;
  }
  last_us_ = mono_us();
  buf_.append(buf, (size_t)n);
  return true;
}

ssize_t LineReader::read_some(char* out, size_t n, int timeout_ms) {
  if (n == 0) return 0;
  if (!buf_.empty()) {
    size_t c = std::min(n, buf_.size());
    std::memcpy(out, buf_.data(), c);
    buf_.erase(0, c);
    return (ssize_t)c;
  }
  if (eof_) return 0;
  ssize_t r = ds::read_some(fd_, out, n, timeout_ms);
  if (r == -2) return -2;
  if (r <= 0) {
    eof_ = true;
    return r;
  }
  last_us_ = mono_us();
  return r;
}

bool LineReader::read_line(std::string* line, int timeout_ms) {
  long deadline = timeout_ms < 0 ? -1 : mono_us() + (long)timeout_ms * 1000;
  while (true) {
    size_t nl = buf_.find('\n');
    if (nl != std::string::npos) {
      *line = buf_.substr(0, nl);
      buf_.erase(0, nl + 1);
      return true;
    }
    int left = -1;
    if (deadline >= 0) {
      long l = (deadline - mono_us()) / 1000;
      if (l <= 0) return false;
      left = (int)l;
    }
    if (!fill(left)) return false;
  }
}

bool LineReader::wait_for(const std::string& keyword, int timeout_ms, std::string* before, bool partial) {
  long deadline = timeout_ms < 0 ? -1 : mono_us() + (long)timeout_ms * 1000;
  while (true) {
    size_t nl;
    while ((nl = buf_.find('\n')) != std::string::npos) {
      std::string line = buf_.substr(0, nl);
      buf_.erase(0, nl + 1);
      if (line == keyword) return true;
      if (before && !line.empty()) *before += line + "\n";
    }
    if (partial && buf_ == keyword) {
      buf_.clear();
      return true;
    }
    int left = -1;
    if (deadline >= 0) {
      long l = (deadline - mono_us()) / 1000;
      if (l <= 0) return false;
      left = (int)l;
    }
    if (!fill(left)) return false;
  }
}

bool LineReader::read_exact(std::string* out, size_t n, int timeout_ms) {
  out->clear();
  return read_to(
      n,
      [&](const char* d, size_t k) {
        out->append(d, k);
        return true;
      },
      timeout_ms);
}

bool LineReader::read_to(size_t n, const std::function<bool(const char*, size_t)>& sink, int timeout_ms,
                         int64_t rate_limit) {
  RateLimiter rl(rate_limit);
  size_t take = std::min(n, buf_.size());
  if (take) {
    if (rate_limit > 0) rl.take(take);
    if (!sink(buf_.data(), take)) return false;
    buf_.erase(0, take);
    n -= take;
  }
  char buf[65536];
  while (n > 0) {
    ssize_t r = ds::read_some(fd_, buf, std::min(n, sizeof(buf)), timeout_ms);
    if (r <= 0) {
      if (r == 0) eof_ = true;
      return false;
    }
    last_us_ = mono_us();
    if (rate_limit > 0) rl.take((size_t)r);
    if (!sink(buf, (size_t)r)) return false;
    n -= (size_t)r;
  }
  return true;
}

void RateLimiter::take(size_t n) {
  if (rate_ <= 0) return;
  long now = mono_us();
  if (last_us_ == 0) {
    last_us_ = now;
    tokens_ = (double)rate_;  // bucket capacity = rate (one second burst)
  }
  tokens_ = std::min((double)rate_, tokens_ + (double)(now - last_us_) * (double)rate_ / 1e6);
  last_us_ = now;
  tokens_ -= (double)n;
  if (tokens_ < 0) {
    long wait_us = (long)(-tokens_ * 1e6 / (double)rate_);
    std::this_thread::sleep_for(std::chrono::microseconds(wait_us));
  }
}

}  // namespace sync
}  // namespace ds

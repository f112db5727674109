// Remote shell transports for the sync engine.
//
// The reference runs `sh` in the container over SPDY exec (sync/upstream.go:47) and, in tests,
// a local `sh` (sync/upstream.go:67-95 `testing` flag). Here that seam is a first-class
// interface: LocalShellTransport (local-pod backend + tests), kube::ExecTransport (WebSocket
// exec), FaultInjectingTransport (drop/stall/corrupt streams for recovery tests).
#pragma once

#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "core/proc.h"

namespace ds {
namespace sync {

class Shell {
 public:
  virtual ~Shell() = default;
  virtual int in() = 0;   // write commands / payload
  virtual int out() = 0;  // remote stdout
  virtual int err() = 0;  // remote stderr
  virtual void close() = 0;
  virtual bool alive() = 0;
  // Ends the remote side without closing local fds, so readers blocked in other threads see
  // EOF; close() afterwards releases the fds.
  virtual void terminate() = 0;
};

class Transport {
 public:
  virtual ~Transport() = default;
  // Starts `argv` (default: sh) in the target container with piped stdio.
  virtual std::unique_ptr<Shell> open(const std::vector<std::string>& argv = {"sh"}) = 0;
  virtual std::string describe() const = 0;
  // Prefix that maps container paths to what the shell sees (local-pod backend roots
  // every pod under a directory; real containers use "").
  virtual std::string path_prefix() const { return ""; }
  // Pod behind this transport ("" when not a pod).
  virtual std::string pod_name() const { return ""; }
};

// Runs commands as local processes (optionally chrooted-by-convention under `root`).
class LocalShellTransport : public Transport {
 public:
  explicit LocalShellTransport(std::string cwd = "", std::string root_prefix = "",
                               std::map<std::string, std::string> env = {});
  std::unique_ptr<Shell> open(const std::vector<std::string>& argv) override;
  std::string describe() const override { return "local-shell"; }
  std::string path_prefix() const override { return root_; }

 private:
  std::string cwd_, root_;
  std::map<std::string, std::string> env_;
};

struct FaultPlan {
  // Kill the shell once this many bytes were written to its stdin (0 = never).
  size_t kill_after_stdin_bytes = 0;
  // Kill the shell once this many bytes were read from its stdout (0 = never).
  size_t kill_after_stdout_bytes = 0;
  // Delay every chunk read from remote stdout by this many ms.
  int stall_stdout_ms = 0;
  // Replace the first occurrence of `corrupt_from` in stdout with `corrupt_to`.
  std::string corrupt_from, corrupt_to;
  // Only the n-th opened shell (1-based) gets the fault; 0 = all shells.
  int only_shell = 0;
};

class FaultInjectingTransport : public Transport {
 public:
  FaultInjectingTransport(std::shared_ptr<Transport> inner, FaultPlan plan)
      : inner_(std::move(inner)), plan_(std::move(plan)) {}
  std::unique_ptr<Shell> open(const std::vector<std::string>& argv) override;
  std::string describe() const override { return "fault(" + inner_->describe() + ")"; }
  std::string path_prefix() const override { return inner_->path_prefix(); }
  int opened() const { return opened_; }

 private:
  std::shared_ptr<Transport> inner_;
  FaultPlan plan_;
  int opened_ = 0;
};

// Buffered line/byte reader over an fd; keeps read-ahead so binary payloads following a
// text line are not lost (the reference's waitTill discards overlap, sync/util.go:178).
class LineReader {
 public:
  explicit LineReader(int fd = -1) : fd_(fd) {}
  void reset(int fd);
  // Reads one '\n'-terminated line (without it). false on EOF/timeout/error.
  bool read_line(std::string* line, int timeout_ms = -1);
  // Waits for a line equal to keyword, or (partial=true) a trailing unterminated chunk equal to
  // keyword (reference `printf "DONE"` acks). Collects preceding lines into `before`.
  bool wait_for(const std::string& keyword, int timeout_ms = -1, std::string* before = nullptr,
                bool partial = false);
  bool read_exact(std::string* out, size_t n, int timeout_ms = -1);
  // Streams exactly n bytes to a sink.
  bool read_to(size_t n, const std::function<bool(const char*, size_t)>& sink, int timeout_ms = -1,
               int64_t rate_limit = 0);
  // Up to n bytes (buffered read-ahead first). Returns bytes, 0 on EOF, -1 on error, -2 on
  // timeout.
  ssize_t read_some(char* out, size_t n, int timeout_ms = -1);
  // Puts bytes back in front of the read-ahead (a parser that pulled past its own data).
  void unread(const std::string& data) { buf_.insert(0, data); }
  int fd() const { return fd_; }
  bool eof() const { return eof_; }
  // Monotonic time (us) of the last byte received; the reset time before any.
  long last_activity_us() const { return last_us_; }
  std::string take_buffer() {
    std::string b;
    b.swap(buf_);
    return b;
  }

 private:
  bool fill(int timeout_ms);
  int fd_;
  std::string buf_;
  bool eof_ = false;
  long last_us_ = 0;
};

// Token-bucket rate limiter (juju/ratelimit in the reference; bytes/second).
class RateLimiter {
 public:
  explicit RateLimiter(int64_t rate) : rate_(rate) {}
  void take(size_t n);

 private:
  int64_t rate_;
  double tokens_ = 0;
  long last_us_ = 0;
};

}  // namespace sync
}  // namespace ds

// Child processes and fd-level I/O.
//
// Every remote stream in the tool (local `sh`, Kubernetes exec over WebSocket, port-forward
// channels) is surfaced as plain file descriptors, so the sync engine can use poll() with
// timeouts uniformly instead of goroutine-per-pipe (sync/upstream.go:47, kubectl/exec.go:20).
#pragma once

#include <sys/types.h>

#include <map>
#include <memory>
#include <string>
#include <vector>

namespace ds {

// Owned file descriptor.
class Fd {
 public:
  Fd() = default;
  explicit Fd(int fd) : fd_(fd) {}
  ~Fd() { reset(); }
  Fd(const Fd&) = delete;
  Fd& operator=(const Fd&) = delete;
  Fd(Fd&& o) noexcept : fd_(o.release()) {}
  Fd& operator=(Fd&& o) noexcept {
    if (this != &o) {
      reset();
      fd_ = o.release();
    }
    return *this;
  }
  int get() const { return fd_; }
  bool valid() const { return fd_ >= 0; }
  int release() {
    int f = fd_;
    fd_ = -1;
    return f;
  }
  void reset(int fd = -1);

 private:
  int fd_ = -1;
};

// Creates a pipe; returns false on failure. Both ends are O_CLOEXEC.
bool make_pipe(Fd* read_end, Fd* write_end);

// Write everything (handles EINTR / partial writes; blocks on full pipes). false on error.
bool write_all(int fd, const void* data, size_t n);
inline bool write_all(int fd, const std::string& s) { return write_all(fd, s.data(), s.size()); }
// Read up to n bytes waiting at most timeout_ms (-1 = forever). Returns bytes, 0 on EOF,
// -1 on error, -2 on timeout.
ssize_t read_some(int fd, void* buf, size_t n, int timeout_ms = -1);
// Read exactly n bytes (or fail).
bool read_exact(int fd, void* buf, size_t n, int timeout_ms = -1);
// Read until EOF.
std::string read_all(int fd);
void set_nonblocking(int fd, bool nb);

struct ProcOptions {
  std::string cwd;
  std::map<std::string, std::string> env;  // added/overridden on top of the current env
  bool clear_env = false;
  bool pipe_stdin = true;
  bool pipe_stdout = true;
  bool pipe_stderr = true;
  bool merge_stderr = false;  // stderr -> stdout pipe
  bool new_process_group = true;
  int stdin_fd = -1;   // inherit this fd as stdin when !pipe_stdin (-1 = /dev/null)
  int stdout_fd = -1;  // when !pipe_stdout (-1 = inherit parent's)
  int stderr_fd = -1;  // when !pipe_stderr (-1 = inherit parent's)
};

class Process {
 public:
  Process() = default;
  ~Process();
  Process(const Process&) = delete;
  Process& operator=(const Process&) = delete;

  // argv[0] is looked up in PATH. Returns false (with error()) if the spawn failed.
  bool start(const std::vector<std::string>& argv, const ProcOptions& opts = {});
  pid_t pid() const { return pid_; }
  int stdin_fd() const { return in_.get(); }
  int stdout_fd() const { return out_.get(); }
  int stderr_fd() const { return err_.get(); }
  void close_stdin() { in_.reset(); }
  void close_stdout() { out_.reset(); }
  void close_stderr() { err_.reset(); }
  // Wait for exit; returns exit code (128+signal when killed). timeout_ms<0 waits forever;
  // returns -1 on timeout.
  int wait(int timeout_ms = -1);
  bool running();
  void kill(int sig = 15);  // signals the whole process group when started in one
  const std::string& error() const { return error_; }
  int exit_code() const { return exit_code_; }

 private:
  pid_t pid_ = -1;
  bool group_ = false;
  bool reaped_ = false;
  int exit_code_ = -1;
  Fd in_, out_, err_;
  std::string error_;
};

struct RunResult {
  int code = -1;
  std::string out;
  std::string err;
  bool spawn_failed = false;
};

// Run to completion capturing stdout/stderr; optional stdin data.
RunResult run(const std::vector<std::string>& argv, const std::string& input = "", const ProcOptions& opts = {},
              int timeout_ms = -1);

// Locate an executable in PATH ("" if absent).
std::string which(const std::string& name);

}  // namespace ds

#include "core/proc.h"

#include <fcntl.h>
#include <poll.h>
#include <signal.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>
#include <thread>

#include "core/fs.h"
#include "core/strutil.h"
#include "platform/platform.h"

extern char** environ;

namespace ds {

void Fd::reset(int fd) {
  if (fd_ >= 0) ::close(fd_);
  fd_ = fd;
}

bool make_pipe(Fd* r, Fd* w) {
  int p[2];
  if (plat::pipe_cloexec(p) != 0) return false;
  r->reset(p[0]);
  w->reset(p[1]);
  return true;
}

bool write_all(int fd, const void* data, size_t n) {
  const char* p = (const char*)data;
  while (n > 0) {
    ssize_t w = ::write(fd, p, n);
    if (w < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN) {
        struct pollfd pf{fd, POLLOUT, 0};
        ::poll(&pf, 1, 100);
        continue;
      }
      return false;
    }
    p += w;
    n -= (size_t)w;
  }
  return true;
}

ssize_t read_some(int fd, void* buf, size_t n, int timeout_ms) {
  while (true) {
    if (timeout_ms >= 0) {
      struct pollfd pf{fd, POLLIN, 0};
      int r = ::poll(&pf, 1, timeout_ms);
      if (r < 0) {
        if (errno == EINTR) continue;
        return -1;
      }
      if (r == 0) return -2;
    }
    ssize_t got = ::read(fd, buf, n);
    if (got < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN) {
        struct pollfd pf{fd, POLLIN, 0};
        ::poll(&pf, 1, timeout_ms < 0 ? 1000 : timeout_ms);
        continue;
      }
      return -1;
    }
    return got;
  }
}

bool read_exact(int fd, void* buf, size_t n, int timeout_ms) {
  char* p = (char*)buf;
  while (n > 0) {
    ssize_t r = read_some(fd, p, n, timeout_ms);
    if (r <= 0) return false;
    p += r;
    n -= (size_t)r;
  }
  return true;
}

std::string read_all(int fd) {
  std::string out;
  char buf[65536];
  while (true) {
    ssize_t r = read_some(fd, buf, sizeof(buf));
    if (r <= 0) break;
    out.append(buf, (size_t)r);
  }
  return out;
}

void set_nonblocking(int fd, bool nb) {
  int fl = ::fcntl(fd, F_GETFL);
  if (nb)
    ::fcntl(fd, F_SETFL, fl | O_NONBLOCK);
  else
    ::fcntl(fd, F_SETFL, fl & ~O_NONBLOCK);
}

std::string which(const std::string& name) {
  if (name.find('/') != std::string::npos) return ::access(name.c_str(), X_OK) == 0 ? name : "";
  const char* path = getenv("PATH");
  if (!path) path = "/usr/local/bin:/usr/bin:/bin";
  for (auto& dir : split(path, ":")) {
    if (dir.empty()) continue;
    std::string cand = dir + "/" + name;
    if (::access(cand.c_str(), X_OK) == 0 && !fs::is_dir(cand)) return cand;
  }
  return "";
}

Process::~Process() {
  if (pid_ > 0 && !reaped_) {
    kill(SIGKILL);
    wait(2000);
  }
}

bool Process::start(const std::vector<std::string>& argv, const ProcOptions& opts) {
  if (argv.empty()) {
    error_ = "empty argv";
    return false;
  }
  std::string exe = which(argv[0]);
  if (exe.empty()) {
    error_ = "executable file not found in $PATH: " + argv[0];
    return false;
  }
  Fd in_r, in_w, out_r, out_w, err_r, err_w;
  if (opts.pipe_stdin && !make_pipe(&in_r, &in_w)) return false;
  if (opts.pipe_stdout && !make_pipe(&out_r, &out_w)) return false;
  if (opts.pipe_stderr && !opts.merge_stderr && !make_pipe(&err_r, &err_w)) return false;
  // exec status pipe to report exec failures
  Fd st_r, st_w;
  make_pipe(&st_r, &st_w);

  std::vector<std::string> envs;
  if (!opts.clear_env) {
    for (char** e = environ; e && *e; ++e) {
      std::string kv = *e;
      size_t eq = kv.find('=');
      std::string k = kv.substr(0, eq);
      if (opts.env.count(k)) continue;
      envs.push_back(kv);
    }
  }
  for (auto& kv : opts.env) envs.push_back(kv.first + "=" + kv.second);
  std::vector<char*> cargv, cenv;
  for (auto& a : argv) cargv.push_back(const_cast<char*>(a.c_str()));
  cargv.push_back(nullptr);
  for (auto& e : envs) cenv.push_back(const_cast<char*>(e.c_str()));
  cenv.push_back(nullptr);
  int devnull = -1;
  if (!opts.pipe_stdin && opts.stdin_fd < 0) devnull = ::open("/dev/null", O_RDONLY | O_CLOEXEC);

  pid_t pid = ::fork();
  if (pid < 0) {
    error_ = std::string("fork: ") + std::strerror(errno);
    if (devnull >= 0) ::close(devnull);
    return false;
  }
  if (pid == 0) {
    if (opts.new_process_group) ::setpgid(0, 0);
    // restore default signal handling
    signal(SIGPIPE, SIG_DFL);
    signal(SIGINT, SIG_DFL);
    signal(SIGTERM, SIG_DFL);
    if (opts.pipe_stdin)
      ::dup2(in_r.get(), 0);
    else if (opts.stdin_fd >= 0)
      ::dup2(opts.stdin_fd, 0);
    else if (devnull >= 0)
      ::dup2(devnull, 0);
    if (opts.pipe_stdout)
      ::dup2(out_w.get(), 1);
    else if (opts.stdout_fd >= 0)
      ::dup2(opts.stdout_fd, 1);
    if (opts.merge_stderr && opts.pipe_stdout)
      ::dup2(out_w.get(), 2);
    else if (opts.pipe_stderr)
      ::dup2(err_w.get(), 2);
    else if (opts.stderr_fd >= 0)
      ::dup2(opts.stderr_fd, 2);
    if (!opts.cwd.empty() && ::chdir(opts.cwd.c_str()) != 0) {
      int e = errno;
      ssize_t ignored = ::write(st_w.get(), &e, sizeof(e));
      (void)ignored;
      _exit(127);
    }
    plat::close_fds_in_child(st_w.get());
    ::execve(exe.c_str(), cargv.data(), cenv.data());
    int e = errno;
    ssize_t ignored = ::write(st_w.get(), &e, sizeof(e));
    (void)ignored;
    _exit(127);
  }
  if (devnull >= 0) ::close(devnull);
  st_w.reset();
  int child_errno = 0;
  ssize_t n = ::read(st_r.get(), &child_errno, sizeof(child_errno));
  if (n == (ssize_t)sizeof(child_errno)) {
    error_ = std::string("exec ") + argv[0] + ": " + std::strerror(child_errno);
    int status;
    ::waitpid(pid, &status, 0);
    return false;
  }
  pid_ = pid;
  group_ = opts.new_process_group;
  in_ = std::move(in_w);
  out_ = std::move(out_r);
  err_ = std::move(err_r);
  return true;
}

int Process::wait(int timeout_ms) {
  if (pid_ <= 0) return -1;
  if (reaped_) return exit_code_;
  struct timespec start;
  clock_gettime(CLOCK_MONOTONIC, &start);
  while (true) {
    int status = 0;
    pid_t r = ::waitpid(pid_, &status, timeout_ms < 0 ? 0 : WNOHANG);
    if (r == pid_) {
      reaped_ = true;
      if (WIFEXITED(status))
        exit_code_ = WEXITSTATUS(status);
      else if (WIFSIGNALED(status))
        exit_code_ = 128 + WTERMSIG(status);
      return exit_code_;
    }
    if (r < 0 && errno != EINTR) {
      reaped_ = true;
      return exit_code_;
    }
    if (timeout_ms >= 0) {
      struct timespec now;
      clock_gettime(CLOCK_MONOTONIC, &now);
      long ms = (now.tv_sec - start.tv_sec) * 1000 + (now.tv_nsec - start.tv_nsec) / 1000000;
      if (ms >= timeout_ms) return -1;
      std::this_thread::sleep_for(std::chrono::milliseconds(5));
    }
  }
}

bool Process::running() {
  if (pid_ <= 0 || reaped_) return false;
  return wait(0) == -1;
}

void Process::kill(int sig) {
  if (pid_ <= 0 || reaped_) return;
  if (group_)
    ::kill(-pid_, sig);
  else
    ::kill(pid_, sig);
}

RunResult run(const std::vector<std::string>& argv, const std::string& input, const ProcOptions& o,
              int timeout_ms) {
  RunResult res;
  Process p;
  ProcOptions opts = o;
  opts.pipe_stdin = true;
  opts.pipe_stdout = true;
  opts.pipe_stderr = true;
  if (!p.start(argv, opts)) {
    res.spawn_failed = true;
    res.err = p.error();
    res.code = 127;
    return res;
  }
  std::thread writer([&] {
    if (!input.empty()) write_all(p.stdin_fd(), input);
    p.close_stdin();
  });
  // drain both pipes with poll
  int ofd = p.stdout_fd(), efd = p.stderr_fd();
  struct timespec start;
  clock_gettime(CLOCK_MONOTONIC, &start);
  bool timed_out = false;
  while (ofd >= 0 || efd >= 0) {
    struct pollfd pf[2];
    int nf = 0;
    if (ofd >= 0) pf[nf++] = {ofd, POLLIN, 0};
    if (efd >= 0) pf[nf++] = {efd, POLLIN, 0};
    int r = ::poll(pf, nf, 200);
    if (r < 0 && errno != EINTR) break;
    for (int i = 0; i < nf; ++i) {
      if (!(pf[i].revents & (POLLIN | POLLHUP | POLLERR))) continue;
      char buf[65536];
      ssize_t n = ::read(pf[i].fd, buf, sizeof(buf));
      if (n <= 0) {
        if (pf[i].fd == ofd)
          ofd = -1;
        else
          efd = -1;
      } else {
        (pf[i].fd == ofd ? res.out : res.err).append(buf, (size_t)n);
      }
    }
    if (timeout_ms >= 0) {
      struct timespec now;
      clock_gettime(CLOCK_MONOTONIC, &now);
      long ms = (now.tv_sec - start.tv_sec) * 1000 + (now.tv_nsec - start.tv_nsec) / 1000000;
      if (ms > timeout_ms) {
        timed_out = true;
        p.kill(9);
        break;
      }
    }
  }
  writer.join();
  res.code = p.wait();
  if (timed_out) res.code = 124;
  return res;
}

}  // namespace ds

// POSIX.1-2008 implementation of platform/platform.h (-DDEVSPACE_PORTABLE=ON): no Linux-only
// system calls, so it is the starting point of the darwin client (docs/platforms.md lists what
// darwin and windows still need).
#include <fcntl.h>
#include <signal.h>
#include <netdb.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <climits>
#include <cstdint>
#include <cstdlib>
#include <mutex>
#include <thread>

#include "platform/platform.h"

namespace ds {
namespace plat {

namespace {

bool set_cloexec(int fd) {
  int fl = ::fcntl(fd, F_GETFD);
  return fl >= 0 && ::fcntl(fd, F_SETFD, fl | FD_CLOEXEC) == 0;
}

bool set_nonblock(int fd) {
  int fl = ::fcntl(fd, F_GETFL);
  return fl >= 0 && ::fcntl(fd, F_SETFL, fl | O_NONBLOCK) == 0;
}

// A fork elsewhere in the process can catch a descriptor between its creation and the fcntl
// below; the CLI's own children close every inherited descriptor before exec
// (close_fds_in_child, called by core/proc.cc), so such a window leaks nothing.
int finish(int fd) {
  if (fd >= 0) set_cloexec(fd);
  return fd;
}

std::mutex g_exe_mu;
std::string g_exe;

}  // namespace

const char* name() { return "posix"; }

int pipe_cloexec(int fds[2], bool nonblock) {
  if (::pipe(fds) != 0) return -1;
  for (int i = 0; i < 2; ++i) {
    set_cloexec(fds[i]);
    if (nonblock) set_nonblock(fds[i]);
  }
  return 0;
}

void grow_pipe(int, int) {}  // macOS and the BSDs grow a pipe's buffer with its backlog

int socket_cloexec(int family, int type, int protocol) { return finish(::socket(family, type, protocol)); }

int accept_cloexec(int listen_fd) {
  while (true) {
    int fd = ::accept(listen_fd, nullptr, nullptr);
    if (fd < 0 && errno == EINTR) continue;
    return finish(fd);
  }
}

void close_fds_in_child(int keep) {
  long max = ::sysconf(_SC_OPEN_MAX);
  if (max < 0 || max > 65536) max = 65536;
  for (int fd = 3; fd < max; ++fd)
    if (fd != keep) ::close(fd);
}

// SIGPIPE is ignored process-wide by the CLI (cli/common.cc install_signal_handlers) and by
// CPython for the module, so a plain send returns EPIPE.
ssize_t send_nosignal(int fd, const void* data, size_t n) { return ::send(fd, data, n, 0); }

Waker::Waker() {
  int p[2];
  if (pipe_cloexec(p, true) == 0) {
    rfd_ = p[0];
    wfd_ = p[1];
  }
}

Waker::~Waker() {
  if (rfd_ >= 0) ::close(rfd_);
  if (wfd_ >= 0) ::close(wfd_);
}

void Waker::poke() {
  if (wfd_ < 0) return;
  char c = 1;
  ssize_t w = ::write(wfd_, &c, 1);  // a full pipe is already readable: nothing is lost
  (void)w;
}

void Waker::drain() {
  if (rfd_ < 0) return;
  char buf[64];
  while (::read(rfd_, buf, sizeof(buf)) > 0) {
  }
}

void tie_to_parent(long parent_pid) {
  if (parent_pid <= 1 || ::getppid() != (pid_t)parent_pid) return;
  std::thread([parent_pid] {
    while (::getppid() == (pid_t)parent_pid) ::usleep(200000);  // re-parented: the parent died
    ::kill(::getpid(), SIGTERM);
  }).detach();
}

void set_argv0(const char* argv0) {
  if (!argv0 || !*argv0) return;
  std::string a = argv0, found;
  if (a.find('/') != std::string::npos) {
    found = a;
  } else if (const char* path = getenv("PATH")) {
    std::string p = path;
    size_t start = 0;
    while (start <= p.size()) {
      size_t end = p.find(':', start);
      if (end == std::string::npos) end = p.size();
      std::string dir = p.substr(start, end - start);
      std::string cand = (dir.empty() ? std::string(".") : dir) + "/" + a;
      if (::access(cand.c_str(), X_OK) == 0) {
        found = cand;
        break;
      }
      start = end + 1;
    }
  }
  char buf[PATH_MAX];
  if (found.empty() || !::realpath(found.c_str(), buf)) return;  // resolved now: cwd may change
  std::lock_guard<std::mutex> g(g_exe_mu);
  g_exe = buf;
}

std::string self_exe() {
  std::lock_guard<std::mutex> g(g_exe_mu);
  return g_exe;
}

int open_unlinked_tmp(const std::string& dir) {
  std::string tmpl = dir + "/devspace-spill-XXXXXX";
  int fd = finish(::mkstemp(&tmpl[0]));
  if (fd >= 0) ::unlink(tmpl.c_str());
  return fd;
}

bool system_resolver() { return true; }

}  // namespace plat
}  // namespace ds

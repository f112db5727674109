// Linux implementation of platform/platform.h (the default build).
#include <fcntl.h>
#include <signal.h>
#include <sys/prctl.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <climits>
#include <cstdint>

#include "platform/platform.h"

namespace ds {
namespace plat {

const char* name() { return "linux"; }

int pipe_cloexec(int fds[2], bool nonblock) { return ::pipe2(fds, O_CLOEXEC | (nonblock ? O_NONBLOCK : 0)); }

int socket_cloexec(int family, int type, int protocol) { return ::socket(family, type | SOCK_CLOEXEC, protocol); }

int accept_cloexec(int listen_fd) {
  while (true) {
    int fd = ::accept4(listen_fd, nullptr, nullptr, SOCK_CLOEXEC);
    if (fd < 0 && errno == EINTR) continue;
    return fd;
  }
}

void grow_pipe(int fd, int bytes) {
  if (fd >= 0) ::fcntl(fd, F_SETPIPE_SZ, bytes);
}

void close_fds_in_child(int) {}

ssize_t send_nosignal(int fd, const void* data, size_t n) { return ::send(fd, data, n, MSG_NOSIGNAL); }

Waker::Waker() { rfd_ = wfd_ = ::eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC); }

Waker::~Waker() {
  if (rfd_ >= 0) ::close(rfd_);
}

void Waker::poke() {
  if (wfd_ < 0) return;
  uint64_t one = 1;
  ssize_t w = ::write(wfd_, &one, sizeof(one));
  (void)w;
}

void Waker::drain() {
  if (rfd_ < 0) return;
  uint64_t v;
  ssize_t r = ::read(rfd_, &v, sizeof(v));
  (void)r;
}

void tie_to_parent(long parent_pid) {
  if (parent_pid <= 1) return;
  if (::getppid() != (pid_t)parent_pid) return;  // started by someone else: not ours to tie
  ::prctl(PR_SET_PDEATHSIG, SIGTERM);
  if (::getppid() != (pid_t)parent_pid) ::kill(::getpid(), SIGTERM);  // it died in between
}

void set_argv0(const char*) {}

std::string self_exe() {
  char buf[PATH_MAX];
  ssize_t n = ::readlink("/proc/self/exe", buf, sizeof(buf) - 1);
  if (n <= 0) return "";
  buf[n] = 0;
  return buf;
}

int open_unlinked_tmp(const std::string& dir) {
  int fd = ::open(dir.c_str(), O_TMPFILE | O_RDWR | O_CLOEXEC, 0600);
  if (fd >= 0) return fd;
  // file systems without O_TMPFILE (overlayfs before 4.x, some FUSE mounts)
  std::string tmpl = dir + "/devspace-spill-XXXXXX";
  fd = ::mkostemp(&tmpl[0], O_CLOEXEC);
  if (fd >= 0) ::unlink(tmpl.c_str());
  return fd;
}

bool system_resolver() { return false; }

}  // namespace plat
}  // namespace ds

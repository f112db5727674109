// The operating-system seam of the CLI. Everything the client needs beyond POSIX.1-2008 goes
// through here, so the rest of src/ compiles against POSIX only:
//   * src/platform/linux.cc   — the default build: pipe2/accept4/SOCK_CLOEXEC, MSG_NOSIGNAL,
//                                eventfd wake-ups, /proc/self/exe, O_TMPFILE, the built-in
//                                resolver (the release binary is static, no NSS);
//   * src/platform/posix.cc   — -DDEVSPACE_PORTABLE=ON: the same contracts from plain POSIX
//                                (fcntl(FD_CLOEXEC), a self-pipe, argv[0] + PATH, mkstemp +
//                                unlink, getaddrinfo), the base for the darwin client.
// File watching has its own seam in platform/watch.h.
//
// The reference ships darwin, windows and linux clients from one Go tree
// (/root/reference/scripts/build-all.bash:27-62); Go's runtime is its platform layer. This file
// is ours. The in-container helper (src/helper/) runs in the pod and stays Linux-only.
#pragma once

#include <sys/types.h>

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

struct stat;

namespace ds {
namespace plat {

// "linux" or "posix": which implementation this binary was built with.
const char* name();

// Close-on-exec descriptors, created that way atomically where the OS allows it.
int pipe_cloexec(int fds[2], bool nonblock = false);
int socket_cloexec(int family, int type, int protocol = 0);
// accept(2) of one connection; the new descriptor is close-on-exec. -1 with errno set.
int accept_cloexec(int listen_fd);

// Asks for a pipe buffer of `bytes` (Linux: F_SETPIPE_SZ, up to the unprivileged maximum of
// 1 MiB, so bulk transfers cross the pipe in fewer wake-ups). Elsewhere pipes size themselves:
// a no-op. Best effort: a refusal leaves the default size.
void grow_pipe(int fd, int bytes);

// In a forked child before execve: closes inherited descriptors above 2 that are not
// close-on-exec yet (except `keep`). A no-op where every descriptor is created close-on-exec.
// Async-signal-safe.
void close_fds_in_child(int keep);

// send(2) that never raises SIGPIPE on a peer that went away (EPIPE instead).
ssize_t send_nosignal(int fd, const void* data, size_t n);

// A descriptor poll(2) can wait on next to a socket, made readable by poke() from any thread.
// drain() resets it. eventfd on Linux, a non-blocking self-pipe elsewhere.
class Waker {
 public:
  Waker();
  ~Waker();
  Waker(const Waker&) = delete;
  Waker& operator=(const Waker&) = delete;
  bool ok() const { return rfd_ >= 0; }
  int fd() const { return rfd_; }
  void poke();
  void drain();

 private:
  int rfd_ = -1;
  int wfd_ = -1;  // == rfd_ for an eventfd
};

// When this process's parent is `parent_pid`: SIGTERM to this process once that parent dies
// (however it dies), so a CLI started by a test harness or a script never outlives it. Linux:
// PR_SET_PDEATHSIG; POSIX: a thread that watches getppid(). A parent that already died before
// this call ran: SIGTERM now. Another parent (a grandchild of `parent_pid`): nothing.
void tie_to_parent(long parent_pid);

// Remember argv[0] (main() calls this first): the POSIX build finds its own executable from it.
void set_argv0(const char* argv0);
// Absolute path of the running executable, "" when unknown.
std::string self_exe();

// A read-write temporary file in `dir` that has no name: nothing is left behind whatever way
// the process ends. -1 with errno set.
int open_unlinked_tmp(const std::string& dir);

// Modification time of a stat result in nanoseconds since the epoch.
int64_t mtime_ns(const struct stat& st);

// The release target this binary runs as, go-style "<os>-<arch>" from uname(2): "linux-amd64",
// "darwin-arm64", ... It names the self-update asset (devspace-<target>).
std::string release_target();

// Whether host names go to the system resolver (getaddrinfo: NSS, macOS scoped DNS, VPN split
// DNS) instead of the built-in /etc/hosts + resolv.conf resolver of the static Linux binary.
bool system_resolver();

}  // namespace plat
}  // namespace ds

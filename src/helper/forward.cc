// `devspace-helper forward`: the pod side of port-forwarding through the helper
// (protocol: src/sync/fwd_proto.h). One poll loop: frames from the client on stdin, one socket
// per forwarded connection to localhost in the pod's network namespace, frames back on stdout.
// A connect the app refuses (it is restarting under hot reload) is retried every 2 ms until the
// client's hold runs out, so the connection is made once, within milliseconds of the app
// listening: what the client sent meanwhile is kept here and delivered exactly once.
#include "helper/forward.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <signal.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "sync/fwd_proto.h"

namespace ds {
namespace helper {

namespace {

namespace fwd = ds::sync::fwd;

long mono_us() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1000000L + ts.tv_nsec / 1000;
}

bool write_all(int fd, const std::string& s) {
  const char* p = s.data();
  size_t n = s.size();
  while (n) {
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

struct Conn {
  int port = 0;
  int fd = -1;
  bool connecting = false;  // a non-blocking connect in flight on fd
  bool connected = false;
  int family = AF_INET;     // the address of the attempt in flight (127.0.0.1, then ::1)
  long deadline_us = 0;     // the hold: refused connects are retried until then
  long next_try_us = 0;     // 0: try now
  std::string to_app;       // client bytes not written yet
  bool client_fin = false;  // the client half-closed: shut the socket's write side once drained
  bool shut_wr = false;
  bool app_eof = false;
  uint64_t unacked = 0;     // app bytes sent to the client that it has not acknowledged
};

constexpr long kRetryUs = 2000;

class Forwarder {
 public:
  int run() {
    ::fcntl(0, F_SETFL, ::fcntl(0, F_GETFL) | O_NONBLOCK);
    while (true) {
      long now = mono_us();
      for (auto it = conns_.begin(); it != conns_.end();) {
        Conn& c = it->second;
        if (!c.connected && !c.connecting && c.next_try_us <= now && !try_connect(it->first, c, now)) {
          it = conns_.erase(it);
          continue;
        }
        ++it;
      }
      std::vector<struct pollfd> pf;
      std::vector<uint32_t> ids;
      pf.push_back({0, POLLIN, 0});
      ids.push_back(0);
      int timeout = 200;
      for (auto& kv : conns_) {
        Conn& c = kv.second;
        if (c.fd < 0) {
          if (!c.connected && !c.connecting)
            timeout = std::min<long>(timeout, std::max<long>(0, (c.next_try_us - now + 999) / 1000));
          continue;
        }
        short ev = 0;
        if (c.connecting || (c.connected && !c.to_app.empty())) ev |= POLLOUT;
        if (c.connected && !c.app_eof && c.unacked < fwd::kWindow) ev |= POLLIN;  // else: the client reads slowly
        if (!ev) continue;
        pf.push_back({c.fd, ev, 0});
        ids.push_back(kv.first);
      }
      int r = ::poll(pf.data(), pf.size(), timeout);
      if (r < 0) {
        if (errno == EINTR) continue;
        return 1;
      }
      now = mono_us();
      if (pf[0].revents & (POLLIN | POLLHUP | POLLERR)) {
        if (!read_client()) return 0;  // stdin closed: the client is gone
      }
      for (size_t i = 1; i < pf.size(); ++i) {
        auto it = conns_.find(ids[i]);
        if (it == conns_.end() || it->second.fd != pf[i].fd) continue;  // closed by a frame meanwhile
        if (!on_socket(it->first, it->second, pf[i].revents, now)) conns_.erase(it);
      }
    }
  }

 private:
  // false: the connection is gone (reported)
  bool try_connect(uint32_t id, Conn& c, long now) {
    for (int attempt = 0; attempt < 2; ++attempt) {
      int fd = ::socket(c.family, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
      if (fd < 0) return fail(id, c, std::string("socket: ") + std::strerror(errno));
      int rc;
      if (c.family == AF_INET) {
        struct sockaddr_in a{};
        a.sin_family = AF_INET;
        a.sin_port = htons((uint16_t)c.port);
        a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
        rc = ::connect(fd, (struct sockaddr*)&a, sizeof(a));
      } else {
        struct sockaddr_in6 a{};
        a.sin6_family = AF_INET6;
        a.sin6_port = htons((uint16_t)c.port);
        a.sin6_addr = in6addr_loopback;
        rc = ::connect(fd, (struct sockaddr*)&a, sizeof(a));
      }
      if (rc == 0 || errno == EINPROGRESS) {
        c.fd = fd;
        if (rc == 0) return connected(id, c);
        c.connecting = true;
        return true;
      }
      int e = errno;
      ::close(fd);
      c.family = c.family == AF_INET ? AF_INET6 : AF_INET;  // localhost is either
      if (e != ECONNREFUSED && e != EADDRNOTAVAIL && e != EAFNOSUPPORT && e != ENETUNREACH)
        return fail(id, c, std::string("connect: ") + std::strerror(e));
    }
    return refused(id, c, now);
  }

  bool refused(uint32_t id, Conn& c, long now) {
    if (now >= c.deadline_us) return fail(id, c, "dial tcp 127.0.0.1:" + std::to_string(c.port) + ": connect: connection refused");
    c.next_try_us = now + kRetryUs;
    return true;
  }

  bool connected(uint32_t id, Conn& c) {
    c.connecting = false;
    c.connected = true;
    int one = 1;
    ::setsockopt(c.fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    send(fwd::frame('C', id));
    return flush(id, c);
  }

  bool fail(uint32_t id, Conn& c, const std::string& why) {
    if (c.fd >= 0) ::close(c.fd);
    c.fd = -1;
    send(fwd::frame('E', id, why));
    return false;
  }

  bool flush(uint32_t id, Conn& c) {
    size_t wrote = 0;
    while (!c.to_app.empty()) {
      ssize_t w = ::send(c.fd, c.to_app.data(), c.to_app.size(), MSG_NOSIGNAL);
      if (w < 0) {
        if (errno == EINTR) continue;
        if (errno == EAGAIN) break;
        return fail(id, c, std::string("write: ") + std::strerror(errno));
      }
      c.to_app.erase(0, (size_t)w);
      wrote += (size_t)w;
    }
    if (wrote) send(fwd::ack_frame(id, wrote));  // the client may send that much more
    if (!c.to_app.empty()) return true;
    if (c.client_fin && !c.shut_wr) {
      ::shutdown(c.fd, SHUT_WR);
      c.shut_wr = true;
    }
    return done_if_both_closed(c);
  }

  bool done_if_both_closed(Conn& c) {
    if (c.app_eof && c.shut_wr) {
      ::close(c.fd);
      c.fd = -1;
      return false;  // both sides finished: forget it (the client has its 'F')
    }
    return true;
  }

  bool on_socket(uint32_t id, Conn& c, short rev, long now) {
    if (c.connecting) {
      if (!(rev & (POLLOUT | POLLERR | POLLHUP))) return true;
      int err = 0;
      socklen_t len = sizeof(err);
      ::getsockopt(c.fd, SOL_SOCKET, SO_ERROR, &err, &len);
      if (err == 0) return connected(id, c);
      ::close(c.fd);
      c.fd = -1;
      c.connecting = false;
      c.family = c.family == AF_INET ? AF_INET6 : AF_INET;
      if (err != ECONNREFUSED) return fail(id, c, std::string("connect: ") + std::strerror(err));
      return refused(id, c, now);
    }
    if (rev & POLLIN) {
      char buf[65536];
      ssize_t n = ::recv(c.fd, buf, sizeof(buf), 0);
      if (n > 0) {
        c.unacked += (uint64_t)n;
        send(fwd::frame('D', id, std::string(buf, (size_t)n)));
      } else if (n == 0) {
        c.app_eof = true;
        send(fwd::frame('F', id));
        if (!done_if_both_closed(c)) return false;
      } else if (errno != EAGAIN && errno != EINTR) {
        return fail(id, c, std::string("read: ") + std::strerror(errno));
      }
    } else if (rev & (POLLERR | POLLHUP)) {
      return fail(id, c, "connection reset by the app");
    }
    if ((rev & POLLOUT) && c.connected) return flush(id, c);
    return true;
  }

  // false at the client's end (stdin EOF or a 'Q' frame)
  bool read_client() {
    char buf[1 << 16];
    while (true) {
      ssize_t n = ::read(0, buf, sizeof(buf));
      if (n == 0) return false;
      if (n < 0) {
        if (errno == EINTR) continue;
        if (errno == EAGAIN) break;
        return false;
      }
      in_.append(buf, (size_t)n);
    }
    size_t pos = 0;
    while (in_.size() - pos >= sync::frame::kHeaderSize) {
      char op;
      uint64_t len;
      sync::frame::parse_header((const unsigned char*)in_.data() + pos, &op, &len);
      if (len > fwd::kMaxFramePayload) return false;  // not our protocol: stop
      if (in_.size() - pos - sync::frame::kHeaderSize < len) break;
      std::string body = in_.substr(pos + sync::frame::kHeaderSize, (size_t)len);
      pos += sync::frame::kHeaderSize + (size_t)len;
      if (op == 'Q') return false;
      if (body.size() < 4) continue;
      on_frame(op, fwd::get_u32be(body, 0), body.substr(4));
    }
    in_.erase(0, pos);
    return true;
  }

  void on_frame(char op, uint32_t id, const std::string& rest) {
    long now = mono_us();
    auto it = conns_.find(id);
    switch (op) {
      case 'O': {
        if (rest.size() < 6 || it != conns_.end()) return;
        Conn c;
        c.port = ((unsigned char)rest[0] << 8) | (unsigned char)rest[1];
        c.deadline_us = now + (long)fwd::get_u32be(rest, 2) * 1000L;
        conns_[id] = std::move(c);
        break;
      }
      case 'D':
        if (it == conns_.end()) return;  // gone: the client has (or gets) its 'E'
        it->second.to_app += rest;
        if (it->second.connected && !flush(id, it->second)) conns_.erase(it);
        break;
      case 'F':
        if (it == conns_.end()) return;
        it->second.client_fin = true;
        if (it->second.connected && !flush(id, it->second)) conns_.erase(it);
        break;
      case 'A':
        if (it == conns_.end() || rest.size() < 4) return;
        it->second.unacked -= std::min<uint64_t>(it->second.unacked, fwd::get_u32be(rest, 0));
        break;
      case 'K':
        if (it == conns_.end()) return;
        if (it->second.fd >= 0) ::close(it->second.fd);
        conns_.erase(it);
        break;
      default:
        break;
    }
  }

  void send(const std::string& f) {
    if (!write_all(1, f)) std::_Exit(0);  // the client is gone
  }

  std::map<uint32_t, Conn> conns_;
  std::string in_;
};

}  // namespace

int forward_main() {
  ::signal(SIGPIPE, SIG_IGN);
  write_all(1, "FORWARD READY\n");
  return Forwarder().run();
}

}  // namespace helper
}  // namespace ds

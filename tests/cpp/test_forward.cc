// `devspace-helper forward` (src/helper/forward.cc): a connection the app refuses is held in the
// pod and made once when the app listens; what the client sent meanwhile arrives exactly once;
// the hold ends with a refusal; several connections share the stream.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <map>
#include <mutex>
#include <thread>

#include "core/proc.h"
#include "sync/fwd_proto.h"
#include "sync/transport.h"
#include "testing.h"

using namespace ds;
namespace fwd = ds::sync::fwd;

namespace {

int free_port() {
  int s = ::socket(AF_INET, SOCK_STREAM, 0);
  struct sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  ::bind(s, (struct sockaddr*)&a, sizeof(a));
  socklen_t len = sizeof(a);
  ::getsockname(s, (struct sockaddr*)&a, &len);
  ::close(s);
  return ntohs(a.sin_port);
}

// A one-shot HTTP-ish server: counts connections, reads until the client half-closes, answers.
struct Server {
  int lfd = -1;
  std::atomic<int> conns{0};
  std::mutex mu;
  std::string got_;
  std::string got() {
    std::lock_guard<std::mutex> g(mu);
    return got_;
  }
  std::thread t;
  void start(int port, const std::string& reply) {
    lfd = ::socket(AF_INET, SOCK_STREAM, 0);
    int one = 1;
    ::setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    struct sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    if (::bind(lfd, (struct sockaddr*)&a, sizeof(a)) != 0 || ::listen(lfd, 8) != 0) throw std::runtime_error("bind");
    t = std::thread([this, reply] {
      struct pollfd pf{lfd, POLLIN, 0};
      while (::poll(&pf, 1, 3000) > 0) {
        int c = ::accept(lfd, nullptr, nullptr);
        if (c < 0) return;
        conns++;
        char buf[4096];
        ssize_t n;
        while ((n = ::read(c, buf, sizeof(buf))) > 0) {
          std::lock_guard<std::mutex> g(mu);
          got_.append(buf, (size_t)n);
        }
        ssize_t w = ::write(c, reply.data(), reply.size());
        (void)w;
        ::close(c);
      }
    });
  }
  ~Server() {
    if (lfd >= 0) ::shutdown(lfd, SHUT_RDWR);
    if (t.joinable()) t.join();
    if (lfd >= 0) ::close(lfd);
  }
};

struct Helper {
  Process p;
  sync::LineReader out;
  Helper() {
    ProcOptions o;
    o.pipe_stderr = false;
    if (!p.start({DEVSPACE_SOURCE_DIR "/bin/devspace-helper", "forward"}, o)) throw std::runtime_error(p.error());
    out.reset(p.stdout_fd());
    std::string line;
    if (!out.read_line(&line, 5000) || line != "FORWARD READY") throw std::runtime_error("no ready line: " + line);
  }
  void send(const std::string& f) { write_all(p.stdin_fd(), f); }
  std::map<uint32_t, uint64_t> acked;  // per id: the client's bytes the helper wrote to the app
  // the next frame other than an acknowledgement: (op, id, body); op 0 on timeout
  std::tuple<char, uint32_t, std::string> next(int timeout_ms = 5000) {
    while (true) {
      std::string hdr, body;
      if (!out.read_exact(&hdr, sync::frame::kHeaderSize, timeout_ms)) return {0, 0, ""};
      char op;
      uint64_t len;
      sync::frame::parse_header((const unsigned char*)hdr.data(), &op, &len);
      if (!out.read_exact(&body, (size_t)len, timeout_ms)) return {0, 0, ""};
      uint32_t id = fwd::get_u32be(body, 0);
      if (op == 'A') {
        acked[id] += fwd::get_u32be(body, 4);
        continue;
      }
      return {op, id, body.substr(4)};
    }
  }
};

}  // namespace

TEST(helper_forward_holds_a_refused_connection_in_the_pod_and_delivers_once) {
  Helper h;
  int port = free_port();
  const std::string req = "GET /held HTTP/1.0\r\n\r\n";
  auto t0 = std::chrono::steady_clock::now();
  h.send(fwd::open_frame(1, port, 3000));
  h.send(fwd::frame('D', 1, req));
  h.send(fwd::frame('F', 1));
  std::this_thread::sleep_for(std::chrono::milliseconds(150));  // the app is "restarting"
  Server s;
  s.start(port, "hello");
  auto [op, id, body] = h.next();
  EXPECT_EQ(op, 'C');
  EXPECT_EQ(id, (uint32_t)1);
  auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
  EXPECT_TRUE(ms < 150 + 50);  // connected within a few retry periods of the listen
  std::string reply;
  while (true) {
    auto [op2, id2, b2] = h.next();
    EXPECT_EQ(id2, (uint32_t)1);
    if (op2 == 'D') {
      reply += b2;
      continue;
    }
    EXPECT_EQ(op2, 'F');
    break;
  }
  EXPECT_EQ(reply, std::string("hello"));
  std::this_thread::sleep_for(std::chrono::milliseconds(50));
  EXPECT_EQ(s.conns.load(), 1);
  EXPECT_EQ(s.got(), req);
  EXPECT_EQ(h.acked[1], (uint64_t)req.size());  // written to the app: acknowledged
}

TEST(helper_forward_keeps_at_most_a_window_unacknowledged_per_connection) {
  // the app sends 24 MiB at once; the client reads frames but acknowledges nothing at first: the
  // helper stops reading the app after a window, then goes on as acknowledgements arrive
  int lfd = ::socket(AF_INET, SOCK_STREAM, 0);
  int one = 1;
  ::setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  int port = free_port();
  struct sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  EXPECT_EQ(::bind(lfd, (struct sockaddr*)&a, sizeof(a)), 0);
  EXPECT_EQ(::listen(lfd, 1), 0);
  const size_t total = 24u << 20;
  std::atomic<size_t> sent{0};
  std::thread app([&] {
    int c = ::accept(lfd, nullptr, nullptr);
    std::string chunk(1 << 16, 'z');
    while (sent < total) {
      ssize_t w = ::write(c, chunk.data(), std::min(chunk.size(), total - sent.load()));
      if (w <= 0) break;
      sent += (size_t)w;
    }
    ::close(c);
  });
  Helper h;
  h.send(fwd::open_frame(3, port, 1000));
  size_t got = 0;
  bool ended = false;
  // without acknowledgements: what arrives stops at about a window
  while (true) {
    auto [op, id, body] = h.next(500);
    if (op == 0) break;
    EXPECT_EQ(id, (uint32_t)3);
    if (op == 'D') got += body.size();
    if (op == 'F') ended = true;
  }
  EXPECT_TRUE(!ended);
  EXPECT_TRUE(got >= fwd::kWindow && got < fwd::kWindow + (1u << 17));
  EXPECT_TRUE(sent.load() < total);  // the app is held back by TCP, not buffered in the helper
  // acknowledging as the client writes it out: the rest flows
  uint64_t unacked = got;
  while (!ended) {
    if (unacked) {
      h.send(fwd::ack_frame(3, unacked));
      unacked = 0;
    }
    auto [op, id, body] = h.next(5000);
    EXPECT_TRUE(op != 0);
    if (op == 0) break;
    if (op == 'D') {
      got += body.size();
      unacked += body.size();
    }
    if (op == 'F') ended = true;
  }
  EXPECT_EQ(got, total);
  app.join();
  ::close(lfd);
}

TEST(helper_forward_refuses_after_the_hold_and_multiplexes) {
  Helper h;
  int dead = free_port();
  h.send(fwd::open_frame(7, dead, 60));
  auto t0 = std::chrono::steady_clock::now();
  auto [op, id, body] = h.next();
  auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
  EXPECT_EQ(op, 'E');
  EXPECT_EQ(id, (uint32_t)7);
  EXPECT_TRUE(body.find("connection refused") != std::string::npos);
  EXPECT_TRUE(ms >= 50 && ms < 1000);
  // two connections at once on one stream, each answered on its own id
  int port = free_port();
  Server s;
  s.start(port, "pong");
  for (uint32_t i : {11u, 12u}) {
    h.send(fwd::open_frame(i, port, 1000));
    h.send(fwd::frame('D', i, "ping" + std::to_string(i)));
    h.send(fwd::frame('F', i));
  }
  std::map<uint32_t, std::string> replies;
  int ends = 0;
  while (ends < 2) {
    auto [o, i, b] = h.next();
    EXPECT_TRUE(o != 0);
    if (o == 'D') replies[i] += b;
    if (o == 'F') ends++;
  }
  EXPECT_EQ(replies[11], std::string("pong"));
  EXPECT_EQ(replies[12], std::string("pong"));
  EXPECT_EQ(s.conns.load(), 2);
}

// Port forwarding (services/port_forwarding.go:18, kubectl/client.go:356): local listeners, one
// multiplexed tunnel per pod (or a WebSocket per connection), held connections replayed across
// an app restart, hedged retries of repeatable requests on a remote cluster.
#include "services/services.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstring>

#include "core/compat.h"
#include "core/log.h"
#include "core/resolve.h"
#include "core/strutil.h"
#include "core/codec.h"
#include "core/fs.h"
#include "core/trace.h"
#include "platform/platform.h"
#include "sync/fwd_proto.h"

namespace ds {
namespace services {

static long mono_ms() {
  return (long)std::chrono::duration_cast<std::chrono::milliseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// ---------------------------------------------------------------- port forwarding

PortForwarder::PortForwarder(std::shared_ptr<kube::Client> k, Value pod, std::vector<std::pair<int, int>> ports,
                             std::vector<std::string> addresses, std::string label_selector)
    : k_(std::move(k)), pod_(std::move(pod)), selector_(std::move(label_selector)), ports_(std::move(ports)),
      addrs_(std::move(addresses)) {
  ns_ = pod_.at_path("metadata.namespace").as_string();
}

PortForwarder::~PortForwarder() { close(); }

std::string PortForwarder::describe() const {
  std::vector<std::string> p;
  for (auto& pr : ports_) p.push_back(std::to_string(pr.first) + ":" + std::to_string(pr.second));
  return join(p, ", ");
}

std::string PortForwarder::pod_name() {
  std::lock_guard<std::mutex> g(pod_mu_);
  return pod_.at_path("metadata.name").as_string();
}

size_t PortForwarder::active_connections() {
  std::lock_guard<std::mutex> g(conns_mu_);
  size_t n = 0;
  for (auto& c : conns_) n += !c->done;
  return n;
}

// Listen addresses for one mapping's bindAddress, as `kubectl port-forward --address` reads
// them: "localhost" (the default) is 127.0.0.1 plus ::1, an IPv6 literal ("::1", "[::1]", "::")
// binds an AF_INET6 socket, a host name goes through the resolver. Returns (family, address).
std::vector<std::pair<int, std::string>> listen_addresses(const std::string& bind) {
  std::string a = bind.empty() ? "localhost" : bind;
  if (a.size() > 2 && a.front() == '[' && a.back() == ']') a = a.substr(1, a.size() - 2);
  if (to_lower(a) == "localhost") return {{AF_INET, "127.0.0.1"}, {AF_INET6, "::1"}};
  struct in_addr v4;
  struct in6_addr v6;
  if (inet_pton(AF_INET, a.c_str(), &v4) == 1) return {{AF_INET, a}};
  if (inet_pton(AF_INET6, a.c_str(), &v6) == 1) return {{AF_INET6, a}};
  std::vector<std::pair<int, std::string>> out;
  for (auto& r : net::resolve(a, 0)) out.push_back({r.family, r.text});
  if (out.empty()) throw std::runtime_error("Unable to resolve port-forward address \"" + bind + "\"");
  return out;
}

// One listening socket or -errno. "::" is dual-stack (also takes IPv4), every other IPv6
// address is v6-only so it can sit next to the IPv4 listener on the same port.
static int listen_on(int family, const std::string& addr, int port) {
  int fd = plat::socket_cloexec(family, SOCK_STREAM);
  if (fd < 0) return -errno;
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  struct sockaddr_storage ss{};
  socklen_t len;
  if (family == AF_INET6) {
    auto* a6 = (struct sockaddr_in6*)&ss;
    a6->sin6_family = AF_INET6;
    a6->sin6_port = htons((uint16_t)port);
    inet_pton(AF_INET6, addr.c_str(), &a6->sin6_addr);
    int v6only = addr == "::" ? 0 : 1;
    setsockopt(fd, IPPROTO_IPV6, IPV6_V6ONLY, &v6only, sizeof(v6only));
    len = sizeof(*a6);
  } else {
    auto* a4 = (struct sockaddr_in*)&ss;
    a4->sin_family = AF_INET;
    a4->sin_port = htons((uint16_t)port);
    inet_pton(AF_INET, addr.c_str(), &a4->sin_addr);
    len = sizeof(*a4);
  }
  if (::bind(fd, (struct sockaddr*)&ss, len) != 0 || ::listen(fd, 64) != 0) {
    int err = errno;
    ::close(fd);
    return -err;
  }
  return fd;
}

// One forwarded connection's stream(s), as the connection handler sees them.
class FwdStream {
 public:
  virtual ~FwdStream() = default;
  // client -> pod bytes
  virtual bool send(const std::string& data) = 0;
  // The next event: channel 0 bytes from the pod, channel 1 an error message. false at the end.
  virtual bool recv(int* channel, std::string* data) = 0;
  // the client finished sending (a tunnel stream half-closes; a WebSocket cannot)
  virtual void close_write() {}
  virtual void close() = 0;
  virtual const char* via() const = 0;
  // the stream ended because its tunnel did (no reply, no error from the pod)
  virtual bool tunnel_lost() const { return false; }
};

namespace {

// portforward.k8s.io over a WebSocket of its own: channel byte 0 data / 1 error, and each
// channel's first frame carries the port number (2 bytes LE).
class WsFwd : public FwdStream {
 public:
  explicit WsFwd(std::unique_ptr<net::WebSocket> ws) : ws_(std::move(ws)) {}
  bool send(const std::string& data) override { return ws_->send(std::string(1, '\0') + data); }
  bool recv(int* channel, std::string* data) override {
    std::string msg;
    while (ws_->recv(&msg)) {
      if (msg.empty()) continue;
      int ch = (unsigned char)msg[0];
      std::string d = msg.substr(1);
      if (ch == 0 && first_data_) {
        first_data_ = false;
        if (d.size() == 2) continue;
      }
      if (ch == 1 && first_err_) {
        first_err_ = false;
        if (d.size() == 2) continue;
      }
      *channel = ch;
      *data = std::move(d);
      return true;
    }
    return false;
  }
  void close() override { ws_->close(); }
  const char* via() const override { return "websocket"; }

 private:
  std::unique_ptr<net::WebSocket> ws_;
  bool first_data_ = true, first_err_ = true;
};

// Disk a tunnel connection may use for what its local reader has not taken yet
// (kube::SpdyMailbox): DEVSPACE_PORTFORWARD_SPILL_MB, default 1024; 0 = none (the tunnel's
// reader then waits for a slow reader, holding up the pod's other connections).
uint64_t tunnel_spill_cap() {
  static const uint64_t cap = [] {
    const char* v = std::getenv("DEVSPACE_PORTFORWARD_SPILL_MB");
    long long mb = v && *v ? std::atoll(v) : 1024;
    return (uint64_t)(mb < 0 ? 0 : mb) << 20;
  }();
  return cap;
}

// A stream pair in the pod's tunnel, as kubectl creates it: an error stream (the client never
// writes to it) and a data stream, tied by a request id. The data follows the SYN_STREAM at once.
class TunnelFwd : public FwdStream {
 public:
  TunnelFwd(std::shared_ptr<kube::SpdySession> s, int port, uint64_t request_id) : s_(std::move(s)) {
    box_->spill_cap = tunnel_spill_cap();
    std::string p = std::to_string(port), id = std::to_string(request_id);
    err_ = s_->open({{"streamtype", "error"}, {"port", p}, {"requestid", id}}, box_, 1, true);
    try {
      data_ = s_->open({{"streamtype", "data"}, {"port", p}, {"requestid", id}}, box_, 0);
    } catch (...) {
      // a GOAWAY between the two opens: the error stream must not stay in the session
      s_->reset(err_);
      box_->close();
      throw;
    }
  }
  ~TunnelFwd() override { close(); }
  bool send(const std::string& data) override { return s_->send(data_, data); }
  bool recv(int* channel, std::string* data) override {
    kube::SpdyMailbox::Event e;
    while (!data_done_ && box_->pop(&e)) {
      if (e.end) {
        if (e.channel == 0) {
          data_done_ = true;
          lost_ = e.reset == "tunnel closed" || e.reset == "closed";  // SpdySession::end_all
        }
        continue;
      }
      if (e.channel == 0) s_->consumed(data_, e.data.size());
      *channel = e.channel;
      *data = std::move(e.data);
      return true;
    }
    return false;
  }
  void close_write() override { s_->send(data_, "", true); }
  void close() override {
    if (closed_) return;
    closed_ = true;
    // abandoned (stop, a failed client write): the server stops forwarding; a recv() still
    // waiting in another thread returns, and the session's reader never blocks on this mailbox
    s_->reset(data_);
    s_->reset(err_);
    box_->close();
  }
  const char* via() const override { return "tunnel"; }
  bool tunnel_lost() const override { return lost_; }

 private:
  std::shared_ptr<kube::SpdySession> s_;
  std::shared_ptr<kube::SpdyMailbox> box_ = std::make_shared<kube::SpdyMailbox>();
  std::shared_ptr<kube::SpdySession::Stream> err_, data_;
  bool data_done_ = false, closed_ = false, lost_ = false;
};

bool port_forward_tunnel_enabled() {
  const char* v = std::getenv("DEVSPACE_PORTFORWARD_TUNNEL");
  return !(v && std::string(v) == "0") && !reference_timing();  // the reference dials per stream
}

}  // namespace

std::shared_ptr<kube::SpdySession> PortForwarder::tunnel_for(const std::string& pod) {
  if (tunnel_mode_ == 0) return nullptr;
  std::lock_guard<std::mutex> g(tunnel_mu_);
  if (tunnel_ && tunnel_pod_ == pod && tunnel_->usable()) return tunnel_;
  if (tunnel_) {
    tunnel_->close();
    tunnel_.reset();
  }
  std::vector<int> remote;
  for (auto& pr : ports_) remote.push_back(pr.second);
  auto t = k_->portforward_tunnel(ns_, pod, remote);  // throws when the pod is gone
  if (!t) {
    tunnel_mode_ = 0;
    log::file_logger("portforwarding")->emit("info", "The API server has no multiplexed port-forward "
                                             "(SPDY/3.1+portforward.k8s.io): one WebSocket per connection", {});
    return nullptr;
  }
  tunnel_mode_ = 1;
  tunnels_opened_++;
  t->ping();  // its answer tells a remote cluster from one next door (hedging below)
  tunnel_ = t;
  tunnel_pod_ = pod;
  tunnel_requests_ = 0;
  return t;
}

int64_t PortForwarder::tunnel_rtt_us() {
  std::lock_guard<std::mutex> g(tunnel_mu_);
  // the smallest of several: one PING answered late by a busy API server next door is no link
  return tunnel_ && tunnel_->rtt_samples() >= 5 ? tunnel_->rtt_us() : -1;
}

bool PortForwarder::drop_tunnel_if_pod_gone(const std::string& pod) {
  std::string uid;
  {
    std::lock_guard<std::mutex> g(pod_mu_);
    // re-selected meanwhile: the next stream goes to the new pod's tunnel
    if (pod_.at_path("metadata.name").as_string() != pod) return true;
    uid = pod_.at_path("metadata.uid").as_string();
  }
  std::optional<Value> live;
  try {
    live = k_->try_get("/api/v1/namespaces/" + ns_ + "/pods/" + pod);
  } catch (const std::exception&) {
    return false;  // cannot tell (API server unreachable): keep the tunnel
  }
  if (live) {
    const std::string phase = live->at_path("status.phase").as_string();
    const std::string live_uid = live->at_path("metadata.uid").as_string();
    if (phase != "Succeeded" && phase != "Failed" && live_uid == uid) return false;
    if (live_uid != uid && phase == "Running") {
      // the same name, a new pod (a StatefulSet's replacement): forward to it
      std::lock_guard<std::mutex> g(pod_mu_);
      if (pod_.at_path("metadata.name").as_string() == pod) pod_ = *live;
      reselections_++;
      log::info("Port forwarding " + describe() + " now targets pod " + pod + " (replaced)");
    }
  }
  std::lock_guard<std::mutex> g(tunnel_mu_);
  if (tunnel_ && tunnel_pod_ == pod) {
    tunnel_->close();
    tunnel_.reset();
  }
  return true;
}

std::unique_ptr<FwdStream> PortForwarder::open_to(const std::string& pod, int remote_port) {
  for (int tries = 0; tries < 2 && tunnel_mode_ != 0; ++tries) {
    auto t = tunnel_for(pod);
    if (!t) break;
    try {
      return std::make_unique<TunnelFwd>(t, remote_port, tunnel_requests_++);
    } catch (const net::NetError&) {
      // the tunnel just closed (API server restart, idle timeout): a new one
    }
  }
  return std::make_unique<WsFwd>(k_->portforward(ns_, pod, remote_port, take_spare()));
}

void PortForwarder::spare_loop() {
  const long kMaxAgeMs = 30000;  // below API-server idle timeouts; re-dialed after that
  std::unique_lock<std::mutex> lk(spare_mu_);
  while (!stop_) {
    if (tunnel_mode_ != 0 && port_forward_tunnel_enabled()) {
      // keep the pod's tunnel open (re-opened after the API server closed it), so the first
      // connection after a quiet spell does not pay the upgrade either
      lk.unlock();
      try {
        // and measure its round trip now and then (hedging needs it; the smallest one counts)
        if (auto t = tunnel_for(pod_name())) t->ping();
      } catch (const std::exception&) {
      }
      lk.lock();
      if (tunnel_mode_ == 1) {
        spares_.clear();
        // hedging needs the round trip: PINGs every 100 ms until the tunnel has ten answers (known
        // within a second of opening), then every second; a far end that leaves five unanswered
        // gets one a second. Without hedging, one a second keeps the tunnel warm.
        int samples = 0;
        size_t unanswered = 0;
        {
          std::lock_guard<std::mutex> g(tunnel_mu_);
          if (tunnel_) {
            samples = tunnel_->rtt_samples();
            unanswered = tunnel_->pings_in_flight();
          }
        }
        bool fast = (hedge_ || !helper_file_.empty()) && samples < 10 && unanswered < 5;
        lk.unlock();
        maintain_helper_link();
        lk.lock();
        // the first five round trips within ~0.1 s (the helper link waits for them), the next
        // five at 100 ms, then one a second
        int wait_ms = !fast ? 1000 : samples < 5 ? 20 : 100;
        spare_cv_.wait_for(lk, std::chrono::milliseconds(wait_ms), [this] { return stop_.load(); });
        continue;
      }
    }
    while (!spares_.empty() && mono_ms() - spares_.front().first > kMaxAgeMs) spares_.pop_front();
    if ((int)spares_.size() < want_spares_) {
      lk.unlock();
      std::unique_ptr<net::Conn> c;
      try {
        c = k_->http().connect();
      } catch (const std::exception&) {
      }
      lk.lock();
      if (c) {
        spares_.emplace_back(mono_ms(), std::move(c));
      } else {
        spare_cv_.wait_for(lk, std::chrono::seconds(1), [this] { return stop_.load(); });
      }
      continue;
    }
    spare_cv_.wait_for(lk, std::chrono::seconds(5),
                       [this] { return stop_.load() || (int)spares_.size() < want_spares_; });
  }
  spares_.clear();
}

std::unique_ptr<net::Conn> PortForwarder::take_spare() {
  std::unique_ptr<net::Conn> c;
  {
    std::lock_guard<std::mutex> g(spare_mu_);
    while (!spares_.empty() && !c) {
      c = std::move(spares_.front().second);
      spares_.pop_front();
      if (c->stale()) c.reset();
    }
  }
  spare_cv_.notify_one();
  if (c) spares_used_++;
  return c;
}

void PortForwarder::start() {
  if (const char* v = std::getenv("DEVSPACE_PORTFORWARD_SPARES")) {
    want_spares_ = std::max(0, std::min(8, std::atoi(v)));
  } else {
    want_spares_ = reference_timing() ? 0 : 2;  // the reference dials every stream
  }
  if (!port_forward_tunnel_enabled()) tunnel_mode_ = 0;
  if (hedge_)
    log::file_logger("portforwarding")
        ->emit("info",
               "DEVSPACE_PORTFORWARD_HEDGE=1: a held GET/HEAD/OPTIONS on a remote cluster may reach the app more "
               "than once",
               {});
  if (want_spares_ > 0 || tunnel_mode_ != 0) spare_thread_ = std::thread([this] { spare_loop(); });
  for (size_t i = 0; i < ports_.size(); ++i) {
    std::string bind = i < addrs_.size() ? addrs_[i] : "";
    auto addrs = listen_addresses(bind);
    bool is_default = addrs.size() == 2 && addrs[0].second == "127.0.0.1" && addrs[1].second == "::1";
    int bound = 0;
    int first_err = 0;
    for (size_t k = 0; k < addrs.size(); ++k) {
      int fd = listen_on(addrs[k].first, addrs[k].second, ports_[i].first);
      if (fd < 0) {
        // kubectl tolerates one of localhost's two families failing (a host without IPv6)
        if (is_default && k == 1 && bound > 0) continue;
        if (!first_err) first_err = -fd;
        continue;
      }
      listeners_.push_back(fd);
      ++bound;
      int rp = ports_[i].second;
      threads_.emplace_back([this, fd, rp] { accept_loop(fd, rp); });
    }
    if (bound == (int)addrs.size() || (is_default && bound > 0)) continue;
    // Pods of the bundled local cluster share the host network: a same-number mapping is
    // already served by the container itself.
    if (bound == 0 && first_err == EADDRINUSE && k_->is_local_cluster() && ports_[i].first == ports_[i].second) {
      log::info("Port " + std::to_string(ports_[i].first) +
                " is served directly by the pod (local cluster shares the host network)");
      continue;
    }
    throw std::runtime_error("Unable to listen on " + (bind.empty() ? std::string("localhost") : bind) + ":" +
                             std::to_string(ports_[i].first) + ": " + std::strerror(first_err));
  }
}

void PortForwarder::reap(bool all) {
  std::vector<std::unique_ptr<Conn>> finished;
  {
    std::lock_guard<std::mutex> g(conns_mu_);
    for (auto it = conns_.begin(); it != conns_.end();) {
      if (all || (*it)->done) {
        finished.push_back(std::move(*it));
        it = conns_.erase(it);
      } else {
        ++it;
      }
    }
  }
  for (auto& c : finished)
    if (c->t.joinable()) c->t.join();
}

void PortForwarder::accept_loop(int lfd, int remote_port) {
  while (!stop_) {
    reap(false);
    struct pollfd pf{lfd, POLLIN, 0};
    if (::poll(&pf, 1, 200) <= 0) continue;
    int cfd = plat::accept_cloexec(lfd);
    if (cfd < 0) continue;
    auto c = std::make_unique<Conn>();
    c->fd = cfd;
    Conn* raw = c.get();
    std::lock_guard<std::mutex> g(conns_mu_);
    if (stop_) {
      ::close(cfd);
      break;
    }
    conns_.push_back(std::move(c));
    raw->t = std::thread([this, raw, remote_port] { handle(raw, remote_port); });
  }
}

std::unique_ptr<FwdStream> PortForwarder::open_stream(int remote_port) {
  Value pod;
  {
    std::lock_guard<std::mutex> g(pod_mu_);
    pod = pod_;
  }
  std::string name = pod.at_path("metadata.name").as_string();
  try {
    return open_to(name, remote_port);
  } catch (const std::exception& e) {
    if (selector_.empty() || stop_) throw;
    // the pod is gone or not running any more: follow the selector to its newest pod
    Value fresh = k_->newest_running_pod(ns_, selector_, 60000);
    std::string fresh_name = fresh.at_path("metadata.name").as_string();
    if (fresh_name == name) throw;
    {
      std::lock_guard<std::mutex> g(pod_mu_);
      pod_ = fresh;
    }
    reselections_++;
    log::file_logger("portforwarding")->emit("info", "Pod " + name + " is gone (" + e.what() +
                                             "), forwarding to " + fresh_name, {});
    log::info("Port forwarding " + describe() + " now targets pod " + fresh_name);
    return open_to(fresh_name, remote_port);
  }
}

std::unique_ptr<FwdStream> PortForwarder::open_stream_direct(int remote_port) {
  return open_to(pod_name(), remote_port);
}

namespace {
// The next attempt of a held connection, opened on its own thread while the current attempt
// waits for its reply or refusal. Opening a stream is the bulk of an attempt (the WebSocket
// upgrade through the API server, and the pod-side dial that comes with it), so overlapping
// it with the wait roughly halves the retry period. Only one stream of a connection ever
// carries the client's bytes at a time: the next one gets them only after this one was
// refused, so a request still reaches the app at most once.
class PreOpened {
 public:
  template <class F>
  explicit PreOpened(F open) : t_([this, open] {
      try {
        ws_ = open();
      } catch (const std::exception&) {
        ws_.reset();  // the caller falls back to a synchronous open (with pod re-selection)
      }
      done_ = true;
    }) {}
  // the open finished: take() / discard() will not block
  bool ready() const { return done_; }
  ~PreOpened() { discard(); }
  std::unique_ptr<FwdStream> take() {
    if (t_.joinable()) t_.join();
    return std::move(ws_);
  }
  void discard() {
    auto ws = take();
    if (ws) ws->close();
  }

 private:
  std::unique_ptr<FwdStream> ws_;
  std::atomic<bool> done_{false};
  std::thread t_;  // declared last: the thread starts once ws_ and done_ exist
};
}  // namespace

// ---------------------------------------------------------------- forwarding through the helper
// One exec stream per pod running `devspace-helper forward` (src/helper/forward.cc, protocol
// src/sync/fwd_proto.h): every connection of the forward is multiplexed over it, and a connect
// the restarting app refuses is retried in the pod every 2 ms, so a held request reaches the new
// server within ms of it listening instead of up to a round trip later, and exactly once.

struct HelperBox {
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::pair<char, std::string>> q;
  bool closed = false;     // the link ended
  bool gone = false;       // the connection ended ('E' from the helper, or closed here)
  uint64_t in_flight = 0;  // bytes sent to the helper that it has not acknowledged ('A')
};

class HelperLink {
 public:
  // `sh` in the container, the helper the sync put there (content-addressed `file`) exec'd in
  // forward mode; nullptr with *why when it is not there (the forward never uploads it).
  static std::shared_ptr<HelperLink> open(sync::Transport& t, const std::string& file, std::string* why) {
    auto sh = t.open({"sh"});
    if (!sh) {
      *why = "no shell";
      return nullptr;
    }
    std::string probe = sync::helper_probe_script(file, sync::helper_dirs(), "exec \"$dsd/" + file + "\" forward");
    if (!write_all(sh->in(), probe)) {
      *why = "exec stream closed";
      return nullptr;
    }
    auto link = std::shared_ptr<HelperLink>(new HelperLink(std::move(sh)));
    std::string line;
    if (!link->out_.read_line(&line, 15000) || !starts_with(line, "HAVE ")) {
      *why = line.empty() ? "no answer from the probe" : "helper not in the container (" + line + ")";
      link->close();
      return nullptr;
    }
    if (!link->out_.read_line(&line, 15000) || line != "FORWARD READY") {
      *why = "the helper did not start its forward mode (" + line + ")";
      link->close();
      return nullptr;
    }
    link->th_ = std::thread([l = link.get()] { l->reader(); });
    return link;
  }
  ~HelperLink() { close(); }
  bool usable() const { return !dead_; }
  // Registers a connection and sends its 'O' frame; 0 when the link is gone.
  uint32_t open_conn(int port, uint32_t hold_ms, std::shared_ptr<HelperBox>* box) {
    auto b = std::make_shared<HelperBox>();
    uint32_t id;
    {
      std::lock_guard<std::mutex> g(mu_);
      id = next_++;
      boxes_[id] = b;
    }
    *box = b;
    if (!send(sync::fwd::open_frame(id, port, hold_ms))) return 0;
    return id;
  }
  bool send(const std::string& frame) {
    if (dead_) return false;
    std::lock_guard<std::mutex> g(wmu_);
    if (!write_all(sh_->in(), frame)) {
      dead_ = true;
      return false;
    }
    return true;
  }
  void forget(uint32_t id) {
    std::lock_guard<std::mutex> g(mu_);
    boxes_.erase(id);
  }
  void close() {
    if (closed_.exchange(true)) return;
    dead_ = true;
    if (sh_) sh_->terminate();
    if (th_.joinable()) th_.join();
    if (sh_) sh_->close();
    end_all();
  }

 private:
  explicit HelperLink(std::unique_ptr<sync::Shell> sh) : sh_(std::move(sh)), out_(sh_->out()) {}
  void end_all() {
    std::map<uint32_t, std::shared_ptr<HelperBox>> boxes;
    {
      std::lock_guard<std::mutex> g(mu_);
      boxes.swap(boxes_);
    }
    for (auto& kv : boxes) {
      {
        std::lock_guard<std::mutex> g(kv.second->mu);
        kv.second->closed = true;
      }
      kv.second->cv.notify_all();
    }
  }
  void reader() {
    std::string hdr, body;
    while (!closed_) {
      if (!out_.read_exact(&hdr, sync::frame::kHeaderSize, -1)) break;
      char op;
      uint64_t len;
      sync::frame::parse_header((const unsigned char*)hdr.data(), &op, &len);
      if (len < 4 || len > sync::fwd::kMaxFramePayload || !out_.read_exact(&body, (size_t)len, -1)) break;
      uint32_t id = sync::fwd::get_u32be(body, 0);
      std::shared_ptr<HelperBox> b;
      {
        std::lock_guard<std::mutex> g(mu_);
        auto it = boxes_.find(id);
        if (it != boxes_.end()) b = it->second;
        if (op == 'E' && it != boxes_.end()) boxes_.erase(it);  // the helper forgot it too
      }
      if (!b) continue;
      {
        std::lock_guard<std::mutex> g(b->mu);
        if (op == 'A') {
          if (body.size() >= 8) b->in_flight -= std::min<uint64_t>(b->in_flight, sync::fwd::get_u32be(body, 4));
        } else {
          if (op == 'E') b->gone = true;
          b->q.emplace_back(op, body.substr(4));
        }
      }
      b->cv.notify_all();
    }
    dead_ = true;
    end_all();
  }
  std::unique_ptr<sync::Shell> sh_;
  sync::LineReader out_;
  std::mutex wmu_, mu_;
  std::map<uint32_t, std::shared_ptr<HelperBox>> boxes_;
  uint32_t next_ = 1;
  std::atomic<bool> dead_{false}, closed_{false};
  std::thread th_;
};

namespace {
class HelperFwd : public FwdStream {
 public:
  HelperFwd(std::shared_ptr<HelperLink> link, int port, uint32_t hold_ms) : link_(std::move(link)) {
    id_ = link_->open_conn(port, hold_ms, &box_);
    if (!id_) throw std::runtime_error("helper link closed");
  }
  ~HelperFwd() override { close(); }
  // Blocks while the helper holds a window's worth of this connection's data unwritten to the app.
  bool send(const std::string& data) override {
    constexpr size_t kChunk = 256u << 10;
    for (size_t off = 0; off < data.size(); off += kChunk) {
      const size_t n = std::min(kChunk, data.size() - off);
      {
        std::unique_lock<std::mutex> lk(box_->mu);
        box_->cv.wait(lk, [&] { return box_->in_flight + n <= sync::fwd::kWindow || box_->closed || box_->gone; });
        if (box_->closed || box_->gone) return false;
        box_->in_flight += n;
      }
      if (!link_->send(sync::fwd::frame('D', id_, data.substr(off, n)))) return false;
    }
    return true;
  }
  // The caller writes what a call returns to its local connection before it calls again: what the
  // previous calls returned is acknowledged here, every kAckEvery bytes or before waiting.
  bool recv(int* channel, std::string* data) override {
    uint64_t ack = 0;
    {
      std::lock_guard<std::mutex> g(box_->mu);
      if (unacked_ >= sync::fwd::kAckEvery || (unacked_ && box_->q.empty())) std::swap(ack, unacked_);
    }
    if (ack) link_->send(sync::fwd::ack_frame(id_, ack));  // outside the box's lock: the reader takes it
    std::unique_lock<std::mutex> lk(box_->mu);
    while (true) {
      box_->cv.wait(lk, [this] { return !box_->q.empty() || box_->closed || ended_; });
      if (box_->q.empty()) {
        if (!ended_) lost_ = true;  // the link ended under this connection
        return false;
      }
      auto ev = std::move(box_->q.front());
      box_->q.pop_front();
      switch (ev.first) {
        case 'C':
          connected_ = true;
          continue;
        case 'D':
          *channel = 0;
          *data = std::move(ev.second);
          unacked_ += data->size();
          return true;
        case 'F':
          ended_ = true;
          return false;
        case 'E':
          ended_ = true;  // the next recv ends the stream
          *channel = 1;
          *data = std::move(ev.second);
          return true;
        default:
          continue;
      }
    }
  }
  void close_write() override { link_->send(sync::fwd::frame('F', id_)); }
  void close() override {
    if (closed_) return;
    closed_ = true;
    link_->send(sync::fwd::frame('K', id_));
    link_->forget(id_);
    {
      std::lock_guard<std::mutex> g(box_->mu);
      ended_ = true;
      box_->gone = true;
    }
    box_->cv.notify_all();
  }
  const char* via() const override { return "helper"; }
  bool tunnel_lost() const override { return lost_; }
  // the helper connected to the app: what was sent may have reached it
  bool delivered() const { return connected_; }

 private:
  std::shared_ptr<HelperLink> link_;
  std::shared_ptr<HelperBox> box_;
  uint32_t id_ = 0;
  uint64_t unacked_ = 0;  // data returned by recv() not yet acknowledged to the helper
  bool connected_ = false, ended_ = false, lost_ = false, closed_ = false;
};
}  // namespace

std::string port_forward_via() {
  const char* v = std::getenv("DEVSPACE_PORTFORWARD_VIA");
  std::string s = v && *v ? v : "auto";
  if (reference_timing()) return "kubelet";
  return s == "helper" || s == "kubelet" ? s : "auto";
}

void PortForwarder::set_helper(const std::string& helper_path) {
  std::string bin;
  if (via_ == "kubelet" || helper_path.empty() || !fs::read_file(helper_path, &bin) || bin.empty()) return;
  helper_file_ = "devspace-helper-" + sha256_hex(bin).substr(0, 16);  // as the sync names it
}

bool PortForwarder::want_helper() {
  if (helper_file_.empty()) return false;
  if (via_ == "helper") return true;
  return tunnel_rtt_us() >= 5000;  // next to the cluster the kubelet's retries cost ~nothing
}

std::shared_ptr<HelperLink> PortForwarder::helper_link() {
  if (!want_helper()) return nullptr;
  const std::string pod = pod_name();
  std::lock_guard<std::mutex> g(helper_mu_);
  if (helper_ && helper_->usable() && helper_pod_ == pod) return helper_;
  return nullptr;
}

void PortForwarder::maintain_helper_link() {
  if (stop_ || !want_helper()) return;
  const std::string pod = pod_name();
  {
    std::lock_guard<std::mutex> g(helper_mu_);
    if (helper_ && helper_->usable() && helper_pod_ == pod) return;
    if (mono_ms() < helper_retry_ms_) return;
  }
  std::shared_ptr<HelperLink> old;
  {
    std::lock_guard<std::mutex> g(helper_mu_);
    old.swap(helper_);
  }
  if (old) old->close();
  Value p;
  {
    std::lock_guard<std::mutex> g(pod_mu_);
    p = pod_;
  }
  // the helper lives in the container the sync targets: look in each until it is found
  std::string why = "no containers";
  for (auto& c : p.at_path("spec.containers").items()) {
    kube::ExecTransport t(k_, p, c.get("name").as_string());
    std::shared_ptr<HelperLink> link;
    try {
      link = HelperLink::open(t, helper_file_, &why);
    } catch (const std::exception& e) {
      why = e.what();
    }
    if (link) {
      std::lock_guard<std::mutex> g(helper_mu_);
      helper_ = link;
      helper_pod_ = pod;
      helper_backoff_ms_ = 2000;
      log::file_logger("portforwarding")
          ->emit("info", "Forwarding through the in-container helper of pod " + pod + " (container " +
                             c.get("name").as_string() + "): held connections are retried in the pod", {});
      return;
    }
  }
  // the sync may not have uploaded it yet; a cluster that refuses the exec is not asked every 2 s
  std::lock_guard<std::mutex> g(helper_mu_);
  helper_retry_ms_ = mono_ms() + helper_backoff_ms_;
  helper_backoff_ms_ = std::min(30000L, helper_backoff_ms_ * 2);
}

// True for the error-channel message of a stream whose pod-side connect failed (kubelet /
// CRI: "... dial tcp4 127.0.0.1:8080: connect: connection refused"): nothing reached the
// container, so the client's bytes can be replayed on a new stream.
bool is_dial_refused(const std::string& err) { return contains(to_lower(err), "connection refused"); }

namespace {
// A stream whose first reply bytes were already read (the winner of hedged attempts).
class PrimedFwd : public FwdStream {
 public:
  PrimedFwd(std::unique_ptr<FwdStream> in, std::string first) : in_(std::move(in)), first_(std::move(first)) {}
  bool send(const std::string& data) override { return in_->send(data); }
  bool recv(int* channel, std::string* data) override {
    if (!given_) {
      given_ = true;
      *channel = 0;
      *data = std::move(first_);
      return true;
    }
    return in_->recv(channel, data);
  }
  void close_write() override { in_->close_write(); }
  void close() override { in_->close(); }
  const char* via() const override { return in_->via(); }
  bool tunnel_lost() const override { return in_->tunnel_lost(); }

 private:
  std::unique_ptr<FwdStream> in_;
  std::string first_;
  bool given_ = false;
};
}  // namespace

bool hedgeable_request(const std::string& bytes) {
  if (!(starts_with(bytes, "GET ") || starts_with(bytes, "HEAD ") || starts_with(bytes, "OPTIONS "))) return false;
  size_t end = bytes.find("\r\n\r\n");
  if (end == std::string::npos || end + 4 != bytes.size()) return false;  // one whole request head, nothing after
  std::string head = to_lower(bytes.substr(0, end));
  // a body, or an upgrade (a WebSocket, e.g. a dev server's hot-reload socket): a session on the
  // server, not a request to repeat
  return !contains(head, "\r\ncontent-length:") && !contains(head, "\r\ntransfer-encoding:") &&
         !contains(head, "\r\nupgrade:");
}

// Opt-in (DEVSPACE_PORTFORWARD_HEDGE=1): hedged attempts can each reach the app, and dev apps
// often have GET routes with side effects. By default every request is delivered once, as by
// kubectl port-forward.
bool port_forward_hedge() {
  const char* v = std::getenv("DEVSPACE_PORTFORWARD_HEDGE");
  return v && std::string(v) == "1" && !reference_timing();
}

// A held idempotent request on a slow link (the app restarting behind a remote API server):
// instead of one attempt per round trip, a new attempt (a stream pair in the pod's tunnel with
// the request) goes out every third of a round trip while earlier ones are in flight, so the
// request reaches the new server within a few ms of it listening rather than up to a round trip
// later. The first attempt answered wins; the others are reset. The app may see the request
// more than once (up to about four times), which is why this is opt-in (port_forward_hedge):
// only GET, HEAD and OPTIONS without a body are hedged,
// which HTTP lets a client repeat (RFC 9110 §9.2.2). nullptr: no answer before `deadline_ms`, or
// an attempt ended other than refused (the caller carries on one attempt at a time).
std::unique_ptr<FwdStream> PortForwarder::hedge(int remote_port, const std::string& request, bool fin, int64_t rtt_us,
                                                long deadline_ms, std::string* first) {
  struct Attempt {
    std::unique_ptr<FwdStream> s;
    std::thread t;
    int state = 0;  // 0 in flight, 1 refused, 2 answered, 3 ended otherwise
    std::string data;
    int64_t t_open = 0, t_end = 0;
  };
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::unique_ptr<Attempt>> attempts;
  const long spacing = std::max(8L, std::min(25L, (long)(rtt_us / 3000)));
  Attempt* winner = nullptr;
  bool failed = false;
  const long started = mono_ms();
  long next_open = started;
  while (!stop_ && !winner && !failed && mono_ms() < deadline_ms) {
    size_t in_flight = 0;
    {
      std::lock_guard<std::mutex> g(mu);
      for (auto& a : attempts) in_flight += a->state == 0;
    }
    if (mono_ms() >= next_open && in_flight < 8) {
      auto a = std::make_unique<Attempt>();
      a->t_open = trace::now_us();
      try {
        a->s = open_to(pod_name(), remote_port);
      } catch (const std::exception&) {
        break;
      }
      if (std::string(a->s->via()) != "tunnel" || !a->s->send(request)) {
        a->s->close();
        break;
      }
      if (fin) a->s->close_write();
      Attempt* ap = a.get();
      a->t = std::thread([ap, &mu, &cv] {
        int ch = 0, st = 3;
        std::string d;
        while (ap->s->recv(&ch, &d)) {
          if (ch == 0) {
            st = 2;
            break;
          }
          if (ch == 1 && !d.empty()) {
            st = is_dial_refused(d) ? 1 : 3;
            break;
          }
        }
        {
          std::lock_guard<std::mutex> g(mu);
          ap->state = st;
          ap->t_end = trace::now_us();
          if (st == 2) ap->data = std::move(d);
        }
        cv.notify_all();
      });
      attempts.push_back(std::move(a));
      held_retries_++;
      // an app that takes more than a second to come back is not waited on this closely
      next_open = mono_ms() + (mono_ms() - started < 1000 ? spacing : std::max(spacing, 50L));
    }
    std::unique_lock<std::mutex> lk(mu);
    long wait = std::max(1L, std::min(next_open, deadline_ms) - mono_ms());
    cv.wait_for(lk, std::chrono::milliseconds(wait), [&] {
      for (auto& a : attempts)
        if (a->state >= 2) return true;
      return false;
    });
    for (auto& a : attempts) {
      if (a->state == 2) {
        winner = a.get();
        break;
      }
      if (a->state == 3) failed = true;
    }
  }
  for (auto& a : attempts)
    if (a.get() != winner) a->s->close();  // a reply it may still get is dropped
  for (auto& a : attempts)
    if (a->t.joinable()) a->t.join();
  if (trace::enabled()) {
    int n = 0;
    for (auto& a : attempts) {
      static const char* kOutcome[] = {"abandoned", "refused", "reply", "closed"};
      trace::emit("portforward.stream", a->t_open, (a->t_end ? a->t_end : trace::now_us()) - a->t_open,
                  {{"port", std::to_string(remote_port)},
                   {"attempt", "h" + std::to_string(n++)},
                   {"first_us", a->t_end ? std::to_string(a->t_end - a->t_open) : std::string("-1")},
                   {"outcome", a.get() == winner ? "reply" : kOutcome[a->state]},
                   {"hedged", "1"},
                   {"via", "tunnel"}});
    }
  }
  if (!winner) return nullptr;
  *first = std::move(winner->data);
  return std::move(winner->s);
}

bool port_forward_preopen() {
  const char* v = std::getenv("DEVSPACE_PORTFORWARD_PREOPEN");
  return !(v && std::string(v) == "0");
}

int port_forward_hold_ms() {
  if (const char* v = std::getenv("DEVSPACE_PORTFORWARD_HOLD_MS")) return std::max(0, std::atoi(v));
  return reference_timing() ? 0 : 3000;
}

// One accepted local connection. Restart-tolerant: while the app in the pod is restarting
// (hot reload), its port refuses connections for a moment; kubectl then drops the client's
// connection and a browser shows an error. Here, as long as nothing came back from the pod yet
// and the pod-side connect was refused, the connection is held and its bytes replayed on a
// new stream for up to hold_ms_, so a request sent mid-restart is answered by the new server as
// soon as it listens. For the first 100 ms the next stream is opened while the current attempt
// is in flight (PreOpened) and used as soon as that attempt is refused; after that the attempts
// back off (5 ms, then 25 ms after a second).
void PortForwarder::handle(Conn* conn, int remote_port) {
  int cfd = conn->fd;
  const long hold_start = mono_ms();
  const long hold_deadline = hold_start + hold_ms_;
  std::string replay;           // client bytes of this connection, kept while no reply arrived
  bool replayable = hold_ms_ > 0;
  bool client_eof = false;
  int attempt = 0;
  std::unique_ptr<PreOpened> next;
  std::unique_ptr<FwdStream> hedged;  // the answered attempt of a hedged held request
  bool helper_failed = false;         // a helper link died under this connection: the kubelet's path
  while (!stop_) {
    std::unique_ptr<FwdStream> ws = std::move(hedged);
    const bool primed = ws != nullptr;  // its request went out with it
    // span per stream: open (the WebSocket upgrade, or a stream pair in the tunnel; the pod-side
    // dial happens with it) and the time until the first reply byte or the refusal
    // (trace.jsonl "portforward.stream")
    const int64_t t_open = trace::now_us();
    const std::string target = pod_name();
    bool preopened = false;
    if (next) {
      ws = next->take();
      next.reset();
      preopened = ws != nullptr;
    }
    if (!ws && !helper_failed) {
      // through the in-container helper: the hold happens in the pod (one connect, made within
      // ms of the app listening), so this is the connection's only attempt unless the link dies
      if (auto link = helper_link()) {
        try {
          long left = std::max<long>(0, hold_deadline - mono_ms());
          ws = std::make_unique<HelperFwd>(link, remote_port, replayable ? (uint32_t)left : 0);
          helper_streams_++;
        } catch (const std::exception&) {
          ws.reset();
        }
      }
    }
    if (!ws) {
      try {
        ws = open_stream(remote_port);
      } catch (const std::exception& e) {
        log::file_logger("portforwarding")->emit("error", std::string("Error forwarding ports: ") + e.what(), {});
        break;
      }
    }
    if (preopened) preopened_++;
    const int64_t t_opened = trace::now_us();
    const bool tunneled = std::string(ws->via()) == "tunnel";
    // a held connection (its first stream was refused) within its first 100 ms: open the
    // following attempt's stream now, while this one waits for its reply or refusal. (Not through
    // the tunnel: a stream there opens without a round trip, and its pod-side dial is what an
    // attempt is for.)
    if (preopen_ && !tunneled && attempt > 0 && replayable && !stop_ && mono_ms() - hold_start < 100)
      next = std::make_unique<PreOpened>([this, remote_port] { return open_stream_direct(remote_port); });
    std::atomic<int64_t> t_first{0};
    if (!primed && !replay.empty() && !ws->send(replay)) break;
    if (client_eof && !primed) ws->close_write();
    plat::Waker wake;
    if (!wake.ok()) break;
    std::atomic<bool> down_done{false}, got_reply{false}, refused{false};
    std::string error_text;  // the first error message before any reply (read after the join)
    std::thread down([&] {
      int ch = 0;
      std::string data;
      while (ws->recv(&ch, &data)) {
        if (ch == 0) {
          if (!got_reply) t_first = trace::now_us();
          got_reply = true;
          if (!write_all(cfd, data)) break;
        } else if (ch == 1 && !data.empty()) {
          if (!got_reply && is_dial_refused(data)) {
            t_first = trace::now_us();
            refused = true;
            break;
          }
          if (!got_reply && error_text.empty()) error_text = data;
          log::file_logger("portforwarding")->emit("error", data, {});
        }
      }
      down_done = true;
      wake.poke();
    });
    char buf[65536];
    while (!down_done && !stop_ && !client_eof) {
      // answered: the spare attempt is not needed (dropped once its open is done, so the
      // forwarding never waits on it; else at the end of the connection)
      if (next && got_reply && next->ready()) next.reset();
      struct pollfd pf[2] = {{cfd, POLLIN, 0}, {wake.fd(), POLLIN, 0}};
      int r = ::poll(pf, 2, 200);
      if (r <= 0 || !(pf[0].revents & (POLLIN | POLLHUP | POLLERR))) continue;
      ssize_t n = ::recv(cfd, buf, sizeof(buf), 0);
      if (n <= 0) {
        client_eof = true;  // half-close: the request is complete, keep reading the reply
        ws->close_write();
        break;
      }
      if (replayable && !got_reply) {
        replay.append(buf, (size_t)n);
        if (replay.size() > (4u << 20)) replayable = false;  // a large upload: do not buffer it
      }
      if (!ws->send(std::string(buf, (size_t)n))) break;
    }
    if (client_eof && !down_done) {
      // the client finished sending: wait for the reply (or the refusal) before closing
      while (!down_done && !stop_) {
        if (next && got_reply && next->ready()) next.reset();
        struct pollfd pw{wake.fd(), POLLIN, 0};
        ::poll(&pw, 1, 200);
      }
    }
    ws->close();
    down.join();
    if (trace::enabled()) {
      int64_t tf = t_first.load();
      trace::emit("portforward.stream", t_open, trace::now_us() - t_open,
                  {{"port", std::to_string(remote_port)},
                   {"attempt", std::to_string(attempt)},
                   {"open_us", std::to_string(t_opened - t_open)},
                   {"first_us", tf ? std::to_string(tf - t_open) : std::string("-1")},
                   {"outcome", refused ? "refused" : got_reply ? "reply" : error_text.empty() ? "closed" : "error"},
                   {"preopened", preopened ? "1" : "0"},
                   {"via", ws->via()}});
    }
    ++attempt;
    if (std::string(ws->via()) == "helper") {
      auto* hf = static_cast<HelperFwd*>(ws.get());
      if (hf->tunnel_lost() && !got_reply && !stop_ && replayable && mono_ms() < hold_deadline &&
          (!hf->delivered() || hedgeable_request(replay))) {
        // the helper's exec stream ended under this connection (the pod went away, the API server
        // closed it) before a reply: the kubelet's path, with the bytes again when they never
        // reached the app (or form a request HTTP lets a client repeat)
        helper_failed = true;
        held_retries_++;
        continue;
      }
      if (refused)  // the helper held it in the pod for the whole hold
        log::file_logger("portforwarding")->emit("error", "connection refused by the pod", {});
      break;
    }
    if (tunneled && ws->tunnel_lost() && !got_reply && !refused && error_text.empty() && replayable && !stop_ &&
        mono_ms() < hold_deadline && hedgeable_request(replay)) {
      // the tunnel ended under this stream before anything came back (an API server's idle
      // timeout or restart): a request HTTP lets a client repeat goes out again, on a new tunnel
      held_retries_++;
      continue;
    }
    if (tunneled && !got_reply && !refused && !error_text.empty() && !stop_ && drop_tunnel_if_pod_gone(target)) {
      // A tunnel outlives its pod: once the pod was replaced every stream fails with the
      // kubelet's "failed to find sandbox"-type error instead of a 404 at the upgrade. The tunnel
      // is dropped and the next stream re-selects the pod (open_stream); nothing reached the
      // app, so a held connection is replayed there.
      if (replayable && mono_ms() < hold_deadline) {
        held_retries_++;
        continue;
      }
    }
    // the link's round trip: the smallest of the tunnel's PINGs (unknown until one came back:
    // then this is not taken for a remote cluster)
    const int64_t link_rtt_us = tunnel_rtt_us();
    if (refused && replayable && !stop_ && mono_ms() < hold_deadline && tunneled && hedge_ && link_rtt_us >= 5000 &&
        hedgeable_request(replay)) {
      // a remote cluster and a request HTTP lets a client repeat
      std::string first;
      auto win = hedge(remote_port, replay, client_eof, link_rtt_us, hold_deadline, &first);
      if (win) {
        hedged = std::make_unique<PrimedFwd>(std::move(win), std::move(first));
        continue;
      }
    }
    if (refused && replayable && !stop_ && mono_ms() < hold_deadline) {
      // a hot-reloading app is back within tens of ms: retry at once for the first 100 ms
      // (a refusal takes a round trip, which paces the attempts; so does a pre-opened stream),
      // then back off
      long held = mono_ms() - hold_start;
      int delay = next || tunneled ? (held < 100 ? 0 : held < 1000 ? 5 : 25) : held < 100 ? 1 : held < 1000 ? 5 : 25;
      if (delay) std::this_thread::sleep_for(std::chrono::milliseconds(delay));
      held_retries_++;
      continue;
    }
    if (refused) log::file_logger("portforwarding")->emit("error", "connection refused by the pod", {});
    break;
  }
  ::shutdown(cfd, SHUT_RDWR);
  ::close(cfd);
  conn->done = true;
}

void PortForwarder::close() {
  if (stop_.exchange(true)) return;
  {
    std::lock_guard<std::mutex> g(spare_mu_);  // no lost wake-up between its check and wait
  }
  spare_cv_.notify_all();
  if (spare_thread_.joinable()) spare_thread_.join();
  for (auto& t : threads_)
    if (t.joinable()) t.join();
  for (int fd : listeners_) ::close(fd);
  listeners_.clear();
  reap(true);  // every connection thread ends within one poll interval once stop_ is set
  std::shared_ptr<HelperLink> h;
  {
    std::lock_guard<std::mutex> g(helper_mu_);
    h.swap(helper_);
  }
  if (h) h->close();
}

std::vector<std::unique_ptr<PortForwarder>> start_port_forwarding(const Value& cfg, std::shared_ptr<kube::Client> k,
                                                                  int pod_wait_ms, int poll_ms,
                                                                  const std::string& helper_path) {
  std::vector<std::unique_ptr<PortForwarder>> out;
  for (auto& pf : cfg.at_path("dev.ports").items()) {
    config::SelectorRef ref = config::resolve_selector(cfg, pf);
    log::start_wait("Port-Forwarding: Waiting for pods...");
    Value pod;
    try {
      pod = k->newest_running_pod(ref.namespace_, ref.labels.to_query(), pod_wait_ms, poll_ms);
    } catch (const std::exception& e) {
      log::stop_wait();
      throw std::runtime_error(std::string("Error starting port-forwarding: Unable to list devspace pods: ") + e.what());
    }
    log::stop_wait();
    std::vector<std::pair<int, int>> ports;
    std::vector<std::string> addrs;
    for (auto& m : pf.get("portMappings").items()) {
      ports.emplace_back((int)m.get("localPort").as_int(), (int)m.get("remotePort").as_int());
      // Deliberate deviation (PARITY.md): the reference defaults to "127.0.0.1"
      // (port_forwarding.go:64-67); an unset bindAddress here listens on localhost, i.e.
      // 127.0.0.1 and ::1, as `kubectl port-forward` does, so http://localhost:<port> works on
      // hosts that resolve localhost to ::1 first. An explicit bindAddress is used as given.
      addrs.push_back(m.get("bindAddress").as_string("localhost"));
    }
    auto fwd = std::make_unique<PortForwarder>(k, pod, ports, addrs, ref.labels.to_query());
    if (!helper_path.empty()) fwd->set_helper(helper_path);
    fwd->start();
    log::done("Port forwarding started on " + fwd->describe());
    out.push_back(std::move(fwd));
  }
  return out;
}

}  // namespace services
}  // namespace ds

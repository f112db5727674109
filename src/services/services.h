// Dev-time services on selected pods (pkg/devspace/services/*.go): sync, port-forwarding,
// terminal, attach, logs, and pod/container selection.
#pragma once

#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "config/config.h"
#include "kube/client.h"
#include "sync/sync.h"

namespace ds {
namespace services {

struct Target {
  std::string namespace_, label_selector, container;
};

// services/attach.go:75 getSelectorNamespaceLabelSelector + container preference.
Target resolve_target(const Value& cfg, const std::string& selector_flag, const std::string& label_selector_flag,
                      const std::string& namespace_flag, const std::string& container_flag);

// Interactive pod/container pick among running pods (services/pod_selector.go).
Value select_pod(kube::Client& k, const std::string& ns, const std::string& label_selector);
std::string select_container(const Value& pod, const std::string& preferred);

struct SyncOptions {
  bool verbose = false;
  sync::Mode mode = sync::Mode::Helper;
  std::string helper_path;
  int pod_wait_ms = 120000;
  int poll_ms = 100;  // pod discovery poll (1000 = reference timing)
};

// Every dev.sync path, started concurrently; the first failure is thrown.
std::vector<std::unique_ptr<sync::Session>> start_sync(const Value& cfg, std::shared_ptr<kube::Client> k,
                                                        const SyncOptions& o);
// One dev.sync entry; nullptr when its container is not in the pod (a warning).
std::unique_ptr<sync::Session> start_sync_path(const Value& cfg, const Value& sync_path,
                                               std::shared_ptr<kube::Client> k, const SyncOptions& o);

// Listen addresses (family, literal) for a port mapping's bindAddress ("" = localhost: both
// 127.0.0.1 and ::1, like kubectl port-forward's default).
std::vector<std::pair<int, std::string>> listen_addresses(const std::string& bind);

// How long a local connection is held while the pod refuses it (app restarting):
// DEVSPACE_PORTFORWARD_HOLD_MS, default 3000; 0 with DEVSPACE_REFERENCE_TIMING (kubectl drops it).
int port_forward_hold_ms();
// Whether a held connection opens its next attempt's stream while the current one is in flight
// (DEVSPACE_PORTFORWARD_PREOPEN=0 turns it off).
bool port_forward_preopen();
bool is_dial_refused(const std::string& error_channel_message);
// Whether a held connection on a slow link may be retried on several streams at once
// (opt-in, DEVSPACE_PORTFORWARD_HEDGE=1: the app may see such a request more than once), and whether its bytes so far are one request that
// HTTP lets a client repeat: GET, HEAD or OPTIONS, the whole head and no body.
bool port_forward_hedge();
bool hedgeable_request(const std::string& bytes);

class FwdStream;   // one forwarded connection's stream(s) (portforward.cc)
class HelperLink;  // connections through the in-container helper (portforward.cc)

// How forwarded connections reach the pod (DEVSPACE_PORTFORWARD_VIA): "auto" (default) goes
// through the in-container helper when the sync has put it in the container and the cluster is
// remote (the tunnel's round trip is 5 ms or more), else the kubelet's port-forward; "helper"
// whenever the helper is there; "kubelet" never through the helper.
std::string port_forward_via();

// Local listeners forwarding to a pod port (services/port_forwarding.go:18, kubectl/client.go:356):
// through one multiplexed tunnel per pod (SPDY/3.1 over a WebSocket, kube/spdy.h) where the API
// server speaks it, else over a portforward.k8s.io WebSocket per connection. Every accepted
// connection gets its own stream and thread; the forwarder owns those threads and joins them in
// close(). When the
// pod goes away (restart, rollout) new connections re-select the newest running pod of the
// selector instead of failing forever (the reference keeps forwarding to the dead pod).
class PortForwarder {
 public:
  PortForwarder(std::shared_ptr<kube::Client> k, Value pod, std::vector<std::pair<int, int>> ports,
                std::vector<std::string> addresses, std::string label_selector = "");
  ~PortForwarder();
  // Binds all listeners; throws on failure.
  void start();
  void close();
  std::string describe() const;
  std::string pod_name();
  int reselections() const { return reselections_; }
  // Connections replayed on a new stream because the pod refused them mid-restart.
  int held_retries() const { return held_retries_; }
  // Streams opened on a pre-dialed connection.
  int spares_used() const { return spares_used_; }
  // Held-connection attempts whose stream was opened while the previous attempt was in flight.
  int preopened_attempts() const { return preopened_; }
  size_t active_connections();
  // The static helper binary the sync uploads (its content-addressed name in the container is
  // what the forward looks for); enables forwarding through it (port_forward_via).
  void set_helper(const std::string& helper_path);
  // Connections that went through the helper.
  int helper_streams() const { return helper_streams_; }

 private:
  struct Conn {
    std::thread t;
    int fd = -1;
    std::atomic<bool> done{false};
  };
  void accept_loop(int lfd, int remote_port);
  // Pre-dialed API-server connections (TCP + TLS done): a new local connection only pays the
  // WebSocket upgrade round trip, not a handshake — kubectl gets the same by multiplexing
  // its streams over one SPDY connection.
  void spare_loop();
  std::unique_ptr<net::Conn> take_spare();
  void handle(Conn* c, int remote_port);
  void reap(bool all);
  std::unique_ptr<FwdStream> open_stream(int remote_port);
  // The current pod's stream without pod re-selection (the hold's pre-opened next attempt).
  std::unique_ptr<FwdStream> open_stream_direct(int remote_port);
  // A stream to `pod`: a stream pair in the pod's multiplexed tunnel, or (an API server without
  // the tunnel, DEVSPACE_PORTFORWARD_TUNNEL=0) a WebSocket of its own.
  std::unique_ptr<FwdStream> open_to(const std::string& pod, int remote_port);
  // The pod's tunnel, opened (or re-opened after it closed) on demand; nullptr when unsupported.
  std::shared_ptr<kube::SpdySession> tunnel_for(const std::string& pod);
  // A tunnel stream failed with an error before any reply: true when `pod` is gone, replaced
  // (same name, new uid) or finished, or was re-selected away from; its tunnel is then dropped.
  bool drop_tunnel_if_pod_gone(const std::string& pod);
  // the current tunnel's PING round trip (-1: none measured)
  int64_t tunnel_rtt_us();
  std::unique_ptr<FwdStream> hedge(int remote_port, const std::string& request, bool fin, int64_t rtt_us,
                                   long deadline_ms, std::string* first);
  std::shared_ptr<kube::Client> k_;
  std::mutex pod_mu_;
  Value pod_;
  std::string ns_, selector_;
  std::vector<std::pair<int, int>> ports_;
  std::vector<std::string> addrs_;
  std::vector<int> listeners_;
  std::vector<std::thread> threads_;
  std::mutex conns_mu_;
  std::vector<std::unique_ptr<Conn>> conns_;
  std::atomic<bool> stop_{false};
  std::atomic<int> reselections_{0};
  std::atomic<int> held_retries_{0};
  std::mutex spare_mu_;
  std::condition_variable spare_cv_;
  std::deque<std::pair<long, std::unique_ptr<net::Conn>>> spares_;  // (dialed at ms, conn)
  std::thread spare_thread_;
  int want_spares_ = 0;
  std::atomic<int> spares_used_{0};
  std::atomic<int> preopened_{0};
  int hold_ms_ = port_forward_hold_ms();
  bool preopen_ = port_forward_preopen();
  bool hedge_ = port_forward_hedge();
  // the multiplexed tunnel (SPDY/3.1 over one WebSocket): -1 not tried, 0 unsupported, 1 in use
  std::atomic<int> tunnel_mode_{-1};
  std::mutex tunnel_mu_;
  std::shared_ptr<kube::SpdySession> tunnel_;
  std::string tunnel_pod_;
  std::atomic<uint64_t> tunnel_requests_{0};  // request ids of the current tunnel
  std::atomic<int> tunnels_opened_{0};
  // forwarding through the in-container helper
  std::shared_ptr<HelperLink> helper_link();  // a usable link to the current pod, or nullptr
  void maintain_helper_link();                // (spare_loop) opens / re-opens it when wanted
  bool want_helper();
  std::string helper_file_;                   // devspace-helper-<sha16>, "" when not enabled
  std::string via_ = port_forward_via();
  std::mutex helper_mu_;
  std::shared_ptr<HelperLink> helper_;
  std::string helper_pod_;
  long helper_retry_ms_ = 0;                  // not before this (monotonic ms) after a failed probe
  long helper_backoff_ms_ = 2000;             // doubling up to 30 s while it keeps failing
  std::atomic<int> helper_streams_{0};

 public:
  // Tunnels opened (1 for a forward whose API server speaks it and whose pod never changed).
  int tunnels_opened() const { return tunnels_opened_; }
  bool tunneled() const { return tunnel_mode_ == 1; }
};

// helper_path: the sync's static helper (set when the sync runs in helper mode), for
// forwarding through it (PortForwarder::set_helper).
std::vector<std::unique_ptr<PortForwarder>> start_port_forwarding(const Value& cfg, std::shared_ptr<kube::Client> k,
                                                                  int pod_wait_ms = 120000, int poll_ms = 100,
                                                                  const std::string& helper_path = "");

// Runs an interactive command in the container with a TTY when stdin is a terminal
// (services/terminal.go). `interrupt` is polled; returns the remote exit code.
int start_terminal(const Value& cfg, std::shared_ptr<kube::Client> k, const std::string& selector,
                   const std::string& container, const std::string& label_selector, const std::string& ns, bool pick,
                   std::vector<std::string> cmd, const std::function<bool()>& interrupt);

// Attach to the container output (services/attach.go:18). With follow_restarts (dev) a
// stream that ends because the container restarted or the pod was replaced re-attaches to the
// newest running pod until `interrupt` fires.
int start_attach(const Value& cfg, std::shared_ptr<kube::Client> k, const std::string& selector,
                 const std::string& container, const std::string& label_selector, const std::string& ns,
                 const std::function<bool()>& interrupt, bool follow_restarts = false);

// Print last N lines, optionally follow (services/logs.go:17).
int start_logs(const Value& cfg, std::shared_ptr<kube::Client> k, const std::string& selector,
               const std::string& container, const std::string& label_selector, const std::string& ns, bool pick,
               bool follow, int tail, const std::function<bool()>& interrupt);

}  // namespace services
}  // namespace ds

// Kubernetes API client: REST over HTTP/1.1(+TLS), exec/attach/port-forward over the
// WebSocket channel protocols (v4.channel.k8s.io, portforward.k8s.io), pod status logic.
//
// Reference equivalents: kubectl/client.go (NewClient, getClientConfig, GetNewestRunningPod,
// GetPodStatus), kubectl/exec.go (ExecStream*), kubectl/attach.go, kubectl/logs.go,
// kubectl/util.go (EnsureDefaultNamespace, EnsureGoogleCloudClusterRoleBinding),
// kubectl/client.go:356 (NewPortForwarder). client-go/SPDY are replaced by native code.
#pragma once

#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <memory>
#include <optional>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "kube/spdy.h"

#include "core/net.h"
#include "core/proc.h"
#include "core/value.h"
#include "kube/kubeconfig.h"
#include "sync/transport.h"

namespace ds {
namespace kube {

struct ApiError : std::runtime_error {
  int code;
  std::string reason;
  ApiError(int c, const std::string& r, const std::string& msg) : std::runtime_error(msg), code(c), reason(r) {}
  bool not_found() const { return code == 404; }
  bool conflict() const { return code == 409; }
  bool invalid() const { return code == 422; }
};

// How `apply` treats an object whose changed fields the API server refuses as immutable.
struct ApplyOptions {
  // Delete and re-create the object (`kubectl apply --force`). Never done for
  // PersistentVolumeClaims, PersistentVolumes or Namespaces (data / whole-namespace loss).
  bool recreate_on_immutable = false;
  std::string field_manager = "devspace";
};

// Kinds whose delete-and-recreate would destroy data: apply never recreates them.
bool never_recreate(const std::string& kind);

// Pod status string exactly like `kubectl get pods` (kubectl/client.go:224 GetPodStatus).
std::string pod_status(const Value& pod);
bool pod_status_is_fatal(const std::string& status);

// REST path for a manifest object (apiVersion/kind/namespace/name).
std::string resource_path(const std::string& api_version, const std::string& kind, const std::string& ns,
                          const std::string& name = "");
std::string plural_of(const std::string& kind);
bool is_cluster_scoped(const std::string& kind);

// client-go's REST retry rule (k8s.io/client-go/rest/request.go checkWait with maxRetries 10;
// the reference gets it through kubernetes.NewForConfig, kubectl/client.go:34-51): a
// `429 Too Many Requests` (API Priority and Fairness throttling) or a 5xx carrying Retry-After
// is sent again after the server's delay. Unlike client-go, a POST is retried only on 429 (the
// server did not act on it), never on a 5xx, where it may have. Returns the wait in ms before
// the retry, or -1 for "do not retry". Retry-After: delta-seconds (an HTTP-date or garbage counts
// as 1 s), capped at kMaxRetryAfterS; a 429 without the header waits 1 s.
constexpr int kMaxApiRetries = 10;
constexpr int kMaxRetryAfterS = 10;
int retry_wait_ms(int status, const std::string& retry_after, const std::string& method);

class ExecSession;

class Client {
 public:
  explicit Client(RestConfig cfg);
  // getClientConfig semantics (kubectl/client.go:63): devspace config cluster.* or kube
  // context (optionally switching the current context in ~/.kube/config).
  static std::shared_ptr<Client> from_devspace_config(const Value& cfg, bool switch_context = false);

  const RestConfig& rest() const { return cfg_; }
  std::string default_namespace() const { return cfg_.namespace_.empty() ? "default" : cfg_.namespace_; }
  bool is_local_cluster();  // the bundled local cluster (process pods on the host network)
  bool is_minikube() const { return cfg_.context == "minikube"; }

  // REST (JSON bodies). Throw ApiError on non-2xx.
  Value get(const std::string& path);
  Value post(const std::string& path, const Value& body);
  Value put(const std::string& path, const Value& body);
  Value patch(const std::string& path, const Value& body,
              const std::string& type = "application/merge-patch+json");
  Value del(const std::string& path, const Value& body = Value());
  // Returns nullopt for 404.
  std::optional<Value> try_get(const std::string& path);
  net::Response raw(const std::string& method, const std::string& path, const std::string& body = "",
                    const std::string& content_type = "application/json", int timeout_ms = 60000);
  // Stream a GET (logs -f, watch).
  int stream(const std::string& path, const std::function<bool(const std::string&)>& on_data, int timeout_ms = -1);

  // List + watch (the client-go informer pattern without the cache): lists `collection`
  // (a collection path, `query` without '?'), then follows `?watch=1` from the list's
  // resourceVersion, re-listing on 410 Gone and re-watching when the server ends the watch.
  // `done` sees the current object set (ordered by creationTimestamp) after the list and
  // after every event; returns true as soon as `done` does, false on timeout. Servers without
  // watch support are polled instead (back-off, 5 ms -> 250 ms).
  bool list_watch(const std::string& collection, const std::string& query, int timeout_ms,
                  const std::function<bool(const std::vector<Value>&)>& done);
  // Waits until the single object at `object_path` satisfies `pred` (nullopt = absent).
  bool wait_object(const std::string& object_path, int timeout_ms,
                   const std::function<bool(const std::optional<Value>&)>& pred);

  // Pods
  std::vector<Value> list_pods(const std::string& ns, const std::string& label_selector);
  // Newest pod by creationTimestamp that is Running; fails fast on fatal states
  // (kubectl/client.go:171). poll_ms: 1000 reproduces the reference's 1 s sleeps.
  Value newest_running_pod(const std::string& ns, const std::string& label_selector, int max_wait_ms,
                           int poll_ms = 100);
  std::string logs(const std::string& ns, const std::string& pod, const std::string& container, int tail,
                   bool previous = false);

  // Namespaces / RBAC helpers (kubectl/util.go)
  void ensure_namespace(const std::string& ns);
  void ensure_gcloud_cluster_role_binding();
  // Largest per-pod amd.com/gpu request among workload manifests vs. the largest node
  // allocatable (AMD device plugin); warns before deploying something unschedulable.
  // Returns the warning text ("" when fine).
  std::string check_gpu_requests(const std::vector<Value>& objs);
  // Largest per-pod amd.com/gpu request among workload manifests (0 = no GPU workload).
  static int64_t max_gpu_request(const std::vector<Value>& objs);

  // Server-side apply (PATCH application/apply-patch+yaml, fieldManager=devspace, force):
  // fields set by other managers (the PV binder's spec.volumeName, a Service's clusterIP,
  // the HPA's replicas) are left alone. Servers without SSA get a strategic-merge (built-in
  // kinds) or JSON merge patch, or a create. Immutable-field rejections are reported, and only
  // with opts.recreate_on_immutable turned into delete + create (never for never_recreate()).
  Value apply(Value obj, const std::string& default_ns, const ApplyOptions& opts);
  Value apply(Value obj, const std::string& default_ns) { return apply(std::move(obj), default_ns, apply_opts_); }
  // Defaults for apply() (the CLI's --force-recreate).
  void set_apply_options(const ApplyOptions& o) { apply_opts_ = o; }
  bool delete_object(const Value& obj, const std::string& default_ns);

  // Streams
  std::unique_ptr<ExecSession> exec(const std::string& ns, const std::string& pod, const std::string& container,
                                    const std::vector<std::string>& cmd, bool tty, bool stdin = true);
  std::unique_ptr<ExecSession> attach(const std::string& ns, const std::string& pod, const std::string& container,
                                      bool tty, bool stdin = false);
  // `spare`: a pre-dialed connection to the API server to upgrade (saves the TLS handshake).
  // One multiplexed port-forward tunnel to `pod` (WebSocket subprotocol
  // "SPDY/3.1+portforward.k8s.io", Kubernetes >= 1.30): every forwarded connection becomes a
  // stream pair in it. nullptr when the API server does not speak it (then: portforward()).
  std::shared_ptr<SpdySession> portforward_tunnel(const std::string& ns, const std::string& pod,
                                                  const std::vector<int>& ports);
  std::unique_ptr<net::WebSocket> portforward(const std::string& ns, const std::string& pod, int port,
                                              std::unique_ptr<net::Conn> spare = nullptr);

  net::HttpClient& http() { return http_; }

  // Dials `n` connections to the API server (TCP + TLS) in the background for the WebSocket
  // upgrades that follow (exec, attach, port-forward): `devspace dev` asks for them before it
  // builds and deploys, so opening its sync shells and streams costs the upgrade round trip
  // only, not a handshake each. Unused ones are dropped after a minute.
  void prewarm_upgrades(int n);
  ~Client();

  // Credential refresh (exec plugins: on expiry and on 401; tokenFile: every minute and on 401).
  // ensure_fresh_credentials() returns the credentials' generation a request is about to use;
  // after a 401, refresh_after_unauthorized(that generation) is true when the request should be
  // sent again: another thread already replaced those credentials, or this call did.
  uint64_t ensure_fresh_credentials();
  bool refresh_after_unauthorized(uint64_t used_generation);
  int credential_refreshes() const { return refreshes_; }
  // Requests sent again after a 429 / 5xx + Retry-After (all verbs, all streams).
  int throttle_retries() const { return throttle_retries_; }

 private:
  // Before retry `attempt` (1-based) of a throttled request: counts it, logs the first
  // throttling of the process once, sleeps `wait_ms`.
  void throttled(const std::string& what, int status, int wait_ms, int attempt);
  void refresh_exec_credentials();
  void apply_auth_locked();
  std::unique_ptr<net::WebSocket> ws_connect(const std::string& path, const std::vector<std::string>& protocols,
                                             std::unique_ptr<net::Conn> spare = nullptr);
  // a pre-dialed connection, or nullptr; waits for one still being dialed (never slower than a
  // new dial)
  std::unique_ptr<net::Conn> take_prewarmed();
  RestConfig cfg_;
  std::mutex warm_mu_;
  std::condition_variable warm_cv_;
  std::deque<std::pair<int64_t, std::unique_ptr<net::Conn>>> warm_;  // (dialed at ms, conn)
  int warm_pending_ = 0;
  std::vector<std::pair<std::thread, std::shared_ptr<std::atomic<bool>>>> warm_threads_;  // (dialer, done)
  int local_cluster_ = -1;  // is_local_cluster() cache
  net::HttpClient http_;
  ApplyOptions apply_opts_;
  std::mutex auth_mu_;
  int64_t token_expiry_ = 0;      // unix seconds, 0 = no expiry
  int64_t token_file_read_ = 0;   // unix seconds of the last tokenFile read
  std::atomic<int> refreshes_{0};
  uint64_t auth_gen_ = 0;  // bumped whenever the credentials change (under auth_mu_)
  std::atomic<int> throttle_retries_{0};
};

// A running exec/attach: stdin/stdout/stderr exposed as pipes (so the sync engine and the
// terminal proxy can poll() them), remote exit code from the error channel.
class ExecSession : public sync::Shell {
 public:
  ExecSession(std::unique_ptr<net::WebSocket> ws, bool tty);
  ~ExecSession() override;
  int in() override { return in_w_.get(); }
  int out() override { return out_r_.get(); }
  int err() override { return err_r_.get(); }
  bool alive() override { return !done_; }
  void terminate() override;
  void close() override;
  void resize(int width, int height);
  void close_stdin_if_any() { in_w_.reset(); }
  // Waits for the remote process; returns its exit code (or -1 if unknown / stream died).
  int wait(int timeout_ms = -1);
  std::string error_message();

 private:
  void pump_in();
  void pump_out();
  std::unique_ptr<net::WebSocket> ws_;
  bool tty_;
  Fd in_r_, in_w_, out_r_, out_w_, err_r_, err_w_;
  std::thread t_in_, t_out_;
  std::atomic<bool> done_{false};
  std::atomic<int> exit_code_{-1};
  std::string error_;
  std::mutex mu_;
  std::condition_variable cv_;
};

// sync::Transport running `sh` in a pod container via exec. Pods of the devspace local
// cluster carry the annotation devspace.sh/local-root; container paths are mapped under it.
class ExecTransport : public sync::Transport {
 public:
  ExecTransport(std::shared_ptr<Client> c, Value pod, std::string container);
  std::unique_ptr<sync::Shell> open(const std::vector<std::string>& argv) override;
  std::string describe() const override { return "exec(" + pod_name_ + "/" + container_ + ")"; }
  std::string path_prefix() const override { return prefix_; }
  std::string pod_name() const override { return pod_name_; }

 private:
  std::shared_ptr<Client> c_;
  std::string ns_, pod_name_, container_, prefix_;
};

extern const char* const kLocalRootAnnotation;  // "devspace.sh/local-root"

}  // namespace kube
}  // namespace ds

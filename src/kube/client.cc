#include "kube/client.h"

#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <map>

#include "core/codec.h"
#include "core/fs.h"
#include "core/log.h"
#include "core/proc.h"
#include "core/strutil.h"

namespace ds {
namespace kube {

const char* const kLocalRootAnnotation = "devspace.sh/local-roots";

static void sleep_ms(int ms) { std::this_thread::sleep_for(std::chrono::milliseconds(ms)); }

// ---------------------------------------------------------------- pod status

std::string pod_status(const Value& pod) {
  const Value& st = pod.get("status");
  std::string reason = st.get("phase").as_string();
  if (!st.get("reason").as_string().empty()) reason = st.get("reason").as_string();
  bool initializing = false;
  const Value& inits = st.get("initContainerStatuses");
  size_t n_init = pod.at_path("spec.initContainers").size();
  for (size_t i = 0; i < inits.size(); ++i) {
    const Value& c = inits[i];
    const Value& term = c.at_path("state.terminated");
    const Value& wait = c.at_path("state.waiting");
    if (term.is_map() && term.get("exitCode").as_int() == 0) continue;
    if (term.is_map()) {
      if (term.get("reason").as_string().empty()) {
        if (term.get("signal").as_int() != 0)
          reason = "Init:Signal:" + std::to_string(term.get("signal").as_int());
        else
          reason = "Init:ExitCode:" + std::to_string(term.get("exitCode").as_int());
      } else {
        reason = "Init:" + term.get("reason").as_string();
      }
      initializing = true;
    } else if (wait.is_map() && !wait.get("reason").as_string().empty() &&
               wait.get("reason").as_string() != "PodInitializing") {
      reason = "Init:" + wait.get("reason").as_string();
      initializing = true;
    } else {
      reason = "Init:" + std::to_string(i) + "/" + std::to_string(n_init);
      initializing = true;
    }
    break;
  }
  if (!initializing) {
    bool has_running = false;
    const Value& cs = st.get("containerStatuses");
    for (size_t k = cs.size(); k-- > 0;) {
      const Value& c = cs[k];
      const Value& wait = c.at_path("state.waiting");
      const Value& term = c.at_path("state.terminated");
      if (wait.is_map() && !wait.get("reason").as_string().empty()) {
        reason = wait.get("reason").as_string();
      } else if (term.is_map() && !term.get("reason").as_string().empty()) {
        reason = term.get("reason").as_string();
      } else if (term.is_map()) {
        if (term.get("signal").as_int() != 0)
          reason = "Signal:" + std::to_string(term.get("signal").as_int());
        else
          reason = "ExitCode:" + std::to_string(term.get("exitCode").as_int());
      } else if (c.get("ready").as_bool() && c.at_path("state.running").is_map()) {
        has_running = true;
      }
    }
    if (reason == "Completed" && has_running) reason = "Running";
  }
  if (!pod.at_path("metadata.deletionTimestamp").is_null()) {
    reason = st.get("reason").as_string() == "NodeLost" ? "Unknown" : "Terminating";
  }
  return reason;
}

bool pod_status_is_fatal(const std::string& s) {
  return s == "Error" || s == "Unknown" || s == "ImagePullBackOff" || s == "CrashLoopBackOff" ||
         s == "RunContainerError" || s == "ErrImagePull" || s == "CreateContainerConfigError" ||
         s == "InvalidImageName";
}

// ---------------------------------------------------------------- resource paths

bool is_cluster_scoped(const std::string& kind) {
  static const char* k[] = {"Namespace", "Node", "PersistentVolume", "ClusterRole", "ClusterRoleBinding",
                            "StorageClass", "CustomResourceDefinition", "PriorityClass",
                            "MutatingWebhookConfiguration", "ValidatingWebhookConfiguration", "APIService"};
  for (auto* x : k)
    if (kind == x) return true;
  return false;
}

std::string plural_of(const std::string& kind) {
  static const std::map<std::string, std::string> special = {
      {"Endpoints", "endpoints"}, {"Ingress", "ingresses"}, {"NetworkPolicy", "networkpolicies"},
      {"PodSecurityPolicy", "podsecuritypolicies"}, {"StorageClass", "storageclasses"},
      {"PriorityClass", "priorityclasses"}};
  auto it = special.find(kind);
  if (it != special.end()) return it->second;
  std::string l = to_lower(kind);
  if (ends_with(l, "y") && !ends_with(l, "ey")) return l.substr(0, l.size() - 1) + "ies";
  if (ends_with(l, "s") || ends_with(l, "x") || ends_with(l, "ch")) return l + "es";
  return l + "s";
}

std::string resource_path(const std::string& api_version, const std::string& kind, const std::string& ns,
                          const std::string& name) {
  std::string base = api_version.find('/') == std::string::npos ? "/api/" + api_version : "/apis/" + api_version;
  std::string p = base;
  if (!is_cluster_scoped(kind)) p += "/namespaces/" + ns;
  p += "/" + plural_of(kind);
  if (!name.empty()) p += "/" + name;
  return p;
}

// ---------------------------------------------------------------- client

static net::TlsOptions tls_for(const RestConfig& c) {
  net::TlsOptions t;
  t.insecure = c.insecure;
  t.ca_pem = c.ca_pem;
  t.cert_pem = c.client_cert_pem;
  t.key_pem = c.client_key_pem;
  return t;
}

Client::Client(RestConfig cfg) : cfg_(std::move(cfg)), http_(cfg_.server, tls_for(cfg_)) {
  if (cfg_.token.empty() && !cfg_.exec_command.empty()) refresh_exec_token();
  if (!cfg_.token.empty()) http_.set_header("Authorization", "Bearer " + cfg_.token);
  if (!cfg_.username.empty())
    http_.set_header("Authorization", "Basic " + base64_encode(cfg_.username + ":" + cfg_.password));
  http_.set_header("Accept", "application/json");
  http_.set_header("User-Agent", "devspace-amd/0.1");
}

void Client::refresh_exec_token() {
  ProcOptions o;
  for (auto& kv : cfg_.exec_env) o.env[kv.first] = kv.second;
  RunResult r = run(cfg_.exec_command, "", o, 30000);
  if (r.code != 0) throw std::runtime_error("exec credential plugin failed: " + r.err);
  Value v = json_parse(r.out);
  cfg_.token = v.at_path("status.token").as_string();
}

bool Client::is_local_cluster() const { return contains(cfg_.context, "devspace-local") || contains(cfg_.server, "127.0.0.1"); }

std::shared_ptr<Client> Client::from_devspace_config(const Value& cfg, bool switch_context) {
  const Value& cl = cfg.get("cluster");
  RestConfig rc;
  if (cl.get("apiServer").is_null()) {
    KubeConfig kc = KubeConfig::load();
    std::string active = kc.current_context();
    std::string want = cl.get("kubeContext").as_string();
    if (!want.empty() && want != active) {
      active = want;
      if (switch_context) {
        kc.set_current_context(active);
        try {
          kc.save();
        } catch (const std::exception& e) {
          throw std::runtime_error(std::string("Error saving kube config: ") + e.what());
        }
      }
    }
    if (!kc.has_context(active)) throw std::runtime_error("Active Context doesn't exist");
    rc = kc.resolve(active);
  } else {
    rc.server = cl.get("apiServer").as_string();
    rc.ca_pem = cl.get("caCert").as_string();
    rc.client_cert_pem = cl.at_path("user.clientCert").as_string();
    rc.client_key_pem = cl.at_path("user.clientKey").as_string();
    rc.token = cl.at_path("user.token").as_string();
    rc.context = "devspace";
  }
  if (!cl.get("namespace").as_string().empty()) rc.namespace_ = cl.get("namespace").as_string();
  return std::make_shared<Client>(rc);
}

net::Response Client::raw(const std::string& method, const std::string& path, const std::string& body,
                          const std::string& content_type, int timeout_ms) {
  net::Request r;
  r.method = method;
  r.path = path;
  r.body = body;
  r.timeout_ms = timeout_ms;
  if (!body.empty()) r.headers.push_back({"Content-Type", content_type});
  return http_.request(r);
}

static Value check(const net::Response& r, const std::string& what) {
  if (r.status >= 200 && r.status < 300) {
    if (r.body.empty()) return Value::map();
    try {
      return json_parse(r.body);
    } catch (...) {
      return Value(r.body);
    }
  }
  std::string msg = r.body, reason;
  try {
    Value v = json_parse(r.body);
    if (v.get("message").is_string()) msg = v.get("message").as_string();
    reason = v.get("reason").as_string();
  } catch (...) {
  }
  throw ApiError(r.status, reason, what + ": " + std::to_string(r.status) + " " + msg);
}

Value Client::get(const std::string& path) { return check(raw("GET", path), "GET " + path); }
Value Client::post(const std::string& path, const Value& body) {
  return check(raw("POST", path, json_dump(body)), "POST " + path);
}
Value Client::put(const std::string& path, const Value& body) {
  return check(raw("PUT", path, json_dump(body)), "PUT " + path);
}
Value Client::patch(const std::string& path, const Value& body, const std::string& type) {
  return check(raw("PATCH", path, json_dump(body), type), "PATCH " + path);
}
Value Client::del(const std::string& path, const Value& body) {
  return check(raw("DELETE", path, body.is_null() ? "" : json_dump(body)), "DELETE " + path);
}
std::optional<Value> Client::try_get(const std::string& path) {
  try {
    return get(path);
  } catch (const ApiError& e) {
    if (e.not_found()) return std::nullopt;
    throw;
  }
}

int Client::stream(const std::string& path, const std::function<bool(const std::string&)>& on_data, int timeout_ms) {
  net::Request r;
  r.path = path;
  r.timeout_ms = timeout_ms;
  return http_.stream(r, on_data).status;
}

std::vector<Value> Client::list_pods(const std::string& ns, const std::string& sel) {
  std::string p = "/api/v1/namespaces/" + ns + "/pods";
  if (!sel.empty()) p += "?labelSelector=" + net::url_encode(sel);
  Value v = get(p);
  return v.get("items").items();
}

Value Client::newest_running_pod(const std::string& ns, const std::string& sel, int max_wait_ms, int poll_ms) {
  auto t0 = std::chrono::steady_clock::now();
  bool compat = poll_ms >= 1000;
  while (true) {
    if (compat) sleep_ms(poll_ms);  // the reference sleeps before the first list
    auto pods = list_pods(ns, sel);
    const Value* newest = nullptr;
    for (auto& p : pods) {
      // (the reference keeps &pod of the range variable, i.e. the last pod; intent: newest)
      if (!newest || p.at_path("metadata.creationTimestamp").as_string() >
                         newest->at_path("metadata.creationTimestamp").as_string())
        newest = &p;
    }
    if (newest) {
      std::string s = pod_status(*newest);
      if (s == "Running") return *newest;
      if (pod_status_is_fatal(s)) throw std::runtime_error("Selected Pod(s) cannot start (Status: " + s + ")");
    }
    sleep_ms(poll_ms);
    auto el = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
    if (el >= max_wait_ms)
      throw std::runtime_error("Waiting for pod with selector " + sel + " in namespace " + ns + " timed out");
  }
}

std::string Client::logs(const std::string& ns, const std::string& pod, const std::string& container, int tail,
                         bool previous) {
  std::string p = "/api/v1/namespaces/" + ns + "/pods/" + pod + "/log?container=" + net::url_encode(container);
  if (tail > 0) p += "&tailLines=" + std::to_string(tail);
  if (previous) p += "&previous=true";
  net::Response r = raw("GET", p);
  if (r.status != 200) check(r, "GET logs");
  return r.body;
}

void Client::ensure_namespace(const std::string& ns) {
  if (ns.empty() || ns == "default") return;
  if (try_get("/api/v1/namespaces/" + ns)) return;
  Value body = Value::map();
  body["apiVersion"] = "v1";
  body["kind"] = "Namespace";
  body["metadata"]["name"] = ns;
  try {
    post("/api/v1/namespaces", body);
    log::done("Created namespace: " + ns);
  } catch (const ApiError& e) {
    if (!e.conflict()) throw;
  }
}

static int64_t pod_gpu_request(const Value& pod_spec) {
  int64_t n = 0;
  for (auto& c : pod_spec.get("containers").items()) {
    const Value* lim = c.at_path("resources.limits").find("amd.com/gpu");
    const Value* req = c.at_path("resources.requests").find("amd.com/gpu");
    const Value* v = lim ? lim : req;
    int64_t x = 0;
    if (v && (v->is_int() || parse_int64(v->as_string(), &x))) n += v->is_int() ? v->as_int() : x;
  }
  return n;
}

std::string Client::check_gpu_requests(const std::vector<Value>& objs) {
  int64_t want = 0;
  std::string who;
  for (auto& o : objs) {
    const Value& spec = o.get("kind").as_string() == "Pod" ? o.get("spec") : o.at_path("spec.template.spec");
    if (!spec.is_map()) continue;
    int64_t n = pod_gpu_request(spec);
    if (n > want) {
      want = n;
      who = o.get("kind").as_string() + " " + o.at_path("metadata.name").as_string();
    }
  }
  if (want == 0) return "";
  int64_t best = 0;
  try {
    Value nodes = get("/api/v1/nodes");
    for (auto& n : nodes.get("items").items()) {
      int64_t a = 0;
      const Value& v = n.at_path("status.allocatable").get("amd.com/gpu");
      if (v.is_int()) a = v.as_int();
      else parse_int64(v.as_string(), &a);
      best = std::max(best, a);
    }
  } catch (const std::exception&) {
    return "";  // no permission to list nodes: nothing to say
  }
  std::string msg;
  if (best == 0)
    msg = who + " requests " + std::to_string(want) +
          " amd.com/gpu but no node advertises amd.com/gpu (is the AMD GPU device plugin running?)";
  else if (want > best)
    msg = who + " requests " + std::to_string(want) + " amd.com/gpu but the largest node offers " +
          std::to_string(best) + " — the pod cannot be scheduled";
  if (!msg.empty()) log::warn(msg);
  return msg;
}

void Client::ensure_gcloud_cluster_role_binding() {
  // kubectl/util.go:47 — GKE users need cluster-admin to create RBAC for the dev pods.
  if (!starts_with(cfg_.context, "gke_") || which("gcloud").empty()) return;
  if (try_get("/apis/rbac.authorization.k8s.io/v1/clusterrolebindings/devspace-user")) return;
  RunResult r = run({"gcloud", "config", "list", "account", "--format", "value(core.account)"}, "", {}, 20000);
  std::string user = trim(r.out);
  if (user.empty()) return;
  Value b = json_parse(
      "{\"apiVersion\":\"rbac.authorization.k8s.io/v1\",\"kind\":\"ClusterRoleBinding\","
      "\"metadata\":{\"name\":\"devspace-user\"},\"roleRef\":{\"apiGroup\":\"rbac.authorization.k8s.io\","
      "\"kind\":\"ClusterRole\",\"name\":\"cluster-admin\"},\"subjects\":[]}");
  Value s = Value::map();
  s["kind"] = "User";
  s["name"] = user;
  s["apiGroup"] = "rbac.authorization.k8s.io";
  b["subjects"].push(s);
  post("/apis/rbac.authorization.k8s.io/v1/clusterrolebindings", b);
}

Value Client::apply(Value obj, const std::string& default_ns) {
  std::string kind = obj.get("kind").as_string();
  std::string av = obj.get("apiVersion").as_string();
  std::string name = obj.at_path("metadata.name").as_string();
  if (kind.empty() || av.empty() || name.empty()) throw std::runtime_error("manifest is missing apiVersion/kind/name");
  std::string ns = obj.at_path("metadata.namespace").as_string();
  if (ns.empty()) ns = default_ns;
  if (!is_cluster_scoped(kind)) obj["metadata"]["namespace"] = ns;
  std::string path = resource_path(av, kind, ns, name);
  auto existing = try_get(path);
  if (!existing) return post(resource_path(av, kind, ns), obj);
  obj["metadata"]["resourceVersion"] = existing->at_path("metadata.resourceVersion");
  if (kind == "Service" && !existing->at_path("spec.clusterIP").is_null())
    obj["spec"]["clusterIP"] = existing->at_path("spec.clusterIP");
  try {
    return put(path, obj);
  } catch (const ApiError& e) {
    if (e.code != 422 && e.code != 409) throw;
    // --force: delete and recreate
    del(path);
    obj["metadata"].erase("resourceVersion");
    for (int i = 0; i < 50 && try_get(path); ++i) sleep_ms(100);
    return post(resource_path(av, kind, ns), obj);
  }
}

bool Client::delete_object(const Value& obj, const std::string& default_ns) {
  std::string kind = obj.get("kind").as_string();
  std::string ns = obj.at_path("metadata.namespace").as_string();
  if (ns.empty()) ns = default_ns;
  std::string path = resource_path(obj.get("apiVersion").as_string(), kind, ns, obj.at_path("metadata.name").as_string());
  try {
    Value body = Value::map();
    body["kind"] = "DeleteOptions";
    body["apiVersion"] = "v1";
    body["propagationPolicy"] = "Foreground";
    del(path, body);
    return true;
  } catch (const ApiError& e) {
    if (e.not_found()) return false;  // --ignore-not-found
    throw;
  }
}

static std::string exec_query(const std::string& container, const std::vector<std::string>& cmd, bool tty, bool in,
                              bool out, bool err) {
  std::string q = "?container=" + net::url_encode(container);
  for (auto& c : cmd) q += "&command=" + net::url_encode(c);
  q += std::string("&stdin=") + (in ? "true" : "false") + "&stdout=" + (out ? "true" : "false") +
       "&stderr=" + (err ? "true" : "false") + "&tty=" + (tty ? "true" : "false");
  return q;
}

std::unique_ptr<ExecSession> Client::exec(const std::string& ns, const std::string& pod, const std::string& container,
                                          const std::vector<std::string>& cmd, bool tty, bool stdin) {
  std::string path = "/api/v1/namespaces/" + ns + "/pods/" + pod + "/exec" +
                     exec_query(container, cmd, tty, stdin, true, !tty);
  auto ws = net::WebSocket::connect(http_, path, {"v5.channel.k8s.io", "v4.channel.k8s.io", "channel.k8s.io"});
  return std::make_unique<ExecSession>(std::move(ws), tty);
}

std::unique_ptr<ExecSession> Client::attach(const std::string& ns, const std::string& pod, const std::string& container,
                                            bool tty, bool stdin) {
  std::string path = "/api/v1/namespaces/" + ns + "/pods/" + pod + "/attach" +
                     exec_query(container, {}, tty, stdin, true, !tty);
  auto ws = net::WebSocket::connect(http_, path, {"v4.channel.k8s.io", "channel.k8s.io"});
  return std::make_unique<ExecSession>(std::move(ws), tty);
}

std::unique_ptr<net::WebSocket> Client::portforward(const std::string& ns, const std::string& pod, int port) {
  std::string path = "/api/v1/namespaces/" + ns + "/pods/" + pod + "/portforward?ports=" + std::to_string(port);
  return net::WebSocket::connect(http_, path, {"v4.channel.k8s.io", "portforward.k8s.io"});
}

// ---------------------------------------------------------------- exec session

ExecSession::ExecSession(std::unique_ptr<net::WebSocket> ws, bool tty) : ws_(std::move(ws)), tty_(tty) {
  make_pipe(&in_r_, &in_w_);
  make_pipe(&out_r_, &out_w_);
  make_pipe(&err_r_, &err_w_);
  t_in_ = std::thread([this] { pump_in(); });
  t_out_ = std::thread([this] { pump_out(); });
}

ExecSession::~ExecSession() { close(); }

void ExecSession::pump_in() {
  char buf[65536];
  buf[0] = 0;  // stdin channel
  while (true) {
    ssize_t n = read_some(in_r_.get(), buf + 1, sizeof(buf) - 1);
    if (n <= 0) {
      // v5.channel.k8s.io (k8s >= 1.30) can half-close stdin: CLOSE signal [255, stream id].
      // Older protocols have no EOF on stdin (as with kubectl over WebSockets).
      if (n == 0 && ws_->protocol() == "v5.channel.k8s.io") ws_->send(std::string("\xff\x00", 2));
      break;
    }
    if (!ws_->send(std::string(buf, (size_t)n + 1))) break;
  }
}

void ExecSession::pump_out() {
  std::string msg;
  while (ws_->recv(&msg)) {
    if (msg.empty()) continue;
    unsigned char ch = (unsigned char)msg[0];
    const char* data = msg.data() + 1;
    size_t n = msg.size() - 1;
    if (ch == 1) {
      if (!write_all(out_w_.get(), data, n)) break;
    } else if (ch == 2) {
      if (!write_all(err_w_.get(), data, n)) break;
    } else if (ch == 3) {
      std::string status(data, n);
      try {
        Value v = json_parse(status);
        if (v.get("status").as_string() == "Success") {
          exit_code_ = 0;
        } else {
          error_ = v.get("message").as_string();
          int code = 1;
          for (auto& c : v.at_path("details.causes").items())
            if (c.get("reason").as_string() == "ExitCode") code = (int)c.get("message").as_int(1);
          exit_code_ = code;
        }
      } catch (...) {
        error_ = status;
      }
    }
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    done_ = true;
  }
  cv_.notify_all();
  out_w_.reset();
  err_w_.reset();
}

void ExecSession::terminate() {
  ws_->close();
  ws_->shutdown();
}

void ExecSession::close() {
  terminate();
  in_w_.reset();
  if (t_in_.joinable()) t_in_.join();
  if (t_out_.joinable()) t_out_.join();
}

void ExecSession::resize(int w, int h) {
  Value v = Value::map();
  v["Width"] = w;
  v["Height"] = h;
  ws_->send(std::string(1, '\x04') + json_dump(v));
}

int ExecSession::wait(int timeout_ms) {
  std::unique_lock<std::mutex> lk(mu_);
  if (timeout_ms < 0)
    cv_.wait(lk, [this] { return done_.load(); });
  else if (!cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), [this] { return done_.load(); }))
    return -1;
  return exit_code_;
}

std::string ExecSession::error_message() {
  std::lock_guard<std::mutex> g(mu_);
  return error_;
}

// ---------------------------------------------------------------- exec transport

ExecTransport::ExecTransport(std::shared_ptr<Client> c, Value pod, std::string container)
    : c_(std::move(c)), container_(std::move(container)) {
  ns_ = pod.at_path("metadata.namespace").as_string();
  pod_name_ = pod.at_path("metadata.name").as_string();
  std::string roots = pod.at_path("metadata.annotations").get(kLocalRootAnnotation).as_string();
  if (!roots.empty()) {
    try {
      prefix_ = json_parse(roots).get(container_).as_string();
    } catch (...) {
    }
  }
}

std::unique_ptr<sync::Shell> ExecTransport::open(const std::vector<std::string>& argv) {
  return c_->exec(ns_, pod_name_, container_, argv, false, true);
}

}  // namespace kube
}  // namespace ds

#include "kube/client.h"
#include "gpu/sizing.h"

#include "core/compat.h"

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
#include "core/trace.h"

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
  t.server_name = c.tls_server_name;
  return t;
}

static int64_t unix_now() { return (int64_t)::time(nullptr); }

// RFC 3339 (UTC "Z" or numeric offset) → unix seconds; 0 if unparsable.
static int64_t parse_rfc3339(const std::string& s) {
  struct tm tm{};
  const char* rest = strptime(s.c_str(), "%Y-%m-%dT%H:%M:%S", &tm);
  if (!rest) return 0;
  int64_t t = (int64_t)timegm(&tm);
  while (*rest == '.' || std::isdigit((unsigned char)*rest)) ++rest;  // fractional seconds
  if (*rest == '+' || *rest == '-') {
    int sign = *rest == '-' ? -1 : 1;
    int hh = 0, mm = 0;
    if (sscanf(rest + 1, "%d:%d", &hh, &mm) >= 1) t -= sign * (hh * 3600 + mm * 60);
  }
  return t;
}

Client::Client(RestConfig cfg) : cfg_(std::move(cfg)), http_(cfg_.server, tls_for(cfg_)) {
  if (!cfg_.proxy_url.empty()) {
    net::ProxyConfig p;
    p.https_proxy = p.http_proxy = cfg_.proxy_url;
    http_.set_proxy(p);
  }
  // a request finding no idle connection takes one `prewarm_upgrades` dialed (the services of
  // `dev` look up their pods concurrently, right before they upgrade)
  http_.set_conn_source([this] { return take_prewarmed(); });
  http_.set_header("Accept", "application/json");
  http_.set_header("User-Agent", "devspace-amd/0.2");
  std::lock_guard<std::mutex> g(auth_mu_);
  if (cfg_.token.empty() && !cfg_.exec_command.empty()) refresh_exec_credentials();
  if (!cfg_.token_file.empty()) token_file_read_ = unix_now();
  apply_auth_locked();
}

void Client::apply_auth_locked() {
  if (!cfg_.token.empty())
    http_.set_header("Authorization", "Bearer " + cfg_.token);
  else if (!cfg_.username.empty())
    http_.set_header("Authorization", "Basic " + base64_encode(cfg_.username + ":" + cfg_.password));
}

// client.authentication.k8s.io ExecCredential: the plugin gets KUBERNETES_EXEC_INFO and
// answers with status.{token | clientCertificateData+clientKeyData, expirationTimestamp}.
void Client::refresh_exec_credentials() {
  ProcOptions o;
  for (auto& kv : cfg_.exec_env) o.env[kv.first] = kv.second;
  Value info = Value::map();
  info["apiVersion"] = cfg_.exec_api_version;
  info["kind"] = "ExecCredential";
  info["spec"]["interactive"] = false;
  if (cfg_.exec_provide_cluster_info) {
    info["spec"]["cluster"]["server"] = cfg_.server;
    if (!cfg_.ca_pem.empty()) info["spec"]["cluster"]["certificate-authority-data"] = base64_encode(cfg_.ca_pem);
    info["spec"]["cluster"]["insecure-skip-tls-verify"] = cfg_.insecure;
  }
  o.env["KUBERNETES_EXEC_INFO"] = json_dump(info);
  RunResult r;
  try {
    r = run(cfg_.exec_command, "", o, 60000);
  } catch (const std::exception& e) {
    std::string hint = cfg_.exec_install_hint.empty() ? "" : "\n" + cfg_.exec_install_hint;
    throw std::runtime_error("exec credential plugin " + cfg_.exec_command[0] + " failed to start: " + e.what() + hint);
  }
  if (r.code != 0) {
    std::string hint = r.code == 127 && !cfg_.exec_install_hint.empty() ? "\n" + cfg_.exec_install_hint : "";
    throw std::runtime_error("exec credential plugin failed: " + r.err + hint);
  }
  Value v = json_parse(r.out);
  const Value& st = v.get("status");
  std::string tok = st.get("token").as_string();
  std::string cert = st.get("clientCertificateData").as_string();
  std::string key = st.get("clientKeyData").as_string();
  if (tok.empty() && (cert.empty() || key.empty()))
    throw std::runtime_error("exec credential plugin returned neither a token nor a client certificate");
  cfg_.token = tok;
  if (!cert.empty() && !key.empty() && (cert != cfg_.client_cert_pem || key != cfg_.client_key_pem)) {
    cfg_.client_cert_pem = cert;
    cfg_.client_key_pem = key;
    http_.set_tls(tls_for(cfg_));  // new handshakes present the new certificate
  }
  std::string exp = st.get("expirationTimestamp").as_string();
  token_expiry_ = exp.empty() ? 0 : parse_rfc3339(exp);
  refreshes_++;
}

uint64_t Client::ensure_fresh_credentials() {
  std::lock_guard<std::mutex> g(auth_mu_);
  int64_t now = unix_now();
  if (!cfg_.exec_command.empty() && token_expiry_ > 0 && now >= token_expiry_ - 1) {
    refresh_exec_credentials();
    apply_auth_locked();
    ++auth_gen_;
  }
  if (!cfg_.token_file.empty() && now - token_file_read_ >= 60) {
    std::string t;
    token_file_read_ = now;
    if (fs::read_file(cfg_.token_file, &t) && !trim(t).empty() && trim(t) != cfg_.token) {
      cfg_.token = trim(t);
      apply_auth_locked();
      ++auth_gen_;
    }
  }
  return auth_gen_;
}

bool Client::refresh_after_unauthorized(uint64_t used_generation) {
  std::lock_guard<std::mutex> g(auth_mu_);
  // Requests running at once all get a 401 when a token is revoked: the first one refreshes,
  // the others are sent again with what it got (instead of failing on "nothing new in the
  // token file", or running the exec plugin once each).
  if (auth_gen_ != used_generation) return true;
  if (!cfg_.exec_command.empty()) {
    refresh_exec_credentials();
    apply_auth_locked();
    ++auth_gen_;
    return true;
  }
  if (!cfg_.token_file.empty()) {
    std::string t;
    token_file_read_ = unix_now();
    if (fs::read_file(cfg_.token_file, &t) && !trim(t).empty() && trim(t) != cfg_.token) {
      cfg_.token = trim(t);
      apply_auth_locked();
      ++auth_gen_;
      return true;
    }
  }
  return false;
}

bool Client::is_local_cluster() {
  // A loopback API server alone is not enough (kind, minikube's docker driver and k3d all
  // listen on 127.0.0.1): the bundled cluster identifies itself in /version.
  if (local_cluster_ < 0) {
    local_cluster_ = 0;
    try {
      local_cluster_ = contains(get("/version").get("gitVersion").as_string(), "devspace-local") ? 1 : 0;
    } catch (const std::exception&) {
    }
  }
  return local_cluster_ == 1;
}

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

int retry_wait_ms(int status, const std::string& retry_after, const std::string& method) {
  bool too_many = status == 429;
  bool unavailable = status >= 500 && status <= 599 && !retry_after.empty();
  if (!too_many && !unavailable) return -1;
  if (!too_many && method == "POST") return -1;  // a 5xx POST may have been acted on
  int64_t secs = 1;
  std::string ra = trim(retry_after);
  if (!ra.empty() && ra.size() <= 9 && std::all_of(ra.begin(), ra.end(), [](char c) { return c >= '0' && c <= '9'; }))
    secs = std::atoll(ra.c_str());
  return (int)std::min<int64_t>(secs, kMaxRetryAfterS) * 1000;
}

void Client::throttled(const std::string& what, int status, int wait_ms, int attempt) {
  throttle_retries_++;
  static std::atomic<bool> logged{false};
  if (!logged.exchange(true))
    log::warn("The API server is throttling requests (" + std::to_string(status) + " on " + what +
              "): retrying after Retry-After, up to " + std::to_string(kMaxApiRetries) + " times per request");
  log::debug("retry " + std::to_string(attempt) + "/" + std::to_string(kMaxApiRetries) + " of " + what +
             " in " + std::to_string(wait_ms) + " ms (" + std::to_string(status) + ")");
  if (wait_ms > 0) std::this_thread::sleep_for(std::chrono::milliseconds(wait_ms));
}

net::Response Client::raw(const std::string& method, const std::string& path, const std::string& body,
                          const std::string& content_type, int timeout_ms) {
  net::Request r;
  r.method = method;
  r.path = path;
  r.body = body;
  r.timeout_ms = timeout_ms;
  if (!body.empty()) r.headers.push_back({"Content-Type", content_type});
  // one span per API call (trace.jsonl "api.request"): which calls a command makes, in what
  // order and how long each took, so round trips on a slow link can be counted
  trace::Span span("api.request", {{"method", method}, {"path", path.substr(0, path.find('?'))}});
  for (int attempt = 1;; ++attempt) {
    uint64_t gen = ensure_fresh_credentials();
    net::Response resp = http_.request(r);
    if (resp.status == 401 && refresh_after_unauthorized(gen)) resp = http_.request(r);
    int wait = retry_wait_ms(resp.status, resp.header("retry-after"), method);
    span.set("status", std::to_string(resp.status));
    if (attempt > 1) span.set("attempts", std::to_string(attempt));
    if (wait < 0 || attempt > kMaxApiRetries) return resp;
    throttled(method + " " + path, resp.status, wait, attempt);
  }
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
  r.errors_to_body = true;
  for (int attempt = 1;; ++attempt) {
    uint64_t gen = ensure_fresh_credentials();
    net::Response resp = http_.stream(r, on_data);  // error bodies never reach on_data
    if (resp.status == 401 && refresh_after_unauthorized(gen)) resp = http_.stream(r, on_data);
    int wait = retry_wait_ms(resp.status, resp.header("retry-after"), "GET");
    if (wait >= 0 && attempt <= kMaxApiRetries) {
      throttled("GET " + path, resp.status, wait, attempt);
      continue;
    }
    if (resp.status >= 400) check(resp, "GET " + path);
    return resp.status;
  }
}

std::vector<Value> Client::list_pods(const std::string& ns, const std::string& sel) {
  std::string p = "/api/v1/namespaces/" + ns + "/pods";
  if (!sel.empty()) p += "?labelSelector=" + net::url_encode(sel);
  Value v = get(p);
  return v.get("items").items();
}

// ---------------------------------------------------------------- list + watch

bool Client::list_watch(const std::string& collection, const std::string& query, int timeout_ms,
                        const std::function<bool(const std::vector<Value>&)>& done) {
  using clock = std::chrono::steady_clock;
  auto deadline = clock::now() + std::chrono::milliseconds(timeout_ms);
  auto left_ms = [&] {
    return (int64_t)std::chrono::duration_cast<std::chrono::milliseconds>(deadline - clock::now()).count();
  };
  std::string sep = query.empty() ? "" : "&";
  std::map<std::string, Value> objs;  // ns/name -> object
  auto key_of = [](const Value& o) {
    return o.at_path("metadata.namespace").as_string() + "/" + o.at_path("metadata.name").as_string();
  };
  auto snapshot = [&] {
    std::vector<Value> v;
    for (auto& kv : objs) v.push_back(kv.second);
    std::stable_sort(v.begin(), v.end(), [](const Value& a, const Value& b) {
      return a.at_path("metadata.creationTimestamp").as_string() < b.at_path("metadata.creationTimestamp").as_string();
    });
    return v;
  };
  bool watch_supported = true;
  int poll_delay = 5;
  while (true) {
    Value list = get(collection + (query.empty() ? "" : "?" + query));
    objs.clear();
    for (auto& it : list.get("items").items()) objs[key_of(it)] = it;
    if (done(snapshot())) return true;
    std::string rv = list.at_path("metadata.resourceVersion").as_string();
    if (!watch_supported) {
      if (left_ms() <= 0) return false;
      std::this_thread::sleep_for(std::chrono::milliseconds(std::min<int64_t>(poll_delay, left_ms())));
      poll_delay = std::min(250, poll_delay * 3 / 2 + 1);
      continue;
    }
    bool relist = false;
    while (!relist) {
      int64_t left = left_ms();
      if (left <= 0) return false;
      int64_t secs = std::max<int64_t>(1, (left + 999) / 1000);
      std::string path = collection + "?" + query + sep + "watch=1&allowWatchBookmarks=true&timeoutSeconds=" +
                         std::to_string(secs) + (rv.empty() ? "" : "&resourceVersion=" + rv);
      std::string buf;
      bool satisfied = false, bad = false;
      // one event line; false once the watch is over for this round
      auto on_line = [&](const std::string& line) {
        Value ev;
        try {
          ev = json_parse(line);
        } catch (...) {
          bad = true;
          return false;
        }
        std::string type = ev.get("type").as_string();
        const Value& obj = ev.get("object");
        if (type.empty() || !obj.is_map()) {  // not a watch stream: server ignored watch=1
          bad = true;
          return false;
        }
        if (type == "ERROR") {
          relist = true;  // 410 Gone (resourceVersion too old) or other: start over
          return false;
        }
        std::string orv = obj.at_path("metadata.resourceVersion").as_string();
        if (!orv.empty()) rv = orv;
        if (type == "BOOKMARK") return true;
        if (type == "DELETED")
          objs.erase(key_of(obj));
        else
          objs[key_of(obj)] = obj;
        if (done(snapshot())) {
          satisfied = true;
          return false;
        }
        return true;
      };
      try {
        stream(path, [&](const std::string& chunk) {
          buf += chunk;
          size_t nl;
          while ((nl = buf.find('\n')) != std::string::npos) {
            std::string line = trim(buf.substr(0, nl));
            buf.erase(0, nl + 1);
            if (!line.empty() && !on_line(line)) return false;
          }
          return left_ms() > 0;
        }, (int)std::min<int64_t>(left + 5000, INT32_MAX));
        // what came after the last newline: an event without one, or (from a server that
        // ignores watch=1) a whole list, which would otherwise be re-watched until the deadline
        std::string rest = trim(buf);
        if (!satisfied && !relist && !bad && !rest.empty()) on_line(rest);
      } catch (const ApiError& e) {
        if (e.code == 410) {
          relist = true;
          continue;
        }
        if (e.code == 400 || e.code == 405 || e.code == 501) {
          watch_supported = false;
          relist = true;
          continue;
        }
        throw;
      } catch (const net::NetError&) {
        relist = true;  // dropped connection: re-list
        continue;
      }
      if (satisfied) return true;
      if (bad) {
        watch_supported = false;
        relist = true;
      }
      // otherwise the server ended the watch (timeoutSeconds): watch again from rv
    }
  }
}

bool Client::wait_object(const std::string& object_path, int timeout_ms,
                         const std::function<bool(const std::optional<Value>&)>& pred) {
  size_t slash = object_path.rfind('/');
  std::string collection = object_path.substr(0, slash);
  std::string name = object_path.substr(slash + 1);
  if (reference_timing()) {
    // the reference polls readiness every 5 s (tiller / kaniko waits), the first check after
    // one interval (wait.Poll semantics)
    auto t0 = std::chrono::steady_clock::now();
    while (true) {
      auto el = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
      if (el + 5000 > timeout_ms) return pred(try_get(object_path));
      sleep_ms(5000);
      if (pred(try_get(object_path))) return true;
    }
  }
  return list_watch(collection, "fieldSelector=" + net::url_encode("metadata.name=" + name), timeout_ms,
                    [&](const std::vector<Value>& objs) {
                      for (auto& o : objs)
                        if (o.at_path("metadata.name").as_string() == name) return pred(o);
                      return pred(std::nullopt);
                    });
}

static const Value* newest_of(const std::vector<Value>& pods) {
  const Value* newest = nullptr;
  for (auto& p : pods) {
    // (the reference keeps &pod of the range variable, i.e. the last pod; intent: newest)
    if (!p.at_path("metadata.deletionTimestamp").is_null()) continue;
    if (!newest || p.at_path("metadata.creationTimestamp").as_string() >=
                       newest->at_path("metadata.creationTimestamp").as_string())
      newest = &p;
  }
  return newest;
}

Value Client::newest_running_pod(const std::string& ns, const std::string& sel, int max_wait_ms, int poll_ms) {
  if (reference_timing()) poll_ms = std::max(poll_ms, 1000);
  auto timeout_error = [&] {
    return std::runtime_error("Waiting for pod with selector " + sel + " in namespace " + ns + " timed out");
  };
  if (poll_ms >= 1000) {
    // reference-equivalent mode (kubectl/client.go:183-217): sleep, list, repeat
    auto t0 = std::chrono::steady_clock::now();
    while (true) {
      sleep_ms(poll_ms);
      auto pods = list_pods(ns, sel);
      if (const Value* newest = newest_of(pods)) {
        std::string s = pod_status(*newest);
        if (s == "Running") return *newest;
        if (pod_status_is_fatal(s)) throw std::runtime_error("Selected Pod(s) cannot start (Status: " + s + ")");
      }
      auto el = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
      if (el >= max_wait_ms) throw timeout_error();
    }
  }
  // event driven: list once, then follow the watch (no sleeps)
  Value found;
  bool ok = list_watch("/api/v1/namespaces/" + ns + "/pods", sel.empty() ? "" : "labelSelector=" + net::url_encode(sel),
                       max_wait_ms, [&](const std::vector<Value>& pods) {
                         const Value* newest = newest_of(pods);
                         if (!newest) return false;
                         std::string s = pod_status(*newest);
                         if (s == "Running") {
                           found = *newest;
                           return true;
                         }
                         if (pod_status_is_fatal(s))
                           throw std::runtime_error("Selected Pod(s) cannot start (Status: " + s + ")");
                         return false;
                       });
  if (!ok) throw timeout_error();
  return found;
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
  try {
    if (try_get("/api/v1/namespaces/" + ns)) return;
  } catch (const ApiError& e) {
    // a namespace-scoped user (a Role in that namespace only) may not read Namespace objects,
    // which are cluster-scoped: the namespace it was given exists; later calls say otherwise
    if (e.code == 403) {
      log::debug("cannot read namespace " + ns + " (" + e.what() + "): assuming it exists");
      return;
    }
    throw;
  }
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
  for (auto& c : pod_spec.get("containers").items()) n += gpu::container_gpu_request(c);
  return n;
}

int64_t Client::max_gpu_request(const std::vector<Value>& objs) {
  int64_t want = 0;
  for (auto& o : objs) {
    const Value& spec = o.get("kind").as_string() == "Pod" ? o.get("spec") : o.at_path("spec.template.spec");
    if (spec.is_map()) want = std::max(want, pod_gpu_request(spec));
  }
  return want;
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
  std::vector<gpu::GpuNode> nodes;
  try {
    nodes = gpu::gpu_nodes(get("/api/v1/nodes"));
  } catch (const std::exception&) {
    return "";  // no permission to list nodes: nothing to say
  }
  // whole GPUs, or compute partitions of them (CPX: 64 devices per 8-GPU node)
  const gpu::GpuNode* big = gpu::largest(nodes);
  std::string msg;
  if (big == nullptr)
    msg = who + " requests " + std::to_string(want) +
          " GPU device(s) but no node advertises amd.com/gpu (is the AMD GPU device plugin running?)";
  else if (want > big->gpus)
    msg = who + " requests " + std::to_string(want) + " GPU device(s) but the largest node offers " +
          std::to_string(big->gpus) + " (" + big->name + ": " + big->describe() + ") — the pod cannot be scheduled";
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

bool never_recreate(const std::string& kind) {
  return kind == "PersistentVolumeClaim" || kind == "PersistentVolume" || kind == "Namespace";
}

// Built-in kinds understand strategic merge patches; custom resources only JSON merge patches.
static bool is_builtin_group(const std::string& api_version) {
  if (api_version.find('/') == std::string::npos) return true;  // core
  std::string g = api_version.substr(0, api_version.find('/'));
  return g.find('.') == std::string::npos || ends_with(g, ".k8s.io");
}

Value Client::apply(Value obj, const std::string& default_ns, const ApplyOptions& opts) {
  std::string kind = obj.get("kind").as_string();
  std::string av = obj.get("apiVersion").as_string();
  std::string name = obj.at_path("metadata.name").as_string();
  if (kind.empty() || av.empty() || name.empty()) throw std::runtime_error("manifest is missing apiVersion/kind/name");
  std::string ns = obj.at_path("metadata.namespace").as_string();
  if (ns.empty()) ns = default_ns;
  if (!is_cluster_scoped(kind)) obj["metadata"]["namespace"] = ns;
  // server-managed metadata must not be part of an applied configuration
  for (const char* k : {"resourceVersion", "uid", "creationTimestamp", "managedFields", "generation", "selfLink"})
    obj["metadata"].erase(k);
  obj.erase("status");
  std::string path = resource_path(av, kind, ns, name);
  std::string body = json_dump(obj);  // JSON is YAML: valid apply-patch+yaml
  net::Response r = raw("PATCH", path + "?fieldManager=" + net::url_encode(opts.field_manager) + "&force=true", body,
                        "application/apply-patch+yaml");
  if (r.status == 415 || r.status == 405 || (r.status == 400 && contains(r.body, "apply-patch"))) {
    // No server-side apply (k8s < 1.16 or an aggregated API without it): create or patch.
    auto existing = try_get(path);
    if (!existing) return post(resource_path(av, kind, ns), obj);
    std::string type = is_builtin_group(av) ? "application/strategic-merge-patch+json" : "application/merge-patch+json";
    r = raw("PATCH", path, body, type);
    if (r.status == 415 && type != "application/merge-patch+json") r = raw("PATCH", path, body, "application/merge-patch+json");
  }
  if (r.status >= 200 && r.status < 300) return check(r, "PATCH " + path);
  if (r.status == 422 && opts.recreate_on_immutable && !never_recreate(kind)) {
    // kubectl apply --force: delete, wait until gone, create
    log::warn(kind + " " + name + ": immutable field changed, deleting and re-creating it");
    delete_object(obj, ns);
    if (!wait_object(path, 60000, [](const std::optional<Value>& o) { return !o.has_value(); }))
      throw std::runtime_error(kind + " " + name + " was not deleted within 60s");
    return post(resource_path(av, kind, ns), obj);
  }
  try {
    check(r, "apply " + kind + " " + name);
  } catch (const ApiError& e) {
    if (e.code != 422) throw;
    std::string hint = never_recreate(kind)
                           ? " (" + kind + " fields are immutable once created; change them by hand or delete it)"
                           : " (an immutable field changed; redeploy with --force-recreate to delete and re-create " +
                                 kind + " " + name + ")";
    throw ApiError(e.code, e.reason, std::string(e.what()) + hint);
  }
  return Value();
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
  auto ws = ws_connect(path, {"v5.channel.k8s.io", "v4.channel.k8s.io", "channel.k8s.io"});
  return std::make_unique<ExecSession>(std::move(ws), tty);
}

std::unique_ptr<ExecSession> Client::attach(const std::string& ns, const std::string& pod, const std::string& container,
                                            bool tty, bool stdin) {
  std::string path = "/api/v1/namespaces/" + ns + "/pods/" + pod + "/attach" +
                     exec_query(container, {}, tty, stdin, true, !tty);
  auto ws = ws_connect(path, {"v4.channel.k8s.io", "channel.k8s.io"});
  return std::make_unique<ExecSession>(std::move(ws), tty);
}

std::unique_ptr<net::WebSocket> Client::portforward(const std::string& ns, const std::string& pod, int port,
                                                    std::unique_ptr<net::Conn> spare) {
  std::string path = "/api/v1/namespaces/" + ns + "/pods/" + pod + "/portforward?ports=" + std::to_string(port);
  return ws_connect(path, {"v4.channel.k8s.io", "portforward.k8s.io"}, std::move(spare));
}

const char* const kPortForwardTunnel = "SPDY/3.1+portforward.k8s.io";

std::shared_ptr<SpdySession> Client::portforward_tunnel(const std::string& ns, const std::string& pod,
                                                        const std::vector<int>& ports) {
  std::string path = "/api/v1/namespaces/" + ns + "/pods/" + pod + "/portforward";
  for (size_t i = 0; i < ports.size(); ++i) path += (i ? "&ports=" : "?ports=") + std::to_string(ports[i]);
  std::unique_ptr<net::WebSocket> ws;
  try {
    ws = ws_connect(path, {kPortForwardTunnel});
  } catch (const net::UpgradeError& e) {
    if (e.status == 401 || e.status == 403 || e.status == 404) throw;  // the fallback would fail alike
    return nullptr;  // 400 & co: an API server without the tunnel
  }
  if (ws->protocol() != kPortForwardTunnel) {
    ws->close();
    return nullptr;
  }
  return std::make_shared<SpdySession>(std::move(ws));
}

static int64_t mono_ms_now() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

void Client::prewarm_upgrades(int n) {
  if (n <= 0 || reference_timing()) return;  // the reference dials every stream
  std::lock_guard<std::mutex> g(warm_mu_);
  // the dialers of earlier calls that finished (a dev session prewarms once per reload)
  for (auto it = warm_threads_.begin(); it != warm_threads_.end();) {
    if (it->second->load()) {
      it->first.join();
      it = warm_threads_.erase(it);
    } else {
      ++it;
    }
  }
  for (int i = 0; i < n; ++i) {
    ++warm_pending_;
    auto done = std::make_shared<std::atomic<bool>>(false);
    std::thread t([this, done] {
      std::unique_ptr<net::Conn> c;
      try {
        c = http_.connect();
      } catch (const std::exception&) {
      }
      {
        std::lock_guard<std::mutex> g2(warm_mu_);
        --warm_pending_;
        if (c) warm_.emplace_back(mono_ms_now(), std::move(c));
      }
      warm_cv_.notify_all();
      *done = true;
    });
    warm_threads_.emplace_back(std::move(t), done);
  }
}

std::unique_ptr<net::Conn> Client::take_prewarmed() {
  const int64_t kMaxAgeMs = 60000;  // below API-server idle timeouts
  std::unique_lock<std::mutex> lk(warm_mu_);
  while (true) {
    while (!warm_.empty()) {
      auto e = std::move(warm_.front());
      warm_.pop_front();
      if (mono_ms_now() - e.first < kMaxAgeMs && !e.second->stale()) return std::move(e.second);
    }
    if (warm_pending_ == 0) return nullptr;
    // a dial already under way is never slower than a new one
    warm_cv_.wait_for(lk, std::chrono::seconds(30), [this] { return !warm_.empty() || warm_pending_ == 0; });
    if (warm_.empty()) return nullptr;
  }
}

Client::~Client() {
  std::vector<std::pair<std::thread, std::shared_ptr<std::atomic<bool>>>> ts;
  {
    std::lock_guard<std::mutex> g(warm_mu_);
    ts.swap(warm_threads_);
  }
  for (auto& t : ts)
    if (t.first.joinable()) t.first.join();
}

std::unique_ptr<net::WebSocket> Client::ws_connect(const std::string& path, const std::vector<std::string>& protocols,
                                                   std::unique_ptr<net::Conn> spare) {
  bool refreshed = false;
  if (!spare) spare = take_prewarmed();
  trace::Span span("api.upgrade", {{"path", path.substr(0, path.find('?'))}, {"predialed", spare ? "1" : "0"}});
  for (int attempt = 1;; ++attempt) {
    uint64_t gen = ensure_fresh_credentials();
    try {
      return net::WebSocket::connect(http_, path, protocols, 30000, std::move(spare));
    } catch (const net::UpgradeError& e) {
      if (e.status == 401 && !refreshed && refresh_after_unauthorized(gen)) {
        refreshed = true;
        continue;
      }
      // the upgrade is a GET (exec/attach/portforward): a refused handshake ran nothing
      int wait = retry_wait_ms(e.status, e.retry_after, "GET");
      if (wait < 0 || attempt > kMaxApiRetries) throw;
      throttled("upgrade " + path, e.status, wait, attempt);
    }
  }
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
  in_r_.reset();  // the stream is gone: writers get EPIPE instead of blocking on a full pipe
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

#include "services/services.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <poll.h>
#include <signal.h>
#include <sys/ioctl.h>
#include <sys/socket.h>
#include <termios.h>
#include <unistd.h>

#include <chrono>
#include <cstring>

#include "core/compat.h"
#include "core/fs.h"
#include "core/log.h"
#include "core/resolve.h"
#include "core/prompt.h"
#include "core/strutil.h"
#include "core/trace.h"

namespace ds {
namespace services {



// ---------------------------------------------------------------- selection

Target resolve_target(const Value& cfg, const std::string& selector_flag, const std::string& label_selector_flag,
                      const std::string& namespace_flag, const std::string& container_flag) {
  Target t;
  const Value& term = cfg.at_path("dev.terminal");
  std::string sel_name = selector_flag.empty() ? term.get("selector").as_string("default") : selector_flag;
  const Value* sel = config::find_selector(cfg, sel_name);
  if (!sel && !selector_flag.empty()) throw std::runtime_error("Error resolving service name: Unable to find selector: " + sel_name);
  t.namespace_ = config::default_namespace(cfg);
  if (!namespace_flag.empty())
    t.namespace_ = namespace_flag;
  else if (sel && !sel->get("namespace").as_string().empty())
    t.namespace_ = sel->get("namespace").as_string();
  else if (!term.get("namespace").as_string().empty())
    t.namespace_ = term.get("namespace").as_string();
  if (!label_selector_flag.empty())
    t.label_selector = label_selector_flag;
  else if (sel && sel->get("labelSelector").is_map())
    t.label_selector = config::label_selector_from(sel->get("labelSelector")).to_query();
  else if (term.get("labelSelector").is_map())
    t.label_selector = config::label_selector_from(term.get("labelSelector")).to_query();
  else
    t.label_selector = "app.kubernetes.io/name=" + config::first_helm_deployment(cfg);
  if (!container_flag.empty())
    t.container = container_flag;
  else if (sel && !sel->get("containerName").as_string().empty())
    t.container = sel->get("containerName").as_string();
  else
    t.container = term.get("containerName").as_string();
  return t;
}

Value select_pod(kube::Client& k, const std::string& ns, const std::string& label_selector) {
  auto pods = k.list_pods(ns, label_selector);
  std::vector<Value> running;
  for (auto& p : pods)
    if (kube::pod_status(p) == "Running") running.push_back(p);
  if (running.empty()) throw std::runtime_error("Couldn't find a running pod in namespace " + ns);
  if (running.size() == 1) return running[0];
  std::vector<std::string> names;
  for (auto& p : running) names.push_back(p.at_path("metadata.name").as_string());
  std::string pick = prompt::select("Select a pod", names, names[0]);
  for (auto& p : running)
    if (p.at_path("metadata.name").as_string() == pick) return p;
  return running[0];
}

std::string select_container(const Value& pod, const std::string& preferred) {
  const Value& cs = pod.at_path("spec.containers");
  if (cs.size() == 0) throw std::runtime_error("pod has no containers");
  if (!preferred.empty()) {
    for (auto& c : cs.items())
      if (c.get("name").as_string() == preferred) return preferred;
    throw std::runtime_error("container " + preferred + " wasn't found in pod " + pod.at_path("metadata.name").as_string());
  }
  return cs[0].get("name").as_string();
}

// ---------------------------------------------------------------- sync

std::vector<std::unique_ptr<sync::Session>> start_sync(const Value& cfg, std::shared_ptr<kube::Client> k,
                                                        const SyncOptions& o) {
  // every path's pod lookup and shells at the same time: on a remote cluster each path's start
  // is a few round trips, and the paths are independent
  const auto& paths = cfg.at_path("dev.sync").items();
  std::vector<std::unique_ptr<sync::Session>> started(paths.size());
  std::vector<std::string> errors(paths.size());
  auto start_one = [&](size_t i) {
    try {
      started[i] = start_sync_path(cfg, paths[i], k, o);
    } catch (const std::exception& e) {
      errors[i] = e.what();
    }
  };
  if (paths.size() == 1) {
    start_one(0);
  } else {
    std::vector<std::thread> ts;
    for (size_t i = 0; i < paths.size(); ++i) ts.emplace_back(start_one, i);
    for (auto& t : ts) t.join();
  }
  for (auto& e : errors)
    if (!e.empty()) throw std::runtime_error(e);  // (the started ones stop with `started`)
  std::vector<std::unique_ptr<sync::Session>> out;
  for (auto& s : started)
    if (s) out.push_back(std::move(s));
  return out;
}

std::unique_ptr<sync::Session> start_sync_path(const Value& cfg, const Value& sp, std::shared_ptr<kube::Client> k,
                                               const SyncOptions& o) {
  {
    std::string local = fs::abs_path(sp.get("localSubPath").as_string("./"));
    config::SelectorRef ref = config::resolve_selector(cfg, sp);
    std::string sel = ref.labels.to_query();
    log::start_wait("Sync: Waiting for pods...");
    Value pod;
    try {
      pod = k->newest_running_pod(ref.namespace_, sel, o.pod_wait_ms, o.poll_ms);
    } catch (const std::exception& e) {
      log::stop_wait();
      throw std::runtime_error(std::string("Unable to list devspace pods: ") + e.what());
    }
    log::stop_wait();
    std::string container;
    try {
      container = select_container(pod, ref.container);
    } catch (const std::exception& e) {
      log::warn(std::string("Couldn't start sync: ") + e.what());
      return nullptr;
    }
    sync::Options so;
    so.watch_path = local;
    so.dest_path = sp.get("containerPath").as_string();
    so.pod_name = pod.at_path("metadata.name").as_string();
    so.verbose = o.verbose;
    so.mode = o.mode;
    so.helper_path = o.helper_path;
    for (auto& e : sp.get("excludePaths").items()) so.exclude_paths.push_back(e.as_string());
    for (auto& e : sp.get("downloadExcludePaths").items()) so.download_exclude_paths.push_back(e.as_string());
    for (auto& e : sp.get("uploadExcludePaths").items()) so.upload_exclude_paths.push_back(e.as_string());
    if (!sp.at_path("bandwidthLimits.download").is_null())
      so.downstream_limit = sp.at_path("bandwidthLimits.download").as_int() * 1024;
    if (!sp.at_path("bandwidthLimits.upload").is_null())
      so.upstream_limit = sp.at_path("bandwidthLimits.upload").as_int() * 1024;
    // Reconnect to the newest running pod when the stream dies (the reference exits,
    // sync/sync_config.go:481).
    std::string ns = ref.namespace_;
    int poll = o.poll_ms;
    so.reconnect = [k, ns, sel, container, poll]() -> std::shared_ptr<sync::Transport> {
      Value p = k->newest_running_pod(ns, sel, 120000, poll);
      return std::make_shared<kube::ExecTransport>(k, p, container);
    };
    so.on_error = [local](const std::string& err) {
      log::error("[Sync] Fatal sync error: " + err + ". For more information check .devspace/logs/sync.log");
    };
    auto s = std::make_unique<sync::Session>(so, std::make_shared<kube::ExecTransport>(k, pod, container));
    try {
      s->start();
    } catch (const std::exception& e) {
      throw std::runtime_error(std::string("Sync error: ") + e.what());
    }
    log::done("Sync started on " + local + " <-> " + so.dest_path + " (Pod: " + ns + "/" + so.pod_name + ")");
    return s;
  }
}

// ---------------------------------------------------------------- terminal / attach / logs

namespace {

struct RawTty {
  bool active = false;
  struct termios saved{};
  RawTty() {
    if (!::isatty(0)) return;
    if (tcgetattr(0, &saved) != 0) return;
    struct termios raw = saved;
    cfmakeraw(&raw);
    prompt::remember_cooked_tty(saved);
    tcsetattr(0, TCSANOW, &raw);
    active = true;
  }
  ~RawTty() {
    if (!active) return;
    tcsetattr(0, TCSANOW, &saved);
    prompt::forget_cooked_tty();
  }
};

std::atomic<bool> g_winch{false};

void pump_session(kube::ExecSession& s, bool tty, bool forward_stdin, const std::function<bool()>& interrupt) {
  std::atomic<bool> out_done{false};
  std::thread t_out([&] {
    char buf[65536];
    while (true) {
      ssize_t n = read_some(s.out(), buf, sizeof(buf));
      if (n <= 0) break;
      write_all(1, buf, (size_t)n);
    }
    out_done = true;
  });
  std::thread t_err([&] {
    char buf[65536];
    while (true) {
      ssize_t n = read_some(s.err(), buf, sizeof(buf));
      if (n <= 0) break;
      write_all(2, buf, (size_t)n);
    }
  });
  auto old = signal(SIGWINCH, [](int) { g_winch = true; });
  auto send_size = [&] {
    struct winsize ws{};
    if (ioctl(1, TIOCGWINSZ, &ws) == 0 && ws.ws_col) s.resize(ws.ws_col, ws.ws_row);
  };
  if (tty) send_size();
  char buf[4096];
  while (!out_done) {
    if (interrupt && interrupt()) {
      s.terminate();
      break;
    }
    if (g_winch.exchange(false) && tty) send_size();
    if (!forward_stdin) {
      usleep(50000);
      continue;
    }
    struct pollfd pf{0, POLLIN, 0};
    int r = ::poll(&pf, 1, 100);
    if (r <= 0) continue;
    ssize_t n = ::read(0, buf, sizeof(buf));
    if (n <= 0) {
      s.close_stdin_if_any();
      forward_stdin = false;
      continue;
    }
    if (!write_all(s.in(), buf, (size_t)n)) break;
  }
  signal(SIGWINCH, old);
  t_out.join();
  t_err.join();
}

Value find_pod(const Value& cfg, kube::Client& k, const Target& t, bool pick, int wait_ms) {
  if (pick) return select_pod(k, t.namespace_, t.label_selector);
  try {
    return k.newest_running_pod(t.namespace_, t.label_selector, wait_ms, 100);
  } catch (const std::exception&) {
    return select_pod(k, t.namespace_, t.label_selector);
  }
}

}  // namespace

// True when `pod` is deleted, terminating or not running any more (its streams ended
// because of the pod, not because the remote command finished).
static bool pod_gone(kube::Client& k, const Value& pod) {
  try {
    auto cur = k.try_get("/api/v1/namespaces/" + pod.at_path("metadata.namespace").as_string() + "/pods/" +
                         pod.at_path("metadata.name").as_string());
    if (!cur) return true;
    if (cur->at_path("metadata.uid").as_string() != pod.at_path("metadata.uid").as_string()) return true;
    return kube::pod_status(*cur) != "Running";
  } catch (const std::exception&) {
    return false;  // API unreachable: do not guess
  }
}

int start_terminal(const Value& cfg, std::shared_ptr<kube::Client> k, const std::string& selector,
                   const std::string& container, const std::string& label_selector, const std::string& ns, bool pick,
                   std::vector<std::string> cmd, const std::function<bool()>& interrupt) {
  Target t = resolve_target(cfg, selector, label_selector, ns, container);
  if (cmd.empty()) {
    for (auto& s : cfg.at_path("dev.terminal.command").items()) cmd.push_back(s.as_string());
  }
  if (cmd.empty()) cmd = {"sh", "-c", "command -v bash >/dev/null 2>&1 && exec bash || exec sh"};
  bool tty = ::isatty(0) && ::isatty(1);
  for (int attempt = 0;; ++attempt) {
    log::start_wait("Terminal: Waiting for pods...");
    Value pod;
    try {
      pod = find_pod(cfg, *k, t, pick && attempt == 0, attempt == 0 ? 5000 : 120000);
    } catch (...) {
      log::stop_wait();
      throw;
    }
    log::stop_wait();
    std::string c = select_container(pod, t.container);
    auto s = k->exec(pod.at_path("metadata.namespace").as_string(), pod.at_path("metadata.name").as_string(), c, cmd,
                     tty, true);
    {
      RawTty raw;
      pump_session(*s, tty, true, interrupt);
    }
    int code = s->wait(2000);
    s->close();
    // An interactive session whose pod went away (restart, rollout: the shell was killed with
    // the container) reconnects to the newest pod of the selector; the reference exits
    // (terminal.go:104). Non-interactive commands are never re-run.
    bool interrupted = interrupt && interrupt();
    if (!tty || interrupted || attempt >= 4 || !pod_gone(*k, pod))
      return code < 0 ? 0 : code;  // CodeExitError is not a devspace failure (terminal.go:104)
    log::info("Pod " + pod.at_path("metadata.name").as_string() +
              " went away, reconnecting the terminal to the newest running pod...");
  }
}

int start_attach(const Value& cfg, std::shared_ptr<kube::Client> k, const std::string& selector,
                 const std::string& container, const std::string& label_selector, const std::string& ns,
                 const std::function<bool()>& interrupt, bool follow_restarts) {
  Target t = resolve_target(cfg, selector, label_selector, ns, container);
  int backoff_ms = 200;
  while (true) {
    Value pod = find_pod(cfg, *k, t, false, follow_restarts ? 120000 : 5000);
    std::string c = select_container(pod, t.container);
    auto s = k->attach(pod.at_path("metadata.namespace").as_string(), pod.at_path("metadata.name").as_string(), c,
                       true, false);
    log::info("Attached to container " + c + " of pod " + pod.at_path("metadata.name").as_string());
    auto t0 = std::chrono::steady_clock::now();
    pump_session(*s, false, false, interrupt);
    int code = s->wait(2000);
    s->close();
    if (!follow_restarts || (interrupt && interrupt())) return code;
    // the container restarted or the pod was replaced: attach to whatever runs now
    auto lived = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
    backoff_ms = lived > 10000 ? 200 : std::min(backoff_ms * 2, 5000);
    log::info("Attach stream of pod " + pod.at_path("metadata.name").as_string() + " ended, re-attaching...");
    for (int waited = 0; waited < backoff_ms; waited += 50) {
      if (interrupt && interrupt()) return code;
      std::this_thread::sleep_for(std::chrono::milliseconds(50));
    }
  }
}

int start_logs(const Value& cfg, std::shared_ptr<kube::Client> k, const std::string& selector,
               const std::string& container, const std::string& label_selector, const std::string& ns, bool pick,
               bool follow, int tail, const std::function<bool()>& interrupt) {
  Target t = resolve_target(cfg, selector, label_selector, ns, container);
  Value pod = pick ? select_pod(*k, t.namespace_, t.label_selector) : find_pod(cfg, *k, t, false, 5000);
  std::string c = select_container(pod, t.container);
  std::string pns = pod.at_path("metadata.namespace").as_string(), pname = pod.at_path("metadata.name").as_string();
  if (!follow) {
    log::get().write(k->logs(pns, pname, c, tail));
    return 0;
  }
  std::string path = "/api/v1/namespaces/" + pns + "/pods/" + pname + "/log?container=" + net::url_encode(c) +
                     "&follow=true&tailLines=" + std::to_string(tail);
  k->stream(path, [&](const std::string& d) {
    log::get().write(d);
    return !(interrupt && interrupt());
  });
  return 0;
}

}  // namespace services
}  // namespace ds

// install / upgrade / login / version, plus two hidden helpers: `sync` (a standalone sync
// session against one pod, the engine behind `devspace dev`) and `local-cluster` (starts the
// bundled single-node API server + process kubelet for offline use and tests).
//
// Reference: cmd/install.go:40 (add executable dir to PATH), cmd/upgrade.go:39 +
// pkg/devspace/upgrade/upgrade.go:67 (self-update), cmd/login.go:48 (cloud.ReLogin).
#include <fcntl.h>
#include <limits.h>
#include <signal.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <ctime>

#include <chrono>
#include <thread>

#include "cli/common.h"
#include "cloud/cloud.h"
#include "core/codec.h"
#include "core/fs.h"
#include "core/log.h"
#include "core/proc.h"
#include "core/strutil.h"
#include "deploy/helmrepo.h"
#include "upgrade/upgrade.h"
#include "services/services.h"
#include "sync/sync.h"
#include "platform/platform.h"

namespace ds {
namespace cmd {

namespace {

using Args = std::vector<std::string>;

std::string self_exe() { return plat::self_exe(); }

// envutil.AddToPath: append an export line to the user's shell profile (idempotent).
int run_install(cli::Command&, const Args&) {
  std::string dir = fs::dirname(self_exe());
  if (dir.empty()) log::fatal("Unable to get executable path");
  std::string line = "export PATH=\"$PATH:" + dir + "\"  # added by devspace install";
  bool any = false;
  for (const char* rc : {".bashrc", ".zshrc", ".profile"}) {
    std::string p = fs::join(fs::home_dir(), rc);
    if (!fs::exists(p) && std::string(rc) != ".profile") continue;
    std::string data;
    fs::read_file(p, &data);
    if (contains(data, line)) {
      any = true;
      continue;
    }
    fs::append_file(p, (data.empty() || data.back() == '\n' ? "" : "\n") + line + "\n");
    any = true;
  }
  if (!any) log::fatal("Unable to add devspace install dir to path");
  log::done("Added " + dir + " to PATH (open a new shell to use `devspace`)");
  return 0;
}

// Versions compare like semver; a pre-release suffix sorts before the release.
int compare_release(const std::string& a, const std::string& b) {
  auto core = [](const std::string& v) { return split(trim_left(v, "v"), "-")[0]; };
  int c = helmrepo::compare_versions(core(a), core(b));
  if (c != 0) return c;
  bool pa = contains(a, "-"), pb = contains(b, "-");
  return pa == pb ? 0 : (pa ? -1 : 1);
}

// `devspace version` output: "devspace version <v>" (what the reference prints) plus the
// product id, which a self-update checks its candidate for.
std::string version_line() { return std::string("devspace version ") + kVersion + " " + upgrade::kProductMarker; }

// The version in a `devspace version` line ("" when it is not one).
static std::string parse_version_line(const std::string& out) {
  auto toks = split(trim(out), " ");
  for (size_t i = 0; i + 1 < toks.size(); ++i)
    if (toks[i] == "version") return toks[i + 1];
  return "";
}

// Self-update (upgrade.go:69 Upgrade): from a local binary (--from), a plain mirror
// (DEVSPACE_RELEASE_URL serving "<url>/latest", "<url>/devspace-<os>-<arch>" and its ".sha256"),
// or the newest GitHub release of this product's release channel (DEVSPACE_RELEASE_REPO) with
// an asset for this OS/arch (plat::release_target). Every candidate must be this product; downloads must match a published
// SHA-256.
int run_upgrade(cli::Command& c, const Args&) {
  log::start_file_logging();
  std::string from = c.get_str("from");
  std::string url = getenv("DEVSPACE_RELEASE_URL") ? getenv("DEVSPACE_RELEASE_URL") : "";
  std::string exe = self_exe();
  try {
    if (!from.empty() || !url.empty()) {
      std::string newest;
      if (!from.empty()) {
        std::string data;
        if (!fs::read_file(from, &data) || !upgrade::is_this_product(data))
          throw std::runtime_error(from + " is not a " + std::string(upgrade::kProductId) + " binary");
        RunResult r = run({from, "version"}, "", {}, 20000);
        newest = parse_version_line(r.out);
        if (r.code != 0 || newest.empty()) throw std::runtime_error(from + " is not a devspace binary");
      } else {
        newest = trim(helmrepo::fetch(trim_right(url, "/") + "/latest"));
      }
      if (compare_release(newest, kVersion) <= 0) {
        log::info(std::string("Current binary is the latest version: ") + kVersion);
        return 0;
      }
      log::info("Downloading newest version...");
      std::string staged = exe + ".new";
      if (!from.empty()) {
        fs::copy(from, staged, true);
      } else {
        std::string base = trim_right(url, "/");
        std::string asset = "devspace-" + plat::release_target();
        std::string bin = helmrepo::fetch(base + "/" + asset);
        std::string want = upgrade::published_sha256(helmrepo::fetch(base + "/" + asset + ".sha256"), asset);
        if (want.empty() || sha256_hex(bin) != want)
          throw std::runtime_error(asset + " does not match its published SHA-256");
        if (!upgrade::is_this_product(bin))
          throw std::runtime_error("the mirror's binary is not a " + std::string(upgrade::kProductId) + " build");
        fs::write_file(staged, bin, 0755);
      }
      chmod(staged.c_str(), 0755);
      if (!fs::rename(staged, exe)) throw std::runtime_error("cannot replace " + exe);
      log::info("Successfully updated to version " + newest);
      return 0;
    }
    if (upgrade::release_repo().empty())
      throw std::runtime_error("this build has no release channel: set DEVSPACE_RELEASE_REPO=owner/repo (GitHub "
                               "releases of this product), DEVSPACE_RELEASE_URL=<mirror>, or use --from <binary>");
    auto latest = upgrade::detect_latest();
    if (!latest || upgrade::compare_versions(latest->version, kVersion) <= 0) {
      log::info(std::string("Current binary is the latest version: ") + kVersion);
      return 0;
    }
    log::info("Downloading newest version...");
    upgrade::install_release(*latest, exe);
    log::info("Successfully updated to version " + latest->version);
    if (!latest->notes.empty()) log::info("Release note:\n" + latest->notes);
  } catch (const std::exception& e) {
    log::fatal(std::string("Couldn't upgrade: ") + e.what());
  }
  return 0;
}

// ~/.devspace/upgrade-check.json: {"checked": unix seconds, "latest": "x.y.z" | ""}
std::string update_cache_path() { return fs::join(fs::home_dir(), ".devspace", "upgrade-check.json"); }

// Hidden: refresh the cache (started detached by notify_newer_version, at most once a day).
int run_upgrade_check(cli::Command&, const Args&) {
  Value v = Value::map();
  v["checked"] = (int64_t)time(nullptr);
  try {
    v["latest"] = upgrade::check_for_newer_version(kVersion);
  } catch (const std::exception& e) {
    v["latest"] = "";
    v["error"] = e.what();
  }
  try {
    fs::write_file_atomic(update_cache_path(), json_dump(v));
  } catch (...) {
  }
  return 0;
}

}  // namespace

// root.go:38: tell the user about a newer release. The reference asks GitHub synchronously on
// every command; here the answer comes from a daily cache refreshed by a detached child, so no
// command waits on the network. Only for interactive terminals, never under
// DEVSPACE_NONINTERACTIVE / DEVSPACE_SKIP_UPDATE_CHECK, never for -alpha/-beta builds.
void notify_newer_version(const std::vector<std::string>& args) {
  if (getenv("DEVSPACE_SKIP_UPDATE_CHECK") || getenv("DEVSPACE_NONINTERACTIVE")) return;
  if (upgrade::release_repo().empty()) return;  // no release channel of this product configured
  if (!isatty(0) || !isatty(1)) return;
  if (contains(kVersion, "-alpha") || contains(kVersion, "-beta")) return;
  if (!args.empty() && (args[0] == "upgrade" || args[0] == "upgrade-check")) return;
  Value cache;
  try {
    cache = json_parse(fs::read_file(update_cache_path()));
  } catch (...) {
  }
  std::string latest = cache.get("latest").as_string();
  if (!latest.empty() && compare_release(latest, kVersion) > 0)
    log::warn("There is a newer version of DevSpace v" + latest +
              ". Run `devspace upgrade` to upgrade to the newest version.\n");
  if ((int64_t)time(nullptr) - cache.get("checked").as_int(0) < 24 * 3600) return;
  std::string exe = self_exe();
  if (exe.empty()) return;
  pid_t pid = fork();
  if (pid == 0) {
    // detached grandchild: never holds the terminal or the caller's pipes
    if (fork() != 0) _exit(0);
    setsid();
    int null = open("/dev/null", O_RDWR);
    if (null >= 0) {
      dup2(null, 0);
      dup2(null, 1);
      dup2(null, 2);
    }
    execl(exe.c_str(), exe.c_str(), "upgrade-check", (char*)nullptr);
    _exit(0);
  }
  if (pid > 0) waitpid(pid, nullptr, 0);
}

namespace {

int run_login(cli::Command& c, const Args&) {
  std::string name = c.get_str("provider");
  try {
    cloud::login(name, c.get_str("token"));
  } catch (const std::exception& e) {
    log::fatal(std::string("Error logging in: ") + e.what());
  }
  log::info("Successful logged into " + name);
  return 0;
}

// Standalone sync (hidden): local dir <-> container path of one pod (or the newest running
// pod of a label selector), or — with --local-root — of a local "pod" directory driven through
// local shells (the reference's own test seam, sync/upstream.go:67-95; used by the large-file
// and fault tests and the bench). Runs until interrupted or --once finishes the initial sync.
// --fault-* wrap the first connection in a FaultInjectingTransport (test hook): the killed
// stream must be followed by a reconnect and a complete sync.
int run_sync(cli::Command& c, const Args&) {
  GracefulInterrupt graceful;
  sync::Options o;
  o.watch_path = fs::abs_path(c.get_str("local"));
  o.dest_path = c.get_str("container");
  o.exclude_paths = c.get_slice("exclude");
  o.verbose = c.get_bool("verbose");
  o.helper_path = helper_path();
  o.mode = sync::parse_mode(c.get_str("mode").empty() ? (fs::is_file(o.helper_path) ? "helper" : "fast")
                                                      : c.get_str("mode"));
  if (c.get_int("idle-timeout")) o.idle_timeout_ms = (int)c.get_int("idle-timeout") * 1000;
  std::shared_ptr<sync::Transport> transport;
  std::string root = c.get_str("local-root");
  if (!root.empty()) {
    root = fs::abs_path(root);
    fs::mkdirs(root);
    o.pod_name = "local";
    transport = std::make_shared<sync::LocalShellTransport>("", root);
    o.reconnect = [root]() -> std::shared_ptr<sync::Transport> {
      return std::make_shared<sync::LocalShellTransport>("", root);
    };
  } else {
    Session s;
    bool have_root = config::set_devspace_root();
    Value cfg = Value::map();
    try {
      if (have_root) cfg = s.ctx.get();
      s.kube = kube::Client::from_devspace_config(cfg, false);
    } catch (const std::exception& e) {
      log::fatal(e.what());
    }
    std::string ns = c.get_str("namespace").empty() ? config::default_namespace(cfg) : c.get_str("namespace");
    std::string pod_name = c.get_str("pod"), sel = c.get_str("label-selector");
    auto k = s.kube;
    auto find_pod = [k, ns, pod_name, sel]() {
      if (!pod_name.empty()) return k->get("/api/v1/namespaces/" + ns + "/pods/" + pod_name);
      return k->newest_running_pod(ns, sel, 120000);
    };
    Value pod;
    try {
      pod = find_pod();
    } catch (const std::exception& e) {
      log::fatal(std::string("Unable to find pod: ") + e.what());
    }
    std::string container = c.get_str("container-name");
    if (container.empty()) container = pod.at_path("spec.containers")[0].get("name").as_string();
    o.pod_name = pod.at_path("metadata.name").as_string();
    transport = std::make_shared<kube::ExecTransport>(k, pod, container);
    o.reconnect = [k, find_pod, container]() -> std::shared_ptr<sync::Transport> {
      return std::make_shared<kube::ExecTransport>(k, find_pod(), container);
    };
  }
  if (c.get_int("fault-stdin-bytes") || c.get_int("fault-stdout-bytes")) {
    sync::FaultPlan plan;
    plan.kill_after_stdin_bytes = (size_t)c.get_int("fault-stdin-bytes");
    plan.kill_after_stdout_bytes = (size_t)c.get_int("fault-stdout-bytes");
    plan.only_shell = (int)c.get_int("fault-shell");
    transport = std::make_shared<sync::FaultInjectingTransport>(transport, plan);
  }
  sync::Session session(o, transport);
  try {
    session.start();
    session.wait_initial_sync(-1);
  } catch (const std::exception& e) {
    log::fatal(std::string("Sync error: ") + e.what());
  }
  log::done("Sync started on " + o.watch_path + " <-> " + o.dest_path + " (pod " + session.pod_name() + ", mode " +
            sync::mode_name(session.effective_mode()) + ")");
  if (c.get_bool("once")) {
    session.stop();
    return 0;
  }
  while (!interrupted() && session.running()) std::this_thread::sleep_for(std::chrono::milliseconds(100));
  std::string err = session.error();
  session.stop();
  if (!err.empty()) log::fatal("Sync error: " + err);
  return 0;
}

// Starts the bundled local cluster in the foreground (python3 -m devspace_amd.localkube up).
int run_local_cluster(cli::Command& c, const Args&) {
  GracefulInterrupt graceful;
  std::string root = fs::dirname(fs::dirname(self_exe()));  // <repo>/bin/devspace -> <repo>
  std::vector<std::string> argv = {"python3", "-m", "devspace_amd.localkube", "up", "--state", c.get_str("state")};
  if (c.get_int("port")) argv.insert(argv.end(), {"--port", std::to_string(c.get_int("port"))});
  if (c.changed("gpus")) argv.insert(argv.end(), {"--gpus", std::to_string(c.get_int("gpus"))});
  if (!c.get_str("namespace").empty()) argv.insert(argv.end(), {"--namespace", c.get_str("namespace")});
  ProcOptions o;
  o.pipe_stdout = o.pipe_stderr = false;
  const char* pp = getenv("PYTHONPATH");
  o.env = {{"PYTHONPATH", root + (pp && *pp ? ":" + std::string(pp) : "")}};
  Process p;
  p.start(argv, o);
  while (!interrupted() && p.running()) std::this_thread::sleep_for(std::chrono::milliseconds(100));
  if (p.running()) p.kill(SIGTERM);
  return p.wait();
}

}  // namespace

void register_misc(cli::Command& root) {
  {
    auto c = std::make_unique<cli::Command>("install", "Installs the DevSpace.cli",
                                            "Adds the directory of the devspace binary to PATH in your shell profile");
    c->max_args = 0;
    c->run = run_install;
    root.add(std::move(c));
  }
  {
    auto c = std::make_unique<cli::Command>("upgrade", "Upgrade the DevSpace.cli to the newest version",
                                            "Upgrades the DevSpace.cli to the newest version");
    c->max_args = 0;
    c->str("from", "", "", "Path of a newer devspace binary to install");
    c->run = run_upgrade;
    root.add(std::move(c));
  }
  {
    auto c = std::make_unique<cli::Command>("upgrade-check", "Refreshes the cached newest-release check");
    c->hidden = true;
    c->max_args = 0;
    c->run = run_upgrade_check;
    root.add(std::move(c));
  }
  {
    auto c = std::make_unique<cli::Command>(
        "login", "Log into DevSpace.cloud",
        "If no --token is supplied the browser will be opened\nand the login page is shown\n\nExample:\ndevspace "
        "login\ndevspace login --token 123456789");
    c->max_args = 0;
    c->str("token", "", "", "Token to use for login")
        .str("provider", "", cloud::kDefaultProviderName, "Cloud provider to use");
    c->run = run_login;
    root.add(std::move(c));
  }
  {
    auto c = std::make_unique<cli::Command>("version", "Prints the devspace version");
    c->max_args = 0;
    c->run = [](cli::Command&, const Args&) {
      log::get().write(version_line() + "\n");
      return 0;
    };
    root.add(std::move(c));
  }
  {
    auto c = std::make_unique<cli::Command>("sync", "Starts a bi-directional sync with a container");
    c->hidden = true;
    c->max_args = 0;
    c->str("local", "", ".", "Local directory")
        .str("container", "", "/app", "Container path")
        .str("pod", "", "", "Pod name (default: newest running pod matching --label-selector)")
        .str("label-selector", "l", "", "Label selector")
        .str("namespace", "n", "", "Namespace")
        .str("container-name", "c", "", "Container name")
        .str("mode", "", "", "Sync protocol: compat | fast | helper")
        .slice("exclude", "e", "Exclude paths (gitignore syntax)")
        .boolean("verbose", "", false, "Log every change")
        .boolean("once", "", false, "Exit after the initial sync")
        .str("local-root", "", "", "Sync into a local directory that stands for the container's root (no cluster)")
        .integer("idle-timeout", "", 0, "Seconds without data after which a stream counts as dead (default 120)")
        .integer("fault-stdin-bytes", "", 0, "Test hook: kill the stream after this many bytes sent")
        .integer("fault-stdout-bytes", "", 0, "Test hook: kill the stream after this many bytes received")
        .integer("fault-shell", "", 1, "Test hook: which opened shell (1-based) gets the fault, 0 = all");
    c->run = run_sync;
    root.add(std::move(c));
  }
  {
    auto c = std::make_unique<cli::Command>("local-cluster", "Runs the bundled single-node cluster");
    c->hidden = true;
    c->max_args = 0;
    c->str("state", "", ".devspace-cluster", "State directory")
        .integer("port", "", 0, "API server port (0 = random)")
        .integer("gpus", "", 0, "amd.com/gpu capacity (default: detected)")
        .str("namespace", "", "", "Namespace for the kube context");
    c->run = run_local_cluster;
    root.add(std::move(c));
  }
}

}  // namespace cmd
}  // namespace ds

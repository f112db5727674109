// Core workflow commands: deploy, dev (+ deprecated `up`), enter, logs, analyze, purge
// (+ deprecated `down`), reset.
//
// Reference: cmd/deploy.go:71 (Run) + :166 (prepareConfig), cmd/dev.go:135-384 (Run,
// buildAndDeploy, startServices, GetPaths), cmd/enter.go:63, cmd/logs.go:58,
// cmd/analyze.go:48, cmd/purge.go:69-159, cmd/reset.go:58-269.
#include <unistd.h>

#include <chrono>
#include <thread>

#include "analyze/analyze.h"
#include "build/image.h"
#include "cli/common.h"
#include "cloud/cloud.h"
#include "core/fs.h"
#include "core/log.h"
#include "core/prompt.h"
#include "core/strutil.h"
#include "core/watch.h"
#include "deploy/deploy.h"
#include "services/services.h"

namespace ds {
namespace cmd {

namespace {

// Shared start-up for commands that operate on the project (root discovery, --config,
// file logging, cloud configuration).
void open_project(Session& s, const cli::Command& c, bool file_logging = true) {
  apply_config_flag(s.ctx, c);
  require_devspace_root();
  if (file_logging) log::start_file_logging();
}

std::string ns_of(Session& s) { return config::default_namespace(s.cfg()); }

// deploy.go:166 prepareConfig: flag overrides applied to the in-memory config.
void apply_deploy_flags(Session& s, const cli::Command& c) {
  Value& cfg = s.ctx.mutable_config();
  if (!c.get_str("namespace").empty()) {
    cfg["cluster"]["namespace"] = c.get_str("namespace");
    log::info("Using " + c.get_str("namespace") + " namespace for deploying");
  }
  if (!c.get_str("kube-context").empty()) {
    cfg["cluster"]["kubeContext"] = c.get_str("kube-context");
    log::info("Using " + c.get_str("kube-context") + " kube context for deploying");
  }
  if (!c.get_str("docker-target").empty() && cfg.get("images").is_map())
    for (auto& e : cfg["images"].entries()) e.second["build"]["options"]["target"] = c.get_str("docker-target");
}

void connect(Session& s, bool switch_context) {
  s.kube = make_kube(s.cfg(), switch_context);
  std::string ns = ns_of(s);
  try {
    s.kube->ensure_namespace(ns);
  } catch (const std::exception& e) {
    log::fatal(std::string("Unable to create namespace: ") + e.what());
  }
  try {
    s.kube->ensure_gcloud_cluster_role_binding();
  } catch (const std::exception& e) {
    log::fatal(std::string("Unable to ensure cluster-admin role binding: ") + e.what());
  }
}

void set_apply_flags(Session& s, const cli::Command& c) {
  kube::ApplyOptions ao;
  ao.recreate_on_immutable = c.get_bool("force-recreate");
  s.kube->set_apply_options(ao);
}

void print_space_domain(Session& s) {
  if (s.cfg().at_path("cluster.cloudProvider").is_null()) return;
  config::Generated& g = s.ctx.generated();
  if (g.has_space() && !g.space().get("domain").as_string().empty())
    log::info("The Space is now reachable via ingress on this URL: https://" + g.space().get("domain").as_string());
}

// Build + deploy pipeline shared by deploy and dev (dev.go:186 buildAndDeploy).
void pipeline(Session& s, bool is_dev, bool force_build, bool force_deploy, const std::string& docker_target) {
  config::Generated& gen = s.ctx.generated();
  build::BuildOptions bo;
  bo.is_dev = is_dev;
  bo.force_rebuild = force_build;
  bo.docker_target = docker_target;
  bo.interrupted = [] { return interrupted().load(); };
  // a kaniko build polls the flag and deletes its build pod when interrupted
  std::unique_ptr<GracefulInterrupt> kaniko_cleanup;
  for (auto& kv : s.cfg().get("images").entries())
    if (!kv.second.at_path("build.kaniko").is_null()) kaniko_cleanup.reset(new GracefulInterrupt());
  bool rebuilt = build::build_all(s.cfg(), gen, s.kube, bo);
  kaniko_cleanup.reset();
  if (rebuilt) s.ctx.save_generated();
  if (s.cfg().get("deployments").size() > 0 || !is_dev) {
    deploy::deploy_all(s.cfg(), gen, s.kube, is_dev, rebuilt || force_deploy);
    s.ctx.save_generated();
  }
}

int run_deploy(cli::Command& c, const std::vector<std::string>& args) {
  Session s;
  open_project(s, c);
  try {
    apply_deploy_flags(s, c);
    s.ctx.validate(s.cfg());
  } catch (const std::exception& e) {
    log::fatal(e.what());
  }
  cloud_configure(s.ctx, args.empty() ? "" : args[0]);
  connect(s, c.get_bool("switch-context"));
  set_apply_flags(s, c);
  try {
    build::init_registries(s.cfg(), s.kube, ns_of(s));
    pipeline(s, false, c.get_bool("force-build"), c.get_bool("force-deploy"), c.get_str("docker-target"));
  } catch (const std::exception& e) {
    log::fatal(e.what());
  }
  print_space_domain(s);
  log::done("Successfully deployed!");
  log::info("Run `devspace analyze` to check for potential issues");
  return 0;
}

// dev.go:331 GetPaths
std::vector<std::string> auto_reload_paths(const Value& cfg) {
  std::vector<std::string> paths;
  const Value& ar = cfg.at_path("dev.autoReload");
  if (!ar.is_map()) return paths;
  for (auto& dn : ar.get("deployments").items())
    for (auto& d : cfg.get("deployments").items()) {
      if (d.get("name").as_string() != dn.as_string()) continue;
      std::string chart = d.at_path("helm.chartPath").as_string();
      if (!chart.empty()) {
        if (chart.back() != '/') chart += "/";
        paths.push_back(chart + "**");
      } else {
        for (auto& m : d.at_path("kubectl.manifests").items()) paths.push_back(m.as_string());
      }
    }
  for (auto& in : ar.get("images").items()) {
    const Value* img = cfg.get("images").find(in.as_string());
    if (!img) continue;
    std::string df = img->at_path("build.dockerfilePath").as_string("./Dockerfile");
    paths.push_back(df);
  }
  for (auto& p : ar.get("paths").items()) paths.push_back(p.as_string());
  return paths;
}

services::SyncOptions dev_sync_options(bool verbose) {
  services::SyncOptions o;
  o.verbose = verbose;
  o.helper_path = helper_path();
  const char* env = getenv("DEVSPACE_SYNC_MODE");
  if (env && *env)
    o.mode = sync::parse_mode(env);
  else
    o.mode = fs::is_file(o.helper_path) ? sync::Mode::Helper : sync::Mode::Fast;
  return o;
}

int run_dev(cli::Command& c, const std::vector<std::string>& args) {
  GracefulInterrupt graceful;
  Session s;
  open_project(s, c);
  cloud_configure(s.ctx);
  connect(s, c.get_bool("switch-context"));
  set_apply_flags(s, c);
  if (c.get_bool("init-registries")) {
    try {
      build::init_registries(s.cfg(), s.kube, ns_of(s));
    } catch (const std::exception& e) {
      log::fatal(e.what());
    }
  }
  bool skip = c.get_bool("skip-pipeline");
  while (true) {
    {
      // the WebSocket upgrades the services below open: two sync shells per path, one
      // port-forward tunnel per forward, the attach or terminal stream, plus one for the pod
      // lookups they make at the same time. Dialed now, while the pipeline runs, they cost the
      // upgrade round trip only on a remote cluster.
      const Value& dev = s.cfg().get("dev");
      int n = (c.get_bool("sync") ? 2 * (int)dev.get("sync").size() : 0) +
              (c.get_bool("portforwarding") ? (int)dev.get("ports").size() : 0) + 2;
      s.kube->prewarm_upgrades(std::min(n, 8));
    }
    if (!skip) {
      try {
        pipeline(s, true, c.get_bool("force-build"), c.get_bool("force-deploy"), "");
      } catch (const std::exception& e) {
        log::fatal(std::string("Error deploying: ") + e.what());
      }
    }
    if (c.get_bool("exit-after-deploy")) return 0;

    // dev.go:249 startServices — port-forwarding and sync each look up their pods and open
    // their streams; on a real cluster that is a few API round trips apiece, so both start
    // concurrently instead of one after the other as in the reference.
    std::vector<std::unique_ptr<services::PortForwarder>> forwards;
    std::vector<std::unique_ptr<sync::Session>> syncs;
    std::string pf_err, sync_err;
    {
      bool want_pf = c.get_bool("portforwarding"), want_sync = c.get_bool("sync");
      auto opts = dev_sync_options(c.get_bool("verbose-sync"));
      std::thread pf_thread([&] {
        try {
          // the sync's helper in the container also carries forwarded connections on a remote
          // cluster (services::port_forward_via)
          if (want_pf)
            forwards = services::start_port_forwarding(s.cfg(), s.kube, 120000, 100,
                                                       want_sync && opts.mode == sync::Mode::Helper ? opts.helper_path
                                                                                                    : "");
        } catch (const std::exception& e) {
          pf_err = e.what();
        }
      });
      try {
        if (want_sync) syncs = services::start_sync(s.cfg(), s.kube, opts);
      } catch (const std::exception& e) {
        sync_err = e.what();
      }
      pf_thread.join();
    }
    if (!pf_err.empty()) log::fatal("Unable to start portforwarding: " + pf_err);
    if (!sync_err.empty()) log::fatal("Unable to start sync: " + sync_err);
    print_space_domain(s);

    std::atomic<bool> reload{false};
    std::unique_ptr<PollWatcher> watcher;
    std::vector<std::string> paths = auto_reload_paths(s.cfg());
    if (!skip && !paths.empty()) {
      auto once = std::make_shared<std::atomic<bool>>(false);
      watcher = std::make_unique<PollWatcher>(paths, [&reload, once](const std::vector<std::string>&,
                                                                     const std::vector<std::string>&) {
        if (once->exchange(true)) return;
        log::info("Change detected, will reload in 2 seconds");
        std::this_thread::sleep_for(std::chrono::seconds(2));
        reload = true;
      });
      watcher->start();
    }
    auto stop_now = [&] { return reload.load() || interrupted().load(); };
    int rc = 0;
    const Value& term = s.cfg().at_path("dev.terminal");
    bool terminal = c.get_bool("terminal") && !term.get("disabled").as_bool(false);
    try {
      if (terminal) {
        rc = services::start_terminal(s.cfg(), s.kube, c.get_str("selector"), c.get_str("container"),
                                      c.get_str("label-selector"), c.get_str("namespace"), false, args, stop_now);
      } else {
        log::done("Services started (Press Ctrl+C to abort port-forwarding and sync)");
        log::info("Will now try to print the logs of a running pod...");
        try {
          services::start_attach(s.cfg(), s.kube, c.get_str("selector"), c.get_str("container"),
                                 c.get_str("label-selector"), c.get_str("namespace"), stop_now, true);
        } catch (const std::exception& e) {
          log::info(std::string("Couldn't print logs of running pod: ") + e.what());
        }
        while (!stop_now()) std::this_thread::sleep_for(std::chrono::milliseconds(100));
      }
    } catch (const std::exception& e) {
      if (watcher) watcher->stop();
      log::fatal(e.what());
    }
    if (watcher) watcher->stop();
    for (auto& sy : syncs) sy->stop();
    for (auto& f : forwards) f->close();
    if (!reload) return rc;
    s.ctx.reset();  // re-read config (charts/manifests/Dockerfiles may have changed)
  }
}

int run_enter(cli::Command& c, const std::vector<std::string>& args) {
  GracefulInterrupt graceful;
  Session s;
  open_project(s, c);
  cloud_configure(s.ctx);
  s.kube = make_kube(s.cfg(), c.get_bool("switch-context"));
  try {
    return services::start_terminal(s.cfg(), s.kube, c.get_str("selector"), c.get_str("container"),
                                    c.get_str("label-selector"), c.get_str("namespace"), c.get_bool("pick"), args,
                                    [] { return interrupted().load(); });
  } catch (const std::exception& e) {
    log::fatal(e.what());
  }
}

int run_logs(cli::Command& c, const std::vector<std::string>&) {
  GracefulInterrupt graceful;
  Session s;
  apply_config_flag(s.ctx, c);
  if (!config::set_devspace_root()) log::fatal("Couldn't find any devspace configuration. Please run `devspace init`");
  log::start_file_logging();
  cloud_configure(s.ctx);
  s.kube = make_kube(s.cfg(), false);
  try {
    return services::start_logs(s.cfg(), s.kube, c.get_str("selector"), c.get_str("container"),
                                c.get_str("label-selector"), c.get_str("namespace"), c.get_bool("pick"),
                                c.get_bool("follow"), (int)c.get_int("lines"), [] { return interrupted().load(); });
  } catch (const std::exception& e) {
    log::fatal(e.what());
  }
}

int run_analyze(cli::Command& c, const std::vector<std::string>&) {
  Session s;
  bool exists = config::set_devspace_root();
  std::string ns;
  try {
    if (exists) {
      cloud_configure(s.ctx);
      s.kube = make_kube(s.cfg(), false);
      ns = ns_of(s);
    } else {
      s.kube = kube::Client::from_devspace_config(Value::map(), false);
      ns = s.kube->default_namespace();
    }
  } catch (const std::exception& e) {
    log::fatal(e.what());
  }
  if (!c.get_str("namespace").empty()) ns = c.get_str("namespace");
  analyze::Options o;
  o.wait = c.get_bool("wait");
  o.gpu_probe = c.get_bool("gpu-probe");
  try {
    std::string report = analyze::analyze(*s.kube, ns, o);
    if (report.empty()) {
      log::done("No problems found");
    } else {
      log::get().write(report);
    }
  } catch (const std::exception& e) {
    log::fatal(std::string("Error during analyze: ") + e.what());
  }
  return 0;
}

std::vector<std::string> split_list(const std::string& v) {
  std::vector<std::string> out;
  for (auto& p : split(v, ","))
    if (!trim(p).empty()) out.push_back(trim(p));
  return out;
}

int run_purge(cli::Command& c, const std::vector<std::string>&) {
  Session s;
  apply_config_flag(s.ctx, c);
  if (!config::set_devspace_root()) log::fatal("Couldn't find any devspace configuration. Please run `devspace init`");
  log::start_file_logging();
  cloud_configure(s.ctx);
  s.kube = make_kube(s.cfg(), false);
  deploy::purge(s.cfg(), s.kube, split_list(c.get_str("deployment")));
  return 0;
}

bool ask_yes(const std::string& q) {
  prompt::Params p;
  p.question = q;
  p.default_value = "yes";
  p.options = {"yes", "no"};
  return prompt::ask(p) == "yes";
}

int run_reset(cli::Command& c, const std::vector<std::string>&) {
  Session s;
  open_project(s, c, false);
  cloud_configure(s.ctx);
  try {
    s.kube = kube::Client::from_devspace_config(s.cfg(), false);
  } catch (const std::exception& e) {
    log::fail(std::string("Failed to initialize kubectl client: ") + e.what());
  }
  const Value& cfg = s.cfg();
  if (!cfg.at_path("cluster.cloudProvider").is_null() && !cfg.at_path("cluster.namespace").as_string().empty()) {
    // reset.go:107 deleteCloudSpace
    if (ask_yes("Should the Space be deleted from DevSpace.cloud?")) {
      auto providers = cloud::load_providers();
      auto it = providers.find(cfg.at_path("cluster.cloudProvider").as_string());
      config::Generated& g = s.ctx.generated();
      if (it != providers.end()) {
        if (!g.has_space()) {
          log::info("Didn't remove Space since there is no Space configured");
        } else {
          try {
            cloud::Client(it->second).delete_space(g.space().get("spaceID").as_int());
            log::done("Successfully deleted Space " + cfg.at_path("cluster.namespace").as_string());
          } catch (const std::exception& e) {
            log::fail(std::string("Error deleting Space: ") + e.what());
          }
        }
      }
    }
  } else if (s.kube) {
    deploy::purge(cfg, s.kube, {});
    // reset.go:220 deleteClusterRoleBinding
    const std::string crb = "/apis/rbac.authorization.k8s.io/v1/clusterrolebindings/devspace-user";
    try {
      if (s.kube->try_get(crb) && ask_yes("\n\nShould the ClusterRoleBinding 'devspace-user' be removed?")) {
        s.kube->del(crb);
        log::done("Successfully deleted ClusterRoleBinding 'devspace-user'");
      }
    } catch (const std::exception& e) {
      log::fail(std::string("Failed to remove ClusterRoleBinding: ") + e.what());
    }
  }
  // reset.go:151 deleteDeploymentFiles
  for (auto& d : cfg.get("deployments").items()) {
    std::string chart = d.at_path("helm.chartPath").as_string();
    if (chart.empty() || !fs::exists(chart)) continue;
    if (ask_yes("Should the Chart (" + chart + "/*) be removed?")) {
      fs::remove_all(fs::abs_path(chart));
      log::done("Successfully deleted " + chart);
    }
  }
  // reset.go:177 deleteImageFiles
  for (auto& e : cfg.get("images").entries()) {
    std::string df = e.second.at_path("build.dockerfilePath").as_string("Dockerfile");
    if (fs::exists(df) && ask_yes("Should " + df + " be removed?")) {
      fs::remove(fs::abs_path(df));
      log::done("Successfully deleted " + fs::abs_path(df));
    }
    std::string ctxp = e.second.at_path("build.contextPath").as_string(".");
    std::string di = fs::join(fs::abs_path(ctxp), ".dockerignore");
    if (fs::exists(di) && ask_yes("\n\nShould " + di + " be removed?")) {
      fs::remove(di);
      log::done("Successfully deleted " + di);
    }
  }
  if (ask_yes("\n\nShould the .devspace folder be removed?")) {
    fs::remove_all(".devspace");
    log::done("Successfully deleted .devspace folder");
  }
  return 0;
}

std::unique_ptr<cli::Command> banner_cmd(const std::string& use, const std::string& short_desc,
                                         const std::string& body) {
  std::string title = "devspace " + use;
  std::string bar(55, '#');
  size_t pad = (55 - title.size() - 2) / 2;
  std::string mid = std::string(pad, '#') + " " + title + " " + std::string(55 - pad - title.size() - 2, '#');
  return std::make_unique<cli::Command>(use, short_desc, "\n" + bar + "\n" + mid + "\n" + bar + "\n" + body + "\n" + bar);
}

}  // namespace

void register_core(cli::Command& root) {
  const std::string cfg_usage = "The DevSpace config file to load (default: '.devspace/config.yaml'";
  {
    auto c = banner_cmd("deploy", "Deploy the project",
                        "Deploys the current project to a Space or namespace:\n\ndevspace deploy --namespace=deploy\n"
                        "devspace deploy --kube-context=deploy-context");
    c->max_args = 1;
    c->str("namespace", "", "", "The namespace to deploy to")
        .str("kube-context", "", "", "The kubernetes context to use for deployment")
        .str("config", "", config::kDefaultConfigPath, cfg_usage)
        .str("docker-target", "", "", "The docker target to use for building")
        .boolean("switch-context", "", false, "Switches the kube context to the deploy context")
        .boolean("force-build", "b", false, "Forces to (re-)build every image")
        .boolean("force-deploy", "d", false, "Forces to (re-)deploy every deployment")
        .boolean("force-recreate", "", false,
                 "Delete and re-create objects whose immutable fields changed (never PVCs, PVs or namespaces)");
    c->run = run_deploy;
    root.add(std::move(c));
  }
  auto dev_flags = [&](cli::Command& c) {
    c.boolean("init-registries", "", true, "Initialize registries (and install internal one)")
        .boolean("force-build", "b", false, "Forces to build every image")
        .boolean("force-deploy", "d", false, "Forces to deploy every deployment")
        .boolean("force-recreate", "", false,
                 "Delete and re-create objects whose immutable fields changed (never PVCs, PVs or namespaces)")
        .boolean("skip-pipeline", "x", false, "Skips build & deployment and only starts sync, portforwarding & terminal")
        .boolean("sync", "", true, "Enable code synchronization")
        .boolean("verbose-sync", "", false, "When enabled the sync will log every file change")
        .boolean("portforwarding", "", true, "Enable port forwarding")
        .boolean("terminal", "", true, "Enable terminal (true or false)")
        .str("selector", "s", "", "Selector name (in config) to select pods/container for terminal")
        .str("container", "c", "", "Container name where to open the shell")
        .str("label-selector", "l", "",
             "Comma separated key=value selector list to use for terminal (e.g. release=test)")
        .str("namespace", "n", "", "Namespace where to select pods for terminal")
        .boolean("switch-context", "", false, "Switch kubectl context to the DevSpace context")
        .boolean("exit-after-deploy", "", false,
                 "Exits the command after building the images and deploying the project")
        .str("config", "", config::kDefaultConfigPath, cfg_usage);
  };
  {
    auto c = banner_cmd("dev", "Starts the development mode",
                        "Starts your project in development mode:\n1. Builds your Docker images and override "
                        "entrypoints if specified\n2. Deploys the deployments via helm or kubectl\n3. Forwards "
                        "container ports to the local computer\n4. Starts the sync client\n5. Enters the container "
                        "shell");
    dev_flags(*c);
    c->run = run_dev;
    root.add(std::move(c));
    auto up = std::make_unique<cli::Command>("up", "alias for `devspace dev` (deprecated)");
    dev_flags(*up);
    up->run = [](cli::Command& cc, const std::vector<std::string>& a) {
      log::warn("`devspace up` is deprecated, please use `devspace dev` in future");
      return run_dev(cc, a);
    };
    root.add(std::move(up));
  }
  {
    auto c = banner_cmd("enter", "Open a shell to a container",
                        "Execute a command or start a new terminal in your\ndevspace:\n\ndevspace enter\ndevspace enter "
                        "-p # Select pod to enter\ndevspace enter bash\ndevspace enter -s my-selector\ndevspace enter "
                        "-c my-container\ndevspace enter bash -n my-namespace\ndevspace enter bash -l release=test");
    c->str("selector", "s", "", "Selector name (in config) to select pod/container for terminal")
        .str("container", "c", "", "Container name within pod where to execute command")
        .str("label-selector", "l", "", "Comma separated key=value selector list (e.g. release=test)")
        .str("namespace", "n", "", "Namespace where to select pods")
        .boolean("switch-context", "", false, "Switch kubectl context to the DevSpace context")
        .boolean("pick", "p", false, "Select a pod to stream logs from")
        .str("config", "", config::kDefaultConfigPath, cfg_usage);
    c->run = run_enter;
    root.add(std::move(c));
  }
  {
    auto c = banner_cmd("logs", "Prints the logs of a pod and attaches to it",
                        "Logs prints the last log of a pod container and attachs\nto it\n\nExample:\ndevspace "
                        "logs\ndevspace logs --namespace=mynamespace");
    c->max_args = 0;
    c->str("selector", "s", "", "Selector name (in config) to select pod/container for terminal")
        .str("container", "c", "", "Container name within pod where to execute command")
        .str("label-selector", "l", "", "Comma separated key=value selector list (e.g. release=test)")
        .str("namespace", "n", "", "Namespace where to select pods")
        .boolean("pick", "p", false, "Select a pod to stream logs from")
        .boolean("follow", "f", false, "Attach to logs afterwards")
        .integer("lines", "", 200, "Max amount of lines to print from the last log")
        .str("config", "", config::kDefaultConfigPath, cfg_usage);
    c->run = run_logs;
    root.add(std::move(c));
  }
  {
    auto c = banner_cmd("analyze", "Analyzes a kubernetes namespace and checks for potential problems",
                        "Analyze checks a namespaces events, replicasets, services\nand pods for potential problems "
                        "(including AMD GPU scheduling\nand ROCm runtime failures)\n\nExample:\ndevspace "
                        "analyze\ndevspace analyze --namespace=mynamespace");
    c->max_args = 0;
    c->str("namespace", "n", "", "The kubernetes namespace to analyze")
        .boolean("wait", "", true, "Wait for pods to get ready if they are just starting")
        .boolean("gpu-probe", "", false, "Run the GPU probe inside pods that request amd.com/gpu");
    c->run = run_analyze;
    root.add(std::move(c));
  }
  auto purge_flags = [&](cli::Command& c) {
    c.max_args = 0;
    c.str("deployment", "d", "",
          "The deployment to delete (You can specify multiple deployments comma-separated, e.g. "
          "devspace-default,devspace-database etc.)")
        .str("config", "", config::kDefaultConfigPath, cfg_usage);
  };
  {
    auto c = banner_cmd("purge", "Delete all deployed kubernetes resources",
                        "Deletes the deployed kuberenetes resources.\nWarning: will delete everything that is defined "
                        "in the\nlocal chart, including persistent volume claims!");
    purge_flags(*c);
    c->run = run_purge;
    root.add(std::move(c));
    auto down = std::make_unique<cli::Command>("down", "alias for devspace purge (deprecated)");
    purge_flags(*down);
    down->run = [](cli::Command& cc, const std::vector<std::string>& a) {
      log::warn("`devspace down` is deprecated, please use `devspace purge` in future");
      return run_purge(cc, a);
    };
    root.add(std::move(down));
  }
  {
    auto c = banner_cmd("reset", "Remove DevSpace completely from your project",
                        "Resets your project by removing all DevSpace related\ndata from your project and your "
                        "cluster, including:\n1. DevSpace deployments\n2. DevSpace config files in .devspace/ "
                        "(local)\n\nIf you simply want to shutdown your DevSpace, use the\ncommand: devspace purge");
    c->max_args = 0;
    c->str("config", "", config::kDefaultConfigPath, cfg_usage);
    c->run = run_reset;
    root.add(std::move(c));
  }
}

}  // namespace cmd
}  // namespace ds

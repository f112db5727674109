// Config management commands: add / remove / list / status / use / update / create.
//
// Reference: cmd/add/*.go, cmd/remove/*.go, cmd/list/*.go, cmd/status/{deployments,sync}.go,
// cmd/use/{config,context,registry,space}.go, cmd/update/config.go, cmd/create/space.go.
#include <ctime>
#include <regex>

#include "cli/common.h"
#include "cloud/cloud.h"
#include "configure/configure.h"
#include "core/codec.h"
#include "core/fs.h"
#include "core/log.h"
#include "core/prompt.h"
#include "core/safe_regex.h"
#include "core/strutil.h"
#include "deploy/deploy.h"
#include "deploy/helmrepo.h"
#include "kube/kubeconfig.h"
#include "build/docker.h"

namespace ds {
namespace cmd {

namespace {

using Args = std::vector<std::string>;

void need_root() { require_devspace_root(); }

config::Context& ctx_for(cli::Command& c) {
  static config::Context ctx;
  ctx.reset();
  apply_config_flag(ctx, c);
  return ctx;
}

template <typename F>
int guarded(F f) {
  try {
    f();
  } catch (const std::exception& e) {
    log::fatal(e.what());
  }
  return 0;
}

std::string labels_str(const Value& m) {
  std::vector<std::string> parts;
  for (auto& e : m.entries()) parts.push_back(e.first + "=" + e.second.as_string());
  return join(parts, ", ");
}

// cloud.GetCurrentProvider: provider of the project config, else the default one.
cloud::Provider current_provider() {
  std::string name = cloud::kDefaultProviderName;
  if (config::set_devspace_root()) {
    try {
      config::Context ctx;
      std::string p = ctx.base().at_path("cluster.cloudProvider").as_string();
      if (!p.empty()) name = p;
    } catch (...) {
    }
  }
  return cloud::ensure_logged_in(name);
}

std::unique_ptr<cli::Command> group(const std::string& use, const std::string& short_desc) {
  auto g = std::make_unique<cli::Command>(use, short_desc);
  g->max_args = 0;
  g->run = [](cli::Command& c, const Args&) {
    log::get().write(c.help());
    return 0;
  };
  return g;
}

std::unique_ptr<cli::Command> leaf(const std::string& use, const std::string& short_desc, int min_args, int max_args,
                                   cli::RunFn fn) {
  auto c = std::make_unique<cli::Command>(use, short_desc);
  c->min_args = min_args;
  c->max_args = max_args;
  c->run = std::move(fn);
  return c;
}

// ---------------------------------------------------------------- add

std::unique_ptr<cli::Command> make_add() {
  auto add = group("add", "Change the DevSpace configuration");
  {
    auto c = leaf("deployment", "Add a deployment", 1, 1, [](cli::Command& c, const Args& a) {
      need_root();
      return guarded([&] {
        config::Context& ctx = ctx_for(c);
        configure::add_deployment(ctx, a[0], c.get_str("namespace"), c.get_str("manifests"), c.get_str("chart"));
        log::donef("Successfully added %s as new deployment", a[0].c_str());
      });
    });
    c->str("namespace", "", "", "The namespace to use for deploying")
        .str("manifests", "", "", "The kubernetes manifests to deploy (glob pattern are allowed, comma separated)")
        .str("chart", "", "", "The helm chart to deploy");
    add->add(std::move(c));
  }
  {
    auto c = leaf("image", "Add an image", 1, 1, [](cli::Command& c, const Args& a) {
      need_root();
      return guarded([&] {
        configure::add_image(ctx_for(c), a[0], c.get_str("image"), c.get_str("tag"), c.get_str("context"),
                             c.get_str("dockerfile"), c.get_str("buildengine"));
        log::donef("Successfully added image %s", a[0].c_str());
      });
    });
    c->str("image", "", "", "The image name of the image (e.g. myusername/devspace)")
        .str("tag", "", "", "The tag of the image")
        .str("context", "", "", "The path of the images' context")
        .str("dockerfile", "", "", "The path of the images' dockerfile")
        .str("buildengine", "", "", "Specify which engine should build the file. Should match this regex: docker|kaniko")
        .required("image");
    add->add(std::move(c));
  }
  {
    auto c = leaf("package", "Add a helm chart", 0, 1, [](cli::Command& c, const Args& a) {
      need_root();
      return guarded([&] {
        config::Context& ctx = ctx_for(c);
        if (a.empty()) {
          helmrepo::update();
          std::vector<std::vector<std::string>> rows;
          std::string last;
          for (auto& cv : helmrepo::all_charts()) {
            if (cv.name == last) continue;
            last = cv.name;
            rows.push_back({cv.name, cv.version, cv.app_version, cv.description});
          }
          log::get().print_table({"NAME", "CHART VERSION", "APP VERSION", "DESCRIPTION"}, rows);
          return;
        }
        configure::add_package(ctx, a[0], c.get_str("chart-version"), c.get_str("app-version"),
                               c.get_str("deployment"), c.get_bool("skip-question"));
      });
    });
    c->str("app-version", "", "", "App version")
        .str("chart-version", "", "", "Chart version")
        .str("deployment", "d", "", "The deployment name to use")
        .boolean("skip-question", "", false, "Skips the question to show the readme in a browser");
    add->add(std::move(c));
  }
  {
    auto c = leaf("port", "Add a new port forward configuration", 1, 1, [](cli::Command& c, const Args& a) {
      need_root();
      return guarded([&] {
        configure::add_port(ctx_for(c), c.get_str("namespace"), c.get_str("label-selector"), c.get_str("selector"),
                            a[0]);
        log::donef("Successfully added port %s", a[0].c_str());
      });
    });
    c->str("namespace", "", "", "Namespace to use")
        .str("label-selector", "", "", "Comma separated key=value label-selector list (e.g. release=test)")
        .str("selector", "", "", "Name of a selector defined in your DevSpace config");
    add->add(std::move(c));
  }
  {
    auto c = leaf("provider", "Adds a new cloud provider to the configuration", 1, 1, [](cli::Command& c, const Args& a) {
      return guarded([&] {
        std::string name = c.get_str("name").empty() ? a[0] : c.get_str("name");
        auto ps = cloud::load_providers();
        if (ps.count(name)) throw std::runtime_error("Provider " + name + " does already exist");
        cloud::Provider p;
        p.name = name;
        p.host = a[0];
        if (!starts_with(p.host, "http://") && !starts_with(p.host, "https://")) p.host = "https://" + p.host;
        ps[name] = p;
        cloud::save_providers(ps);
        log::donef("Successfully added cloud provider %s", name.c_str());
      });
    });
    c->str("name", "", "", "Cloud provider name to use");
    add->add(std::move(c));
  }
  {
    auto c = leaf("selector", "Add a selector", 1, 1, [](cli::Command& c, const Args& a) {
      need_root();
      return guarded([&] {
        configure::add_selector(ctx_for(c), a[0], c.get_str("label-selector"), c.get_str("namespace"));
        log::donef("Successfully added new service %s", a[0].c_str());
      });
    });
    c->str("namespace", "", "", "The namespace of the selector")
        .str("label-selector", "", "", "The label-selector of the selector");
    add->add(std::move(c));
  }
  {
    auto c = leaf("sync", "Add a sync path", 0, 0, [](cli::Command& c, const Args&) {
      need_root();
      return guarded([&] {
        configure::add_sync(ctx_for(c), c.get_str("local"), c.get_str("container"), c.get_str("namespace"),
                            c.get_str("label-selector"), c.get_str("exclude"), c.get_str("selector"));
        log::donef("Successfully added sync between local path %s and container path %s", c.get_str("local").c_str(),
                   c.get_str("container").c_str());
      });
    });
    c->str("label-selector", "", "", "Comma separated key=value selector list (e.g. release=test)")
        .str("local", "", "", "Relative local path")
        .str("namespace", "", "", "Namespace to use")
        .str("container", "", "", "Absolute container path")
        .str("exclude", "", "", "Comma separated list of paths to exclude (e.g. node_modules/,bin,*.exe)")
        .str("selector", "", "", "Name of a selector defined in your DevSpace config")
        .required("local")
        .required("container");
    add->add(std::move(c));
  }
  return add;
}

// ---------------------------------------------------------------- remove

void delete_space_contexts(const std::vector<cloud::Space>& spaces) {
  for (auto& s : spaces) cloud::delete_kube_context(s);
}

std::unique_ptr<cli::Command> make_remove() {
  auto rm = group("remove", "Changes devspace configuration");
  {
    auto c = leaf("context", "Removes a cloud space kubectl context", 0, 1, [](cli::Command& c, const Args& a) {
      return guarded([&] {
        cloud::Provider p = current_provider();
        cloud::Client cl(p);
        if (c.get_bool("all")) {
          auto spaces = cl.spaces();
          delete_space_contexts(spaces);
          log::donef("Deleted all kubectl contexts for spaces");
          return;
        }
        cloud::Space s;
        if (a.empty()) {
          config::Context ctx;
          if (!config::set_devspace_root() || !ctx.generated().has_space())
            throw std::runtime_error("Please provide a space name or id for this command");
          s = cloud::Space::from_generated(ctx.generated().space());
        } else {
          s = cl.space_by_name(a[0]);
        }
        cloud::delete_kube_context(s);
        log::donef("Successfully deleted kubectl context for space %s", s.name.c_str());
      });
    });
    c->boolean("all", "", false, "Delete all kubectl contexts created from spaces");
    rm->add(std::move(c));
  }
  {
    auto c = leaf("deployment", "Removes one or all deployments from the devspace", 0, 1,
                  [](cli::Command& c, const Args& a) {
                    need_root();
                    return guarded([&] {
                      std::string name = a.empty() ? "" : a[0];
                      configure::remove_deployment(ctx_for(c), c.get_bool("all"), name);
                      if (c.get_bool("all"))
                        log::done("Successfully removed all deployments");
                      else
                        log::donef("Successfully removed deployment %s", name.c_str());
                    });
                  });
    c->boolean("all", "", false, "Remove all deployments");
    rm->add(std::move(c));
  }
  {
    auto c = leaf("image", "Removes one or all images from the devspace", 0, 1, [](cli::Command& c, const Args& a) {
      need_root();
      return guarded([&] {
        configure::remove_image(ctx_for(c), c.get_bool("all"), a);
        log::done("Successfully removed image");
      });
    });
    c->boolean("all", "", false, "Remove all images");
    rm->add(std::move(c));
  }
  {
    auto c = leaf("package", "Removes one or all packages from a devspace", 0, 1, [](cli::Command& c, const Args& a) {
      need_root();
      return guarded([&] {
        configure::remove_package(ctx_for(c), c.get_bool("all"), c.get_str("deployment"), a.empty() ? "" : a[0]);
      });
    });
    c->boolean("all", "", false, "Remove all packages").str("deployment", "d", "", "The deployment name to use");
    rm->add(std::move(c));
  }
  {
    auto c = leaf("port", "Removes forwarded ports from a devspace", 0, 1, [](cli::Command& c, const Args& a) {
      need_root();
      return guarded([&] {
        configure::remove_port(ctx_for(c), c.get_bool("all"), c.get_str("label-selector"), a.empty() ? "" : a[0]);
        log::done("Successfully removed port");
      });
    });
    c->str("label-selector", "", "", "Comma separated key=value selector list (e.g. release=test)")
        .boolean("all", "", false, "Remove all configured ports");
    rm->add(std::move(c));
  }
  {
    auto c = leaf("provider", "Removes a cloud provider from the configuration", 1, 1,
                  [](cli::Command& c, const Args& a) {
                    return guarded([&] {
                      std::string name = c.get_str("name").empty() ? a[0] : c.get_str("name");
                      auto ps = cloud::load_providers();
                      if (!ps.count(name)) throw std::runtime_error("Couldn't find cloud provider " + name);
                      ps.erase(name);
                      cloud::save_providers(ps);
                      log::donef("Successfully removed cloud provider %s", name.c_str());
                    });
                  });
    c->str("name", "", "", "Cloud provider name to use");
    rm->add(std::move(c));
  }
  {
    auto c = leaf("selector", "Removes one or all selectors from the devspace", 0, 1,
                  [](cli::Command& c, const Args& a) {
                    need_root();
                    return guarded([&] {
                      configure::remove_selector(ctx_for(c), c.get_bool("all"), a.empty() ? "" : a[0],
                                                 c.get_str("label-selector"), c.get_str("namespace"));
                      log::done("Successfully removed selector");
                    });
                  });
    c->boolean("all", "", false, "Remove all selectors")
        .str("namespace", "", "", "Namespace of the selector")
        .str("label-selector", "", "", "Label-selector of the selector");
    rm->add(std::move(c));
  }
  {
    auto c = leaf("space", "Removes a cloud space", 0, 1, [](cli::Command& c, const Args& a) {
      return guarded([&] {
        cloud::Provider p = c.get_str("provider").empty() ? current_provider()
                                                          : cloud::ensure_logged_in(c.get_str("provider"));
        cloud::Client cl(p);
        std::vector<cloud::Space> targets;
        if (c.get_bool("all")) {
          targets = cl.spaces();
        } else if (!c.get_str("id").empty()) {
          int64_t id;
          if (!parse_int64(c.get_str("id"), &id)) throw std::runtime_error("invalid space id " + c.get_str("id"));
          targets.push_back(cl.space(id));
        } else if (!a.empty()) {
          targets.push_back(cl.space_by_name(a[0]));
        } else {
          throw std::runtime_error("Please provide a space name or id for this command");
        }
        for (auto& s : targets) {
          cl.delete_space(s.id);
          cloud::delete_kube_context(s);
          if (config::set_devspace_root()) {
            config::Context ctx;
            if (ctx.generated().has_space() && ctx.generated().space().get("spaceID").as_int() == s.id) {
              ctx.generated().clear_space();
              ctx.save_generated();
            }
          }
          log::donef("Deleted space %s", s.name.c_str());
        }
      });
    });
    c->str("id", "", "", "SpaceID id to use")
        .str("provider", "", "", "Provider to use")
        .boolean("all", "", false, "Delete all spaces");
    rm->add(std::move(c));
  }
  {
    auto c = leaf("sync", "Remove sync paths from the devspace", 0, 0, [](cli::Command& c, const Args&) {
      need_root();
      return guarded([&] {
        configure::remove_sync(ctx_for(c), c.get_bool("all"), c.get_str("local"), c.get_str("container"),
                               c.get_str("label-selector"));
        log::done("Successfully removed sync");
      });
    });
    c->str("label-selector", "", "", "Comma separated key=value selector list (e.g. release=test)")
        .str("local", "", "", "Relative local path to remove")
        .str("container", "", "", "Absolute container path to remove")
        .boolean("all", "", false, "Remove all configured sync paths");
    rm->add(std::move(c));
  }
  return rm;
}

// ---------------------------------------------------------------- list

std::unique_ptr<cli::Command> make_list() {
  auto ls = group("list", "Lists configuration");
  ls->add(leaf("configs", "Lists all DevSpace configurations", 0, 0, [](cli::Command&, const Args&) {
    need_root();
    return guarded([&] {
      if (!fs::exists(config::kDefaultConfigsPath)) {
        log::info(std::string("Please create a '") + config::kDefaultConfigsPath +
                  "' to define multiple configurations");
        return;
      }
      Value configs = yaml_load_file(config::kDefaultConfigsPath);
      config::Context ctx;
      std::string active = ctx.generated().active_config();
      std::vector<std::vector<std::string>> rows;
      for (auto& e : configs.entries()) {
        std::string path = e.second.at_path("config.path").as_string(e.second.get("config").has("data") ? "data" : "");
        std::string vars = e.second.get("vars").is_null() ? "false" : "true";
        std::string ov = std::to_string(e.second.get("overrides").size());
        rows.push_back({e.first, e.first == active ? "true" : "false", path, vars, ov});
      }
      log::get().print_table({"Name", "Active", "Path", "Vars", "Overwrites"}, rows);
    });
  }));
  ls->add(leaf("packages", "Lists all added packages", 0, 0, [](cli::Command&, const Args&) {
    need_root();
    return guarded([&] {
      config::Context ctx;
      std::vector<std::vector<std::string>> rows;
      for (auto& d : ctx.get().get("deployments").items()) {
        std::string chart = d.at_path("helm.chartPath").as_string();
        if (chart.empty()) continue;
        std::string req = fs::join(chart, "requirements.yaml");
        if (!fs::exists(req)) continue;
        Value reqs = yaml_load_file(req);
        for (auto& dep : reqs.get("dependencies").items())
          rows.push_back({dep.get("name").as_string(), dep.get("version").as_string(),
                          dep.get("repository").as_string()});
      }
      if (rows.empty()) {
        log::info("No packages found");
        return;
      }
      log::get().print_table({"Name", "Version", "Repository"}, rows);
    });
  }));
  ls->add(leaf("ports", "Lists port forwarding configurations", 0, 0, [](cli::Command&, const Args&) {
    need_root();
    return guarded([&] {
      config::Context ctx;
      const Value& ports = ctx.get().at_path("dev.ports");
      if (ports.size() == 0) {
        log::info("No ports are forwarded. Run `devspace add port` to add a port that should be forwarded");
        return;
      }
      std::vector<std::vector<std::string>> rows;
      for (auto& p : ports.items()) {
        std::vector<std::string> pm;
        for (auto& m : p.get("portMappings").items())
          pm.push_back(std::to_string(m.get("localPort").as_int()) + ":" + std::to_string(m.get("remotePort").as_int()));
        rows.push_back({p.get("selector").as_string(), labels_str(p.get("labelSelector")), join(pm, ", ")});
      }
      log::get().print_table({"Selector", "LabelSelector", "Ports (Local:Remote)"}, rows);
    });
  }));
  ls->add(leaf("selectors", "Lists all selectors", 0, 0, [](cli::Command&, const Args&) {
    need_root();
    return guarded([&] {
      config::Context ctx;
      const Value& sels = ctx.get().at_path("dev.selectors");
      if (sels.size() == 0) {
        log::info("No selectors are configured. Run `devspace add selector` to add new selector");
        return;
      }
      std::vector<std::vector<std::string>> rows;
      for (auto& s : sels.items())
        rows.push_back({s.get("name").as_string(), s.get("namespace").as_string(), labels_str(s.get("labelSelector")),
                        s.get("containerName").as_string()});
      log::get().print_table({"Name", "Namespace", "Label Selector", "Container"}, rows);
    });
  }));
  {
    auto c = leaf("spaces", "Lists all user spaces", 0, 0, [](cli::Command& c, const Args&) {
      return guarded([&] {
        cloud::Client cl(current_provider());
        std::vector<std::vector<std::string>> rows;
        for (auto& s : cl.spaces()) {
          if (!c.get_str("name").empty() && s.name != c.get_str("name")) continue;
          rows.push_back({std::to_string(s.id), s.name, s.namespace_, s.domain, s.created});
        }
        if (rows.empty()) {
          log::info("No spaces found. You can create a space with `devspace create space [NAME]`");
          return;
        }
        log::get().print_table({"SpaceID", "Name", "Namespace", "Domain", "Created"}, rows);
      });
    });
    c->str("name", "", "", "Space name to show (default: all)");
    ls->add(std::move(c));
  }
  ls->add(leaf("sync", "Lists sync configuration", 0, 0, [](cli::Command&, const Args&) {
    need_root();
    return guarded([&] {
      config::Context ctx;
      const Value& sync = ctx.get().at_path("dev.sync");
      if (sync.size() == 0) {
        log::info("No sync paths are configured. Run `devspace add sync` to add new sync path");
        return;
      }
      std::vector<std::vector<std::string>> rows;
      for (auto& s : sync.items()) {
        std::vector<std::string> ex;
        for (auto& e : s.get("excludePaths").items()) ex.push_back(e.as_string());
        rows.push_back({s.get("selector").as_string(), labels_str(s.get("labelSelector")),
                        s.get("localSubPath").as_string(), s.get("containerPath").as_string(), join(ex, ", ")});
      }
      log::get().print_table({"Selector", "Label Selector", "Local Path", "Container Path", "Excluded Paths"}, rows);
    });
  }));
  ls->add(leaf("vars", "Lists the vars in the active config", 0, 0, [](cli::Command&, const Args&) {
    need_root();
    return guarded([&] {
      config::Context ctx;
      ctx.get();  // asks missing vars
      Value& vars = ctx.generated().vars();
      if (vars.size() == 0) {
        log::info("No vars found");
        return;
      }
      std::vector<std::vector<std::string>> rows;
      for (auto& e : vars.entries()) rows.push_back({e.first, e.second.is_scalar() ? e.second.as_string() : json_dump(e.second)});
      log::get().print_table({"Variable", "Value"}, rows);
    });
  }));
  return ls;
}

// ---------------------------------------------------------------- status

std::string ago(int64_t secs) {
  if (secs >= 86400) return std::to_string(secs / 86400) + "d";
  if (secs >= 3600) return std::to_string(secs / 3600) + "h";
  if (secs >= 60) return std::to_string(secs / 60) + "m";
  return std::to_string(secs > 0 ? secs : 0) + "s";
}

int64_t parse_rfc3339(const std::string& s) {
  struct tm tm{};
  if (!strptime(s.c_str(), "%Y-%m-%dT%H:%M:%S", &tm)) return 0;
  return timegm(&tm);
}

std::unique_ptr<cli::Command> make_status() {
  auto st = group("status", "Show the current status");
  st->add(leaf("deployments", "Shows the status of all deployments", 0, 0, [](cli::Command&, const Args&) {
    need_root();
    return guarded([&] {
      Session s;
      cloud_configure(s.ctx);
      s.kube = make_kube(s.cfg(), false);
      std::vector<std::vector<std::string>> rows;
      for (auto& d : s.cfg().get("deployments").items()) {
        auto dep = deploy::make_deployer(s.cfg(), d, s.kube);
        for (auto& r : dep->status()) rows.push_back(r);
      }
      log::get().print_table({"TYPE", "STATUS", "NAMESPACE", "INFO"}, rows);
    });
  }));
  st->add(leaf("sync", "Shows the sync status", 0, 0, [](cli::Command&, const Args&) {
    need_root();
    return guarded([&] {
      std::string path = fs::join(fs::cwd(), ".devspace", "logs", "sync.log");
      std::string data;
      if (!fs::read_file(path, &data))
        throw std::runtime_error("Couldn't read " + path +
                                 ". Do you have a sync path configured? (check `devspace list sync`)");
      struct Status {
        std::string pod, local, container, status, error, last, last_time;
        int64_t total = 0;
      };
      std::vector<std::string> order;
      std::map<std::string, Status> m;
      static const std::regex down("^\\[Downstream\\] Successfully processed (\\d+) change\\(s\\)$");
      static const std::regex up("^\\[Upstream\\] Successfully processed (\\d+) change\\(s\\)$");
      static const std::regex stopped("^\\[Sync\\] Sync stopped$");
      for (auto& line : split(data, "\n")) {
        if (trim(line).empty()) continue;
        Value j = json_parse(line);
        std::string pod = j.get("pod").as_string(), local = j.get("local").as_string(),
                    container = j.get("container").as_string(), msg = j.get("msg").as_string(),
                    level = j.get("level").as_string(), time = j.get("time").as_string();
        if (container.empty() || local.empty() || pod.empty() || level.empty() || time.empty() || msg.empty())
          throw std::runtime_error("Error parsing " + path + ": Json object is invalid " + line);
        std::string id = pod + ":" + local + ":" + container;
        if (!m.count(id)) {
          order.push_back(id);
          m[id] = Status{pod, local, container};
        }
        Status& s = m[id];
        std::smatch sm;
        if (level == "error") {
          s.status = "Error";
          s.error = msg;
          s.last_time = time;
        } else if (safe_regex_match(msg, &sm, down)) {
          s.last = "Downloaded " + sm[1].str() + " changes";
          s.last_time = time;
          s.total += std::stoll(sm[1].str());
        } else if (safe_regex_match(msg, &sm, up)) {
          s.last = "Uploaded " + sm[1].str() + " changes";
          s.last_time = time;
          s.total += std::stoll(sm[1].str());
        } else if (safe_regex_match(msg, stopped)) {
          s.status = "Stopped";
          s.last = "Sync stopped";
          s.last_time = time;
        }
      }
      if (m.empty()) {
        log::info("No sync activity found. Did you run `devspace dev`?");
        return;
      }
      std::vector<std::vector<std::string>> rows;
      int64_t now = ::time(nullptr);
      for (auto& id : order) {
        Status s = m[id];
        std::string act = s.error.empty() ? s.last : s.error;
        int64_t t = parse_rfc3339(s.last_time);
        if (t == 0) t = now;
        act += " (" + ago(now - t) + " ago)";
        if (s.pod.size() > 15) s.pod = s.pod.substr(0, 15) + "...";
        if (s.local.size() > 20) s.local = "..." + s.local.substr(s.local.size() - 20);
        if (s.container.size() > 20) s.container = "..." + s.container.substr(s.container.size() - 20);
        rows.push_back({s.status.empty() ? "Active" : s.status, s.pod, s.local, s.container, act,
                        std::to_string(s.total)});
      }
      log::get().print_table({"Status", "Pod", "Local", "Container", "Latest Activity", "Total Changes"}, rows);
    });
  }));
  return st;
}

// ---------------------------------------------------------------- use / update / create

std::unique_ptr<cli::Command> make_use() {
  auto use = group("use", "Use specific config");
  use->add(leaf("config", "Use a specific DevSpace configuration", 1, 1, [](cli::Command&, const Args& a) {
    need_root();
    return guarded([&] {
      Value configs;
      try {
        configs = yaml_load_file(config::kDefaultConfigsPath);
      } catch (const std::exception& e) {
        throw std::runtime_error(std::string("Cannot load ") + config::kDefaultConfigsPath + ": " + e.what());
      }
      if (!configs.has(a[0]))
        throw std::runtime_error("Config '" + a[0] + "' does not exist in " + config::kDefaultConfigsPath);
      config::Context ctx;
      ctx.generated().set_active_config(a[0]);
      ctx.save_generated();
      log::info("Successfully switched to config '" + a[0] + "'");
    });
  }));
  use->add(leaf("context", "Change current kubectl context to space", 0, 1, [](cli::Command&, const Args& a) {
    return guarded([&] {
      cloud::Space s;
      if (a.empty()) {
        if (!config::set_devspace_root()) throw std::runtime_error("No space configured");
        config::Context ctx;
        if (!ctx.generated().has_space())
          throw std::runtime_error("No space configured. Run `devspace use space` to configure space for active project");
        s = cloud::Space::from_generated(ctx.generated().space());
      } else {
        s = cloud::Client(current_provider()).space_by_name(a[0]);
      }
      cloud::update_kube_config(cloud::kube_context_for(s), s, true);
      log::info("Successfully changed kubectl context to space " + s.name);
    });
  }));
  use->add(leaf("registry", "Configure docker to use a specific registry", 1, 1, [](cli::Command&, const Args& a) {
    return guarded([&] {
      cloud::Provider p = current_provider();
      build::DockerConfigFile dcf = build::DockerConfigFile::load();
      build::AuthConfig auth;
      auth.server_address = a[0];
      auth.username = cloud::token_account(p.token);
      auth.password = p.token;
      auth.auth = base64_encode(auth.username + ":" + auth.password);
      dcf.store(auth);
      dcf.save();
      log::info("Successfully logged into registry " + a[0]);
    });
  }));
  {
    auto c = leaf("space", "Use an existing space for the current configuration", 1, 1,
                  [](cli::Command& c, const Args& a) {
                    need_root();
                    return guarded([&] {
                      config::Context ctx;
                      if (a[0] == "none") {
                        ctx.generated().clear_space();
                        ctx.save_generated();
                        log::info("Successfully erased space");
                        return;
                      }
                      log::start_wait("Retrieving Space details");
                      cloud::Space s = cloud::Client(current_provider()).space_by_name(a[0]);
                      log::stop_wait();
                      ctx.generated().space() = s.to_generated();
                      ctx.save_generated();
                      if (c.get_bool("context")) cloud::update_kube_config(cloud::kube_context_for(s), s, true);
                      log::donef("Successfully configured config to use space %s", s.name.c_str());
                    });
                  });
    c->boolean("context", "", true, "Create/Update kubectl context for space");
    use->add(std::move(c));
  }
  return use;
}

std::unique_ptr<cli::Command> make_update() {
  auto up = group("update", "Updates the current config");
  up->add(leaf("config", "Converts the active config to the current config version", 0, 0,
               [](cli::Command&, const Args&) {
                 need_root();
                 return guarded([&] {
                   config::Context ctx;
                   ctx.base();
                   try {
                     ctx.save_base();
                   } catch (const std::exception& e) {
                     throw std::runtime_error(std::string("Error saving config: ") + e.what());
                   }
                   log::info("Successfully converted base config to current version");
                 });
               }));
  return up;
}

std::unique_ptr<cli::Command> make_create() {
  auto cr = group("create", "Create spaces in the cloud");
  auto c = leaf("space", "Create a new cloud space", 1, 1, [](cli::Command& c, const Args& a) {
    return guarded([&] {
      bool exists = config::set_devspace_root();
      cloud::Client cl(current_provider());
      log::start_wait("Creating space " + a[0]);
      auto projects = cl.projects();
      int64_t project_id;
      if (projects.empty()) {
        auto clusters = cl.clusters();
        if (clusters.empty()) throw std::runtime_error("Cannot create project, because no public cluster was found");
        int64_t cluster_id = clusters[0].first;
        if (clusters.size() > 1) {
          log::stop_wait();
          std::vector<std::string> names;
          for (auto& k : clusters) names.push_back(k.second.empty() ? "Cluster-" + std::to_string(k.first) : k.second);
          std::string pick = prompt::select("Which cluster do you want to use?", names, names[0]);
          for (size_t i = 0; i < names.size(); i++)
            if (names[i] == pick) cluster_id = clusters[i].first;
        }
        project_id = cl.create_project("default", cluster_id);
      } else {
        project_id = projects[0].first;
      }
      int64_t id = cl.create_space(a[0], project_id, 0);
      cloud::Space s = cl.space(id);
      log::stop_wait();
      if (c.get_bool("context")) cloud::update_kube_config(cloud::kube_context_for(s), s, true);
      if (c.get_bool("active") && exists) {
        config::Context ctx;
        ctx.generated().space() = s.to_generated();
        ctx.save_generated();
      }
      log::info("Successfully created space " + s.name);
      log::info("\nYou can now run: \n- `" + log::color("devspace deploy", "white+b") +
                "` to deploy the app to the cloud\n- `" + log::color("devspace dev", "white+b") +
                "` to develop the app in the cloud");
    });
  });
  c->boolean("context", "", true, "Create/Update kubectl context for Space")
      .boolean("active", "", true, "Use the new Space as active Space for the current project");
  cr->add(std::move(c));
  return cr;
}

}  // namespace

void register_config(cli::Command& root) {
  root.add(make_add());
  root.add(make_remove());
  root.add(make_list());
  root.add(make_status());
  root.add(make_use());
  root.add(make_update());
  root.add(make_create());
}

}  // namespace cmd
}  // namespace ds

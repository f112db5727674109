#include "configure/configure.h"

#include <regex>

#include "build/docker.h"
#include "cloud/cloud.h"
#include "core/codec.h"
#include "core/fs.h"
#include "core/log.h"
#include "core/prompt.h"
#include "core/proc.h"
#include "core/strutil.h"
#include "deploy/helmrepo.h"

namespace ds {
namespace configure {

Value parse_selectors(const std::string& s) {
  Value m = Value::map();
  if (s.empty()) return m;
  for (auto& kv : split(s, ",")) {
    auto p = split(kv, "=");
    if (p.size() != 2) throw std::runtime_error("Wrong selector format: " + s);
    m[trim(p[0])] = Value(trim(p[1]));
  }
  return m;
}

bool label_maps_equal(const Value& a, const Value& b) {
  if (a.size() != b.size()) return false;
  for (auto& e : a.entries()) {
    const Value* o = b.find(e.first);
    if (!o || o->as_string() != e.second.as_string()) return false;
  }
  return true;
}

Value parse_port_mappings(const std::string& s) {
  Value out = Value::seq();
  for (auto& m : split(s, ",")) {
    auto p = split(trim(m), ":");
    if (p.size() != 1 && p.size() != 2) throw std::runtime_error("Error parsing port mapping: " + m);
    int64_t a, b;
    if (!parse_int64(p[0], &a)) throw std::runtime_error("strconv.Atoi: parsing \"" + p[0] + "\": invalid syntax");
    b = a;
    if (p.size() == 2 && !parse_int64(p[1], &b))
      throw std::runtime_error("strconv.Atoi: parsing \"" + p[1] + "\": invalid syntax");
    Value pm = Value::map();
    pm["localPort"] = a;
    pm["remotePort"] = b;
    out.push(pm);
  }
  return out;
}

static void save(config::Context& ctx) {
  try {
    ctx.save_base();
  } catch (const std::exception& e) {
    throw std::runtime_error(std::string("Couldn't save config file: ") + e.what());
  }
}

// ---------------------------------------------------------------- deployments

void add_deployment(config::Context& ctx, const std::string& name, const std::string& ns,
                    const std::string& manifests, const std::string& chart) {
  if (manifests.empty() && chart.empty()) throw std::runtime_error("Either manifests or chart flag has to be specified");
  if (!manifests.empty() && !chart.empty())
    throw std::runtime_error("The --manifests flag and --chart flag cannot be used together");
  Value& cfg = ctx.base();
  for (auto& d : cfg.get("deployments").items())
    if (d.get("name").as_string() == name) throw std::runtime_error("Deployment " + name + " already exists");
  Value d = Value::map();
  d["name"] = name;
  if (!ns.empty()) d["namespace"] = ns;
  if (!chart.empty()) {
    d["helm"]["chartPath"] = chart;
  } else {
    Value ms = Value::seq();
    for (auto& m : split(manifests, ",")) ms.push(Value(trim(m)));
    d["kubectl"]["manifests"] = ms;
  }
  if (!cfg.get("deployments").is_seq()) cfg["deployments"] = Value::seq();
  cfg["deployments"].push(d);
  save(ctx);
}

void remove_deployment(config::Context& ctx, bool all, const std::string& name) {
  if (name.empty() && !all) throw std::runtime_error("You have to specify either a deployment name or the --all flag");
  Value& cfg = ctx.base();
  if (cfg.get("deployments").is_seq()) {
    Value keep = Value::seq();
    for (auto& d : cfg["deployments"].items())
      if (!all && d.get("name").as_string() != name) keep.push(d);
    cfg["deployments"] = keep;
  }
  save(ctx);
}

// ---------------------------------------------------------------- images

void add_image(config::Context& ctx, const std::string& name_in_config, const std::string& image,
               const std::string& tag, const std::string& context_path, const std::string& dockerfile,
               const std::string& engine) {
  Value& cfg = ctx.base();
  Value img = Value::map();
  img["image"] = image;
  if (!tag.empty()) img["tag"] = tag;
  Value b = Value::map();
  if (!context_path.empty()) b["contextPath"] = context_path;
  if (!dockerfile.empty()) b["dockerfilePath"] = dockerfile;
  if (engine == "docker")
    b["docker"] = Value::map();
  else if (engine == "kaniko")
    b["kaniko"] = Value::map();
  else if (!engine.empty())
    log::error("BuildEngine " + engine + " unknown. Please select one of docker|kaniko");
  img["build"] = b;
  cfg["images"][name_in_config] = img;
  save(ctx);
}

void remove_image(config::Context& ctx, bool all, const std::vector<std::string>& names) {
  if (names.empty() && !all) throw std::runtime_error("You have to specify at least one image");
  Value& cfg = ctx.base();
  Value keep = Value::map();
  if (!all)
    for (auto& e : cfg.get("images").entries())
      if (std::find(names.begin(), names.end(), e.first) == names.end()) keep[e.first] = e.second;
  cfg["images"] = keep;
  save(ctx);
}

// ---------------------------------------------------------------- selectors

static const Value* selector_named(const Value& cfg, const std::string& name) {
  for (auto& s : cfg.at_path("dev.selectors").items())
    if (s.get("name").as_string() == name) return &s;
  return nullptr;
}

// The label selector used when none is given: the named selector, the first selector, or
// release=<first helm deployment> (port.go:27, sync.go:30).
static Value default_labels(const Value& cfg, const std::string& selector_name, std::string* label_selector) {
  if (!label_selector->empty()) return parse_selectors(*label_selector);
  const Value& sels = cfg.at_path("dev.selectors");
  if (sels.size() > 0) {
    const Value* s = &sels[0];
    if (!selector_name.empty()) {
      s = selector_named(cfg, selector_name);
      if (!s) throw std::runtime_error("no service with name " + selector_name + " exists");
    }
    return s->get("labelSelector").is_map() ? s->get("labelSelector") : Value::map();
  }
  *label_selector = "release=" + config::first_helm_deployment(cfg);
  return parse_selectors(*label_selector);
}

void add_selector(config::Context& ctx, const std::string& name, const std::string& label_selector,
                  const std::string& ns, bool do_save) {
  Value& cfg = ctx.base();
  Value labels;
  if (label_selector.empty()) {
    const Value& sels = cfg.at_path("dev.selectors");
    if (sels.size() > 0 && sels[0].get("labelSelector").is_map())
      labels = sels[0].get("labelSelector");
    else
      labels = parse_selectors("release=" + config::first_helm_deployment(cfg));
  } else {
    try {
      labels = parse_selectors(label_selector);
    } catch (const std::exception& e) {
      throw std::runtime_error(std::string("Error parsing selectors: ") + e.what());
    }
  }
  Value s = Value::map();
  s["name"] = name;
  s["labelSelector"] = labels;
  if (!ns.empty()) s["namespace"] = ns;
  Value& sels = cfg.ensure_path("dev.selectors");
  if (!sels.is_seq()) sels = Value::seq();
  sels.push(s);
  if (do_save) save(ctx);
}

void remove_selector(config::Context& ctx, bool all, const std::string& name, const std::string& label_selector,
                     const std::string& ns) {
  Value labels;
  try {
    labels = parse_selectors(label_selector);
  } catch (const std::exception& e) {
    throw std::runtime_error(std::string("Error parsing selectors: ") + e.what());
  }
  if (labels.size() == 0 && !all && name.empty() && ns.empty())
    throw std::runtime_error("You have to specify at least one of the supported flags or specify the selectors' name");
  Value& cfg = ctx.base();
  if (cfg.at_path("dev.selectors").size() == 0) return;
  Value keep = Value::seq();
  for (auto& s : cfg["dev"]["selectors"].items()) {
    if (all || (!name.empty() && s.get("name").as_string() == name) ||
        (!ns.empty() && s.get("namespace").as_string() == ns) ||
        (labels.size() > 0 && label_maps_equal(labels, s.get("labelSelector"))))
      continue;
    keep.push(s);
  }
  cfg["dev"]["selectors"] = keep;
  save(ctx);
}

// ---------------------------------------------------------------- ports

void add_port(config::Context& ctx, const std::string& ns, const std::string& label_selector,
              const std::string& selector_name, const std::string& mappings) {
  if (!label_selector.empty() && !selector_name.empty())
    throw std::runtime_error(
        "both service and label-selector specified. This is illegal because the label-selector is already specified "
        "in the referenced service. Therefore defining both is redundant");
  Value& cfg = ctx.base();
  std::string ls = label_selector;
  Value labels;
  try {
    labels = default_labels(cfg, selector_name, &ls);
  } catch (const std::runtime_error& e) {
    if (starts_with(e.what(), "no service")) throw;
    throw std::runtime_error(std::string("Error parsing selectors: ") + e.what());
  }
  Value pms;
  try {
    pms = parse_port_mappings(mappings);
  } catch (const std::exception& e) {
    throw std::runtime_error(std::string("Error parsing port mappings: ") + e.what());
  }
  Value& ports = cfg.ensure_path("dev.ports");
  if (!ports.is_seq()) ports = Value::seq();
  // port.go:131 insertOrReplacePortMapping: extend an entry with the same label selector
  for (auto& p : ports.items()) {
    Value sel = p.get("labelSelector").is_map() ? p.get("labelSelector") : Value::map();
    if (label_maps_equal(sel, labels)) {
      if (!p.get("portMappings").is_seq()) p["portMappings"] = Value::seq();
      for (auto& m : pms.items()) p["portMappings"].push(m);
      save(ctx);
      return;
    }
  }
  Value e = Value::map();
  if (selector_name.empty()) e["labelSelector"] = labels;
  e["portMappings"] = pms;
  if (!ns.empty()) e["namespace"] = ns;
  if (!selector_name.empty()) e["selector"] = selector_name;
  ports.push(e);
  save(ctx);
}

void remove_port(config::Context& ctx, bool all, const std::string& label_selector, const std::string& ports_arg) {
  Value labels = parse_selectors(label_selector);
  if (labels.size() == 0 && !all && ports_arg.empty())
    throw std::runtime_error("You have to specify at least one of the supported flags");
  std::vector<std::string> ports;
  for (auto& p : split(ports_arg, ",")) ports.push_back(trim(p));
  auto has = [&](int64_t v) { return std::find(ports.begin(), ports.end(), std::to_string(v)) != ports.end(); };
  Value& cfg = ctx.base();
  if (cfg.at_path("dev.ports").size() == 0) return;
  Value keep = Value::seq();
  for (auto& p : cfg["dev"]["ports"].items()) {
    if (all) continue;
    if (labels.size() > 0 && label_maps_equal(labels, p.get("labelSelector"))) continue;
    Value pms = Value::seq();
    for (auto& m : p.get("portMappings").items())
      if (!has(m.get("localPort").as_int()) && !has(m.get("remotePort").as_int())) pms.push(m);
    if (pms.size() > 0) {
      Value np = p;
      np["portMappings"] = pms;
      keep.push(np);
    }
  }
  cfg["dev"]["ports"] = keep;
  save(ctx);
}

// ---------------------------------------------------------------- sync

void add_sync(config::Context& ctx, const std::string& local_path, const std::string& container_path,
              const std::string& ns, const std::string& label_selector, const std::string& excluded,
              const std::string& selector_name) {
  if (!label_selector.empty() && !selector_name.empty())
    throw std::runtime_error(
        "both service and label-selector specified. This is illegal because the label-selector is already specified "
        "in the referenced service. Therefore defining both is redundant");
  Value& cfg = ctx.base();
  std::string ls = label_selector;
  Value labels = default_labels(cfg, selector_name, &ls);
  Value ex = Value::seq();
  if (!excluded.empty())
    for (auto& e : split(excluded, ",")) ex.push(Value(trim(e)));
  std::string lp = local_path;
  std::string wd = fs::cwd();
  if (starts_with(lp, wd)) lp = lp.substr(wd.size());
  if (container_path.empty() || container_path[0] != '/')
    throw std::runtime_error(
        "ContainerPath (--container) must start with '/'. Info: There is an issue with MINGW based terminals like git "
        "bash");
  Value s = Value::map();
  if (selector_name.empty()) s["labelSelector"] = labels;
  s["containerPath"] = container_path;
  s["localSubPath"] = lp;
  s["excludePaths"] = ex;
  if (!ns.empty()) s["namespace"] = ns;
  if (!selector_name.empty()) s["selector"] = selector_name;
  Value& sync = cfg.ensure_path("dev.sync");
  if (!sync.is_seq()) sync = Value::seq();
  sync.push(s);
  save(ctx);
}

void remove_sync(config::Context& ctx, bool all, const std::string& local_path, const std::string& container_path,
                 const std::string& label_selector) {
  Value labels;
  try {
    labels = parse_selectors(label_selector);
  } catch (const std::exception& e) {
    throw std::runtime_error(std::string("Error parsing selectors: ") + e.what());
  }
  if (labels.size() == 0 && !all && local_path.empty() && container_path.empty())
    throw std::runtime_error("You have to specify at least one of the supported flags");
  Value& cfg = ctx.base();
  if (cfg.at_path("dev.sync").size() == 0) return;
  Value keep = Value::seq();
  for (auto& s : cfg["dev"]["sync"].items()) {
    if (all || (!local_path.empty() && s.get("localSubPath").as_string() == local_path) ||
        (!container_path.empty() && s.get("containerPath").as_string() == container_path) ||
        (labels.size() > 0 && label_maps_equal(labels, s.get("labelSelector"))))
      continue;
    keep.push(s);
  }
  cfg["dev"]["sync"] = keep;
  save(ctx);
}

// ---------------------------------------------------------------- packages

static const char* kPackageComment =
    "\n# Values of the package (subchart); see the subchart's values.yaml for all options\n";

std::string package_default_values(const std::string& name) {
  static const std::string reset_resources =
      "\n  resources:\n    limits:\n      cpu: 0\n      memory: 0\n    requests:\n      cpu: 0\n      memory: 0";
  static const std::map<std::string, std::string> m = {
      {"mysql",
       "\n  mysqlRootPassword: \"YOUR_ROOT_PASSWORD\"\n  mysqlDatabase: \"YOUR_DATABASE_NAME\"\n  mysqlUser: "
       "\"YOUR_USERNAME\"\n  mysqlPassword: \"YOUR_PASSWORD\"\n  persistence:\n    enabled: true\n    size: 3Gi" +
           reset_resources},
      {"mariadb",
       "\n  rootUser:\n    password: \"YOUR_ROOT_PASSWORD\"\n  db:\n    name: \"YOUR_DATABASE_NAME\"\n    user: "
       "\"YOUR_USERNAME\"\n    password: \"YOUR_PASSWORD\"\n  master:\n    persistence:\n      enabled: true\n      "
       "size: 3Gi"},
      {"postgresql",
       "\n  postgresqlPassword: \"YOUR_PASSWORD\"\n  postgresqlDatabase: \"YOUR_DATABASE_NAME\"\n  persistence:\n    "
       "enabled: true\n    size: 3Gi"},
      {"redis", "\n  usePassword: false\n  cluster:\n    enabled: false\n  master:\n    persistence:\n      enabled: true"},
      {"mongodb", "\n  usePassword: false\n  persistence:\n    enabled: true\n    size: 3Gi"},
      {"rabbitmq", "\n  rabbitmq:\n    username: \"YOUR_USERNAME\"\n    password: \"YOUR_PASSWORD\""},
      {"influxdb", "\n  setDefaultUser:\n    enabled: true\n  persistence:\n    enabled: true\n    size: 3Gi"},
  };
  auto it = m.find(name);
  return it == m.end() ? "" : it->second;
}

Value package_default_selector(const std::string& name, const std::string& deployment) {
  Value s = Value::map();
  if (name == "mariadb")
    s["app"] = "mariadb";
  else if (name == "redis" || name == "postgresql" || name == "mongodb" || name == "rabbitmq")
    s["app"] = name;
  else
    s["app"] = deployment + "-" + name;
  return s;
}

static Value* helm_deployment(config::Context& ctx, const std::string& deployment) {
  Value& cfg = ctx.base();
  if (!cfg.get("deployments").is_seq() || (cfg.get("deployments").size() != 1 && deployment.empty()))
    throw std::runtime_error("Please specify the deployment via the -d flag");
  for (auto& d : cfg["deployments"].items())
    if (deployment.empty() || d.get("name").as_string() == deployment) {
      if (d.at_path("helm.chartPath").as_string().empty())
        throw std::runtime_error("Selected deployment " + d.get("name").as_string() + " is not a valid helm deployment");
      return &d;
    }
  throw std::runtime_error("Deployment " + deployment + " not found");
}

static void write_requirements(const std::string& chart, const Value& deps) {
  Value v = Value::map();
  v["dependencies"] = deps;
  fs::write_file(fs::join(chart, "requirements.yaml"), yaml_dump(v), 0600);
}

// `helm dependency update`: download every dependency archive into charts/.
static void update_dependencies(const std::string& chart, const Value& deps) {
  std::string dir = fs::join(chart, "charts");
  fs::mkdirs(dir);
  for (auto& d : deps.items()) {
    std::string name = d.get("name").as_string(), ver = d.get("version").as_string();
    if (fs::exists(fs::join(dir, name + "-" + ver + ".tgz"))) continue;
    helmrepo::ChartVersion cv;
    try {
      cv = helmrepo::search(name, ver);
    } catch (const std::exception&) {
      std::string repo = d.get("repository").as_string();
      helmrepo::add_repo({"dep-" + name, repo});
      helmrepo::update();
      cv = helmrepo::search(name, ver);
    }
    helmrepo::download(cv, dir);
  }
}

void add_package(config::Context& ctx, const std::string& name, const std::string& chart_version,
                 const std::string& app_version, const std::string& deployment, bool skip_question) {
  Value* d = helm_deployment(ctx, deployment);
  std::string dep_name = d->get("name").as_string();
  std::string chart = fs::abs_path(d->at_path("helm.chartPath").as_string());
  log::start_wait("Search Chart");
  helmrepo::update();
  helmrepo::ChartVersion cv;
  try {
    cv = helmrepo::search(name, chart_version, app_version);
  } catch (...) {
    log::stop_wait();
    throw;
  }
  log::stop_wait();
  log::done("Chart found");

  std::string req = fs::join(chart, "requirements.yaml");
  Value deps = Value::seq();
  if (fs::exists(req)) {
    Value y;
    try {
      y = yaml_load_file(req);
    } catch (const std::exception& e) {
      throw std::runtime_error("Error parsing " + req + ": " + e.what());
    }
    if (!y.get("dependencies").is_null() && !y.get("dependencies").is_seq())
      throw std::runtime_error("Error parsing " + req + ": Key dependencies is not an array");
    deps = y.get("dependencies").is_seq() ? y.get("dependencies") : Value::seq();
    for (auto& x : deps.items())
      if (x.get("name").as_string() == cv.name) throw std::runtime_error("Package " + cv.name + " already added");
  }
  Value e = Value::map();
  e["name"] = cv.name;
  e["version"] = cv.version;
  e["repository"] = cv.repo_url;
  deps.push(e);
  write_requirements(chart, deps);
  log::start_wait("Update chart dependencies");
  try {
    update_dependencies(chart, deps);
  } catch (...) {
    log::stop_wait();
    throw;
  }
  log::stop_wait();

  std::string values_path = fs::join(chart, "values.yaml");
  Value values = fs::exists(values_path) ? yaml_load_file(values_path) : Value::map();
  if (!values.is_map() || !values.has(cv.name)) {
    std::string defaults = package_default_values(cv.name);
    fs::append_file(values_path, std::string(kPackageComment) + cv.name + ":" + (defaults.empty() ? " {}" : defaults) + "\n");
  }
  Value& cfg = ctx.base();
  if (!selector_named(cfg, cv.name)) {
    Value s = Value::map();
    s["name"] = cv.name;
    s["labelSelector"] = package_default_selector(cv.name, dep_name);
    Value& sels = cfg.ensure_path("dev.selectors");
    if (!sels.is_seq()) sels = Value::seq();
    sels.push(s);
  }
  save(ctx);
  log::done("Successfully added package " + cv.name + ", you can now modify the configuration in '" + chart +
            "/values.yaml'");
  if (!skip_question) {
    prompt::Params q;
    q.question = "Do you want to open the package README to see configuration options?";
    q.default_value = "yes";
    q.options = {"yes", "no"};
    if (prompt::ask(q) == "yes") {
      // package.go:506 showReadme: <chart>/charts/<name>-<version>.tgz -> <name>/README.md
      std::string tgz = fs::join(chart, "charts", cv.name + "-" + cv.version + ".tgz");
      std::string readme = extract_from_tgz(tgz, cv.name + "/README.md");
      if (readme.empty())
        log::warn("The package has no README.md");
      else
        log::get().write("\n" + readme + "\n");
    }
  }
}

std::string extract_from_tgz(const std::string& tgz_path, const std::string& member) {
  std::string data;
  if (!fs::read_file(tgz_path, &data)) return "";
  GzipReader gz(string_source(&data));
  TarReader tr([&](char* b, size_t n) { return gz.read(b, n); });
  TarEntry te;
  while (tr.next(&te)) {
    if (fs::clean(te.name) == fs::clean(member)) return tr.read_all();
  }
  return "";
}

void remove_package(config::Context& ctx, bool all, const std::string& deployment, const std::string& name) {
  if (!all && name.empty()) throw std::runtime_error("You need to specify a package name or the --all flag");
  Value* d = helm_deployment(ctx, deployment);
  std::string chart = fs::abs_path(d->at_path("helm.chartPath").as_string());
  std::string req = fs::join(chart, "requirements.yaml");
  if (!fs::exists(req)) {
    log::done("No dependencies found");
    return;
  }
  Value y = yaml_load_file(req);
  Value deps = y.get("dependencies").is_seq() ? y.get("dependencies") : Value::seq();
  Value keep = Value::seq();
  bool removed = false;
  for (auto& x : deps.items()) {
    if (all || x.get("name").as_string() == name) {
      std::string tgz = fs::join(chart, "charts", x.get("name").as_string() + "-" + x.get("version").as_string() + ".tgz");
      if (!fs::remove(tgz)) log::warn("Unable to delete package file: " + tgz);
      removed = true;
      continue;
    }
    keep.push(x);
  }
  write_requirements(chart, keep);
  if (all)
    log::done("Successfully removed all dependencies");
  else if (removed)
    log::done("Successfully removed dependency " + name);
  else
    log::done("No dependencies found");
}

// ---------------------------------------------------------------- init image

void init_image(config::Context& ctx, const std::string& docker_username_in, bool is_cloud) {
  Value& cfg = ctx.base();
  std::string username = docker_username_in;
  std::string registry;
  if (!is_cloud) {
    prompt::Params p;
    p.question = "Which registry do you want to push to? ('hub.docker.com' or URL)";
    p.default_value = "hub.docker.com";
    p.key = "registry";
    p.env = "DEVSPACE_INIT_REGISTRY";
    registry = prompt::ask(p);
  } else {
    std::string provider = cfg.at_path("cluster.cloudProvider").as_string(cloud::kDefaultProviderName);
    cloud::Provider pr = cloud::ensure_logged_in(provider);
    auto regs = cloud::Client(pr).registries();
    registry = regs.empty() ? "hub.docker.com" : regs[0];
  }
  build::DockerConfigFile dcf = build::DockerConfigFile::load();
  // an image named up front (--image / DEVSPACE_INIT_IMAGE) needs no account to derive it from
  const char* env_image = getenv("DEVSPACE_INIT_IMAGE");
  prompt::Params image_q;
  image_q.key = "image";
  image_q.env = "DEVSPACE_INIT_IMAGE";
  bool image_given = prompt::has_answer("image") || (env_image && *env_image);
  if (!image_given && registry != "hub.docker.com") {
    build::AuthConfig a = dcf.get(registry);
    if (a.username.empty() && !is_cloud && fs::exists(registry) == false) {
      // A local/insecure registry (e.g. the devspace local cluster) needs no credentials.
      log::warn("No credentials found for " + registry + " (run `docker login " + registry + "` if it needs auth)");
    }
    if (!a.username.empty()) username = a.username;
  } else if (!image_given && username.empty()) {
    build::AuthConfig a = dcf.get("https://index.docker.io/v1/");
    username = a.username;
    if (username.empty()) {
      log::warn("No dockerhub credentials were found in the credentials store");
      log::warn("Please make sure you have a https://hub.docker.com account");
      log::warn("Installing docker is NOT required\n");
      // a Docker Hub image needs an account namespace (the reference loops on docker login,
      // configure/init_image.go:63-90): never fall through to an image named "/devspace"
      for (int attempt = 0; attempt < 3 && username.empty(); ++attempt) {
        prompt::Params u;
        u.question = "What is your docker hub username?";
        u.optional = true;
        username = trim(prompt::ask(u));
        if (prompt::noninteractive_env()) break;
      }
      if (username.empty())
        throw std::runtime_error(
            "a Docker Hub username is required to push to Docker Hub: set --image (DEVSPACE_INIT_IMAGE) to name "
            "the image, or --registry (DEVSPACE_INIT_REGISTRY) for another registry, or run `docker login`");
      prompt::Params pw;
      pw.question = "What is your docker hub password?";
      pw.is_password = true;
      std::string password = prompt::ask(pw);
      build::AuthConfig na;
      na.server_address = "https://index.docker.io/v1/";
      na.username = username;
      na.password = password;
      na.auth = base64_encode(username + ":" + password);
      dcf.store(na);
      dcf.save();
    }
  }
  std::string image;
  prompt::Params p = image_q;
  if (image_given) {
    p.question = "Which image name do you want to push to?";
    p.validation_regex = "[a-zA-Z0-9\\.:/_-]{1,200}";
    image = prompt::ask(p);
  } else if (registry == "hub.docker.com") {
    p.question = "Which image name do you want to use on Docker Hub?";
    p.default_value = username + "/devspace";
    p.validation_regex = "[a-zA-Z0-9/-]{4,60}";
    image = prompt::ask(p);
  } else if (std::regex_match(registry, std::regex("(.+\\.)?gcr\\.io"))) {
    std::string project = "myGCloudProject";
    if (!which("gcloud").empty()) {
      RunResult r = run({"gcloud", "config", "get-value", "project"}, "", {}, 20000);
      if (r.code == 0 && !trim(r.out).empty()) project = trim(r.out);
    }
    p.question = "Which image name do you want to push to?";
    p.default_value = registry + "/" + project + "/devspace";
    image = prompt::ask(p);
  } else if (is_cloud) {
    p = prompt::Params();
    image = registry + "/" + username + "/devspace";
  } else {
    p.question = "Which image name do you want to push to?";
    p.default_value = registry + "/" + (username.empty() ? "" : username + "/") + "devspace";
    p.validation_regex = "[a-zA-Z0-9\\.:/-]{4,90}";
    image = prompt::ask(p);
  }
  bool pull_secret = true;
  if (!is_cloud) {
    prompt::Params q;
    q.question = "Do you want to enable automatic creation of pull secrets for this image? (yes | no)";
    q.default_value = "yes";
    q.validation_regex = "(yes|no)";
    q.key = "pullSecret";
    q.env = "DEVSPACE_INIT_PULL_SECRET";
    pull_secret = prompt::ask(q) == "yes";
  }
  std::string why = build::image_reference_problem(image);
  if (!why.empty()) throw std::runtime_error("invalid image name \"" + image + "\": " + why);
  cfg["images"]["default"]["image"] = image;
  if (pull_secret) cfg["images"]["default"]["createPullSecret"] = true;
}

}  // namespace configure
}  // namespace ds

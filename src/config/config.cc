#include "config/config.h"

#include <algorithm>
#include <cstdlib>
#include <regex>

#include "core/fs.h"
#include "core/log.h"
#include "core/prompt.h"
#include "core/strutil.h"
#include "kube/kubeconfig.h"

namespace ds {
namespace config {

const char* const kLatestVersion = "v1alpha2";
const char* const kDefaultConfigPath = ".devspace/config.yaml";
const char* const kDefaultConfigsPath = ".devspace/configs.yaml";
const char* const kDefaultVarsPath = ".devspace/vars.yaml";
const char* const kGeneratedPath = ".devspace/generated.yaml";
const char* const kDefaultDeploymentName = "devspace-app";
const char* const kVarEnvPrefix = "DEVSPACE_VAR_";

// ======================================================================= schema DSL

namespace {

using SP = std::shared_ptr<Schema>;

SP str() {
  auto s = std::make_shared<Schema>();
  s->kind = Schema::Str;
  return s;
}
SP integer() {
  auto s = std::make_shared<Schema>();
  s->kind = Schema::Int;
  return s;
}
SP boolean() {
  auto s = std::make_shared<Schema>();
  s->kind = Schema::Bool;
  return s;
}
SP any() {
  auto s = std::make_shared<Schema>();
  s->kind = Schema::Any;
  return s;
}
SP list(SP e) {
  auto s = std::make_shared<Schema>();
  s->kind = Schema::List;
  s->elem = std::move(e);
  return s;
}
SP dict(SP e) {
  auto s = std::make_shared<Schema>();
  s->kind = Schema::Dict;
  s->elem = std::move(e);
  return s;
}
SP st(const std::string& name, std::vector<std::pair<std::string, SP>> fields) {
  auto s = std::make_shared<Schema>();
  s->kind = Schema::Struct;
  s->type_name = name;
  s->fields = std::move(fields);
  return s;
}

SP build_latest() {
  auto cluster_user = st("latest.ClusterUser", {{"clientCert", str()}, {"clientKey", str()}, {"token", str()}});
  auto cluster = st("latest.Cluster", {{"cloudProvider", str()},
                                       {"kubeContext", str()},
                                       {"namespace", str()},
                                       {"apiServer", str()},
                                       {"caCert", str()},
                                       {"user", cluster_user}});
  auto helm = st("latest.HelmConfig", {{"chartPath", str()},
                                       {"wait", boolean()},
                                       {"timeout", integer()},
                                       // revisions kept per release (helm --history-max; 0 = all)
                                       {"maxHistory", integer()},
                                       {"tillerNamespace", str()},
                                       {"overrides", list(str())},
                                       {"overrideValues", any()}});
  auto kubectl = st("latest.KubectlConfig", {{"cmdPath", str()}, {"manifests", list(str())}});
  auto deployment =
      st("latest.DeploymentConfig", {{"name", str()}, {"namespace", str()}, {"helm", helm}, {"kubectl", kubectl}});
  auto labels = dict(str());
  auto terminal = st("latest.Terminal", {{"disabled", boolean()},
                                         {"selector", str()},
                                         {"labelSelector", labels},
                                         {"namespace", str()},
                                         {"containerName", str()},
                                         {"command", list(str())}});
  auto autoreload =
      st("latest.AutoReloadConfig", {{"paths", list(str())}, {"deployments", list(str())}, {"images", list(str())}});
  auto override_image = st("latest.ImageOverrideConfig", {{"name", str()}, {"entrypoint", list(str())}});
  auto selector = st("latest.SelectorConfig",
                     {{"name", str()}, {"namespace", str()}, {"labelSelector", labels}, {"containerName", str()}});
  auto port_mapping =
      st("latest.PortMapping", {{"localPort", integer()}, {"remotePort", integer()}, {"bindAddress", str()}});
  auto ports = st("latest.PortForwardingConfig", {{"selector", str()},
                                                  {"namespace", str()},
                                                  {"labelSelector", labels},
                                                  {"portMappings", list(port_mapping)}});
  auto bw = st("latest.BandwidthLimits", {{"download", integer()}, {"upload", integer()}});
  auto sync = st("latest.SyncConfig", {{"selector", str()},
                                       {"namespace", str()},
                                       {"labelSelector", labels},
                                       {"containerName", str()},
                                       {"localSubPath", str()},
                                       {"containerPath", str()},
                                       {"excludePaths", list(str())},
                                       {"downloadExcludePaths", list(str())},
                                       {"uploadExcludePaths", list(str())},
                                       {"bandwidthLimits", bw}});
  auto dev = st("latest.DevConfig", {{"terminal", terminal},
                                     {"autoReload", autoreload},
                                     {"overrideImages", list(override_image)},
                                     {"selectors", list(selector)},
                                     {"ports", list(ports)},
                                     {"sync", list(sync)}});
  auto kaniko = st("latest.KanikoConfig",
                   {{"cache", boolean()}, {"namespace", str()}, {"pullSecret", str()}, {"image", str()}});
  auto docker = st("latest.DockerConfig", {{"preferMinikube", boolean()}});
  auto opts = st("latest.BuildOptions", {{"buildArgs", dict(str())}, {"target", str()}, {"network", str()}});
  auto build = st("latest.BuildConfig", {{"disabled", boolean()},
                                         {"contextPath", str()},
                                         {"dockerfilePath", str()},
                                         {"kaniko", kaniko},
                                         {"docker", docker},
                                         {"options", opts}});
  auto image = st("latest.ImageConfig", {{"image", str()},
                                         {"tag", str()},
                                         {"createPullSecret", boolean()},
                                         {"insecure", boolean()},
                                         {"skipPush", boolean()},
                                         {"build", build}});
  return st("latest.Config", {{"version", str()},
                              {"cluster", cluster},
                              {"dev", dev},
                              {"deployments", list(deployment)},
                              {"images", dict(image)}});
}

SP build_v1alpha1() {
  auto labels = dict(str());
  auto cluster_user = st("v1alpha1.ClusterUser", {{"clientCert", str()}, {"clientKey", str()}, {"token", str()}});
  auto cluster = st("v1alpha1.Cluster", {{"cloudProvider", str()},
                                         {"kubeContext", str()},
                                         {"namespace", str()},
                                         {"apiServer", str()},
                                         {"caCert", str()},
                                         {"user", cluster_user}});
  auto ar = st("v1alpha1.AutoReloadConfig", {{"disabled", boolean()}});
  auto helm = st("v1alpha1.HelmConfig", {{"chartPath", str()},
                                         {"wait", boolean()},
                                         {"tillerNamespace", str()},
                                         {"devOverwrite", str()},
                                         {"override", str()},
                                         {"overrideValues", any()}});
  auto kubectl = st("v1alpha1.KubectlConfig", {{"cmdPath", str()}, {"manifests", list(str())}});
  auto deployment = st("v1alpha1.DeploymentConfig", {{"name", str()},
                                                     {"namespace", str()},
                                                     {"autoReload", ar},
                                                     {"helm", helm},
                                                     {"kubectl", kubectl}});
  auto terminal = st("v1alpha1.Terminal", {{"disabled", boolean()},
                                           {"service", str()},
                                           {"resourceType", str()},
                                           {"labelSelector", labels},
                                           {"namespace", str()},
                                           {"containerName", str()},
                                           {"command", list(str())}});
  auto arp = st("v1alpha1.AutoReloadPathsConfig", {{"paths", list(str())}});
  auto service = st("v1alpha1.ServiceConfig", {{"name", str()},
                                               {"namespace", str()},
                                               {"resourceType", str()},
                                               {"labelSelector", labels},
                                               {"containerName", str()}});
  auto pm = st("v1alpha1.PortMapping", {{"localPort", integer()}, {"remotePort", integer()}, {"bindAddress", str()}});
  auto ports = st("v1alpha1.PortForwardingConfig", {{"service", str()},
                                                    {"namespace", str()},
                                                    {"resourceType", str()},
                                                    {"labelSelector", labels},
                                                    {"portMappings", list(pm)}});
  auto bw = st("v1alpha1.BandwidthLimits", {{"download", integer()}, {"upload", integer()}});
  auto sync = st("v1alpha1.SyncConfig", {{"service", str()},
                                         {"namespace", str()},
                                         {"labelSelector", labels},
                                         {"containerName", str()},
                                         {"localSubPath", str()},
                                         {"containerPath", str()},
                                         {"excludePaths", list(str())},
                                         {"downloadExcludePaths", list(str())},
                                         {"uploadExcludePaths", list(str())},
                                         {"bandwidthLimits", bw}});
  auto devspace = st("v1alpha1.DevSpaceConfig", {{"terminal", terminal},
                                                 {"autoReload", arp},
                                                 {"services", list(service)},
                                                 {"deployments", list(deployment)},
                                                 {"ports", list(ports)},
                                                 {"sync", list(sync)}});
  auto kaniko = st("v1alpha1.KanikoConfig", {{"cache", boolean()}, {"namespace", str()}, {"pullSecret", str()}});
  auto docker = st("v1alpha1.DockerConfig", {{"preferMinikube", boolean()}});
  auto opts = st("v1alpha1.BuildOptions", {{"buildArgs", dict(str())}, {"target", str()}, {"network", str()}});
  auto build = st("v1alpha1.BuildConfig", {{"disabled", boolean()},
                                           {"contextPath", str()},
                                           {"dockerfilePath", str()},
                                           {"kaniko", kaniko},
                                           {"docker", docker},
                                           {"options", opts}});
  auto image = st("v1alpha1.ImageConfig", {{"name", str()},
                                           {"tag", str()},
                                           {"registry", str()},
                                           {"createPullSecret", boolean()},
                                           {"skipPush", boolean()},
                                           {"autoReload", ar},
                                           {"build", build}});
  auto rauth = st("v1alpha1.RegistryAuth", {{"username", str()}, {"password", str()}});
  auto registry = st("v1alpha1.RegistryConfig", {{"url", str()}, {"auth", rauth}, {"insecure", boolean()}});
  auto tiller = st("v1alpha1.TillerConfig", {{"namespace", str()}});
  auto ireg = st("v1alpha1.InternalRegistryConfig", {{"deploy", boolean()}, {"namespace", str()}});
  return st("v1alpha1.Config", {{"version", str()},
                                {"devSpace", devspace},
                                {"images", dict(image)},
                                {"registries", dict(registry)},
                                {"cluster", cluster},
                                {"tiller", tiller},
                                {"internalRegistry", ireg}});
}

SP build_vars() {
  return list(st("configs.Variable", {{"name", str()}, {"default", str()}, {"question", str()}, {"regexPattern", str()}}));
}

SP build_configs() {
  auto wrapper = st("configs.ConfigWrapper", {{"path", str()}, {"data", any()}});
  auto vars = st("configs.VarsWrapper", {{"path", str()}, {"data", build_vars()}});
  auto def = st("configs.ConfigDefinition", {{"config", wrapper}, {"vars", vars}, {"overrides", list(wrapper)}});
  return dict(def);
}

}  // namespace

const Schema* Schema::field(const std::string& k) const {
  for (auto& f : fields)
    if (f.first == k) return f.second.get();
  return nullptr;
}

const Schema& schema_latest() {
  static SP s = build_latest();
  return *s;
}
const Schema& schema_v1alpha1() {
  static SP s = build_v1alpha1();
  return *s;
}
const Schema& schema_configs() {
  static SP s = build_configs();
  return *s;
}
const Schema& schema_vars() {
  static SP s = build_vars();
  return *s;
}

void validate_strict(const Value& v, const Schema& s, const std::string& where) {
  if (v.is_null()) return;
  auto here = [&](const std::string& child) { return where.empty() ? child : where + "." + child; };
  switch (s.kind) {
    case Schema::Any: return;
    case Schema::Str:
      if (!v.is_scalar())
        throw ConfigError("cannot unmarshal " + std::string(type_name(v.type())) + " into string at " + where);
      return;
    case Schema::Int:
      if (!v.is_int() && !(v.is_string() && !v.quoted() && v.as_int(INT64_MIN) != INT64_MIN))
        throw ConfigError("cannot unmarshal !!" + std::string(type_name(v.type())) + " `" + v.as_string() +
                          "` into int at " + where);
      return;
    case Schema::Bool:
      if (!v.is_bool())
        throw ConfigError("cannot unmarshal !!" + std::string(type_name(v.type())) + " `" + v.as_string() +
                          "` into bool at " + where);
      return;
    case Schema::List:
      if (!v.is_seq()) throw ConfigError("cannot unmarshal " + std::string(type_name(v.type())) + " into a list at " + where);
      for (size_t i = 0; i < v.size(); ++i) validate_strict(v[i], *s.elem, where + "[" + std::to_string(i) + "]");
      return;
    case Schema::Dict:
      if (!v.is_map()) throw ConfigError("cannot unmarshal " + std::string(type_name(v.type())) + " into a map at " + where);
      for (auto& e : v.entries()) validate_strict(e.second, *s.elem, here(e.first));
      return;
    case Schema::Struct:
      if (!v.is_map())
        throw ConfigError("cannot unmarshal " + std::string(type_name(v.type())) + " into " + s.type_name + " at " +
                          (where.empty() ? "<root>" : where));
      for (auto& e : v.entries()) {
        const Schema* f = s.field(e.first);
        if (!f) throw ConfigError("field " + e.first + " not found in type " + s.type_name);
        validate_strict(e.second, *f, here(e.first));
      }
      return;
  }
}

// Normalises scalar types to the schema (e.g. unquoted "3000" stays int; ints where strings
// are expected become strings) so the tree is well-typed after loading.
static void coerce(Value& v, const Schema& s) {
  if (v.is_null()) return;
  switch (s.kind) {
    case Schema::Str:
      if (!v.is_string()) {
        Value n(v.as_string());
        n.set_quoted(true);
        v = n;
      }
      return;
    case Schema::Int:
      if (v.is_string()) v = Value(v.as_int());
      return;
    case Schema::List:
      for (auto& it : v.items()) coerce(it, *s.elem);
      return;
    case Schema::Dict:
      for (auto& e : v.entries()) coerce(e.second, *s.elem);
      return;
    case Schema::Struct:
      for (auto& e : v.entries()) {
        const Schema* f = s.field(e.first);
        if (f) coerce(e.second, *f);
      }
      return;
    default: return;
  }
}

// ======================================================================= upgrade

Value upgrade_v1alpha1(const Value& c) {
  Value next = Value::map();
  next["version"] = kLatestVersion;
  // Fields that convert 1:1 (util.Convert JSON round trip): cluster, images (minus removed keys)
  if (c.get("cluster").is_map()) next["cluster"] = c.get("cluster");
  Value dev = Value::map();
  auto ensure_ar = [&]() -> Value& {
    Value& ar = dev["autoReload"];
    if (ar.is_null()) ar = Value::map();
    return ar;
  };
  const Value& ds = c.get("devSpace");
  if (ds.get("deployments").is_seq()) {
    Value deps = Value::seq();
    for (auto& d : ds.get("deployments").items()) {
      Value nd = Value::map();
      nd["name"] = d.get("name");
      if (!d.get("namespace").is_null()) nd["namespace"] = d.get("namespace");
      // upgrade.go:32 adds the deployment to autoReload when auto reload is *not disabled*
      // (the reference's condition is inverted; intent per docs: enabled unless disabled).
      const Value& dis = d.at_path("autoReload.disabled");
      if (dis.is_null() || !dis.as_bool()) ensure_ar()["deployments"].push(d.get("name"));
      if (d.get("kubectl").is_map()) {
        Value k = Value::map();
        if (!d.at_path("kubectl.cmdPath").is_null()) k["cmdPath"] = d.at_path("kubectl.cmdPath");
        if (!d.at_path("kubectl.manifests").is_null()) k["manifests"] = d.at_path("kubectl.manifests");
        nd["kubectl"] = k;
      } else if (d.get("helm").is_map()) {
        const Value& h = d.get("helm");
        Value nh = Value::map();
        if (!h.get("chartPath").is_null()) nh["chartPath"] = h.get("chartPath");
        if (!h.get("wait").is_null()) nh["wait"] = h.get("wait");
        if (!h.get("overrideValues").is_null()) nh["overrideValues"] = h.get("overrideValues");
        if (!h.get("devOverwrite").is_null()) nh["overrides"] = Value::seq_of({h.get("devOverwrite")});
        if (!h.get("override").is_null()) nh["overrides"] = Value::seq_of({h.get("override")});
        nd["helm"] = nh;
      }
      deps.push(nd);
    }
    next["deployments"] = deps;
  }
  if (ds.is_map()) {
    if (ds.get("sync").is_seq()) {
      Value out = Value::seq();
      for (auto& s : ds.get("sync").items()) {
        Value n = Value::map();
        if (!s.get("service").is_null()) n["selector"] = s.get("service");
        for (const char* k : {"namespace", "labelSelector", "localSubPath", "containerName", "containerPath",
                              "excludePaths", "downloadExcludePaths", "uploadExcludePaths", "bandwidthLimits"})
          if (!s.get(k).is_null()) n[k] = s.get(k);
        out.push(n);
      }
      dev["sync"] = out;
    }
    if (ds.get("ports").is_seq()) {
      Value out = Value::seq();
      for (auto& p : ds.get("ports").items()) {
        Value n = Value::map();
        if (!p.get("service").is_null()) n["selector"] = p.get("service");
        for (const char* k : {"namespace", "labelSelector", "portMappings"})
          if (!p.get(k).is_null()) n[k] = p.get(k);
        out.push(n);
      }
      dev["ports"] = out;
    }
    if (ds.get("terminal").is_map()) {
      const Value& t = ds.get("terminal");
      Value n = Value::map();
      if (!t.get("disabled").is_null()) n["disabled"] = t.get("disabled");
      if (!t.get("service").is_null()) n["selector"] = t.get("service");
      for (const char* k : {"labelSelector", "namespace", "containerName", "command"})
        if (!t.get(k).is_null()) n[k] = t.get(k);
      dev["terminal"] = n;
    }
    if (ds.get("services").is_seq()) {
      Value out = Value::seq();
      for (auto& s : ds.get("services").items()) {
        Value n = Value::map();
        for (const char* k : {"name", "namespace", "labelSelector", "containerName"})
          if (!s.get(k).is_null()) n[k] = s.get(k);
        out.push(n);
      }
      dev["selectors"] = out;
    }
    if (ds.at_path("autoReload.paths").is_seq() && ds.at_path("autoReload.paths").size() > 0)
      ensure_ar()["paths"] = ds.at_path("autoReload.paths");
  }
  if (c.get("images").is_map()) {
    Value images = Value::map();
    for (auto& e : c.get("images").entries()) {
      const Value& img = e.second;
      Value ni = Value::map();
      ni["image"] = img.get("name");
      for (const char* k : {"tag", "createPullSecret", "skipPush", "build"})
        if (!img.get(k).is_null()) ni[k] = img.get(k);
      if (!img.get("registry").is_null()) {
        std::string reg = img.get("registry").as_string();
        const Value& regs = c.get("registries");
        if (!regs.is_map()) throw ConfigError("Registries is nil in config");
        const Value* r = regs.find(reg);
        if (!r) throw ConfigError("Couldn't find registry " + reg + " in registries");
        if (!r->get("auth").is_null())
          log::warn("Registry authentication is not supported any longer (Registry " + reg +
                    "). Please use docker login [registry] instead");
        if (r->get("url").is_null() || img.get("name").is_null())
          throw ConfigError("Registry url or image name is nil for image " + e.first);
        ni["image"] = r->get("url").as_string() + "/" + img.get("name").as_string();
      }
      const Value& dis = img.at_path("autoReload.disabled");
      if (dis.is_null() || !dis.as_bool()) ensure_ar()["images"].push(Value(e.first));
      images[e.first] = ni;
    }
    next["images"] = images;
  }
  if (!c.at_path("tiller.namespace").is_null() && next.get("deployments").is_seq()) {
    for (auto& d : next["deployments"].items())
      if (d.get("helm").is_map()) d["helm"]["tillerNamespace"] = c.at_path("tiller.namespace");
  }
  if (!c.get("internalRegistry").is_null()) log::warn("internalRegistry deployment is not supported anymore");
  next["dev"] = dev;
  return next;
}

Value parse_versioned(Value data) {
  if (data.is_null()) data = Value::map();
  if (!data.is_map()) throw ConfigError("Error loading config: config is not a map");
  std::string version = data.get("version").is_string() ? data.get("version").as_string() : "";
  if (version.empty()) {
    // overrides usually don't carry a version (versions.go:21-25)
    data["version"] = kLatestVersion;
    version = kLatestVersion;
  }
  if (version == "v1alpha1") {
    try {
      validate_strict(data, schema_v1alpha1());
    } catch (const ConfigError& e) {
      throw ConfigError(std::string("Error loading config: ") + e.what());
    }
    try {
      data = upgrade_v1alpha1(data);
    } catch (const ConfigError& e) {
      throw ConfigError(std::string("Error upgrading config from version v1alpha1: ") + e.what());
    }
  } else if (version != kLatestVersion) {
    throw ConfigError("Unrecognized config version " + version + ". Please upgrade devspace with `devspace upgrade`");
  }
  try {
    validate_strict(data, schema_latest());
  } catch (const ConfigError& e) {
    throw ConfigError(std::string("Error loading config: ") + e.what());
  }
  coerce(data, schema_latest());
  data["version"] = kLatestVersion;
  return data;
}

// ======================================================================= generated

Generated Generated::load(const std::string& path) {
  Generated g;
  g.path = path;
  std::string data;
  if (fs::read_file(path, &data)) {
    try {
      g.v_ = yaml_parse(data);
    } catch (const std::exception& e) {
      throw ConfigError("Error loading " + path + ": " + e.what());
    }
  }
  if (!g.v_.is_map()) g.v_ = Value::map();
  if (g.v_.get("activeConfig").as_string().empty()) g.v_["activeConfig"] = "default";
  if (!g.v_.get("configs").is_map()) g.v_["configs"] = Value::map();
  return g;
}

void Generated::save() const { fs::write_file_atomic(path, yaml_dump(prune_empty(v_))); }

std::string Generated::active_config() const { return v_.get("activeConfig").as_string("default"); }
void Generated::set_active_config(const std::string& name) { v_["activeConfig"] = name; }

Value& Generated::active() {
  Value& c = v_["configs"][active_config()];
  if (!c.is_map()) c = Value::map();
  return c;
}

Value& Generated::cache(bool dev) {
  Value& c = active()[dev ? "dev" : "deploy"];
  if (!c.is_map()) c = Value::map();
  for (const char* k : {"deployments", "dockerfileTimestamps", "dockerContextPaths", "imageTags"})
    if (!c.get(k).is_map()) c[k] = Value::map();
  return c;
}

Value& Generated::vars() {
  Value& v = active()["vars"];
  if (!v.is_map()) v = Value::map();
  return v;
}

Value& Generated::space() { return v_["space"]; }
bool Generated::has_space() const { return v_.get("space").is_map(); }
void Generated::clear_space() { v_.erase("space"); }

// ======================================================================= vars

Value convert_var_value(const std::string& s) {
  if (s == "true") return Value(true);
  if (s == "false") return Value(false);
  int64_t iv;
  if (parse_int64(s, &iv)) return Value(iv);
  return Value(s);
}

static Value ask_variable(const Variable* v, const std::string& name) {
  prompt::Params p;
  p.question = v && v->question ? *v->question : "Please enter a value for " + name;
  if (v && v->def) p.default_value = *v->def;
  if (v && v->regex) p.validation_regex = *v->regex;
  return convert_var_value(prompt::ask(p));
}

static std::vector<Variable> vars_from_value(const Value& v) {
  std::vector<Variable> out;
  for (auto& it : v.items()) {
    Variable var;
    var.name = it.get("name").as_string();
    if (!it.get("default").is_null()) var.def = it.get("default").as_string();
    if (!it.get("question").is_null()) var.question = it.get("question").as_string();
    if (!it.get("regexPattern").is_null()) var.regex = it.get("regexPattern").as_string();
    out.push_back(var);
  }
  return out;
}

// ======================================================================= context

bool Context::config_exists() const {
  if (fs::exists(kDefaultConfigsPath)) return true;
  if (fs::exists(config_path)) return true;
  return config_path == kDefaultConfigPath && fs::exists("devspace.yaml");
}

Generated& Context::generated() {
  if (!generated_) generated_ = std::make_unique<Generated>(Generated::load(kGeneratedPath));
  return *generated_;
}

void Context::save_generated() {
  if (generated_) generated_->save();
}

void Context::reset() {
  loaded_ = false;
  config_ = Value();
  raw_ = Value();
  loaded_config_.clear();
  generated_.reset();
  var_defs_.clear();
}

void Context::init_empty() {
  reset();
  raw_ = Value::map();
  raw_["version"] = kLatestVersion;
  config_ = raw_;
  loaded_ = true;
  loaded_with_overrides_ = true;
}

void Context::ask_questions(const std::vector<Variable>& vars) {
  bool changed = false;
  Value& cached = generated().vars();
  for (size_t i = 0; i < vars.size(); ++i) {
    const Variable& v = vars[i];
    if (v.name.empty()) throw ConfigError("Name required for variable with index " + std::to_string(i));
    if (cached.has(v.name)) continue;
    const char* env = getenv((std::string(kVarEnvPrefix) + to_upper(v.name)).c_str());
    cached[v.name] = env && *env ? convert_var_value(env) : ask_variable(&v, v.name);
    changed = true;
  }
  if (changed) save_generated();
}

Value Context::resolve_vars(Value raw) {
  static const std::regex var_re("^\\$\\{[^\\}]+\\}$");
  bool changed = false;
  walk_strings(raw, [&](const std::string&, Value& val) {
    const std::string& s = val.str();
    if (!std::regex_match(s, var_re)) return false;
    std::string name = trim(s.substr(2, s.size() - 3));
    const char* env = getenv((std::string(kVarEnvPrefix) + to_upper(name)).c_str());
    Value& cached = generated().vars();
    if (env && *env) {
      val = convert_var_value(env);
      cached[name] = val;
      changed = true;
      return true;
    }
    // The reference looks the cache up by "${NAME}" (load.go:59) and so always misses; the
    // intent is the bare variable name.
    if (const Value* c = cached.find(name)) {
      val = *c;
      return true;
    }
    const Variable* def = nullptr;
    for (auto& v : var_defs_)
      if (v.name == name) def = &v;
    val = ask_variable(def, name);
    cached[name] = val;
    changed = true;
    return true;
  });
  if (changed) save_generated();
  return raw;
}

Value Context::load_from_value(const Value& data) { return parse_versioned(resolve_vars(data)); }

Value Context::load_from_path(const std::string& path) {
  std::string text;
  if (!fs::read_file(path, &text)) throw ConfigError("open " + path + ": no such file or directory");
  Value raw;
  try {
    raw = yaml_parse(text);
  } catch (const std::exception& e) {
    throw ConfigError(std::string(e.what()));
  }
  return load_from_value(raw);
}

Value Context::load_wrapper(const Value& w, const std::string& what) {
  bool has_path = !w.get("path").is_null(), has_data = !w.get("data").is_null();
  if (!has_path && !has_data) throw ConfigError("path & data key are empty for " + what + " " + loaded_config_);
  if (has_path && has_data)
    throw ConfigError("path & data are both defined in " + what + " " + loaded_config_ + ". Only choose one");
  if (has_path) {
    try {
      return load_from_path(w.get("path").as_string());
    } catch (const ConfigError& e) {
      throw ConfigError(std::string("Loading config: ") + e.what());
    }
  }
  try {
    return load_from_value(w.get("data"));
  } catch (const ConfigError& e) {
    throw ConfigError(std::string("Loading config from interface: ") + e.what());
  }
}

std::vector<Variable> Context::load_vars_definitions() const {
  std::string data;
  if (fs::read_file(kDefaultVarsPath, &data)) {
    Value v = yaml_parse(data);
    validate_strict(v, schema_vars());
    return vars_from_value(v);
  }
  return {};
}

const Value& Context::get(bool with_overrides) {
  if (loaded_ && (loaded_with_overrides_ || !with_overrides)) return config_;
  Generated& gen = generated();
  Value definition;
  if (fs::exists(kDefaultConfigsPath)) {
    Value configs;
    try {
      configs = yaml_load_file(kDefaultConfigsPath);
      validate_strict(configs, schema_configs());
    } catch (const std::exception& e) {
      throw ConfigError(std::string("Error loading ") + kDefaultConfigsPath + ": " + e.what());
    }
    loaded_config_ = gen.active_config();
    if (config_path != kDefaultConfigPath) loaded_config_ = config_path;
    const Value* def = configs.find(loaded_config_);
    if (!def)
      throw ConfigError(
          "No active config selected. Run: \n- `devspace list configs` to list all available configs\n- `devspace use "
          "config [NAME]` to use a specific config");
    definition = *def;
    if (definition.get("config").is_null()) throw ConfigError("config " + loaded_config_ + " cannot be found");
    if (definition.get("vars").is_map()) {
      const Value& vw = definition.get("vars");
      bool hp = !vw.get("path").is_null(), hd = !vw.get("data").is_null();
      if (!hp && !hd) throw ConfigError("path & data key are empty for vars " + loaded_config_);
      if (hp && hd) throw ConfigError("path & data are both defined in vars " + loaded_config_ + ". Only choose one");
      Value vv = hd ? vw.get("data") : yaml_load_file(vw.get("path").as_string());
      validate_strict(vv, schema_vars());
      var_defs_ = vars_from_value(vv);
      ask_questions(var_defs_);
    }
    raw_ = load_wrapper(definition.get("config"), "config");
  } else {
    var_defs_ = load_vars_definitions();
    if (!var_defs_.empty()) ask_questions(var_defs_);
    std::string path = config_path;
    if (path == kDefaultConfigPath && !fs::exists(path) && fs::exists("devspace.yaml")) path = "devspace.yaml";
    try {
      raw_ = load_from_path(path);
    } catch (const ConfigError& e) {
      throw ConfigError(std::string("Loading config: ") + e.what());
    }
  }
  config_ = raw_;
  if (with_overrides && definition.get("overrides").is_seq()) {
    size_t idx = 0;
    for (auto& w : definition.get("overrides").items()) {
      Value ov;
      try {
        ov = load_wrapper(w, "override");
      } catch (const ConfigError& e) {
        throw ConfigError("Error loading override config at index " + std::to_string(idx) + ": " + e.what());
      }
      ov.erase("version");
      merge_into(config_, ov);
      ++idx;
    }
  }
  gen.save();
  loaded_ = true;
  loaded_with_overrides_ = with_overrides;
  validate(config_);
  return config_;
}

Value& Context::base() {
  if (!loaded_) get(false);
  if (loaded_with_overrides_) {
    // Mutations target the base config; drop merged overrides.
    config_ = raw_;
    loaded_with_overrides_ = false;
  }
  return config_;
}

void Context::validate(const Value& cfg) const {
  const Value& dev = cfg.get("dev");
  auto idx = [](size_t i) { return std::to_string(i); };
  if (dev.is_map()) {
    const Value& sels = dev.get("selectors");
    for (size_t i = 0; i < sels.size(); ++i)
      if (sels[i].get("name").is_null()) throw ConfigError("Error in config: Unnamed selector at index " + idx(i));
    const Value& ports = dev.get("ports");
    for (size_t i = 0; i < ports.size(); ++i) {
      if (ports[i].get("selector").is_null() && ports[i].get("labelSelector").is_null())
        throw ConfigError("Error in config: selector and label selector are nil in port config at index " + idx(i));
      if (ports[i].get("portMappings").is_null())
        throw ConfigError("Error in config: portMappings is empty in port config at index " + idx(i));
    }
    const Value& sync = dev.get("sync");
    for (size_t i = 0; i < sync.size(); ++i) {
      if (sync[i].get("selector").is_null() && sync[i].get("labelSelector").is_null())
        throw ConfigError("Error in config: selector and label selector are nil in sync config at index " + idx(i));
      if (sync[i].get("containerPath").is_null() || sync[i].get("localSubPath").is_null())
        throw ConfigError("Error in config: containerPath or localSubPath are nil in sync config at index " + idx(i));
    }
    const Value& ovr = dev.get("overrideImages");
    for (size_t i = 0; i < ovr.size(); ++i)
      if (ovr[i].get("name").is_null())
        throw ConfigError("Error in config: Unnamed override image config at index " + idx(i));
  }
  const Value& deps = cfg.get("deployments");
  for (size_t i = 0; i < deps.size(); ++i) {
    const Value& d = deps[i];
    if (d.get("name").is_null()) throw ConfigError("Error in config: Unnamed deployment at index " + idx(i));
    if (d.get("helm").is_null() && d.get("kubectl").is_null())
      throw ConfigError("Please specify either helm or kubectl as deployment type in deployment " +
                        d.get("name").as_string());
    if (d.get("helm").is_map() && d.at_path("helm.chartPath").is_null())
      throw ConfigError("deployments[" + idx(i) + "].helm.chartPath is required");
    if (d.get("kubectl").is_map() && d.at_path("kubectl.manifests").is_null())
      throw ConfigError("deployments[" + idx(i) + "].kubectl.manifests is required");
  }
}

void Context::save_base() {
  if (config_path != kDefaultConfigPath) return;  // custom config files are not rewritten
  Value cfg = prune_empty(base());
  cfg["version"] = kLatestVersion;
  // keep "version" first
  Value ordered = Value::map();
  ordered["version"] = kLatestVersion;
  for (auto& e : cfg.entries())
    if (e.first != "version") ordered[e.first] = e.second;
  std::string save_path = kDefaultConfigPath;
  if (!loaded_config_.empty() && fs::exists(kDefaultConfigsPath)) {
    Value configs = yaml_load_file(kDefaultConfigsPath);
    Value* def = configs.find(loaded_config_);
    if (def && def->at_path("config.data").is_map()) {
      (*def)["config"]["data"] = ordered;
      fs::write_file(kDefaultConfigsPath, yaml_dump(configs));
      return;
    }
    if (def && !def->at_path("config.path").is_null()) save_path = def->at_path("config.path").as_string();
  } else if (!fs::exists(kDefaultConfigPath) && fs::exists("devspace.yaml")) {
    save_path = "devspace.yaml";
  }
  fs::write_file(save_path, yaml_dump(ordered));
}

// ======================================================================= helpers

bool set_devspace_root(std::string* found_dir) {
  std::string cwd = fs::cwd();
  std::string original = cwd;
  std::string home = fs::clean(fs::home_dir());
  size_t last_len = 0;
  while (cwd.size() != last_len) {
    if (cwd != home) {
      if (fs::is_dir(fs::join(cwd, ".devspace")) || fs::is_file(fs::join(cwd, "devspace.yaml"))) {
        fs::chdir(cwd);
        if (original != cwd) log::info("Using devspace config in " + cwd + "/.devspace");
        if (found_dir) *found_dir = cwd;
        return true;
      }
    }
    last_len = cwd.size();
    cwd = fs::dirname(cwd);
  }
  return false;
}

std::string default_namespace(const Value& cfg) {
  std::string ns = cfg.at_path("cluster.namespace").as_string();
  if (!ns.empty()) return ns;
  if (cfg.at_path("cluster.apiServer").is_null()) {
    kube::KubeConfig kc = kube::KubeConfig::load();
    std::string ctx = kc.current_context();
    std::string want = cfg.at_path("cluster.kubeContext").as_string();
    if (!want.empty()) ctx = want;
    std::string cns = kc.context_namespace(ctx);
    if (!cns.empty()) return cns;
  }
  return "default";
}

const Value* find_selector(const Value& cfg, const std::string& name) {
  for (auto& s : cfg.at_path("dev.selectors").items())
    if (s.get("name").as_string() == name) return &s;
  return nullptr;
}

std::string LabelSelector::to_query() const {
  auto l = labels;
  std::sort(l.begin(), l.end());
  std::vector<std::string> parts;
  for (auto& kv : l) parts.push_back(kv.first + "=" + kv.second);
  return join(parts, ",");
}

LabelSelector label_selector_from(const Value& v) {
  LabelSelector ls;
  for (auto& e : v.entries()) ls.labels.emplace_back(e.first, e.second.as_string());
  return ls;
}

std::string first_helm_deployment(const Value& cfg) {
  for (auto& d : cfg.get("deployments").items())
    if (d.get("helm").is_map()) return d.get("name").as_string();
  return kDefaultDeploymentName;
}

SelectorRef resolve_selector(const Value& cfg, const Value& entry) {
  SelectorRef r;
  r.namespace_ = default_namespace(cfg);
  std::string sel_name = entry.get("selector").as_string();
  const Value* sel = nullptr;
  if (!sel_name.empty()) {
    sel = find_selector(cfg, sel_name);
    if (!sel) throw ConfigError("Unable to find selector: " + sel_name);
    r.selector = sel_name;
  }
  if (!entry.get("namespace").as_string().empty())
    r.namespace_ = entry.get("namespace").as_string();
  else if (sel && !sel->get("namespace").as_string().empty())
    r.namespace_ = sel->get("namespace").as_string();
  if (entry.get("labelSelector").is_map())
    r.labels = label_selector_from(entry.get("labelSelector"));
  else if (sel && sel->get("labelSelector").is_map())
    r.labels = label_selector_from(sel->get("labelSelector"));
  else
    r.labels.labels = {{"app.kubernetes.io/name", first_helm_deployment(cfg)}};
  if (!entry.get("containerName").as_string().empty())
    r.container = entry.get("containerName").as_string();
  else if (sel)
    r.container = sel->get("containerName").as_string();
  return r;
}

}  // namespace config
}  // namespace ds

#include "kube/kubeconfig.h"

#include <algorithm>
#include <cstdlib>
#include <set>
#include <stdexcept>

#include "core/codec.h"
#include "core/fs.h"
#include "core/log.h"
#include "core/strutil.h"

namespace ds {
namespace kube {

std::vector<std::string> KubeConfig::default_paths() {
  std::vector<std::string> out;
  const char* kc = getenv("KUBECONFIG");
  if (kc && *kc) {
    for (auto& p : split(kc, ":")) {
      if (p.empty() || std::find(out.begin(), out.end(), p) != out.end()) continue;
      out.push_back(p);
    }
  }
  if (out.empty()) out.push_back(fs::join(fs::home_dir(), ".kube/config"));
  return out;
}

std::string KubeConfig::default_path() {
  auto paths = default_paths();
  for (auto& p : paths)
    if (fs::exists(p)) return p;
  return paths.front();
}

static Value empty_config() {
  Value v = Value::map();
  v["apiVersion"] = "v1";
  v["kind"] = "Config";
  v["clusters"] = Value::seq();
  v["contexts"] = Value::seq();
  v["current-context"] = "";
  v["preferences"] = Value::map();
  v["users"] = Value::seq();
  return v;
}

static Value load_one(const std::string& path) {
  std::string data;
  if (!fs::read_file(path, &data)) return empty_config();
  Value v;
  try {
    v = yaml_parse(data);
    if (!v.is_map()) v = empty_config();
  } catch (const std::exception& e) {
    log::warn("Unable to decode kube config " + path + ": " + e.what() + ". Creating backup " + path + ".backup");
    fs::write_file(path + ".backup", data, 0600);
    v = empty_config();
  }
  for (const char* k : {"clusters", "contexts", "users"})
    if (!v.get(k).is_seq()) v[k] = Value::seq();
  return v;
}

static const char* const kLists[] = {"clusters", "contexts", "users"};

KubeConfig KubeConfig::load(const std::string& p) {
  KubeConfig kc;
  kc.files = p.empty() ? default_paths() : std::vector<std::string>{p};
  kc.path = p.empty() ? default_path() : p;
  kc.v_ = empty_config();
  bool have_prefs = false;
  for (auto& f : kc.files) {
    Value one = load_one(f);
    for (const char* list : kLists) {
      for (auto& e : one.get(list).items()) {
        std::string name = e.get("name").as_string();
        if (kc.origin_[list].count(name)) continue;  // first definition wins
        kc.origin_[list][name] = f;
        kc.v_[list].push(e);
      }
    }
    if (kc.cc_origin_.empty() && !one.get("current-context").as_string().empty()) {
      kc.v_["current-context"] = one.get("current-context");
      kc.cc_origin_ = f;
    }
    if (!have_prefs && one.get("preferences").is_map() && one.get("preferences").size() > 0) {
      kc.v_["preferences"] = one.get("preferences");
      have_prefs = true;
    }
  }
  return kc;
}

void KubeConfig::save(const std::string& p) const {
  if (!p.empty() || files.size() <= 1) {
    std::string target = p.empty() ? path : p;
    if (target.empty()) target = default_path();
    fs::write_file_atomic(target, yaml_dump(v_), 0600);
    return;
  }
  // Multi-file: rewrite each file with its own entries (updated from the merged view);
  // entries without an origin and the current context go to `path`.
  std::string cc_file = cc_origin_.empty() ? path : cc_origin_;
  for (auto& f : files) {
    bool exists = fs::exists(f);
    Value out = exists ? load_one(f) : empty_config();
    bool touched = false;
    for (const char* list : kLists) {
      Value items = Value::seq();
      std::set<std::string> seen;
      // keep this file's entries in place, shadowed duplicates untouched
      for (auto& e : out.get(list).items()) {
        std::string name = e.get("name").as_string();
        auto it = origin_.find(list);
        bool mine = it != origin_.end() && it->second.count(name) && it->second.at(name) == f;
        if (!mine) {
          items.push(e);
          continue;
        }
        seen.insert(name);
        if (const Value* cur = named(list, name)) {
          items.push(*cur);
          touched = touched || !(*cur == e);
        } else {
          touched = true;  // deleted in the merged view
        }
      }
      if (f == path) {
        for (auto& e : v_.get(list).items()) {
          std::string name = e.get("name").as_string();
          auto it = origin_.find(list);
          if (it != origin_.end() && it->second.count(name)) continue;
          items.push(e);
          touched = true;
        }
      }
      out[list] = items;
    }
    if (f == cc_file && out.get("current-context").as_string() != current_context()) {
      out["current-context"] = current_context();
      touched = true;
    }
    if (touched) fs::write_file_atomic(f, yaml_dump(out), 0600);
  }
}

std::string KubeConfig::current_context() const { return v_.get("current-context").as_string(); }
void KubeConfig::set_current_context(const std::string& ctx) { v_["current-context"] = ctx; }

const Value* KubeConfig::named(const std::string& list, const std::string& name) const {
  const Value& l = v_.get(list);
  for (auto& it : l.items())
    if (it.get("name").as_string() == name) return &it;
  return nullptr;
}

Value* KubeConfig::named(const std::string& list, const std::string& name) {
  Value* l = v_.find(list);
  if (!l) return nullptr;
  for (auto& it : l->items())
    if (it.get("name").as_string() == name) return &it;
  return nullptr;
}

bool KubeConfig::has_context(const std::string& ctx) const { return named("contexts", ctx) != nullptr; }

std::vector<std::string> KubeConfig::contexts() const {
  std::vector<std::string> out;
  for (auto& it : v_.get("contexts").items()) out.push_back(it.get("name").as_string());
  return out;
}

std::string KubeConfig::context_namespace(const std::string& ctx) const {
  const Value* c = named("contexts", ctx.empty() ? current_context() : ctx);
  if (!c) return "";
  return c->at_path("context.namespace").as_string();
}

void KubeConfig::set_context_namespace(const std::string& ctx, const std::string& ns) {
  Value* c = named("contexts", ctx);
  if (c) (*c)["context"]["namespace"] = ns;
}

void KubeConfig::set_cluster(const std::string& name, const std::string& server, const std::string& ca_b64,
                             bool insecure) {
  Value* c = named("clusters", name);
  if (!c) {
    Value n = Value::map();
    n["name"] = name;
    v_["clusters"].push(n);
    c = &v_["clusters"].items().back();
  }
  Value cl = Value::map();
  cl["server"] = server;
  if (!ca_b64.empty()) cl["certificate-authority-data"] = ca_b64;
  if (insecure) cl["insecure-skip-tls-verify"] = true;
  (*c)["cluster"] = cl;
}

void KubeConfig::set_user_token(const std::string& name, const std::string& token) {
  Value* u = named("users", name);
  if (!u) {
    Value n = Value::map();
    n["name"] = name;
    v_["users"].push(n);
    u = &v_["users"].items().back();
  }
  Value us = Value::map();
  us["token"] = token;
  (*u)["user"] = us;
}

void KubeConfig::set_context(const std::string& name, const std::string& cluster, const std::string& user,
                             const std::string& ns) {
  Value* c = named("contexts", name);
  if (!c) {
    Value n = Value::map();
    n["name"] = name;
    v_["contexts"].push(n);
    c = &v_["contexts"].items().back();
  }
  Value ctx = Value::map();
  ctx["cluster"] = cluster;
  ctx["user"] = user;
  if (!ns.empty()) ctx["namespace"] = ns;
  (*c)["context"] = ctx;
}

void KubeConfig::delete_context(const std::string& name) {
  for (const char* list : {"contexts", "clusters", "users"}) {
    Value* l = v_.find(list);
    if (!l) continue;
    auto& items = l->items();
    for (auto it = items.begin(); it != items.end(); ++it) {
      if (it->get("name").as_string() == name) {
        items.erase(it);
        break;
      }
    }
  }
  if (current_context() == name) set_current_context("");
}

static std::string read_data_or_file(const Value& obj, const std::string& data_key, const std::string& file_key,
                                     const std::string& base_dir) {
  std::string d = obj.get(data_key).as_string();
  if (!d.empty()) return base64_decode(d);
  std::string f = obj.get(file_key).as_string();
  if (!f.empty()) {
    if (!fs::is_abs(f)) f = fs::join(base_dir, f);
    std::string out;
    if (fs::read_file(f, &out)) return out;
  }
  return "";
}

std::string KubeConfig::base_dir_of(const std::string& list, const std::string& name) const {
  auto it = origin_.find(list);
  if (it != origin_.end()) {
    auto jt = it->second.find(name);
    if (jt != it->second.end()) return fs::dirname(jt->second);
  }
  return fs::dirname(path);
}

RestConfig KubeConfig::resolve(const std::string& ctx_in) const {
  std::string ctx = ctx_in.empty() ? current_context() : ctx_in;
  const Value* c = named("contexts", ctx);
  if (!c) {
    if (ctx.empty()) throw std::runtime_error("kube config has no current context (is ~/.kube/config set up?)");
    throw std::runtime_error("context \"" + ctx + "\" does not exist in kube config " + path);
  }
  RestConfig rc;
  rc.context = ctx;
  rc.namespace_ = c->at_path("context.namespace").as_string();
  std::string cluster_name = c->at_path("context.cluster").as_string();
  std::string user_name = c->at_path("context.user").as_string();
  const Value* cl = named("clusters", cluster_name);
  if (!cl) throw std::runtime_error("cluster \"" + cluster_name + "\" not found in kube config");
  std::string cbase = base_dir_of("clusters", cluster_name);
  const Value& clv = cl->get("cluster");
  rc.server = clv.get("server").as_string();
  rc.insecure = clv.get("insecure-skip-tls-verify").as_bool();
  rc.tls_server_name = clv.get("tls-server-name").as_string();
  rc.proxy_url = clv.get("proxy-url").as_string();
  rc.ca_pem = read_data_or_file(clv, "certificate-authority-data", "certificate-authority", cbase);
  const Value* us = named("users", user_name);
  if (us) {
    std::string ubase = base_dir_of("users", user_name);
    const Value& u = us->get("user");
    rc.token = u.get("token").as_string();
    std::string tf = u.get("tokenFile").as_string();
    if (rc.token.empty() && !tf.empty()) {
      rc.token_file = fs::is_abs(tf) ? tf : fs::join(ubase, tf);
      std::string t;
      if (fs::read_file(rc.token_file, &t)) rc.token = trim(t);
    }
    rc.client_cert_pem = read_data_or_file(u, "client-certificate-data", "client-certificate", ubase);
    rc.client_key_pem = read_data_or_file(u, "client-key-data", "client-key", ubase);
    rc.username = u.get("username").as_string();
    rc.password = u.get("password").as_string();
    // legacy auth-provider (oidc / gcp): use the cached token it carries
    const Value& ap = u.at_path("auth-provider.config");
    if (rc.token.empty() && ap.is_map()) {
      rc.token = ap.get("id-token").as_string();
      if (rc.token.empty()) rc.token = ap.get("access-token").as_string();
    }
    const Value& ex = u.get("exec");
    if (ex.is_map()) {
      std::string cmd = ex.get("command").as_string();
      // a relative command with a path separator is relative to the kubeconfig file
      if (cmd.find('/') != std::string::npos && !fs::is_abs(cmd)) cmd = fs::join(ubase, cmd);
      rc.exec_command.push_back(cmd);
      for (auto& a : ex.get("args").items()) rc.exec_command.push_back(a.as_string());
      for (auto& e : ex.get("env").items())
        rc.exec_env.emplace_back(e.get("name").as_string(), e.get("value").as_string());
      if (!ex.get("apiVersion").as_string().empty()) rc.exec_api_version = ex.get("apiVersion").as_string();
      rc.exec_provide_cluster_info = ex.get("provideClusterInfo").as_bool(false);
      rc.exec_install_hint = ex.get("installHint").as_string();
    }
  }
  return rc;
}

}  // namespace kube
}  // namespace ds

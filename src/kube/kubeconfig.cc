#include "kube/kubeconfig.h"

#include <cstdlib>
#include <stdexcept>

#include "core/codec.h"
#include "core/fs.h"
#include "core/log.h"
#include "core/strutil.h"

namespace ds {
namespace kube {

std::string KubeConfig::default_path() {
  const char* kc = getenv("KUBECONFIG");
  if (kc && *kc) {
    auto parts = split(kc, ":");
    for (auto& p : parts)
      if (!p.empty()) return p;
  }
  return fs::join(fs::home_dir(), ".kube/config");
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

KubeConfig KubeConfig::load(const std::string& p) {
  KubeConfig kc;
  kc.path = p.empty() ? default_path() : p;
  std::string data;
  if (!fs::read_file(kc.path, &data)) {
    kc.v_ = empty_config();
    return kc;
  }
  try {
    kc.v_ = yaml_parse(data);
    if (!kc.v_.is_map()) kc.v_ = empty_config();
  } catch (const std::exception& e) {
    log::warn("Unable to decode kube config " + kc.path + ": " + e.what() + ". Creating backup " + kc.path +
              ".backup");
    fs::write_file(kc.path + ".backup", data, 0600);
    kc.v_ = empty_config();
  }
  for (const char* k : {"clusters", "contexts", "users"})
    if (!kc.v_.get(k).is_seq()) kc.v_[k] = Value::seq();
  return kc;
}

void KubeConfig::save(const std::string& p) const {
  std::string target = p.empty() ? path : p;
  if (target.empty()) target = default_path();
  fs::write_file_atomic(target, yaml_dump(v_), 0600);
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
  std::string base = fs::dirname(path);
  const Value* cl = named("clusters", cluster_name);
  if (!cl) throw std::runtime_error("cluster \"" + cluster_name + "\" not found in kube config");
  const Value& clv = cl->get("cluster");
  rc.server = clv.get("server").as_string();
  rc.insecure = clv.get("insecure-skip-tls-verify").as_bool();
  rc.ca_pem = read_data_or_file(clv, "certificate-authority-data", "certificate-authority", base);
  const Value* us = named("users", user_name);
  if (us) {
    const Value& u = us->get("user");
    rc.token = u.get("token").as_string();
    if (rc.token.empty() && !u.get("tokenFile").as_string().empty()) {
      std::string t;
      if (fs::read_file(u.get("tokenFile").as_string(), &t)) rc.token = trim(t);
    }
    rc.client_cert_pem = read_data_or_file(u, "client-certificate-data", "client-certificate", base);
    rc.client_key_pem = read_data_or_file(u, "client-key-data", "client-key", base);
    rc.username = u.get("username").as_string();
    rc.password = u.get("password").as_string();
    const Value& ex = u.get("exec");
    if (ex.is_map()) {
      rc.exec_command.push_back(ex.get("command").as_string());
      for (auto& a : ex.get("args").items()) rc.exec_command.push_back(a.as_string());
      for (auto& e : ex.get("env").items())
        rc.exec_env.emplace_back(e.get("name").as_string(), e.get("value").as_string());
    }
  }
  return rc;
}

}  // namespace kube
}  // namespace ds

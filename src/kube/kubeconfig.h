// ~/.kube/config reading / writing (util/kubeconfig/kubeconfig.go, kubectl/client.go:63-142).
#pragma once

#include <string>
#include <vector>

#include "core/value.h"

namespace ds {
namespace kube {

// Everything needed to talk to one API server.
struct RestConfig {
  std::string server;           // https://host:port or http://host:port or unix:///path
  std::string ca_pem;           // PEM data (may be empty)
  bool insecure = false;        // insecure-skip-tls-verify
  std::string client_cert_pem;  // PEM data
  std::string client_key_pem;
  std::string token;
  std::string username, password;
  std::string namespace_;       // context default namespace
  std::string context;          // context name (if from kubeconfig)
  // exec credential plugin
  std::vector<std::string> exec_command;
  std::vector<std::pair<std::string, std::string>> exec_env;
};

class KubeConfig {
 public:
  static std::string default_path();  // $KUBECONFIG (first) or ~/.kube/config
  // Missing file => empty config. Undecodable file is backed up to <path>.backup and a fresh
  // config is returned (util/kubeconfig/kubeconfig.go:28-40).
  static KubeConfig load(const std::string& path = "");
  void save(const std::string& path = "") const;

  std::string current_context() const;
  void set_current_context(const std::string& ctx);
  bool has_context(const std::string& ctx) const;
  std::vector<std::string> contexts() const;
  std::string context_namespace(const std::string& ctx) const;
  void set_context_namespace(const std::string& ctx, const std::string& ns);

  void set_cluster(const std::string& name, const std::string& server, const std::string& ca_data_b64, bool insecure);
  void set_user_token(const std::string& name, const std::string& token);
  void set_context(const std::string& name, const std::string& cluster, const std::string& user,
                   const std::string& ns);
  void delete_context(const std::string& name);

  // Resolves a context (empty = current) into a RestConfig; throws if unknown.
  RestConfig resolve(const std::string& ctx = "") const;

  Value& raw() { return v_; }
  const Value& raw() const { return v_; }
  std::string path;

 private:
  Value* named(const std::string& list, const std::string& name);
  const Value* named(const std::string& list, const std::string& name) const;
  Value v_;
};

}  // namespace kube
}  // namespace ds

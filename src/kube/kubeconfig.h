// ~/.kube/config reading / writing (util/kubeconfig/kubeconfig.go, kubectl/client.go:63-142).
//
// $KUBECONFIG may list several files (':'-separated). They are merged the way client-go's
// clientcmd loading rules do: for clusters / contexts / users the first file that defines a
// name wins, `current-context` comes from the first file that sets one, relative paths
// resolve against the file that holds the entry. Saving writes every entry back to the file it
// came from; new entries and the current context go to the first existing file.
#pragma once

#include <map>
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
  std::string tls_server_name;  // cluster.tls-server-name
  std::string proxy_url;        // cluster.proxy-url (overrides HTTPS_PROXY)
  std::string client_cert_pem;  // PEM data
  std::string client_key_pem;
  std::string token;
  std::string token_file;       // re-read periodically (bound service-account tokens rotate)
  std::string username, password;
  std::string namespace_;       // context default namespace
  std::string context;          // context name (if from kubeconfig)
  // exec credential plugin (client.authentication.k8s.io ExecCredential)
  std::vector<std::string> exec_command;
  std::vector<std::pair<std::string, std::string>> exec_env;
  std::string exec_api_version = "client.authentication.k8s.io/v1beta1";
  bool exec_provide_cluster_info = false;
  std::string exec_install_hint;
};

class KubeConfig {
 public:
  static std::vector<std::string> default_paths();  // $KUBECONFIG entries or ~/.kube/config
  static std::string default_path();                // first existing of default_paths()
  // Missing file => empty config. Undecodable file is backed up to <path>.backup and a fresh
  // config is returned (util/kubeconfig/kubeconfig.go:28-40). An explicit path loads only
  // that file; otherwise all default_paths() are merged.
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
  std::string path;                 // where new entries / the current context are written
  std::vector<std::string> files;   // merged files in precedence order

 private:
  Value* named(const std::string& list, const std::string& name);
  const Value* named(const std::string& list, const std::string& name) const;
  std::string base_dir_of(const std::string& list, const std::string& name) const;
  Value v_;
  std::map<std::string, std::map<std::string, std::string>> origin_;  // list -> name -> file
  std::string cc_origin_;  // file that defined current-context
};

}  // namespace kube
}  // namespace ds

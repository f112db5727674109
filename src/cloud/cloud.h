// Cloud "Spaces" provider client (pkg/devspace/cloud): ~/.devspace/clouds.yaml providers,
// GraphQL API (spaces, projects, clusters, registries), browser/token login, kube-context
// management for spaces. The original service is offline; the client is exercised against a
// fake GraphQL server in tests and works with any compatible endpoint.
#pragma once

#include <map>
#include <optional>
#include <string>
#include <vector>

#include "config/config.h"
#include "core/value.h"

namespace ds {
namespace cloud {

extern const char* const kDefaultProviderName;  // "app.devspace.cloud"
extern const char* const kKubeContextPrefix;    // "devspace"

struct Provider {
  std::string name, host, token;
};

struct Space {
  int64_t id = 0;
  std::string name, namespace_, service_account_token, server, ca_cert, provider_name, created, domain;
  Value to_generated() const;
  static Space from_generated(const Value& v);
};

std::map<std::string, Provider> load_providers();
void save_providers(const std::map<std::string, Provider>& p);

class Client {
 public:
  explicit Client(Provider p) : p_(std::move(p)) {}
  Value graphql(const std::string& query, const Value& vars = Value());
  std::vector<Space> spaces();
  Space space(int64_t id);
  Space space_by_name(const std::string& name);
  int64_t create_space(const std::string& name, int64_t project_id, int64_t cluster_id);
  int64_t create_project(const std::string& name, int64_t cluster_id);
  std::vector<std::pair<int64_t, std::string>> projects();
  std::vector<std::pair<int64_t, std::string>> clusters();
  void delete_space(int64_t id);
  std::vector<std::string> registries();
  // Browser login: callback server on :25853 (/token?token=...), cloud/login.go:103.
  std::string login_via_browser(int timeout_s = 300);
  const Provider& provider() const { return p_; }

 private:
  Provider p_;
};

// Returns the provider (logging in when no token is stored).
Provider ensure_logged_in(const std::string& provider_name);
// (Re)login with a token, or via the browser when empty (cloud.ReLogin), then log docker into
// the provider's registries.
Provider login(const std::string& provider_name, const std::string& token);
// cloud/configure.go:79 — no-op without cluster.cloudProvider.
void configure(config::Context& ctx, const std::string& space_name = "");
std::string kube_context_for(const Space& s);
void update_kube_config(const std::string& context, const Space& s, bool set_active);
void delete_kube_context(const Space& s);
// cloud/util.go:94 — JWT "sub" claim (account name).
std::string token_account(const std::string& jwt);

}  // namespace cloud
}  // namespace ds

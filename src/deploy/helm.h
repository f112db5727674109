// Native Helm: chart loading + rendering (gotemplate), releases stored as Secrets
// (`sh.helm.release.v1.<name>.v<rev>`, Helm-3 layout), install / upgrade (with rollback on
// failure) / delete / status / history, and --wait readiness. Replaces the reference's Helm v2
// + Tiller stack (helm/client.go, helm/install.go, helm/tiller.go) — Tiller is obsolete.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "core/value.h"
#include "kube/client.h"

namespace ds {
namespace helm {

struct Chart {
  std::string dir;
  Value metadata;  // Chart.yaml
  Value values;    // values.yaml
  std::vector<std::pair<std::string, std::string>> templates;  // (relative name, text)
  std::vector<Chart> dependencies;                             // charts/<sub>
  std::string name() const { return metadata.get("name").as_string(); }
  std::string version() const { return metadata.get("version").as_string(); }
};

Chart load_chart(const std::string& dir);

struct RenderOptions {
  std::string release_name, namespace_;
  int revision = 1;
  bool is_install = true;
};

// Renders all templates into manifests (parsed YAML docs, empty docs dropped, sorted in
// Helm's install order).
std::vector<Value> render(const Chart& chart, const Value& values, const RenderOptions& o);
std::string render_to_string(const Chart& chart, const Value& values, const RenderOptions& o);

struct Release {
  std::string name, namespace_, status;  // deployed | failed | superseded | uninstalled
  int version = 0;
  std::string chart, chart_version, last_deployed;
  Value config;
  std::string manifest;
};

class Client {
 public:
  explicit Client(std::shared_ptr<kube::Client> k) : k_(std::move(k)) {}
  std::vector<Release> history(const std::string& ns, const std::string& name);
  bool release_exists(const std::string& ns, const std::string& name);
  std::vector<Release> list(const std::string& ns);
  // Install or upgrade; on failure an upgrade rolls back to the last deployed revision and a
  // first install is purged (helm/install.go:100-166).
  Release install_or_upgrade(const std::string& name, const std::string& ns, const std::string& chart_path,
                             const Value& values, bool wait, int timeout_s);
  void rollback(const std::string& ns, const std::string& name, int to_version);
  void delete_release(const std::string& ns, const std::string& name, bool purge = true);
  // Waits for every workload in the manifest to be ready; returns "" or a failure summary.
  std::string wait_ready(const std::vector<Value>& objs, const std::string& ns, int timeout_s);

 private:
  void store(const Release& r);
  std::shared_ptr<kube::Client> k_;
};

// Values.MergeInto (deploy/helm/merge.go:8): deep merge, `over` wins.
void merge_values(Value& base, const Value& over);

// Helm's install order by kind.
int kind_order(const std::string& kind);

}  // namespace helm
}  // namespace ds

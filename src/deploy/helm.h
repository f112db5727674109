// Native Helm: chart loading + rendering (gotemplate), releases stored as Secrets
// (`sh.helm.release.v1.<name>.v<rev>`, the Helm 3 storage layout, readable by `helm list /
// history / rollback`), install / upgrade (with rollback on failure) / delete / status /
// history, lifecycle hooks, and --wait readiness. Replaces the reference's Helm v2 + Tiller
// stack (helm/client.go, helm/install.go:54-166, helm/tiller.go) — Tiller is obsolete.
//
// Chart semantics follow Helm 3's loader and engine:
//  * `.Files` — every non-special chart file (not Chart.yaml / values.yaml / requirements.* /
//    templates/ / charts/, minus .helmignore), with Get/GetBytes/Glob/Lines/AsConfig/AsSecrets;
//  * dependencies from requirements.yaml (apiVersion v1) or Chart.yaml `dependencies` (v2):
//    `alias`, `condition` (first resolvable bool wins), `tags`, `import-values` (exports and
//    child/parent forms; the parent's own values take precedence), nested charts;
//  * library charts (type: library) contribute their defines only;
//  * `.Capabilities` from the API server's /version and /api(s) discovery;
//  * NOTES.txt of the top chart rendered into the release's info.notes;
//  * values.schema.json validation (JSON Schema subset) before rendering;
//  * `lookup` against the live cluster, `helm.sh/resource-policy: keep`.
#pragma once

#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "core/value.h"
#include "kube/client.h"

namespace ds {
namespace helm {

struct Dependency {
  std::string name, version, repository, condition, alias;
  std::vector<std::string> tags;
  Value import_values;  // seq of strings / {child, parent} maps
  bool enabled = true;
};

struct Chart {
  std::string dir;
  Value metadata;  // Chart.yaml
  Value values;    // values.yaml
  std::string values_raw, schema;
  std::vector<std::pair<std::string, std::string>> templates;  // (relative name, text)
  std::vector<std::pair<std::string, std::string>> files;      // .Files (relative name, bytes)
  std::vector<Dependency> requirements;                        // requirements.yaml / Chart.yaml v2
  std::vector<Chart> dependencies;                             // charts/<sub>
  std::string name() const { return metadata.get("name").as_string(); }
  std::string version() const { return metadata.get("version").as_string(); }
  bool is_library() const { return metadata.get("type").as_string() == "library"; }
};

Chart load_chart(const std::string& dir);

// Helm's ProcessDependencies: drops disabled subcharts (condition/tags, against the chart
// defaults coalesced with `user_values`), applies aliases and import-values. Mutates `c`.
void process_dependencies(Chart& c, const Value& user_values);

// values.schema.json of the chart and of every subchart (against its part of the values), as
// Helm 3 does before rendering; throws with Helm's report format when any value is invalid.
void validate_values(const Chart& chart, const Value& coalesced_values);

// CoalesceValues: chart defaults (recursively, each subchart under its name) under the user's
// values, with `global` propagated into every subchart.
Value coalesce_values(const Chart& c, const Value& user_values);

struct RenderOptions {
  std::string release_name, namespace_;
  int revision = 1;
  bool is_install = true;
  // {KubeVersion: {Major, Minor, GitVersion, Version}, APIVersions: [..]}; null = defaults
  Value capabilities;
  // `lookup` against the live cluster (install/upgrade); unset = {} as in `helm template`
  std::function<Value(const std::string& api_version, const std::string& kind, const std::string& ns,
                      const std::string& name)>
      lookup;
};

// Renders all templates into manifests (parsed YAML docs, empty docs dropped, sorted in
// Helm's install order). `values` are the coalesced values (see coalesce_values).
std::vector<Value> render(const Chart& chart, const Value& values, const RenderOptions& o);
std::string render_to_string(const Chart& chart, const Value& values, const RenderOptions& o);
// Rendered templates by path ("<chart>/templates/x.yaml" -> text), NOTES.txt included.
std::vector<std::pair<std::string, std::string>> render_files(const Chart& chart, const Value& values,
                                                              const RenderOptions& o);

// A hook object (`helm.sh/hook` annotation) of a release.
struct Hook {
  std::string name, kind, path, manifest;
  std::vector<std::string> events, delete_policies;
  int weight = 0;
  Value last_run;  // {started_at, completed_at, phase}
};

struct Release {
  std::string name, namespace_, status;  // deployed | failed | superseded | uninstalled | pending-*
  int version = 0;
  std::string chart, chart_version, first_deployed, last_deployed, description, notes;
  Value config;      // user-supplied values
  Value chart_json;  // Helm 3 chart record: metadata, templates, values, files, schema, lock
  std::string manifest;
  std::vector<Hook> hooks;
};

// Helm 3 release JSON (pkg/release/release.go) <-> Release.
Value release_to_json(const Release& r);
Release release_from_json(const Value& v);

class Client {
 public:
  explicit Client(std::shared_ptr<kube::Client> k) : k_(std::move(k)) {}
  std::vector<Release> history(const std::string& ns, const std::string& name);
  bool release_exists(const std::string& ns, const std::string& name);
  std::vector<Release> list(const std::string& ns);
  // Install or upgrade; on failure an upgrade rolls back to the last deployed revision and a
  // first install is purged (helm/install.go:100-166) — unless its only problem is an image
  // pull still in progress: then the failed release is kept and a re-run continues the wait.
  Release install_or_upgrade(const std::string& name, const std::string& ns, const std::string& chart_path,
                             const Value& values, bool wait, int timeout_s);
  void rollback(const std::string& ns, const std::string& name, int to_version);
  // Revisions kept per release after an install/upgrade/rollback (Helm 3's --history-max,
  // default 10; 0 keeps all). Each revision is a Secret holding the gzipped chart, so a long
  // `devspace dev` session with auto-reload would otherwise pile them up.
  void set_max_history(int n) { max_history_ = n; }
  void delete_release(const std::string& ns, const std::string& name, bool purge = true);
  // Outcome of a rollout wait. `err` is "" once every workload is ready. `fatal`: a pod of the
  // release can not start (ErrImagePull, ImagePullBackOff, InvalidImageName, Unschedulable) —
  // reported within seconds, not at the timeout. `pulling`: the wait ran out while a pod was still
  // pulling its image (a first install keeps its release then: the pull goes on in the cluster).
  struct WaitOutcome {
    std::string err;
    bool fatal = false;
    bool pulling = false;
  };
  // Waits for every workload in the manifest to be ready. Pull-aware: past `timeout_s`, a pod
  // whose kubelet reports `Pulling` (and nothing fatal) extends the wait, up to the pull budget
  // (DEVSPACE_PULL_TIMEOUT, default 1800 s, counted from the start of the wait).
  WaitOutcome wait_ready(const std::vector<Value>& objs, const std::string& ns, int timeout_s);
  // .Capabilities from the API server (cached per client).
  Value capabilities();

 private:
  void store(const Release& r);
  // `known`: the revisions this command knows of (its history read plus what it stored); when
  // they fit in max_history_ the list is not read again (one API round trip less per deploy)
  void prune_history(const std::string& ns, const std::string& name, int known = -1);
  int max_history_ = 10;
  // Runs the hooks of one lifecycle event in weight order; throws on a failed hook.
  void run_hooks(std::vector<Hook>& hooks, const std::string& event, const std::string& ns, int timeout_s);
  std::shared_ptr<kube::Client> k_;
  Value caps_;
};

// Values.MergeInto (deploy/helm/merge.go:8): deep merge, `over` wins.
void merge_values(Value& base, const Value& over);

// Helm's install order by kind.
int kind_order(const std::string& kind);

}  // namespace helm
}  // namespace ds

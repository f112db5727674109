// Project configuration: versioned schema, strict parsing, upgrade chain, configs.yaml with
// overrides + variables, generated.yaml runtime cache, save-without-defaults.
//
// Reference: config/versions/versions.go:19 (Parse), config/versions/latest/schema.go:23,
// config/versions/v1alpha1/upgrade.go:14, config/configutil/get.go:104 (load/merge),
// config/configutil/load.go:23-190 (vars), config/configutil/save.go:15 (save),
// config/generated/config.go (generated.yaml), config/configs/schema.go (configs.yaml).
//
// Unlike the reference's process-wide sync.Once singletons (get.go:53-58), all state lives in
// an explicit Context object.
#pragma once

#include <map>
#include <memory>
#include <optional>
#include <stdexcept>
#include <string>
#include <vector>

#include "core/value.h"

namespace ds {
namespace config {

extern const char* const kLatestVersion;  // "v1alpha2"
extern const char* const kDefaultConfigPath;   // ".devspace/config.yaml"
extern const char* const kDefaultConfigsPath;  // ".devspace/configs.yaml"
extern const char* const kDefaultVarsPath;     // ".devspace/vars.yaml"
extern const char* const kGeneratedPath;       // ".devspace/generated.yaml"
extern const char* const kDefaultDeploymentName;  // "devspace-app"
extern const char* const kVarEnvPrefix;        // "DEVSPACE_VAR_"

struct ConfigError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// ---------------------------------------------------------------- schema

struct Schema {
  enum Kind { Str, Int, Bool, Any, Struct, List, Dict } kind = Any;
  std::string type_name;  // for error messages ("latest.SyncConfig")
  std::vector<std::pair<std::string, std::shared_ptr<Schema>>> fields;  // Struct
  std::shared_ptr<Schema> elem;                                          // List / Dict
  const Schema* field(const std::string& k) const;
};

const Schema& schema_latest();
const Schema& schema_v1alpha1();
const Schema& schema_configs();
const Schema& schema_vars();
// Throws ConfigError("field x not found in type T") etc. (yaml.UnmarshalStrict semantics).
void validate_strict(const Value& v, const Schema& s, const std::string& where = "");

// versions.Parse: strict-load any known version and upgrade to latest.
Value parse_versioned(Value data);
// v1alpha1 -> v1alpha2 conversion (config/versions/v1alpha1/upgrade.go:14).
Value upgrade_v1alpha1(const Value& old);

// ---------------------------------------------------------------- generated.yaml

class Generated {
 public:
  static Generated load(const std::string& path = kGeneratedPath);
  void save() const;
  std::string active_config() const;
  void set_active_config(const std::string& name);
  // configs.<active>.dev | deploy with all four cache maps present.
  Value& cache(bool dev);
  Value& vars();
  Value& space();  // may be null
  bool has_space() const;
  void clear_space();
  Value& raw() { return v_; }
  std::string path;

 private:
  Value& active();
  Value v_;
};

// ---------------------------------------------------------------- variables

struct Variable {
  std::string name;
  std::optional<std::string> def, question, regex;
};
// Typed conversion of an answer/env value ("true"/"false"/int) — load.go:34-50.
Value convert_var_value(const std::string& s);

// ---------------------------------------------------------------- loader context

class Context {
 public:
  Context() = default;
  // Config path override (--config flag). Relative to the project root.
  std::string config_path = kDefaultConfigPath;

  bool config_exists() const;
  // Loads the config (base + overrides when with_overrides). Cached; throws ConfigError.
  const Value& get(bool with_overrides = true);
  // The loaded (merged) config for in-memory adjustments by command flags (--namespace,
  // --kube-context, --docker-target, cloud space injection). Not saved.
  Value& mutable_config() {
    get(true);
    return config_;
  }
  // The base config (no overrides), mutable for add/remove/configure commands.
  Value& base();
  // Validation (ValidateOnce, get.go:234) — throws ConfigError with the reference's messages.
  void validate(const Value& cfg) const;
  // Save the base config: defaults/empties stripped, written to config.yaml or back into
  // configs.yaml when the active config is defined inline (save.go:15).
  void save_base();
  Generated& generated();
  void save_generated();
  // Name of the config chosen from configs.yaml ("" when configs.yaml is not used).
  const std::string& loaded_config() const { return loaded_config_; }
  // Fresh config for `init` (latest.New()).
  void init_empty();
  void reset();  // drop cached state (tests)

  // Variables from configs.yaml / vars.yaml, answered up-front (get.go:141-175).
  std::vector<Variable> load_vars_definitions() const;

 private:
  Value load_from_path(const std::string& path);
  Value load_from_value(const Value& data);
  Value resolve_vars(Value raw);
  Value load_wrapper(const Value& wrapper, const std::string& what);
  void ask_questions(const std::vector<Variable>& vars);

  bool loaded_ = false;
  bool loaded_with_overrides_ = false;
  Value config_;  // merged
  Value raw_;     // base
  std::string loaded_config_;
  std::unique_ptr<Generated> generated_;
  std::vector<Variable> var_defs_;
};

// Walk up from cwd to find a directory with `.devspace` (stopping before $HOME) and chdir
// into it (get.go:323). Returns true if found. `devspace.yaml` at a directory also counts.
bool set_devspace_root(std::string* found_dir = nullptr);

// Default namespace: cluster.namespace, else kube context namespace, else "default".
std::string default_namespace(const Value& cfg);
// Selector lookup by name (get.go:363).
const Value* find_selector(const Value& cfg, const std::string& name);

// ---------------------------------------------------------------- typed views

struct LabelSelector {
  std::vector<std::pair<std::string, std::string>> labels;
  std::string to_query() const;  // "a=b,c=d" (sorted)
  bool empty() const { return labels.empty(); }
};
LabelSelector label_selector_from(const Value& v);

struct SelectorRef {
  std::string selector, namespace_, container;
  LabelSelector labels;
};
// Resolve selector/labelSelector/namespace/containerName of a dev.* entry against
// dev.selectors (services/attach.go:75 getSelectorNamespaceLabelSelector). When neither is
// set the default selector is release=<first helm deployment> (services/attach.go:119).
SelectorRef resolve_selector(const Value& cfg, const Value& entry);

std::string first_helm_deployment(const Value& cfg);

}  // namespace config
}  // namespace ds

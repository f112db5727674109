#include "deploy/helm.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <ctime>
#include <map>
#include <regex>
#include <set>
#include <thread>

#include "analyze/analyze.h"
#include "core/codec.h"
#include "core/compat.h"
#include "core/fs.h"
#include "core/log.h"
#include "core/safe_regex.h"
#include "core/strutil.h"
#include "core/trace.h"
#include "core/match.h"
#include "deploy/gotemplate.h"

namespace ds {
namespace helm {

int kind_order(const std::string& kind) {
  static const char* order[] = {"Namespace", "NetworkPolicy", "ResourceQuota", "LimitRange", "PodSecurityPolicy",
                                "PodDisruptionBudget", "ServiceAccount", "Secret", "SecretList", "ConfigMap",
                                "StorageClass", "PersistentVolume", "PersistentVolumeClaim",
                                "CustomResourceDefinition", "ClusterRole", "ClusterRoleList", "ClusterRoleBinding",
                                "ClusterRoleBindingList", "Role", "RoleList", "RoleBinding", "RoleBindingList",
                                "Service", "DaemonSet", "Pod", "ReplicationController", "ReplicaSet", "Deployment",
                                "HorizontalPodAutoscaler", "StatefulSet", "Job", "CronJob", "Ingress", "APIService"};
  for (size_t i = 0; i < sizeof(order) / sizeof(order[0]); ++i)
    if (kind == order[i]) return (int)i;
  return 1000;
}

void merge_values(Value& base, const Value& over) { merge_into(base, over); }

// ============================================================== chart loading

// Helm 3 loader: these names are chart structure, everything else is a `.Files` entry.
static bool special_chart_file(const std::string& rel) {
  return rel == "Chart.yaml" || rel == "values.yaml" || rel == "values.schema.json" || rel == "requirements.yaml" ||
         rel == "requirements.lock" || rel == "Chart.lock" || rel == ".helmignore" || starts_with(rel, "templates/") ||
         starts_with(rel, "charts/");
}

static std::vector<Dependency> parse_requirements(const Value& list) {
  std::vector<Dependency> out;
  for (auto& d : list.items()) {
    Dependency r;
    r.name = d.get("name").as_string();
    r.version = d.get("version").as_string();
    r.repository = d.get("repository").as_string();
    r.condition = d.get("condition").as_string();
    r.alias = d.get("alias").as_string();
    for (auto& t : d.get("tags").items()) r.tags.push_back(t.as_string());
    r.import_values = d.get("import-values").is_seq() ? d.get("import-values") : Value::seq();
    out.push_back(std::move(r));
  }
  return out;
}

Chart load_chart(const std::string& dir) {
  Chart c;
  c.dir = dir;
  std::string cy = fs::join(dir, "Chart.yaml");
  if (!fs::exists(cy)) throw std::runtime_error("Chart.yaml file is missing in " + dir);
  c.metadata = yaml_load_file(cy);
  if (!c.metadata.is_map()) throw std::runtime_error("Chart.yaml in " + dir + " is not a map");
  std::string vy = fs::join(dir, "values.yaml");
  if (fs::exists(vy)) {
    c.values_raw = fs::read_file(vy);
    c.values = yaml_parse(c.values_raw);
  }
  if (!c.values.is_map()) c.values = Value::map();
  if (fs::exists(fs::join(dir, "values.schema.json"))) c.schema = fs::read_file(fs::join(dir, "values.schema.json"));
  // dependencies: Chart.yaml (apiVersion v2) or requirements.yaml (v1)
  if (c.metadata.get("dependencies").is_seq()) {
    c.requirements = parse_requirements(c.metadata.get("dependencies"));
  } else if (fs::exists(fs::join(dir, "requirements.yaml"))) {
    c.requirements = parse_requirements(yaml_load_file(fs::join(dir, "requirements.yaml")).get("dependencies"));
  }
  GitIgnore ignore;
  std::string hi = fs::join(dir, ".helmignore");
  if (fs::exists(hi)) ignore.add_lines(split(fs::read_file(hi), "\n"));
  fs::walk(dir, [&](const std::string& p, const fs::StatInfo& st) {
    if (p == dir) return true;
    std::string rel = fs::relative(dir, p);
    if (rel == "charts") return false;  // subcharts are loaded below
    if (!ignore.empty() && ignore.matches("/" + rel + (st.is_dir ? "/" : ""))) return false;
    if (st.is_dir) return true;
    if (starts_with(rel, "templates/")) {
      // the loader skips hidden files in templates/ (rules.AddDefaults)
      if (!starts_with(fs::basename(rel), ".")) c.templates.emplace_back(rel, fs::read_file(p));
    } else if (!special_chart_file(rel)) {
      c.files.emplace_back(rel, fs::read_file(p));
    }
    return true;
  });
  std::sort(c.templates.begin(), c.templates.end());
  std::sort(c.files.begin(), c.files.end());
  std::string cdir = fs::join(dir, "charts");
  if (fs::is_dir(cdir)) {
    auto entries = fs::list_dir(cdir);
    std::sort(entries.begin(), entries.end(), [](const fs::DirEntry& a, const fs::DirEntry& b) { return a.name < b.name; });
    for (auto& e : entries) {
      std::string sub = fs::join(cdir, e.name);
      if (e.is_dir && fs::exists(fs::join(sub, "Chart.yaml"))) {
        c.dependencies.push_back(load_chart(sub));
      } else if (ends_with(e.name, ".tgz")) {
        // packaged subchart: extract into a temp dir
        std::string data = fs::read_file(sub);
        std::string tmp = fs::make_temp_dir("devspace-chart-");
        GzipReader gz(string_source(&data));
        TarReader tr([&](char* b, size_t n) { return gz.read(b, n); });
        TarEntry te;
        std::string top;
        while (tr.next(&te)) {
          if (te.type != '0' && te.type != '7') continue;
          std::string out = fs::join(tmp, fs::clean("/" + te.name).substr(1));
          fs::write_file(out, tr.read_all());
          if (top.empty()) top = split(te.name, "/")[0];
        }
        if (!top.empty()) {
          // everything the renderer needs is read into memory: the extraction can go
          Chart sub_chart = load_chart(fs::join(tmp, top));
          sub_chart.dir = sub;
          c.dependencies.push_back(std::move(sub_chart));
        }
        fs::remove_all(tmp);
      }
    }
  }
  return c;
}

// ============================================================== values + dependencies

// Helm's coalesce: `over` wins, maps merge recursively, a null in `over` deletes the key.
static void coalesce_into(Value& base, const Value& over) {
  if (!over.is_map()) return;
  if (!base.is_map()) base = Value::map();
  for (auto& e : over.entries()) {
    if (e.second.is_null()) {
      base.erase(e.first);
      continue;
    }
    Value* cur = base.find(e.first);
    if (cur && cur->is_map() && e.second.is_map())
      coalesce_into(*cur, e.second);
    else
      base[e.first] = e.second;
  }
}

// CoalesceTables(dst, src): keys missing in dst are filled from src; dst wins.
static void fill_missing(Value& dst, const Value& src) {
  if (!src.is_map()) return;
  if (!dst.is_map()) dst = Value::map();
  for (auto& e : src.entries()) {
    Value* cur = dst.find(e.first);
    if (!cur)
      dst[e.first] = e.second;
    else if (cur->is_map() && e.second.is_map())
      fill_missing(*cur, e.second);
  }
}

Value coalesce_values(const Chart& c, const Value& user_values) {
  Value v = c.values.is_map() ? c.values : Value::map();
  coalesce_into(v, user_values);
  for (auto& d : c.dependencies) {
    Value sub = coalesce_values(d, v.get(d.name()));
    const Value& g = v.get("global");
    if (g.is_map()) {  // the parent's globals reach every subchart and win over the subchart's own
      Value sg = sub.get("global").is_map() ? sub.get("global") : Value::map();
      coalesce_into(sg, g);
      sub["global"] = sg;
    }
    v[d.name()] = sub;
  }
  return v;
}

static bool version_compatible(const std::string& constraint, const std::string& version) {
  if (constraint.empty() || version.empty()) return true;
  try {
    return tmpl::semver_match(constraint, version);
  } catch (const std::exception&) {
    return constraint == version;
  }
}

// processDependencyEnabled: alias copies, then tags and conditions against the coalesced
// values of the whole tree (`top`), with `path` the chart's position in it ("" or "sub.").
static void dependency_enabled(Chart& c, const Value& top, const std::string& path) {
  if (c.requirements.empty()) return;
  std::vector<Chart> deps;
  for (auto& ex : c.dependencies) {
    bool listed = false;
    for (auto& r : c.requirements) listed |= ex.name() == r.name && version_compatible(r.version, ex.version());
    if (!listed) deps.push_back(ex);  // charts/ entries no requirement names stay enabled
  }
  for (auto& r : c.requirements) {
    for (auto& ex : c.dependencies) {
      if (ex.name() != r.name || !version_compatible(r.version, ex.version())) continue;
      Chart copy = ex;
      if (!r.alias.empty()) copy.metadata["name"] = r.alias;
      deps.push_back(std::move(copy));
      break;
    }
    if (!r.alias.empty()) r.name = r.alias;
    r.enabled = true;
  }
  c.dependencies = std::move(deps);
  const Value& tags = top.get("tags");
  for (auto& r : c.requirements) {
    bool has_true = false, has_false = false;
    for (auto& t : r.tags) {
      const Value* b = tags.is_map() ? tags.find(t) : nullptr;
      if (b && b->is_bool()) (b->as_bool() ? has_true : has_false) = true;
    }
    if (!has_true && has_false) r.enabled = false;
    for (auto& cond : split(r.condition, ",")) {
      std::string k = trim(cond);
      if (k.empty()) continue;
      const Value& v = top.at_path(path + k);
      if (v.is_bool()) {
        r.enabled = v.as_bool();
        break;
      }
    }
  }
  std::set<std::string> off;
  for (auto& r : c.requirements)
    if (!r.enabled) off.insert(r.name);
  std::vector<Chart> keep;
  for (auto& d : c.dependencies)
    if (!off.count(d.name())) keep.push_back(std::move(d));
  c.dependencies = std::move(keep);
  for (auto& d : c.dependencies) dependency_enabled(d, top, path + d.name() + ".");
}

static Value path_to_map(const std::string& path, const Value& data) {
  if (path.empty() || path == ".") return data;
  Value out = Value::map();
  Value* cur = &out;
  auto parts = split(path, ".");
  for (size_t i = 0; i < parts.size(); ++i) {
    if (parts[i].empty()) continue;
    if (i + 1 == parts.size())
      (*cur)[parts[i]] = data;
    else
      cur = &(*cur)[parts[i]];
  }
  return out;
}

// processImportValues (bottom-up): child values copied into the parent's values; the
// parent's own values take precedence over imported ones.
static void import_values(Chart& c) {
  for (auto& d : c.dependencies) import_values(d);
  bool any = false;
  for (auto& r : c.requirements) any |= r.import_values.size() > 0;
  if (!any) return;
  Value cvals = coalesce_values(c, Value::map());
  Value b = Value::map();
  for (auto& r : c.requirements) {
    if (!r.enabled) continue;
    for (auto& iv : r.import_values.items()) {
      if (iv.is_map()) {
        const Value& vv = cvals.at_path(r.name + "." + iv.get("child").as_string());
        if (vv.is_map()) fill_missing(b, path_to_map(iv.get("parent").as_string(), vv));
      } else if (iv.is_string()) {
        const Value& vm = cvals.at_path(r.name + ".exports." + iv.as_string());
        if (vm.is_map()) fill_missing(b, vm);
      }
    }
  }
  Value nv = c.values;
  fill_missing(nv, b);
  c.values = nv;
}

void process_dependencies(Chart& c, const Value& user_values) {
  dependency_enabled(c, coalesce_values(c, user_values), "");
  import_values(c);
}

// ============================================================== values.schema.json

namespace {

std::string json_type_of(const Value& v) {
  switch (v.type()) {
    case Value::Type::Null: return "null";
    case Value::Type::Bool: return "boolean";
    case Value::Type::Int: return "integer";
    case Value::Type::Float: return v.as_double() == std::floor(v.as_double()) ? "integer" : "number";
    case Value::Type::String: return "string";
    case Value::Type::Seq: return "array";
    case Value::Type::Map: return "object";
  }
  return "null";
}

bool type_matches(const Value& v, const std::string& t) {
  std::string vt = json_type_of(v);
  return vt == t || (t == "number" && vt == "integer");
}

// JSON Schema (draft-07 subset Helm charts use): type, enum, const, required, properties,
// additionalProperties, patternProperties, items, min/maxItems, uniqueItems, minimum/maximum
// (+exclusive), multipleOf, min/maxLength, pattern, allOf/anyOf/oneOf/not, $ref into
// #/definitions or #/$defs. Errors are "path: message" lines like Helm's gojsonschema output.
void validate_schema(const Value& v, const Value& schema, const Value& root, const std::string& path,
                     std::vector<std::string>* errs, int depth = 0) {
  if (!schema.is_map() || depth > 64) return;
  auto err = [&](const std::string& m) { errs->push_back((path.empty() ? "(root)" : path) + ": " + m); };
  if (schema.has("$ref")) {
    std::string ref = schema.get("$ref").as_string();
    if (starts_with(ref, "#/")) {
      const Value* cur = &root;
      for (auto& part : split(ref.substr(2), "/")) {
        cur = cur->is_map() ? cur->find(part) : nullptr;
        if (!cur) break;
      }
      if (cur) validate_schema(v, *cur, root, path, errs, depth + 1);
    }
  }
  const Value& type = schema.get("type");
  if (!type.is_null()) {
    bool ok = false;
    if (type.is_seq()) {
      for (auto& t : type.items()) ok |= type_matches(v, t.as_string());
    } else {
      ok = type_matches(v, type.as_string());
    }
    if (!ok) {
      err("Invalid type. Expected: " + (type.is_seq() ? json_dump(type) : type.as_string()) + ", given: " +
          json_type_of(v));
      return;
    }
  }
  if (schema.get("enum").is_seq()) {
    bool ok = false;
    for (auto& e : schema.get("enum").items()) ok |= e == v || (e.is_number() && v.is_number() && e.as_double() == v.as_double());
    if (!ok) err("must be one of the following: " + json_dump(schema.get("enum")));
  }
  if (schema.has("const") && !(schema.get("const") == v)) err("does not match: " + json_dump(schema.get("const")));
  if (v.is_map()) {
    for (auto& r : schema.get("required").items())
      if (!v.has(r.as_string())) err(r.as_string() + " is required");
    const Value& props = schema.get("properties");
    const Value& pprops = schema.get("patternProperties");
    for (auto& e : v.entries()) {
      std::string sub = path.empty() ? e.first : path + "." + e.first;
      bool known = false;
      if (const Value* ps = props.is_map() ? props.find(e.first) : nullptr) {
        known = true;
        validate_schema(e.second, *ps, root, sub, errs, depth + 1);
      }
      for (auto& pp : pprops.entries()) {
        try {
          if (safe_regex_search(e.first, std::regex(pp.first))) {
            known = true;
            validate_schema(e.second, pp.second, root, sub, errs, depth + 1);
          }
        } catch (const std::regex_error&) {
        }
      }
      if (known) continue;
      const Value& ap = schema.get("additionalProperties");
      if (ap.is_bool() && !ap.as_bool())
        err("Additional property " + e.first + " is not allowed");
      else if (ap.is_map())
        validate_schema(e.second, ap, root, sub, errs, depth + 1);
    }
    if (schema.has("minProperties") && (int64_t)v.size() < schema.get("minProperties").as_int())
      err("must have at least " + schema.get("minProperties").as_string() + " properties");
  }
  if (v.is_seq()) {
    if (schema.has("minItems") && (int64_t)v.size() < schema.get("minItems").as_int())
      err("Array must have at least " + schema.get("minItems").as_string() + " items");
    if (schema.has("maxItems") && (int64_t)v.size() > schema.get("maxItems").as_int())
      err("Array must have at most " + schema.get("maxItems").as_string() + " items");
    if (schema.get("uniqueItems").as_bool(false))
      for (size_t i = 0; i < v.size(); ++i)
        for (size_t j = i + 1; j < v.size(); ++j)
          if (v[i] == v[j]) err("array items[" + std::to_string(i) + "," + std::to_string(j) + "] must be unique");
    if (schema.get("items").is_map())
      for (size_t i = 0; i < v.size(); ++i)
        validate_schema(v[i], schema.get("items"), root, path + "." + std::to_string(i), errs, depth + 1);
  }
  if (v.is_number()) {
    double x = v.as_double();
    if (schema.has("minimum") && x < schema.get("minimum").as_double())
      err("Must be greater than or equal to " + schema.get("minimum").as_string());
    if (schema.has("maximum") && x > schema.get("maximum").as_double())
      err("Must be less than or equal to " + schema.get("maximum").as_string());
    if (schema.get("exclusiveMinimum").is_number() && x <= schema.get("exclusiveMinimum").as_double())
      err("Must be greater than " + schema.get("exclusiveMinimum").as_string());
    if (schema.get("exclusiveMaximum").is_number() && x >= schema.get("exclusiveMaximum").as_double())
      err("Must be less than " + schema.get("exclusiveMaximum").as_string());
    if (schema.has("multipleOf") && schema.get("multipleOf").as_double() > 0) {
      double q = x / schema.get("multipleOf").as_double();
      if (std::fabs(q - std::round(q)) > 1e-9) err("Must be a multiple of " + schema.get("multipleOf").as_string());
    }
  }
  if (v.is_string()) {
    size_t n = 0;
    for (unsigned char c : v.str()) n += (c & 0xC0) != 0x80;  // code points
    if (schema.has("minLength") && (int64_t)n < schema.get("minLength").as_int())
      err("String length must be greater than or equal to " + schema.get("minLength").as_string());
    if (schema.has("maxLength") && (int64_t)n > schema.get("maxLength").as_int())
      err("String length must be less than or equal to " + schema.get("maxLength").as_string());
    if (schema.has("pattern")) {
      try {
        if (!safe_regex_search(v.str(), std::regex(schema.get("pattern").as_string(), std::regex::ECMAScript)))
          err("Does not match pattern '" + schema.get("pattern").as_string() + "'");
      } catch (const std::regex_error&) {
      }
    }
  }
  for (auto& s : schema.get("allOf").items()) validate_schema(v, s, root, path, errs, depth + 1);
  auto passes = [&](const Value& s) {
    std::vector<std::string> e;
    validate_schema(v, s, root, path, &e, depth + 1);
    return e.empty();
  };
  if (schema.get("anyOf").is_seq()) {
    bool any = false;
    for (auto& s : schema.get("anyOf").items()) any |= passes(s);
    if (!any) err("Must validate at least one schema (anyOf)");
  }
  if (schema.get("oneOf").is_seq()) {
    int n = 0;
    for (auto& s : schema.get("oneOf").items()) n += passes(s);
    if (n != 1) err("Must validate one and only one schema (oneOf)");
  }
  if (schema.get("not").is_map() && passes(schema.get("not"))) err("Must not validate the schema (not)");
}

void validate_chart_values(const Chart& c, const Value& values, std::string* report) {
  if (!c.schema.empty()) {
    Value schema;
    try {
      schema = json_parse(c.schema);
    } catch (const std::exception& e) {
      *report += c.name() + ":\n- values.schema.json: " + e.what() + "\n";
    }
    std::vector<std::string> errs;
    validate_schema(values, schema, schema, "", &errs);
    if (!errs.empty()) {
      *report += c.name() + ":\n";
      for (auto& e : errs) *report += "- " + e + "\n";
    }
  }
  for (auto& d : c.dependencies) validate_chart_values(d, values.get(d.name()), report);
}

}  // namespace

void validate_values(const Chart& chart, const Value& coalesced_values) {
  std::string report;
  validate_chart_values(chart, coalesced_values, &report);
  if (!report.empty())
    throw std::runtime_error("values don't meet the specifications of the schema(s) in the following chart(s):\n" +
                             report);
}

// ============================================================== rendering

static bool mentions_capabilities(const Chart& c) {
  for (auto& t : c.templates)
    if (t.second.find("Capabilities") != std::string::npos) return true;
  for (auto& d : c.dependencies)
    if (mentions_capabilities(d)) return true;
  return false;
}

static const char* kHelmVersion = "v3.14.0";

static Value capabilities_value(const Value& in) {
  Value caps = Value::map();
  const Value& kv = in.get("KubeVersion");
  std::string git = kv.get("GitVersion").as_string("v1.29.0");
  caps["KubeVersion"]["Major"] = kv.get("Major").as_string("1");
  caps["KubeVersion"]["Minor"] = kv.get("Minor").as_string("29");
  caps["KubeVersion"]["GitVersion"] = git;
  caps["KubeVersion"]["Version"] = git;
  std::vector<std::string> apis;
  for (auto& a : in.get("APIVersions").items()) apis.push_back(a.as_string());
  if (apis.empty())
    apis = {"v1", "apps/v1", "batch/v1", "rbac.authorization.k8s.io/v1", "autoscaling/v1", "autoscaling/v2",
            "networking.k8s.io/v1", "policy/v1", "storage.k8s.io/v1", "apiextensions.k8s.io/v1"};
  caps["APIVersions"] = tmpl::make_api_versions_object(apis);
  caps["HelmVersion"]["Version"] = kHelmVersion;
  caps["HelmVersion"]["GitCommit"] = "";
  caps["HelmVersion"]["GoVersion"] = "";
  return caps;
}

static void add_templates(tmpl::Engine& eng, const Chart& c, const std::string& prefix) {
  for (auto& t : c.templates) eng.add(prefix + t.first, t.second);
  for (auto& d : c.dependencies) add_templates(eng, d, prefix + "charts/" + d.name() + "/");
}

static Value chart_object(const Chart& c) {
  Value chart = Value::map();
  for (auto& e : c.metadata.entries()) {
    std::string k = e.first;
    if (k == "apiVersion") k = "APIVersion";
    if (!k.empty()) k[0] = (char)std::toupper((unsigned char)k[0]);
    chart[k] = e.second;
  }
  return chart;
}

static void render_chart(tmpl::Engine& eng, const Chart& c, const Value& values, const RenderOptions& o,
                         const Value& caps, const std::string& prefix, bool top,
                         std::vector<std::pair<std::string, std::string>>* out) {
  Value dot = Value::map();
  dot["Values"] = values;
  Value rel = Value::map();
  rel["Name"] = o.release_name;
  rel["Namespace"] = o.namespace_;
  rel["Service"] = "Helm";
  rel["IsInstall"] = o.is_install;
  rel["IsUpgrade"] = !o.is_install;
  rel["Revision"] = o.revision;
  rel["Time"] = log::rfc3339_now();
  dot["Release"] = rel;
  dot["Chart"] = chart_object(c);
  dot["Capabilities"] = caps;
  dot["Files"] = tmpl::make_files_object(c.files);
  if (!c.is_library()) {  // library charts only contribute their defines
    for (auto& t : c.templates) {
      std::string base = fs::basename(t.first);
      bool notes = top && t.first == "templates/NOTES.txt";
      if (starts_with(base, "_")) continue;  // partials
      if (!notes && !ends_with(base, ".yaml") && !ends_with(base, ".yml") && !ends_with(base, ".json")) continue;
      Value d = dot;
      d["Template"]["Name"] = c.name() + "/" + t.first;
      d["Template"]["BasePath"] = c.name() + "/templates";
      out->emplace_back(prefix + t.first, eng.execute(prefix + t.first, d));
    }
  }
  for (auto& dep : c.dependencies) {
    // idempotent on already-coalesced values; also accepts plain user values
    Value sub = coalesce_values(dep, values.get(dep.name()));
    if (values.get("global").is_map()) {
      Value sg = sub.get("global").is_map() ? sub.get("global") : Value::map();
      coalesce_into(sg, values.get("global"));
      sub["global"] = sg;
    }
    render_chart(eng, dep, sub, o, caps, prefix + "charts/" + dep.name() + "/", false, out);
  }
}

std::vector<std::pair<std::string, std::string>> render_files(const Chart& chart, const Value& values,
                                                              const RenderOptions& o) {
  tmpl::Engine eng;
  if (o.lookup) eng.lookup = o.lookup;
  add_templates(eng, chart, "");
  std::vector<std::pair<std::string, std::string>> out;
  render_chart(eng, chart, values, o, capabilities_value(o.capabilities), "", true, &out);
  for (auto& kv : out) kv.first = chart.name() + "/" + kv.first;
  return out;
}

// SplitManifests: documents of one rendered file, separated by "---" lines.
static std::vector<std::string> split_documents(const std::string& text) {
  std::vector<std::string> docs;
  std::string cur;
  for (auto& line : split(text, "\n")) {
    if (starts_with(line, "---") && trim(line.substr(3)).empty()) {
      docs.push_back(cur);
      cur.clear();
      continue;
    }
    cur += line + "\n";
  }
  docs.push_back(cur);
  std::vector<std::string> out;
  for (auto& d : docs) {
    std::string t = trim(d);
    bool only_comments = true;
    for (auto& l : split(t, "\n"))
      if (!trim(l).empty() && !starts_with(trim(l), "#")) only_comments = false;
    if (!only_comments) out.push_back(trim_right(d, " \t\r\n"));
  }
  return out;
}

std::string render_to_string(const Chart& chart, const Value& values, const RenderOptions& o) {
  std::string all;
  for (auto& kv : render_files(chart, values, o)) {
    if (ends_with(kv.first, "/NOTES.txt")) continue;
    for (auto& doc : split_documents(kv.second)) all += "---\n# Source: " + kv.first + "\n" + doc + "\n";
  }
  return all;
}

std::vector<Value> render(const Chart& chart, const Value& values, const RenderOptions& o) {
  std::string text = render_to_string(chart, values, o);
  std::vector<Value> objs;
  for (auto& d : yaml_parse_all(text)) {
    if (!d.is_map() || d.get("kind").is_null()) continue;
    objs.push_back(d);
  }
  std::stable_sort(objs.begin(), objs.end(), [](const Value& a, const Value& b) {
    return kind_order(a.get("kind").as_string()) < kind_order(b.get("kind").as_string());
  });
  return objs;
}

// ============================================================== release storage (Helm 3)

static std::string secret_name(const std::string& name, int v) {
  return "sh.helm.release.v1." + name + ".v" + std::to_string(v);
}

static Value file_list(const std::vector<std::pair<std::string, std::string>>& files) {
  Value l = Value::seq();
  for (auto& f : files) {
    Value e = Value::map();
    e["name"] = f.first;
    e["data"] = base64_encode(f.second);  // []byte marshals as base64
    l.push(e);
  }
  return l;
}

static Value chart_record(const Chart& c) {
  Value ch = Value::map();
  ch["metadata"] = c.metadata;
  ch["lock"] = Value();
  ch["templates"] = file_list(c.templates);
  ch["values"] = c.values;
  ch["schema"] = c.schema.empty() ? Value() : Value(base64_encode(c.schema));
  ch["files"] = file_list(c.files);
  return ch;
}

Value release_to_json(const Release& r) {
  Value v = Value::map();
  v["name"] = r.name;
  Value info = Value::map();
  info["first_deployed"] = r.first_deployed.empty() ? r.last_deployed : r.first_deployed;
  info["last_deployed"] = r.last_deployed;
  info["deleted"] = r.status == "uninstalled" ? Value(log::rfc3339_now()) : Value("0001-01-01T00:00:00Z");
  if (!r.description.empty()) info["description"] = r.description;
  info["status"] = r.status;
  if (!r.notes.empty()) info["notes"] = r.notes;
  v["info"] = info;
  Value ch = r.chart_json;
  if (!ch.is_map()) {
    ch = Value::map();
    ch["metadata"]["name"] = r.chart;
    ch["metadata"]["version"] = r.chart_version;
    ch["lock"] = Value();
    ch["templates"] = Value::seq();
    ch["values"] = Value::map();
    ch["schema"] = Value();
    ch["files"] = Value::seq();
  }
  v["chart"] = ch;
  if (r.config.is_map() && r.config.size()) v["config"] = r.config;
  if (!r.manifest.empty()) v["manifest"] = r.manifest;
  if (!r.hooks.empty()) {
    Value hs = Value::seq();
    for (auto& h : r.hooks) {
      Value e = Value::map();
      e["name"] = h.name;
      e["kind"] = h.kind;
      e["path"] = h.path;
      e["manifest"] = h.manifest;
      e["events"] = Value::strings(h.events);
      e["last_run"] = h.last_run.is_map() ? h.last_run : Value::map();
      if (h.weight) e["weight"] = h.weight;
      if (!h.delete_policies.empty()) e["delete_policies"] = Value::strings(h.delete_policies);
      hs.push(e);
    }
    v["hooks"] = hs;
  }
  v["version"] = r.version;
  v["namespace"] = r.namespace_;
  return v;
}

Release release_from_json(const Value& v) {
  Release r;
  r.name = v.get("name").as_string();
  r.namespace_ = v.get("namespace").as_string();
  r.version = (int)v.get("version").as_int();
  r.status = v.at_path("info.status").as_string();
  r.first_deployed = v.at_path("info.first_deployed").as_string();
  r.last_deployed = v.at_path("info.last_deployed").as_string();
  r.description = v.at_path("info.description").as_string();
  r.notes = v.at_path("info.notes").as_string();
  r.chart = v.at_path("chart.metadata.name").as_string();
  r.chart_version = v.at_path("chart.metadata.version").as_string();
  r.chart_json = v.get("chart");
  r.config = v.get("config").is_map() ? v.get("config") : Value::map();
  r.manifest = v.get("manifest").as_string();
  for (auto& h : v.get("hooks").items()) {
    Hook k;
    k.name = h.get("name").as_string();
    k.kind = h.get("kind").as_string();
    k.path = h.get("path").as_string();
    k.manifest = h.get("manifest").as_string();
    for (auto& e : h.get("events").items()) k.events.push_back(e.as_string());
    for (auto& e : h.get("delete_policies").items()) k.delete_policies.push_back(e.as_string());
    k.weight = (int)h.get("weight").as_int(0);
    k.last_run = h.get("last_run");
    r.hooks.push_back(std::move(k));
  }
  return r;
}

static Release decode_release(const Value& secret) {
  std::string data = secret.at_path("data.release").as_string();
  return release_from_json(json_parse(gzip_decompress(base64_decode(base64_decode(data)))));
}

void Client::store(const Release& r) {
  Value s = Value::map();
  s["apiVersion"] = "v1";
  s["kind"] = "Secret";
  s["type"] = "helm.sh/release.v1";
  s["metadata"]["name"] = secret_name(r.name, r.version);
  s["metadata"]["namespace"] = r.namespace_;
  s["metadata"]["labels"]["owner"] = "helm";
  s["metadata"]["labels"]["name"] = r.name;
  s["metadata"]["labels"]["status"] = r.status;
  s["metadata"]["labels"]["version"] = std::to_string(r.version);
  s["metadata"]["labels"]["modifiedAt"] = std::to_string((long long)time(nullptr));
  // Helm 3 stores base64(gzip(json)) inside Secret data (itself base64 on the wire)
  s["data"]["release"] = base64_encode(base64_encode(gzip_compress(json_dump(release_to_json(r)))));
  k_->apply(s, r.namespace_);
}

// Helm 3 (pkg/action/upgrade.go + storage.removeLeastRecent): delete the oldest revisions
// beyond max_history_, never the deployed one.
void Client::prune_history(const std::string& ns, const std::string& name, int known) {
  if (max_history_ <= 0) return;
  // (a revision another client stored meanwhile is pruned by the next deploy)
  if (known >= 0 && known <= max_history_) return;
  Value list = k_->get("/api/v1/namespaces/" + ns + "/secrets?labelSelector=" +
                       net::url_encode("owner=helm,name=" + name));
  std::vector<std::pair<int, std::pair<std::string, std::string>>> revs;  // version, (secret, status)
  for (auto& s : list.get("items").items())
    revs.push_back({(int)std::atoi(s.at_path("metadata.labels.version").as_string("0").c_str()),
                    {s.at_path("metadata.name").as_string(), s.at_path("metadata.labels.status").as_string()}});
  std::sort(revs.begin(), revs.end());
  int excess = (int)revs.size() - max_history_;
  for (auto& r : revs) {
    if (excess <= 0) break;
    if (r.second.second == "deployed") continue;
    try {
      k_->del("/api/v1/namespaces/" + ns + "/secrets/" + r.second.first);
      --excess;
    } catch (const std::exception& e) {
      log::warn("Could not prune release revision " + r.second.first + ": " + e.what());
      return;
    }
  }
}

std::vector<Release> Client::history(const std::string& ns, const std::string& name) {
  std::vector<Release> out;
  Value list = k_->get("/api/v1/namespaces/" + ns + "/secrets?labelSelector=" +
                       net::url_encode("owner=helm,name=" + name));
  for (auto& s : list.get("items").items()) {
    try {
      out.push_back(decode_release(s));
    } catch (...) {
    }
  }
  std::sort(out.begin(), out.end(), [](const Release& a, const Release& b) { return a.version < b.version; });
  return out;
}

bool Client::release_exists(const std::string& ns, const std::string& name) {
  for (auto& r : history(ns, name))
    if (r.status == "deployed") return true;
  return false;
}

std::vector<Release> Client::list(const std::string& ns) {
  std::map<std::string, Release> latest;
  Value list = k_->get("/api/v1/namespaces/" + ns + "/secrets?labelSelector=" + net::url_encode("owner=helm"));
  for (auto& s : list.get("items").items()) {
    try {
      Release r = decode_release(s);
      if (!latest.count(r.name) || latest[r.name].version < r.version) latest[r.name] = r;
    } catch (...) {
    }
  }
  std::vector<Release> out;
  for (auto& kv : latest) out.push_back(kv.second);
  return out;
}

Value Client::capabilities() {
  if (caps_.is_map()) return caps_;
  Value c = Value::map();
  try {
    Value ver = k_->get("/version");
    std::string minor = ver.get("minor").as_string();
    while (!minor.empty() && !std::isdigit((unsigned char)minor.back())) minor.pop_back();  // "29+" (GKE/EKS)
    c["KubeVersion"]["Major"] = ver.get("major").as_string();
    c["KubeVersion"]["Minor"] = minor;
    c["KubeVersion"]["GitVersion"] = ver.get("gitVersion").as_string();
  } catch (const std::exception& e) {
    log::debug(std::string("capabilities: /version: ") + e.what());
  }
  std::vector<std::string> apis;
  try {
    Value core = k_->get("/api"), groups = k_->get("/apis");  // keep the documents alive while iterating
    for (auto& v : core.get("versions").items()) apis.push_back(v.as_string());
    for (auto& g : groups.get("groups").items())
      for (auto& gv : g.get("versions").items()) apis.push_back(gv.get("groupVersion").as_string());
  } catch (const std::exception& e) {
    log::debug(std::string("capabilities: discovery: ") + e.what());
  }
  c["APIVersions"] = Value::strings(apis);
  caps_ = c;
  return caps_;
}

// helm.sh/resource-policy: keep — Helm never deletes such an object on uninstall or when an
// upgrade drops it from the chart (typically PersistentVolumeClaims holding data).
static bool keep_on_delete(const Value& o) {
  return o.at_path("metadata.annotations").get("helm.sh/resource-policy").as_string() == "keep";
}

static std::string object_key(const Value& o) {
  return o.get("apiVersion").as_string() + "/" + o.get("kind").as_string() + "/" +
         o.at_path("metadata.namespace").as_string() + "/" + o.at_path("metadata.name").as_string();
}

// Readiness of one workload object as `kubectl rollout status` sees it; "" when ready.
static std::string not_ready_reason(const std::string& kind, const std::string& name, const std::optional<Value>& cur) {
  if (!cur) return kind + " " + name + " not found";
  if (kind == "PersistentVolumeClaim")
    return cur->at_path("status.phase").as_string() == "Bound" ? "" : "PVC " + name + " not bound";
  // The controller must have seen the new spec before readiness counts (rollout status).
  if (kind != "ReplicaSet" &&
      cur->at_path("status.observedGeneration").as_int(0) < cur->at_path("metadata.generation").as_int(1))
    return kind + " " + name + ": waiting for the controller to observe generation " +
           std::to_string(cur->at_path("metadata.generation").as_int(1));
  int64_t want = cur->at_path("spec.replicas").as_int(1);
  if (kind == "DaemonSet") want = cur->at_path("status.desiredNumberScheduled").as_int(1);
  if (kind == "Deployment" && cur->at_path("status.updatedReplicas").as_int(0) < want)
    return kind + " " + name + ": " + std::to_string(cur->at_path("status.updatedReplicas").as_int(0)) + "/" +
           std::to_string(want) + " updated";
  int64_t ready = cur->at_path("status.readyReplicas").as_int(0);
  if (kind == "DaemonSet") ready = cur->at_path("status.numberReady").as_int(0);
  if (ready < want) return kind + " " + name + ": " + std::to_string(ready) + "/" + std::to_string(want) + " ready";
  return "";
}

// What the pods of one workload are doing, for the rollout wait: a reason they can never start
// (fail fast instead of waiting out the timeout), or an image pull in progress (worth waiting
// for: a first pull of a tens-of-GB rocm/pytorch image onto a fresh node takes minutes).
struct PodProgress {
  std::string fatal;  // "pod p: container c: ImagePullBackOff: <message>" / "pod p: Unschedulable: ..."
  std::string pulling;  // "pod p: Pulling image \"x\"" ("" if none pulls)
  int64_t pulling_since = 0;  // unix seconds of the oldest pull in progress
};

static int64_t event_time(const std::string& ts) {
  struct tm t{};
  if (ts.size() < 19 || !strptime(ts.c_str(), "%Y-%m-%dT%H:%M:%S", &t)) return 0;
  return (int64_t)timegm(&t);
}

static bool pull_failure_reason(const std::string& r) {
  return r == "ErrImagePull" || r == "ImagePullBackOff" || r == "InvalidImageName" || r == "ErrImageNeverPull";
}

// A pull error no retry fixes: the image or tag does not exist, the name is invalid, access is
// denied, or the pod may not pull at all. Anything else (a registry timeout, a 5xx, a reset
// connection, a 429) is retried by the kubelet's back-off and may still succeed.
static bool permanent_pull_error(const std::string& reason, const std::string& msg_in) {
  if (reason == "InvalidImageName" || reason == "ErrImageNeverPull") return true;
  std::string m = to_lower(msg_in);
  for (const char* p : {"not found", "manifest unknown", "does not exist", "repository does not exist",
                        "unauthorized", "denied", "invalid reference format", "no such host"})
    if (contains(m, p)) return true;
  return false;
}

static int env_seconds(const char* name, int def) {
  const char* v = getenv(name);
  int s = v && *v ? atoi(v) : def;
  return s >= 0 ? s : def;
}

// What the rollout wait saw on earlier polls: when a pod first showed a condition that may yet
// clear up (Unschedulable while the cluster autoscaler adds a node, a pull error the kubelet is
// retrying), so it is called fatal only once it has lasted.
struct ProgressMemory {
  std::map<std::string, std::chrono::steady_clock::time_point> first_seen;
  std::map<std::string, std::string> pull_error;  // pod/container -> last ErrImagePull message
  std::set<std::string> told;
  double seen_for(const std::string& key) {
    auto now = std::chrono::steady_clock::now();
    auto it = first_seen.emplace(key, now).first;
    return std::chrono::duration<double>(now - it->second).count();
  }
};

static std::string match_labels_selector(const Value& workload) {
  std::vector<std::string> parts;
  for (auto& kv : workload.at_path("spec.selector.matchLabels").entries())
    parts.push_back(kv.first + "=" + kv.second.as_string());
  return join(parts, ",");
}

static Value pod_events(kube::Client& k, const std::string& ns, const std::string& pod) {
  try {
    return k.get("/api/v1/namespaces/" + ns + "/events?fieldSelector=" +
                 net::url_encode("involvedObject.kind=Pod,involvedObject.name=" + pod));
  } catch (const std::exception&) {
    return Value::map();
  }
}

static PodProgress pod_progress(kube::Client& k, const Value& workload, const std::string& ns,
                                ProgressMemory& mem) {
  PodProgress out;
  std::string sel = match_labels_selector(workload);
  if (sel.empty()) return out;
  std::vector<Value> pods;
  try {
    pods = k.list_pods(ns, sel);
  } catch (const std::exception&) {
    return out;
  }
  // Unschedulable: a node may be on its way (a cluster autoscaler scales GPU node pools from
  // zero: minutes). Fatal only once it lasted DEVSPACE_UNSCHEDULABLE_GRACE_S (10) with no
  // TriggeredScaleUp event for the pod; with one, the wait runs to its timeout.
  const int unsched_grace = env_seconds("DEVSPACE_UNSCHEDULABLE_GRACE_S", 10);
  // ErrImagePull / ImagePullBackOff of an error the kubelet may yet get past (a registry
  // timeout): fatal once it lasted DEVSPACE_PULL_ERROR_GRACE_S (30); a missing image at once.
  const int pull_grace = env_seconds("DEVSPACE_PULL_ERROR_GRACE_S", 30);
  std::vector<const Value*> creating;
  for (auto& p : pods) {
    if (!p.at_path("metadata.deletionTimestamp").is_null()) continue;
    std::string pn = p.at_path("metadata.name").as_string();
    for (auto& c : p.at_path("status.conditions").items())
      if (c.get("type").as_string() == "PodScheduled" && c.get("status").as_string() == "False" &&
          c.get("reason").as_string() == "Unschedulable") {
        std::string msg = "pod " + pn + ": Unschedulable: " + c.get("message").as_string();
        double lasted = mem.seen_for("unsched/" + pn);
        std::string scale_up;
        Value evs = pod_events(k, ns, pn);  // (not iterated as a temporary: it would dangle)
        for (auto& e : evs.get("items").items())
          if (e.get("reason").as_string() == "TriggeredScaleUp") scale_up = e.get("message").as_string();
        if (!scale_up.empty()) {
          if (mem.told.insert("scaleup/" + pn).second)
            log::info(msg + "; the cluster autoscaler is adding a node (" + scale_up + "): waiting");
          return out;
        }
        if (lasted >= unsched_grace) out.fatal = msg;
        return out;
      }
    bool waiting_create = false;
    for (const char* field : {"status.initContainerStatuses", "status.containerStatuses"})
      for (auto& cs : p.at_path(field).items()) {
        std::string r = cs.at_path("state.waiting.reason").as_string();
        std::string cname = cs.get("name").as_string();
        std::string wmsg = cs.at_path("state.waiting.message").as_string();
        if (pull_failure_reason(r)) {
          std::string key = pn + "/" + cname;
          if (r == "ErrImagePull" && !wmsg.empty()) mem.pull_error[key] = wmsg;
          std::string why = mem.pull_error.count(key) ? mem.pull_error[key] : wmsg;
          if (why.empty() || r == "ImagePullBackOff") {
            // the back-off message says nothing about the cause: the kubelet's Failed event does
            Value evs = pod_events(k, ns, pn);
            for (auto& e : evs.get("items").items())
              if (e.get("reason").as_string() == "Failed" && contains(e.get("message").as_string(), "ull image"))
                why = e.get("message").as_string();
          }
          double lasted = mem.seen_for("pull/" + key);
          if (permanent_pull_error(r, why) || lasted >= pull_grace) {
            out.fatal = "pod " + pn + ": container " + cname + ": " + r + (wmsg.empty() ? "" : ": " + wmsg) +
                        (why.empty() || why == wmsg ? "" : " (" + why + ")");
            return out;
          }
          if (mem.told.insert("pullretry/" + key).second)
            log::info("pod " + pn + ": container " + cname + ": " + r + (why.empty() ? "" : " (" + why + ")") +
                      ": the kubelet retries the pull; failing after " + std::to_string(pull_grace) +
                      " s (DEVSPACE_PULL_ERROR_GRACE_S)");
          continue;
        }
        if (r == "ContainerCreating" || r == "PodInitializing") waiting_create = true;
      }
    if (waiting_create || p.at_path("status.containerStatuses").items().empty()) creating.push_back(&p);
  }
  if (creating.empty()) return out;
  // A pod pulls while its kubelet has reported more `Pulling` than `Successfully pulled` events
  // for it (`Pulled` also says "already present on machine": no pull happened then). Only that
  // pod's events are listed (field selector), not the namespace's whole event history.
  for (const Value* p : creating) {
    std::string pn = p->at_path("metadata.name").as_string();
    std::string uid = p->at_path("metadata.uid").as_string();
    Value evs;
    try {
      evs = k.get("/api/v1/namespaces/" + ns + "/events?fieldSelector=" +
                  net::url_encode("involvedObject.kind=Pod,involvedObject.name=" + pn));
    } catch (const std::exception&) {
      continue;
    }
    int64_t pulls = 0, pulled = 0, since = 0;
    std::string what;
    for (auto& e : evs.get("items").items()) {
      const Value& io = e.get("involvedObject");
      if (io.get("kind").as_string() != "Pod" || io.get("name").as_string() != pn) continue;
      if (!uid.empty() && !io.get("uid").as_string().empty() && io.get("uid").as_string() != uid) continue;
      int64_t n = std::max<int64_t>(1, e.get("count").as_int(1));
      std::string reason = e.get("reason").as_string();
      if (reason == "Pulling") {
        pulls += n;
        what = e.get("message").as_string();
        int64_t t = event_time(e.get("firstTimestamp").as_string(e.get("eventTime").as_string()));
        if (t > 0 && (since == 0 || t < since)) since = t;
      } else if (reason == "Pulled" && starts_with(e.get("message").as_string(), "Successfully pulled")) {
        pulled += n;
      }
    }
    if (pulls > pulled) {
      out.pulling = "pod " + pn + ": " + what;
      out.pulling_since = since;
      return out;
    }
  }
  return out;
}

static int pull_budget_s() {
  const char* v = getenv("DEVSPACE_PULL_TIMEOUT");
  int s = v && *v ? atoi(v) : 1800;
  return s > 0 ? s : 1800;
}

Client::WaitOutcome Client::wait_ready(const std::vector<Value>& objs, const std::string& ns, int timeout_s) {
  // One watch per workload object (fieldSelector=metadata.name), in manifest order: the
  // status change that makes a rollout ready is seen the moment the API server commits it,
  // with no polling; the total wait is bounded by the slowest object. A workload not ready
  // within a second gets its pods looked at once a second: a pod that can never start fails the
  // wait at once, and one still pulling its image carries the wait past `timeout_s` (reference:
  // helm/install.go:171-195 explains a timeout with an analyze report; analyze/pods.go:50-117
  // waits on ContainerCreating pods).
  using clock = std::chrono::steady_clock;
  auto start = clock::now();
  auto deadline = start + std::chrono::seconds(timeout_s);
  auto pull_deadline = start + std::chrono::seconds(std::max(timeout_s, pull_budget_s()));
  auto ms_until = [](clock::time_point t) {
    return (int64_t)std::chrono::duration_cast<std::chrono::milliseconds>(t - clock::now()).count();
  };
  bool told = false;
  ProgressMemory mem;
  for (auto& o : objs) {
    std::string kind = o.get("kind").as_string();
    if (kind != "Deployment" && kind != "StatefulSet" && kind != "ReplicaSet" && kind != "DaemonSet" &&
        kind != "PersistentVolumeClaim")
      continue;
    std::string name = o.at_path("metadata.name").as_string();
    std::string ons = o.at_path("metadata.namespace").as_string(ns);
    std::string path = kube::resource_path(o.get("apiVersion").as_string(), kind, ons, name);
    std::string pending = kind + " " + name + " not checked";
    auto ready = [&](const std::optional<Value>& cur) {
      // a PVC that is gone (pvc-protection released it) is nothing to wait for
      if (!cur && kind == "PersistentVolumeClaim") return true;
      pending = not_ready_reason(kind, name, cur);
      return pending.empty();
    };
    if (reference_timing()) {
      // the reference-equivalent column: the original's 5 s readiness polls over the whole
      // timeout and nothing pull-aware (a timeout is analyzed and a first install purged)
      int64_t left = ms_until(deadline);
      if (left > 0 && k_->wait_object(path, (int)left, ready)) continue;
      return {"timed out waiting for the condition (" + pending + ")"};
    }
    while (true) {
      int64_t left = ms_until(deadline);
      int slice = (int)(left > 0 ? std::min<int64_t>(left, 1000) : std::min<int64_t>(1000, ms_until(pull_deadline)));
      if (slice > 0 && k_->wait_object(path, slice, ready)) break;
      if (kind == "PersistentVolumeClaim") {
        if (ms_until(deadline) > 0) continue;
        return {"timed out waiting for the condition (" + pending + ")"};
      }
      PodProgress pp = pod_progress(*k_, o, ons, mem);
      if (!pp.fatal.empty()) {
        WaitOutcome w;
        w.err = "rollout failed: " + pp.fatal + " (" + pending + ")";
        w.fatal = true;
        return w;
      }
      if (ms_until(deadline) > 0) continue;
      if (!pp.pulling.empty() && ms_until(pull_deadline) > 0) {
        if (!told) {
          int64_t secs = pp.pulling_since > 0 ? (int64_t)time(nullptr) - pp.pulling_since : 0;
          log::info(pp.pulling + " (" + std::to_string(secs) + " s so far): waiting for the pull, up to " +
                    std::to_string(std::max(timeout_s, pull_budget_s())) + " s in all (DEVSPACE_PULL_TIMEOUT)");
          told = true;
        }
        continue;
      }
      WaitOutcome w;
      w.err = "timed out waiting for the condition (" + pending + ")";
      if (!pp.pulling.empty()) {
        w.err += "; " + pp.pulling + " is still in progress";
        w.pulling = true;
      }
      return w;
    }
  }
  return {};
}

// ============================================================== hooks

static const char* kHookAnno = "helm.sh/hook";

static bool hook_has_event(const Hook& h, const std::string& ev) {
  for (auto& e : h.events)
    if (e == ev || (ev == "pre-install" && e == "crd-install")) return true;
  return false;
}

static bool has_policy(const Hook& h, const std::string& p) {
  if (h.delete_policies.empty()) return p == "before-hook-creation";  // Helm 3 default
  return std::find(h.delete_policies.begin(), h.delete_policies.end(), p) != h.delete_policies.end();
}

// Completion of a hook object: "" = still running, "Succeeded" or "Failed: <why>".
static std::string hook_phase(const std::string& kind, const std::optional<Value>& cur) {
  if (!cur) return "";
  if (kind == "Job") {
    for (auto& c : cur->at_path("status.conditions").items()) {
      if (c.get("status").as_string() != "True") continue;
      if (c.get("type").as_string() == "Complete") return "Succeeded";
      if (c.get("type").as_string() == "Failed") return "Failed: " + c.get("message").as_string(c.get("reason").as_string());
    }
    if (cur->at_path("status.succeeded").as_int(0) >= cur->at_path("spec.completions").as_int(1)) return "Succeeded";
    return "";
  }
  if (kind == "Pod") {
    std::string ph = cur->at_path("status.phase").as_string();
    if (ph == "Succeeded") return "Succeeded";
    if (ph == "Failed") return "Failed: pod " + cur->at_path("metadata.name").as_string() + " failed";
    return "";
  }
  return "Succeeded";  // other kinds are done once created
}

void Client::run_hooks(std::vector<Hook>& hooks, const std::string& event, const std::string& ns, int timeout_s) {
  std::vector<Hook*> sel;
  for (auto& h : hooks)
    if (hook_has_event(h, event)) sel.push_back(&h);
  std::stable_sort(sel.begin(), sel.end(), [](const Hook* a, const Hook* b) {
    if (a->weight != b->weight) return a->weight < b->weight;
    int ka = kind_order(a->kind), kb = kind_order(b->kind);
    if (ka != kb) return ka < kb;
    return a->name < b->name;
  });
  for (Hook* h : sel) {
    trace::Span span("deploy.helm_hook", {{"event", event}, {"hook", h->kind + "/" + h->name}});
    Value obj = yaml_parse(h->manifest);
    if (obj.at_path("metadata.namespace").is_null() && !kube::is_cluster_scoped(h->kind)) obj["metadata"]["namespace"] = ns;
    std::string path = kube::resource_path(obj.get("apiVersion").as_string(), h->kind,
                                           obj.at_path("metadata.namespace").as_string(ns), h->name);
    int wait_ms = (timeout_s > 0 ? timeout_s : 300) * 1000;
    if (has_policy(*h, "before-hook-creation") && k_->delete_object(obj, ns))
      k_->wait_object(path, wait_ms, [](const std::optional<Value>& o) { return !o.has_value(); });
    h->last_run = Value::map();
    h->last_run["started_at"] = log::rfc3339_now();
    h->last_run["phase"] = "Running";
    log::info("Running " + event + " hook " + h->kind + "/" + h->name);
    k_->apply(obj, ns);
    std::string phase;
    bool done = k_->wait_object(path, wait_ms, [&](const std::optional<Value>& cur) {
      phase = hook_phase(h->kind, cur);
      return !phase.empty();
    });
    if (!done) phase = "Failed: timed out waiting for the condition";
    h->last_run["completed_at"] = log::rfc3339_now();
    h->last_run["phase"] = phase == "Succeeded" ? "Succeeded" : "Failed";
    if (phase != "Succeeded") {
      if (has_policy(*h, "hook-failed")) k_->delete_object(obj, ns);
      throw std::runtime_error(event + " hook " + h->kind + "/" + h->name + " failed: " + phase.substr(phase.find(':') + 2));
    }
    if (has_policy(*h, "hook-succeeded")) k_->delete_object(obj, ns);
  }
}

// Rendered release: manifest text (hooks excluded), hook records, notes.
struct Rendered {
  std::string manifest, notes;
  std::vector<Hook> hooks;
  std::vector<Value> objs;
};

static Rendered render_release(const Chart& chart, const Value& values, const RenderOptions& ro) {
  Rendered out;
  for (auto& kv : render_files(chart, values, ro)) {
    if (ends_with(kv.first, "/NOTES.txt")) {
      if (kv.first == chart.name() + "/templates/NOTES.txt") out.notes = kv.second;
      continue;
    }
    for (auto& doc : split_documents(kv.second)) {
      Value d = yaml_parse(doc);
      if (!d.is_map() || d.get("kind").is_null()) continue;
      const Value& anno = d.at_path("metadata.annotations").get(kHookAnno);
      if (!anno.is_null()) {
        Hook h;
        h.name = d.at_path("metadata.name").as_string();
        h.kind = d.get("kind").as_string();
        h.path = kv.first;
        h.manifest = doc;
        for (auto& e : split(anno.as_string(), ",")) {
          std::string t = trim(e);
          if (!t.empty()) h.events.push_back(t);
        }
        h.weight = (int)d.at_path("metadata.annotations").get("helm.sh/hook-weight").as_int(0);
        for (auto& p : split(d.at_path("metadata.annotations").get("helm.sh/hook-delete-policy").as_string(), ",")) {
          std::string t = trim(p);
          if (!t.empty()) h.delete_policies.push_back(t);
        }
        out.hooks.push_back(std::move(h));
        continue;
      }
      out.manifest += "---\n# Source: " + kv.first + "\n" + doc + "\n";
      out.objs.push_back(d);
    }
  }
  std::stable_sort(out.objs.begin(), out.objs.end(), [](const Value& a, const Value& b) {
    return kind_order(a.get("kind").as_string()) < kind_order(b.get("kind").as_string());
  });
  return out;
}

// ============================================================== install / upgrade / rollback / delete

Release Client::install_or_upgrade(const std::string& name, const std::string& ns_in, const std::string& chart_path,
                                   const Value& values, bool wait, int timeout_s) {
  std::string ns = ns_in.empty() ? k_->default_namespace() : ns_in;
  Chart chart = load_chart(chart_path);
  if (chart.is_library()) throw std::runtime_error("library charts are not installable: " + chart.name());
  process_dependencies(chart, values);
  auto hist = history(ns, name);
  const Release* last_deployed = nullptr;
  for (auto& h : hist)
    if (h.status == "deployed") last_deployed = &h;
  int rev = hist.empty() ? 1 : hist.back().version + 1;
  RenderOptions ro;
  ro.release_name = name;
  ro.namespace_ = ns;
  ro.revision = rev;
  ro.is_install = last_deployed == nullptr;
  if (mentions_capabilities(chart)) ro.capabilities = capabilities();
  // Helm 3 `lookup`: live objects (a single object by name, or a List when name is empty); a
  // missing object or a forbidden read renders as an empty map, as Helm does
  ro.lookup = [this](const std::string& av, const std::string& kind, const std::string& lns,
                     const std::string& lname) -> Value {
    try {
      if (!lname.empty()) {
        auto o = k_->try_get(kube::resource_path(av, kind, lns, lname));
        return o ? *o : Value::map();
      }
      Value list = k_->get(kube::resource_path(av, kind, lns, ""));
      list["kind"] = kind + "List";
      return list;
    } catch (const std::exception&) {
      return Value::map();
    }
  };
  Value merged = coalesce_values(chart, values);
  validate_values(chart, merged);  // values.schema.json, as `helm install` does before rendering
  Rendered rd = render_release(chart, merged, ro);
  std::vector<Value>& objs = rd.objs;
  std::string gpu_issue = k_->check_gpu_requests(objs);
  for (auto& o : objs) {
    o["metadata"]["labels"]["app.kubernetes.io/managed-by"] = o.at_path("metadata.labels").get("app.kubernetes.io/managed-by").is_null()
                                                                  ? Value("Helm")
                                                                  : o.at_path("metadata.labels").get("app.kubernetes.io/managed-by");
    o["metadata"]["annotations"]["meta.helm.sh/release-name"] = name;
    o["metadata"]["annotations"]["meta.helm.sh/release-namespace"] = ns;
    if (o.at_path("metadata.namespace").is_null() && !kube::is_cluster_scoped(o.get("kind").as_string()))
      o["metadata"]["namespace"] = ns;
  }
  Release r;
  r.name = name;
  r.namespace_ = ns;
  r.version = rev;
  r.chart = chart.name();
  r.chart_version = chart.version();
  r.chart_json = chart_record(chart);
  r.config = values.is_map() ? values : Value::map();
  r.manifest = rd.manifest;
  r.notes = rd.notes;
  r.hooks = rd.hooks;
  r.last_deployed = log::rfc3339_now();
  r.first_deployed = hist.empty() ? r.last_deployed : hist.front().first_deployed;
  std::string err;
  bool still_pulling = false, rollout_failed = false;
  try {
    run_hooks(r.hooks, ro.is_install ? "pre-install" : "pre-upgrade", ns, timeout_s);
    for (auto& o : objs) k_->apply(o, ns);
    // objects that disappeared since the previous deployed revision
    if (last_deployed) {
      std::set<std::string> keep;
      for (auto& o : objs) keep.insert(object_key(o));
      for (auto& d : yaml_parse_all(last_deployed->manifest)) {
        if (!d.is_map() || d.get("kind").is_null()) continue;
        if (d.at_path("metadata.namespace").is_null() && !kube::is_cluster_scoped(d.get("kind").as_string()))
          d["metadata"]["namespace"] = ns;
        if (!keep.count(object_key(d)) && !keep_on_delete(d)) k_->delete_object(d, ns);
      }
    }
    if (wait) {
      trace::Span wspan("deploy.helm_wait", {{"release", name}});
      // install.go:28 DeploymentTimeout (40 s) unless the chart sets one; GPU workloads get
      // 300 s (rocm/pytorch images are tens of GB to pull). A GPU request that no node can
      // satisfy (check_gpu_requests) is not waited out: the analyze report follows at once.
      int wait_s = timeout_s > 0 ? timeout_s : (kube::Client::max_gpu_request(objs) > 0 ? 300 : 40);
      if (!gpu_issue.empty()) wait_s = std::min(wait_s, 5);
      WaitOutcome w = wait_ready(objs, ns, wait_s);
      err = w.err;
      still_pulling = w.pulling;
      rollout_failed = w.fatal;
    }
    // install.go:181 analyzeError: a wait timeout (or a pod that can never start) is explained
    // by an analyze report of the namespace; after a plain timeout, no problems found means the
    // release is fine (just slow). A pull still in progress is not analyzed as a problem.
    if ((contains(err, "timed out waiting") && !still_pulling) || rollout_failed) {
      try {
        analyze::Options ao;
        ao.wait = false;
        auto report = analyze::create_report(*k_, ns, ao);
        if (rollout_failed)
          err += report.empty() ? "" : "\n" + analyze::report_to_string(report);
        else
          err = report.empty() ? "" : analyze::report_to_string(report);
      } catch (const std::exception& e) {
        log::warn(std::string("Error creating analyze report: ") + e.what());
      }
    }
    if (err.empty()) run_hooks(r.hooks, ro.is_install ? "post-install" : "post-upgrade", ns, timeout_s);
  } catch (const std::exception& e) {
    err = e.what();
  }
  if (!err.empty()) {
    r.status = "failed";
    r.description = "Release \"" + name + "\" failed: " + err;
    store(r);
    if (last_deployed) {
      log::warn("Upgrade failed (" + err + "), rolling back to revision " + std::to_string(last_deployed->version));
      try {
        rollback(ns, name, last_deployed->version);
      } catch (const std::exception& e) {
        log::error(std::string("Rollback failed: ") + e.what());
      }
    } else if (still_pulling) {
      // a first install whose pods are still pulling is not purged (the reference's purge,
      // install.go:155-161, would delete the pod mid-pull and start the pull over next time)
      log::warn("Keeping release " + name + ": its image pull goes on in the cluster; run the command again "
                "to keep waiting, or raise DEVSPACE_PULL_TIMEOUT");
    } else {
      try {
        delete_release(ns, name, true);
      } catch (...) {
      }
    }
    throw std::runtime_error(err);
  }
  for (auto& h : hist)
    if (h.status == "deployed") {
      Release old = h;
      old.status = "superseded";
      store(old);
    }
  r.status = "deployed";
  r.description = ro.is_install ? "Install complete" : "Upgrade complete";
  store(r);
  prune_history(ns, name, (int)hist.size() + 1);
  return r;
}

void Client::rollback(const std::string& ns, const std::string& name, int to_version) {
  auto hist = history(ns, name);
  const Release* target = nullptr;
  const Release* current = nullptr;
  for (auto& h : hist) {
    if (h.version == to_version) target = &h;
    if (h.status == "deployed") current = &h;
  }
  if (!target) throw std::runtime_error("release " + name + " has no revision " + std::to_string(to_version));
  Release r = *target;
  r.version = hist.back().version + 1;
  r.status = "deployed";
  r.description = "Rollback to " + std::to_string(to_version);
  r.last_deployed = log::rfc3339_now();
  r.first_deployed = hist.front().first_deployed.empty() ? hist.front().last_deployed : hist.front().first_deployed;
  run_hooks(r.hooks, "pre-rollback", ns, 300);
  std::set<std::string> keep;
  for (auto& d : yaml_parse_all(target->manifest)) {
    if (!d.is_map() || d.get("kind").is_null()) continue;
    if (d.at_path("metadata.namespace").is_null() && !kube::is_cluster_scoped(d.get("kind").as_string()))
      d["metadata"]["namespace"] = ns;
    keep.insert(object_key(d));
    k_->apply(d, ns);
  }
  if (current) {  // objects the rolled-back-from revision added
    for (auto& d : yaml_parse_all(current->manifest)) {
      if (!d.is_map() || d.get("kind").is_null()) continue;
      if (d.at_path("metadata.namespace").is_null() && !kube::is_cluster_scoped(d.get("kind").as_string()))
        d["metadata"]["namespace"] = ns;
      if (!keep.count(object_key(d)) && !keep_on_delete(d)) k_->delete_object(d, ns);
    }
  }
  run_hooks(r.hooks, "post-rollback", ns, 300);
  for (auto& h : hist)
    if (h.status == "deployed") {
      Release old = h;
      old.status = "superseded";
      store(old);
    }
  store(r);
  prune_history(ns, name, (int)hist.size() + 1);
}

void Client::delete_release(const std::string& ns, const std::string& name, bool purge) {
  auto hist = history(ns, name);
  if (hist.empty()) throw std::runtime_error("release: \"" + name + "\" not found");
  Release last = hist.back();
  try {
    run_hooks(last.hooks, "pre-delete", ns, 300);
  } catch (const std::exception& e) {
    log::warn(e.what());
  }
  auto docs = yaml_parse_all(last.manifest);
  std::reverse(docs.begin(), docs.end());
  for (auto& d : docs) {
    if (!d.is_map() || d.get("kind").is_null()) continue;
    if (keep_on_delete(d)) {
      log::info("Keeping " + d.get("kind").as_string() + " " + d.at_path("metadata.name").as_string() +
                " (helm.sh/resource-policy: keep)");
      continue;
    }
    k_->delete_object(d, ns);
  }
  try {
    run_hooks(last.hooks, "post-delete", ns, 300);
  } catch (const std::exception& e) {
    log::warn(e.what());
  }
  if (purge) {
    for (auto& h : hist) {
      try {
        k_->del("/api/v1/namespaces/" + ns + "/secrets/" + secret_name(name, h.version));
      } catch (...) {
      }
    }
  } else {
    last.status = "uninstalled";
    last.description = "Uninstallation complete";
    store(last);
  }
}

}  // namespace helm
}  // namespace ds

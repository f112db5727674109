#include "deploy/helm.h"

#include <algorithm>
#include <chrono>
#include <set>
#include <thread>

#include "analyze/analyze.h"
#include "core/codec.h"
#include "core/fs.h"
#include "core/log.h"
#include "core/strutil.h"
#include "core/trace.h"
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

Chart load_chart(const std::string& dir) {
  Chart c;
  c.dir = dir;
  std::string cy = fs::join(dir, "Chart.yaml");
  if (!fs::exists(cy)) throw std::runtime_error("Chart.yaml file is missing in " + dir);
  c.metadata = yaml_load_file(cy);
  std::string vy = fs::join(dir, "values.yaml");
  if (fs::exists(vy)) c.values = yaml_load_file(vy);
  if (!c.values.is_map()) c.values = Value::map();
  std::string tdir = fs::join(dir, "templates");
  if (fs::is_dir(tdir)) {
    fs::walk(tdir, [&](const std::string& p, const fs::StatInfo& st) {
      if (!st.is_dir) c.templates.emplace_back(fs::relative(dir, p), fs::read_file(p));
      return true;
    });
    std::sort(c.templates.begin(), c.templates.end());
  }
  std::string cdir = fs::join(dir, "charts");
  if (fs::is_dir(cdir)) {
    for (auto& e : fs::list_dir(cdir)) {
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
        if (!top.empty()) c.dependencies.push_back(load_chart(fs::join(tmp, top)));
      }
    }
  }
  return c;
}

static void add_templates(tmpl::Engine& eng, const Chart& c, const std::string& prefix) {
  for (auto& t : c.templates) eng.add(prefix + t.first, t.second);
  for (auto& d : c.dependencies) add_templates(eng, d, prefix + "charts/" + d.name() + "/");
}

static void render_chart(tmpl::Engine& eng, const Chart& c, const Value& values, const RenderOptions& o,
                         const std::string& prefix, std::vector<std::pair<std::string, std::string>>* out) {
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
  Value chart = Value::map();
  for (auto& e : c.metadata.entries()) {
    std::string k = e.first;
    if (!k.empty()) k[0] = (char)std::toupper((unsigned char)k[0]);
    chart[k] = e.second;
  }
  dot["Chart"] = chart;
  Value caps = Value::map();
  caps["KubeVersion"]["Major"] = "1";
  caps["KubeVersion"]["Minor"] = "29";
  caps["KubeVersion"]["GitVersion"] = "v1.29.0";
  caps["KubeVersion"]["Version"] = "v1.29.0";
  caps["APIVersions"] = Value::strings({"v1", "apps/v1", "batch/v1", "rbac.authorization.k8s.io/v1",
                                        "autoscaling/v2", "autoscaling/v2beta1", "networking.k8s.io/v1"});
  dot["Capabilities"] = caps;
  for (auto& t : c.templates) {
    std::string base = fs::basename(t.first);
    if (starts_with(base, "_")) continue;  // partials
    if (!ends_with(base, ".yaml") && !ends_with(base, ".yml") && !ends_with(base, ".tpl") && !ends_with(base, ".json"))
      continue;
    if (ends_with(base, ".tpl")) continue;
    Value d = dot;
    d["Template"]["Name"] = c.name() + "/" + t.first;
    d["Template"]["BasePath"] = c.name() + "/templates";
    out->emplace_back(prefix + t.first, eng.execute(prefix + t.first, d));
  }
  for (auto& dep : c.dependencies) {
    Value sub = dep.values;
    merge_into(sub, values.get(dep.name()));
    if (values.get("global").is_map()) merge_into(sub["global"], values.get("global"));
    render_chart(eng, dep, sub, o, prefix + "charts/" + dep.name() + "/", out);
  }
}

std::string render_to_string(const Chart& chart, const Value& values, const RenderOptions& o) {
  tmpl::Engine eng;
  add_templates(eng, chart, "");
  std::vector<std::pair<std::string, std::string>> out;
  render_chart(eng, chart, values, o, "", &out);
  std::string all;
  for (auto& kv : out) {
    std::string body = trim(kv.second);
    if (body.empty()) continue;
    all += "---\n# Source: " + chart.name() + "/" + kv.first + "\n" + kv.second + "\n";
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

// ============================================================== release storage

static std::string secret_name(const std::string& name, int v) {
  return "sh.helm.release.v1." + name + ".v" + std::to_string(v);
}

static Release decode_release(const Value& secret) {
  Release r;
  std::string data = secret.at_path("data.release").as_string();
  Value v = json_parse(gzip_decompress(base64_decode(base64_decode(data))));
  r.name = v.get("name").as_string();
  r.namespace_ = v.get("namespace").as_string();
  r.version = (int)v.get("version").as_int();
  r.status = v.at_path("info.status").as_string();
  r.last_deployed = v.at_path("info.last_deployed").as_string();
  r.chart = v.at_path("chart.metadata.name").as_string();
  r.chart_version = v.at_path("chart.metadata.version").as_string();
  r.config = v.get("config");
  r.manifest = v.get("manifest").as_string();
  return r;
}

void Client::store(const Release& r) {
  Value v = Value::map();
  v["name"] = r.name;
  v["namespace"] = r.namespace_;
  v["version"] = r.version;
  v["info"]["status"] = r.status;
  v["info"]["last_deployed"] = r.last_deployed;
  v["chart"]["metadata"]["name"] = r.chart;
  v["chart"]["metadata"]["version"] = r.chart_version;
  v["config"] = r.config;
  v["manifest"] = r.manifest;
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
  // Helm 3 stores base64(gzip(json)) inside Secret data (itself base64 on the wire)
  s["data"]["release"] = base64_encode(base64_encode(gzip_compress(json_dump(v))));
  k_->apply(s, r.namespace_);
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

std::string Client::wait_ready(const std::vector<Value>& objs, const std::string& ns, int timeout_s) {
  // One watch per workload object (fieldSelector=metadata.name), in manifest order: the
  // status change that makes a rollout ready is seen the moment the API server commits it,
  // with no polling; the total wait is bounded by the slowest object.
  auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(timeout_s);
  for (auto& o : objs) {
    std::string kind = o.get("kind").as_string();
    if (kind != "Deployment" && kind != "StatefulSet" && kind != "ReplicaSet" && kind != "DaemonSet" &&
        kind != "PersistentVolumeClaim")
      continue;
    std::string name = o.at_path("metadata.name").as_string();
    std::string ons = o.at_path("metadata.namespace").as_string(ns);
    std::string path = kube::resource_path(o.get("apiVersion").as_string(), kind, ons, name);
    int64_t left = std::chrono::duration_cast<std::chrono::milliseconds>(deadline - std::chrono::steady_clock::now()).count();
    std::string pending = kind + " " + name + " not checked";
    bool ok = left > 0 && k_->wait_object(path, (int)left, [&](const std::optional<Value>& cur) {
      // a PVC that is gone (pvc-protection released it) is nothing to wait for
      if (!cur && kind == "PersistentVolumeClaim") return true;
      pending = not_ready_reason(kind, name, cur);
      return pending.empty();
    });
    if (!ok) return "timed out waiting for the condition (" + pending + ")";
  }
  return "";
}

Release Client::install_or_upgrade(const std::string& name, const std::string& ns_in, const std::string& chart_path,
                                   const Value& values, bool wait, int timeout_s) {
  std::string ns = ns_in.empty() ? k_->default_namespace() : ns_in;
  Chart chart = load_chart(chart_path);
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
  Value merged = chart.values;
  merge_values(merged, values);
  std::string manifest = render_to_string(chart, merged, ro);
  std::vector<Value> objs;
  for (auto& d : yaml_parse_all(manifest))
    if (d.is_map() && !d.get("kind").is_null()) objs.push_back(d);
  std::stable_sort(objs.begin(), objs.end(), [](const Value& a, const Value& b) {
    return kind_order(a.get("kind").as_string()) < kind_order(b.get("kind").as_string());
  });
  k_->check_gpu_requests(objs);
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
  r.config = values;
  r.manifest = manifest;
  r.last_deployed = log::rfc3339_now();
  std::string err;
  try {
    for (auto& o : objs) k_->apply(o, ns);
    // objects that disappeared since the previous deployed revision
    if (last_deployed) {
      std::set<std::string> keep;
      for (auto& o : objs) keep.insert(object_key(o));
      for (auto& d : yaml_parse_all(last_deployed->manifest)) {
        if (!d.is_map() || d.get("kind").is_null()) continue;
        if (d.at_path("metadata.namespace").is_null() && !kube::is_cluster_scoped(d.get("kind").as_string()))
          d["metadata"]["namespace"] = ns;
        if (!keep.count(object_key(d))) k_->delete_object(d, ns);
      }
    }
    if (wait) {
      trace::Span wspan("deploy.helm_wait", {{"release", name}});
      err = wait_ready(objs, ns, timeout_s > 0 ? timeout_s : 40);
    }
    // install.go:181 analyzeError: a wait timeout is explained by an analyze report of the
    // namespace; no problems found means the release is fine (just slow).
    if (contains(err, "timed out waiting")) {
      try {
        analyze::Options ao;
        ao.wait = false;
        auto report = analyze::create_report(*k_, ns, ao);
        err = report.empty() ? "" : analyze::report_to_string(report);
      } catch (const std::exception& e) {
        log::warn(std::string("Error creating analyze report: ") + e.what());
      }
    }
  } catch (const std::exception& e) {
    err = e.what();
  }
  if (!err.empty()) {
    r.status = "failed";
    store(r);
    if (last_deployed) {
      log::warn("Upgrade failed (" + err + "), rolling back to revision " + std::to_string(last_deployed->version));
      try {
        rollback(ns, name, last_deployed->version);
      } catch (const std::exception& e) {
        log::error(std::string("Rollback failed: ") + e.what());
      }
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
  store(r);
  return r;
}

void Client::rollback(const std::string& ns, const std::string& name, int to_version) {
  auto hist = history(ns, name);
  const Release* target = nullptr;
  for (auto& h : hist)
    if (h.version == to_version) target = &h;
  if (!target) throw std::runtime_error("release " + name + " has no revision " + std::to_string(to_version));
  for (auto& d : yaml_parse_all(target->manifest))
    if (d.is_map() && !d.get("kind").is_null()) k_->apply(d, ns);
  Release r = *target;
  r.version = hist.back().version + 1;
  r.status = "deployed";
  r.last_deployed = log::rfc3339_now();
  for (auto& h : hist)
    if (h.status == "deployed") {
      Release old = h;
      old.status = "superseded";
      store(old);
    }
  store(r);
}

void Client::delete_release(const std::string& ns, const std::string& name, bool purge) {
  auto hist = history(ns, name);
  if (hist.empty()) throw std::runtime_error("release: \"" + name + "\" not found");
  const Release& last = hist.back();
  auto docs = yaml_parse_all(last.manifest);
  std::reverse(docs.begin(), docs.end());
  for (auto& d : docs)
    if (d.is_map() && !d.get("kind").is_null()) k_->delete_object(d, ns);
  if (purge) {
    for (auto& h : hist) {
      try {
        k_->del("/api/v1/namespaces/" + ns + "/secrets/" + secret_name(name, h.version));
      } catch (...) {
      }
    }
  } else {
    Release r = last;
    r.status = "uninstalled";
    store(r);
  }
}

}  // namespace helm
}  // namespace ds

#include "deploy/deploy.h"

#include <cstdlib>
#include <algorithm>

#include "build/docker.h"
#include "build/image.h"
#include "core/codec.h"
#include "core/fs.h"
#include "core/log.h"
#include "core/match.h"
#include "core/proc.h"
#include "core/strutil.h"
#include "core/trace.h"
#include "deploy/helm.h"

namespace ds {
namespace deploy {

static std::string deployment_ns(const Value& cfg, const Value& d) {
  std::string ns = d.get("namespace").as_string();
  return ns.empty() ? config::default_namespace(cfg) : ns;
}

static Value image_values(const Value& cfg, config::Generated& gen, bool is_dev) {
  Value out = Value::map();
  const Value& tags = gen.cache(is_dev).get("imageTags");
  for (auto& e : cfg.get("images").entries()) {
    std::string image = e.second.get("image").as_string();
    std::string tag = tags.get(image).as_string();
    if (!e.second.get("tag").as_string().empty()) tag = e.second.get("tag").as_string();
    Value v = Value::map();
    v["image"] = image + ":" + tag;
    v["tag"] = tag;
    v["repo"] = image;
    out[e.first] = v;
  }
  return out;
}

Value helm_values(const Value& cfg, const Value& d, config::Generated& gen, bool is_dev) {
  std::string chart = d.at_path("helm.chartPath").as_string();
  std::string vpath = fs::join(chart, "values.yaml");
  Value values = Value::map();
  if (fs::exists(vpath)) {
    try {
      values = yaml_load_file(vpath);
    } catch (const std::exception& e) {
      throw std::runtime_error("Couldn't deploy chart, error reading from chart values " + vpath + ": " + e.what());
    }
    if (!values.is_map()) values = Value::map();
  }
  for (auto& ov : d.at_path("helm.overrides").items()) {
    std::string p = fs::abs_path(ov.as_string());
    try {
      helm::merge_values(values, yaml_load_file(p));
    } catch (const std::exception& e) {
      log::warn("Error reading from chart dev overwrite values " + p + ": " + e.what());
    }
  }
  if (d.at_path("helm.overrideValues").is_map()) helm::merge_values(values, d.at_path("helm.overrideValues"));
  // replace known image names (with or without tag) by image:tag (deploy/helm/deploy.go:212)
  const Value& tags = gen.cache(is_dev).get("imageTags");
  walk_strings(values, [&](const std::string&, Value& v) {
    std::string s = trim(v.str());
    std::string base = split(s, ":")[0];
    if (tags.has(base)) {
      v = Value(base + ":" + tags.get(base).as_string());
      return true;
    }
    return false;
  });
  Value imgs = image_values(cfg, gen, is_dev);
  values["images"] = imgs;
  values["containers"] = imgs;
  Value secrets = Value::seq();
  for (auto& s : values.get("pullSecrets").items()) secrets.push(s);
  for (auto& s : build::pull_secret_names()) {
    bool dup = false;
    for (auto& x : secrets.items()) dup |= x.as_string() == s;
    if (!dup) secrets.push(Value(s));
  }
  values["pullSecrets"] = secrets;
  return values;
}

std::vector<Value> kubectl_manifests(const Value& d, config::Generated& gen, bool is_dev) {
  std::vector<Value> out;
  const Value& tags = gen.cache(is_dev).get("imageTags");
  for (auto& pat : d.at_path("kubectl.manifests").items()) {
    for (auto& file : glob_expand(pat.as_string())) {
      if (!ends_with(file, ".yaml") && !ends_with(file, ".yml")) {
        log::warn("Manifest " + file + " skipped because it does not have a valid ending (.yml or .yaml expected)");
        continue;
      }
      if (fs::is_dir(file)) continue;
      for (auto& doc : yaml_parse_all(fs::read_file(file))) {
        if (!doc.is_map()) continue;
        walk_strings(doc, [&](const std::string& key, Value& v) {
          if (key == "image" && tags.has(v.str())) {
            v = Value(v.str() + ":" + tags.get(v.str()).as_string());
            return true;
          }
          return false;
        });
        out.push_back(doc);
      }
    }
  }
  return out;
}

namespace {

class HelmDeployer : public Deployer {
 public:
  HelmDeployer(const Value& cfg, const Value& d, std::shared_ptr<kube::Client> k) : cfg_(cfg), d_(d), k_(std::move(k)) {}

  void deploy(config::Generated& gen, bool is_dev, bool force) override {
    std::string name = d_.get("name").as_string();
    std::string chart = d_.at_path("helm.chartPath").as_string();
    std::string ns = deployment_ns(cfg_, d_);
    Value& cache = gen.cache(is_dev);
    std::string hash = build::hash_directory(chart);
    Value& dep = cache["deployments"][name];
    if (!dep.is_map()) dep = Value::map();
    if (!dep.get("helmOverrideTimestamps").is_map()) dep["helmOverrideTimestamps"] = Value::map();
    bool override_changed = false;
    for (auto& ov : d_.at_path("helm.overrides").items()) {
      fs::StatInfo st = fs::stat(ov.as_string());
      if (!st.exists) throw std::runtime_error("Error stating override file: " + ov.as_string());
      if (dep["helmOverrideTimestamps"].get(ov.as_string()).as_int(-1) != st.mtime_sec) override_changed = true;
    }
    helm::Client hc(k_);
    if (const char* mh = std::getenv("DEVSPACE_HELM_MAX_HISTORY")) hc.set_max_history(std::atoi(mh));
    if (!d_.at_path("helm.maxHistory").is_null()) hc.set_max_history((int)d_.at_path("helm.maxHistory").as_int(10));
    // The values the chart would get are part of the decision too (the reference's rule,
    // deploy/helm/deploy.go:64, looks at the chart and override files only): a pull secret
    // created after the first deploy, or an edit of helm.overrideValues in the config, reaches
    // the release without a chart edit.
    Value values = helm_values(cfg_, d_, gen, is_dev);
    std::string values_hash = sha256_hex(json_dump(values));
    bool redeploy = force || dep.get("helmChartHash").as_string() != hash || override_changed ||
                    (dep.has("helmValuesHash") && dep.get("helmValuesHash").as_string() != values_hash);
    if (!redeploy) redeploy = !hc.release_exists(ns, name);
    if (!redeploy) {
      if (!dep.has("helmValuesHash")) dep["helmValuesHash"] = values_hash;  // (generated.yaml of an older version)
      log::info("Skipping chart " + chart);
      return;
    }
    log::start_wait("Deploying helm chart");
    bool wait = d_.at_path("helm.wait").as_bool(true);
    int timeout = (int)d_.at_path("helm.timeout").as_int(0);  // 0: helm::Client's default
    helm::Release r;
    try {
      r = hc.install_or_upgrade(name, ns, chart, values, wait, timeout);
    } catch (const std::exception& e) {
      log::stop_wait();
      throw std::runtime_error(std::string("Unable to deploy helm chart: ") + e.what());
    }
    log::stop_wait();
    log::done("Deployed helm chart (Release revision: " + std::to_string(r.version) + ")");
    dep["helmChartHash"] = hash;
    dep["helmValuesHash"] = values_hash;
    for (auto& ov : d_.at_path("helm.overrides").items())
      dep["helmOverrideTimestamps"][ov.as_string()] = fs::stat(ov.as_string()).mtime_sec;
  }

  void remove() override {
    helm::Client hc(k_);
    hc.delete_release(deployment_ns(cfg_, d_), d_.get("name").as_string(), true);
  }

  std::vector<std::vector<std::string>> status() override {
    std::string name = d_.get("name").as_string(), ns = deployment_ns(cfg_, d_);
    helm::Client hc(k_);
    std::vector<helm::Release> hist;
    try {
      hist = hc.history(ns, name);
    } catch (const std::exception& e) {
      return {{name, "Error", ns, e.what()}};
    }
    if (hist.empty()) return {{name, "Not Found", ns, "No release found"}};
    const helm::Release& r = hist.back();
    if (r.status != "deployed") return {{name, "Error", ns, "HELM STATUS:" + to_upper(r.status)}};
    return {{name, "Deployed", ns, "Deployed: " + r.last_deployed}};
  }

 private:
  Value cfg_, d_;
  std::shared_ptr<kube::Client> k_;
};

class KubectlDeployer : public Deployer {
 public:
  KubectlDeployer(const Value& cfg, const Value& d, std::shared_ptr<kube::Client> k) : cfg_(cfg), d_(d), k_(std::move(k)) {}

  void deploy(config::Generated& gen, bool is_dev, bool force) override {
    (void)force;
    log::start_wait("Loading manifests");
    auto docs = kubectl_manifests(d_, gen, is_dev);
    log::stop_wait();
    k_->check_gpu_requests(docs);
    std::string ns = deployment_ns(cfg_, d_);
    std::string cmd = d_.at_path("kubectl.cmdPath").as_string();
    if (!cmd.empty()) {
      run_kubectl(cmd, "apply", {"--force"}, docs, ns);
      return;
    }
    log::start_wait("Applying manifests");
    try {
      for (auto& d : docs) {
        Value r = k_->apply(d, ns);
        log::stop_wait();
        log::get().write(to_lower(d.get("kind").as_string()) + "/" + d.at_path("metadata.name").as_string() +
                         " configured\n");
        log::start_wait("Applying manifests");
      }
    } catch (...) {
      log::stop_wait();
      throw;
    }
    log::stop_wait();
    log::done("Applied " + std::to_string(docs.size()) + " manifest(s) for " + d_.get("name").as_string());
  }

  void remove() override {
    config::Generated dummy = config::Generated::load();
    auto docs = kubectl_manifests(d_, dummy, false);
    std::string ns = deployment_ns(cfg_, d_);
    std::string cmd = d_.at_path("kubectl.cmdPath").as_string();
    if (!cmd.empty()) {
      run_kubectl(cmd, "delete", {"--ignore-not-found=true"}, docs, ns);
      return;
    }
    std::reverse(docs.begin(), docs.end());
    log::start_wait("Deleting manifests");
    for (auto& d : docs) k_->delete_object(d, ns);
    log::stop_wait();
  }

  std::vector<std::vector<std::string>> status() override {
    config::Generated dummy = config::Generated::load();
    std::string ns = deployment_ns(cfg_, d_);
    std::vector<std::vector<std::string>> rows;
    for (auto& d : kubectl_manifests(d_, dummy, false)) {
      std::string kind = d.get("kind").as_string(), name = d.at_path("metadata.name").as_string();
      std::string ons = d.at_path("metadata.namespace").as_string(ns);
      auto cur = k_->try_get(kube::resource_path(d.get("apiVersion").as_string(), kind, ons, name));
      rows.push_back({d_.get("name").as_string() + ": " + kind + "/" + name, cur ? "Deployed" : "Not Found", ons,
                      cur ? "created " + cur->at_path("metadata.creationTimestamp").as_string() : "-"});
    }
    return rows;
  }

 private:
  void run_kubectl(const std::string& cmd, const std::string& verb, const std::vector<std::string>& extra,
                   const std::vector<Value>& docs, const std::string& ns) {
    std::vector<std::string> args = {cmd};
    if (!cfg_.at_path("cluster.kubeContext").as_string().empty()) {
      args.push_back("--context");
      args.push_back(cfg_.at_path("cluster.kubeContext").as_string());
    }
    args.push_back("-n");
    args.push_back(ns);
    args.push_back(verb);
    for (auto& e : extra) args.push_back(e);
    args.push_back("-f");
    args.push_back("-");
    std::string joined;
    for (auto& d : docs) joined += "---\n" + yaml_dump(d);
    log::start_wait((verb == "apply" ? "Applying" : "Deleting") + std::string(" manifests with kubectl"));
    RunResult r = run(args, joined);
    log::stop_wait();
    log::get().write(r.out + r.err);
    if (r.code != 0) throw std::runtime_error("kubectl " + verb + " failed with exit code " + std::to_string(r.code));
  }

  Value cfg_, d_;
  std::shared_ptr<kube::Client> k_;
};

}  // namespace

std::unique_ptr<Deployer> make_deployer(const Value& cfg, const Value& d, std::shared_ptr<kube::Client> kube) {
  if (d.get("helm").is_map()) return std::make_unique<HelmDeployer>(cfg, d, kube);
  if (d.get("kubectl").is_map()) return std::make_unique<KubectlDeployer>(cfg, d, kube);
  throw std::runtime_error("Error deploying devspace: deployment " + d.get("name").as_string() +
                           " has no deployment method");
}

void deploy_all(const Value& cfg, config::Generated& gen, std::shared_ptr<kube::Client> kube, bool is_dev, bool force) {
  for (auto& d : cfg.get("deployments").items()) {
    std::string name = d.get("name").as_string();
    if (d.get("kubectl").is_map())
      log::info("Deploying " + name + " with kubectl");
    else
      log::info("Deploying " + name + " with helm");
    auto dep = make_deployer(cfg, d, kube);
    trace::Span span("deploy", {{"deployment", name}, {"engine", d.get("kubectl").is_map() ? "kubectl" : "helm"}});
    try {
      dep->deploy(gen, is_dev, force);
    } catch (const std::exception& e) {
      throw std::runtime_error("Error deploying devspace: " + std::string(e.what()));
    }
    log::done("Finished deploying " + name);
  }
}

void purge(const Value& cfg, std::shared_ptr<kube::Client> kube, const std::vector<std::string>& only) {
  const auto& deps = cfg.get("deployments").items();
  for (size_t i = deps.size(); i-- > 0;) {
    const Value& d = deps[i];
    std::string name = d.get("name").as_string();
    if (!only.empty() && std::find(only.begin(), only.end(), name) == only.end()) continue;
    log::start_wait("Deleting deployment " + name);
    try {
      make_deployer(cfg, d, kube)->remove();
      log::stop_wait();
      log::done("Successfully deleted deployment " + name);
    } catch (const std::exception& e) {
      log::stop_wait();
      log::warn("Error deleting deployment " + name + ": " + e.what());
    }
  }
}

}  // namespace deploy
}  // namespace ds

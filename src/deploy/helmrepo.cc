#include "deploy/helmrepo.h"

#include <algorithm>
#include <map>

#include "core/fs.h"
#include "core/log.h"
#include "core/net.h"
#include "core/strutil.h"

namespace ds {
namespace helmrepo {

const char* const kStableRepoName = "stable";
const char* const kStableRepoURL = "https://charts.helm.sh/stable";

std::string home() {
  const char* e = getenv("DEVSPACE_HELM_HOME");
  if (e && *e) return e;
  return fs::join(fs::home_dir(), ".devspace/helm");
}

static std::string repos_file() { return fs::join(home(), "repositories.yaml"); }

std::vector<Repo> repos() {
  std::vector<Repo> out;
  std::string data;
  if (fs::read_file(repos_file(), &data)) {
    Value v = yaml_parse(data);
    for (auto& r : v.get("repositories").items()) out.push_back({r.get("name").as_string(), r.get("url").as_string()});
  }
  if (out.empty()) out.push_back({kStableRepoName, kStableRepoURL});
  return out;
}

void add_repo(const Repo& r) {
  std::vector<Repo> rs = repos();
  bool replaced = false;
  for (auto& x : rs)
    if (x.name == r.name) {
      x.url = r.url;
      replaced = true;
    }
  if (!replaced) rs.push_back(r);
  Value v = Value::map();
  v["apiVersion"] = "v1";
  v["repositories"] = Value::seq();
  for (auto& x : rs) {
    Value e = Value::map();
    e["name"] = x.name;
    e["url"] = x.url;
    v["repositories"].push(e);
  }
  fs::write_file(repos_file(), yaml_dump(v));
}

std::string fetch(const std::string& url) {
  if (starts_with(url, "file://")) return fs::read_file(url.substr(7));
  std::string cur = url;
  for (int hop = 0; hop < 8; hop++) {
    net::Url u = net::Url::parse(cur);
    net::HttpClient c(u.scheme + "://" + u.host + (u.port ? ":" + std::to_string(u.port) : ""));
    net::Response r = c.get(u.path.empty() ? "/" : u.path);
    if (r.status >= 300 && r.status < 400 && !r.header("location").empty()) {
      std::string loc = r.header("location");
      if (loc[0] == '/') loc = u.scheme + "://" + u.host + (u.port ? ":" + std::to_string(u.port) : "") + loc;
      cur = loc;
      continue;
    }
    if (r.status != 200) throw std::runtime_error("GET " + cur + ": HTTP " + std::to_string(r.status));
    return r.body;
  }
  throw std::runtime_error("too many redirects fetching " + url);
}

static std::string cache_path(const Repo& r) { return fs::join(home(), "cache", r.name + "-index.yaml"); }

void update() {
  for (auto& r : repos()) {
    try {
      std::string idx = fetch(trim_right(r.url, "/") + "/index.yaml");
      fs::write_file_atomic(cache_path(r), idx);
    } catch (const std::exception& e) {
      log::warn("Unable to get an update from the \"" + r.name + "\" chart repository (" + r.url + "): " + e.what());
    }
  }
}

int compare_versions(const std::string& a, const std::string& b) {
  auto parts = [](const std::string& s) { return split(trim_left(s, "v"), "."); };
  auto pa = parts(a), pb = parts(b);
  for (size_t i = 0; i < std::max(pa.size(), pb.size()); i++) {
    std::string x = i < pa.size() ? pa[i] : "0", y = i < pb.size() ? pb[i] : "0";
    int64_t nx, ny;
    bool ix = parse_int64(x, &nx), iy = parse_int64(y, &ny);
    if (ix && iy) {
      if (nx != ny) return nx < ny ? -1 : 1;
    } else if (x != y) {
      return x < y ? -1 : 1;
    }
  }
  return 0;
}

std::vector<ChartVersion> all_charts() {
  std::vector<ChartVersion> out;
  for (auto& r : repos()) {
    std::string data;
    if (!fs::read_file(cache_path(r), &data)) continue;
    Value idx;
    try {
      idx = yaml_parse(data);
    } catch (const std::exception& e) {
      log::warn("Corrupt index for repository " + r.name + ": " + e.what());
      continue;
    }
    for (auto& e : idx.get("entries").entries()) {
      std::vector<ChartVersion> vs;
      for (auto& v : e.second.items()) {
        ChartVersion cv;
        cv.name = v.get("name").as_string(e.first);
        cv.version = v.get("version").as_string();
        cv.app_version = v.get("appVersion").as_string();
        cv.description = v.get("description").as_string();
        cv.repo_url = r.url;
        for (auto& u : v.get("urls").items()) cv.urls.push_back(u.as_string());
        vs.push_back(cv);
      }
      std::stable_sort(vs.begin(), vs.end(), [](const ChartVersion& a, const ChartVersion& b) {
        return compare_versions(a.version, b.version) > 0;
      });
      out.insert(out.end(), vs.begin(), vs.end());
    }
  }
  return out;
}

ChartVersion search(const std::string& name, const std::string& chart_version, const std::string& app_version) {
  for (auto& cv : all_charts()) {
    if (cv.name != name) continue;
    if (!chart_version.empty() && cv.version != chart_version) continue;
    if (!app_version.empty() && cv.app_version != app_version) continue;
    return cv;
  }
  throw std::runtime_error("Chart " + name + " not found" +
                           (chart_version.empty() ? "" : " with chart version " + chart_version) +
                           (app_version.empty() ? "" : " with app version " + app_version) +
                           ". Run `devspace list packages` to list available packages");
}

std::string download(const ChartVersion& v, const std::string& dir) {
  if (v.urls.empty()) throw std::runtime_error("chart " + v.name + " has no download URL");
  std::string url = v.urls[0];
  if (url.find("://") == std::string::npos) url = trim_right(v.repo_url, "/") + "/" + url;
  std::string dst = fs::join(dir, v.name + "-" + v.version + ".tgz");
  fs::write_file(dst, fetch(url));
  return dst;
}

}  // namespace helmrepo
}  // namespace ds

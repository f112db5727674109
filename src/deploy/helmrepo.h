// Helm chart repositories for `devspace add/remove/list package` (helm/client.go UpdateRepos,
// SearchChart, PrintAllAvailableCharts; configure/package.go). Repositories are listed in
// ~/.devspace/helm/repositories.yaml (name/url); `update` caches each repo's index.yaml under
// ~/.devspace/helm/cache/. http(s):// and file:// repository URLs are supported.
#pragma once

#include <string>
#include <vector>

#include "core/value.h"

namespace ds {
namespace helmrepo {

extern const char* const kStableRepoName;  // "stable"
extern const char* const kStableRepoURL;

struct Repo {
  std::string name, url;
};

struct ChartVersion {
  std::string name, version, app_version, description, repo_url;
  std::vector<std::string> urls;
};

std::string home();  // ~/.devspace/helm (DEVSPACE_HELM_HOME overrides)
std::vector<Repo> repos();
void add_repo(const Repo& r);
// Downloads index.yaml of every repository into the cache; failures are per-repo warnings.
void update();
// All chart versions known from cached indexes (newest version first per chart).
std::vector<ChartVersion> all_charts();
// Best match for name (optionally pinned by chart or app version). Throws if not found.
ChartVersion search(const std::string& name, const std::string& chart_version = "",
                    const std::string& app_version = "");
// Fetches the chart archive into dir/<name>-<version>.tgz; returns the path.
std::string download(const ChartVersion& v, const std::string& dir);
// GET (follows redirects) or read file://.
std::string fetch(const std::string& url);
// Semantic version compare (-1/0/1); non-numeric parts compared lexicographically.
int compare_versions(const std::string& a, const std::string& b);

}  // namespace helmrepo
}  // namespace ds

// Self-update from GitHub releases (pkg/devspace/upgrade/upgrade.go, which wraps
// rhysd/go-github-selfupdate): detect the newest release of `devspace-cloud/devspace` that
// ships a binary for this platform, compare it with the running version, download the asset
// (raw, .gz or .tar.gz/.tgz), and atomically replace the running executable.
//
// Endpoints: DEVSPACE_GITHUB_API (default https://api.github.com; a GitHub Enterprise API or a
// mirror works too), GITHUB_TOKEN for rate limits, HTTPS_PROXY/NO_PROXY honoured.
#pragma once

#include <optional>
#include <string>
#include <vector>

namespace ds {
namespace upgrade {

extern const char* const kGithubSlug;  // "devspace-cloud/devspace" (upgrade.go:14)

// eraseVersionPrefix (upgrade.go:17): "v1.2.3-beta" -> "1.2.3-beta"; throws when no x.y.z.
std::string erase_version_prefix(const std::string& version);

// semver precedence of two versions (prefix erased); pre-releases sort before the release.
int compare_versions(const std::string& a, const std::string& b);

struct Release {
  std::string version;  // without prefix
  std::string tag, name, notes;
  std::string asset_name, asset_url;
};

// Asset names this platform accepts, go-github-selfupdate style: "<os><sep><arch><ext>"
// suffixes with sep in {_,-} and ext in {"", .gz, .tar.gz, .tgz} (linux/amd64 here).
std::vector<std::string> asset_suffixes();

// selfupdate.DetectLatest: newest non-draft, non-prerelease release with a matching asset.
std::optional<Release> detect_latest(const std::string& slug = kGithubSlug);

// CheckForNewerVersion (upgrade.go:52): the newer version, or "" when up to date.
std::string check_for_newer_version(const std::string& current);

// Upgrade (upgrade.go:69): downloads `r`'s asset, extracts the `devspace` binary and replaces
// `exe` (the running executable) atomically, keeping nothing behind on failure.
void install_release(const Release& r, const std::string& exe);

// The binary inside a downloaded asset (decompresses .gz, finds `devspace` in a tarball).
std::string extract_binary(const std::string& asset_name, const std::string& data);

}  // namespace upgrade
}  // namespace ds

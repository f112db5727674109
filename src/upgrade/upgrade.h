// Self-update from GitHub releases (pkg/devspace/upgrade/upgrade.go, which wraps
// rhysd/go-github-selfupdate): detect the newest release of this product's own repository that
// ships a binary for this platform, compare it with the running version, download the asset
// (raw, .gz or .tar.gz/.tgz), verify it and atomically replace the running executable.
//
// Unlike the reference, which always follows devspace-cloud/devspace, the release channel is
// this build's own: DEVSPACE_RELEASE_REPO=owner/name (or the compile-time default); with none
// configured there is no update notice and `devspace upgrade` explains how to set one. An
// upstream devspace release is a different product: a candidate must carry kProductId and the
// asset must match a published SHA-256 (<asset>.sha256, checksums.txt or SHA256SUMS).
//
// Endpoints: DEVSPACE_GITHUB_API (default https://api.github.com; a GitHub Enterprise API or a
// mirror works too), GITHUB_TOKEN for rate limits, HTTPS_PROXY/NO_PROXY honoured.
#pragma once

#include <optional>
#include <string>
#include <vector>

namespace ds {
namespace upgrade {

// Product identity embedded in every binary of this build (and printed by `devspace version`):
// a downloaded or local candidate without it is not this product.
extern const char* const kProductId;
extern const char* const kProductMarker;  // "(" kProductId ")"
// The release channel: DEVSPACE_RELEASE_REPO, else the compile-time DEVSPACE_RELEASE_REPO
// definition, else "" (no channel: no update checks).
std::string release_repo();
// True when `binary` (file bytes) carries kProductId.
bool is_this_product(const std::string& binary);
// SHA-256 published for `asset` in a checksum file ("<hex>  <name>" lines, or a lone hex digest
// for <asset>.sha256); "" when absent.
std::string published_sha256(const std::string& checksum_file, const std::string& asset);

// eraseVersionPrefix (upgrade.go:17): "v1.2.3-beta" -> "1.2.3-beta"; throws when no x.y.z.
std::string erase_version_prefix(const std::string& version);

// semver precedence of two versions (prefix erased); pre-releases sort before the release.
int compare_versions(const std::string& a, const std::string& b);

struct Release {
  std::string version;  // without prefix
  std::string tag, name, notes;
  std::string asset_name, asset_url;
  std::string checksum_name, checksum_url;  // the release's checksum asset ("" if none)
};

// Asset names this platform accepts, go-github-selfupdate style: "<os><sep><arch><ext>"
// suffixes with sep in {_,-} and ext in {"", .gz, .tar.gz, .tgz}, for plat::release_target().
std::vector<std::string> asset_suffixes();

// selfupdate.DetectLatest: newest non-draft, non-prerelease release with a matching asset.
std::optional<Release> detect_latest(const std::string& slug = release_repo());

// CheckForNewerVersion (upgrade.go:52): the newer version, or "" when up to date.
std::string check_for_newer_version(const std::string& current);

// Upgrade (upgrade.go:69): downloads `r`'s asset, verifies its published SHA-256, extracts the
// `devspace` binary, checks it is this product, and replaces `exe` (the running executable)
// atomically, keeping nothing behind on failure.
void install_release(const Release& r, const std::string& exe);

// The binary inside a downloaded asset (decompresses .gz, finds `devspace` in a tarball).
std::string extract_binary(const std::string& asset_name, const std::string& data);

}  // namespace upgrade
}  // namespace ds

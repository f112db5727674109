#include "upgrade/upgrade.h"

#include <sys/stat.h>
#include <unistd.h>

#include <cstdlib>
#include <regex>
#include <stdexcept>

#include "core/codec.h"
#include "core/fs.h"
#include "core/net.h"
#include "core/strutil.h"
#include "core/value.h"
#include "platform/platform.h"

namespace ds {
namespace upgrade {

const char* const kProductId = "devspace-mi355x";
const char* const kProductMarker = "(devspace-mi355x)";  // a literal: present in the binary as is

#ifndef DEVSPACE_RELEASE_REPO
#define DEVSPACE_RELEASE_REPO ""
#endif

std::string release_repo() {
  const char* e = getenv("DEVSPACE_RELEASE_REPO");
  return e && *e ? e : DEVSPACE_RELEASE_REPO;
}

bool is_this_product(const std::string& binary) {
  // the marker as the binary stores it (and a release script would print it)
  return binary.find(kProductMarker) != std::string::npos;
}

std::string published_sha256(const std::string& file, const std::string& asset) {
  static const std::regex hex("^[0-9a-fA-F]{64}$");
  std::string lone;
  int lines = 0;
  for (auto& raw : split(file, "\n")) {
    std::string line = trim(raw);
    if (line.empty()) continue;
    ++lines;
    size_t sp = line.find_first_of(" \t");
    std::string digest = line.substr(0, sp);
    if (!std::regex_match(digest, hex)) continue;
    if (sp == std::string::npos) {
      lone = digest;
      continue;
    }
    std::string name = trim(line.substr(sp));
    if (!name.empty() && name[0] == '*') name = name.substr(1);  // sha256sum binary mode
    if (name == asset || fs::basename(name) == asset) return to_lower(digest);
  }
  return lines == 1 ? to_lower(lone) : "";
}

std::string erase_version_prefix(const std::string& version) {
  static const std::regex re(R"(\d+\.\d+\.\d+)");
  std::smatch m;
  if (!std::regex_search(version, m, re)) throw std::runtime_error("Version not adopting semver: " + version);
  return version.substr((size_t)m.position(0));
}

int compare_versions(const std::string& a_in, const std::string& b_in) {
  auto parse = [](const std::string& v) {
    std::string s = erase_version_prefix(v);
    std::string core = s.substr(0, s.find_first_of("-+"));
    std::string pre;
    size_t dash = s.find('-');
    if (dash != std::string::npos) pre = s.substr(dash + 1, s.find('+') == std::string::npos ? std::string::npos
                                                                                           : s.find('+') - dash - 1);
    std::vector<long long> n;
    for (auto& p : split(core, ".")) n.push_back(std::atoll(p.c_str()));
    while (n.size() < 3) n.push_back(0);
    return std::make_pair(n, pre);
  };
  auto a = parse(a_in), b = parse(b_in);
  if (a.first != b.first) return a.first < b.first ? -1 : 1;
  if (a.second == b.second) return 0;
  if (a.second.empty()) return 1;
  if (b.second.empty()) return -1;
  return a.second < b.second ? -1 : 1;
}

std::vector<std::string> asset_suffixes() {
  std::string t = plat::release_target();
  size_t dash = t.find('-');
  std::string os = t.substr(0, dash), arch = t.substr(dash + 1);
  std::vector<std::string> out;
  for (const char* sep : {"_", "-"})
    for (const char* ext : {"", ".gz", ".tar.gz", ".tgz"}) out.push_back(os + sep + arch + ext);
  return out;
}

namespace {

std::string api_base() {
  const char* e = getenv("DEVSPACE_GITHUB_API");
  return trim_right(e && *e ? e : "https://api.github.com", "/");
}

// GET with redirects (release assets redirect to object storage), proxy from the environment,
// GitHub's required User-Agent, and the token when one is set.
std::string http_get(const std::string& url_in, const std::string& accept) {
  std::string cur = url_in;
  for (int hop = 0; hop < 8; ++hop) {
    net::Url u = net::Url::parse(cur);
    std::string origin = u.scheme + "://" + u.host + (u.port ? ":" + std::to_string(u.port) : "");
    net::HttpClient c(origin);
    c.set_proxy(net::ProxyConfig::from_env());
    c.set_header("User-Agent", "devspace-selfupdate");
    c.set_header("Accept", accept);
    const char* tok = getenv("GITHUB_TOKEN");
    if (tok && *tok && hop == 0) c.set_header("Authorization", std::string("token ") + tok);
    net::Request rq;
    rq.path = u.path.empty() ? "/" : u.path;
    rq.timeout_ms = 120000;
    net::Response r = c.request(rq);
    if (r.status >= 300 && r.status < 400 && !r.header("location").empty()) {
      std::string loc = r.header("location");
      cur = loc[0] == '/' ? origin + loc : loc;
      continue;
    }
    if (r.status != 200) throw std::runtime_error("GET " + cur + ": HTTP " + std::to_string(r.status));
    return r.body;
  }
  throw std::runtime_error("too many redirects fetching " + url_in);
}

bool has_suffix_match(const std::string& name) {
  for (auto& s : asset_suffixes())
    if (ends_with(name, s)) return true;
  return false;
}

}  // namespace

std::optional<Release> detect_latest(const std::string& slug) {
  if (slug.empty()) throw std::runtime_error("no release channel configured (set DEVSPACE_RELEASE_REPO=owner/repo)");
  Value rels = json_parse(http_get(api_base() + "/repos/" + slug + "/releases?per_page=100",
                                   "application/vnd.github+json"));
  std::optional<Release> best;
  for (auto& rel : rels.items()) {
    if (rel.get("draft").as_bool() || rel.get("prerelease").as_bool()) continue;
    std::string tag = rel.get("tag_name").as_string();
    std::string ver;
    try {
      ver = erase_version_prefix(tag);
    } catch (const std::exception&) {
      continue;  // not a semver tag
    }
    for (auto& a : rel.get("assets").items()) {
      std::string name = a.get("name").as_string();
      if (!has_suffix_match(name)) continue;
      if (!best || compare_versions(ver, best->version) > 0) {
        Release r;
        r.version = ver;
        r.tag = tag;
        r.name = rel.get("name").as_string();
        r.notes = rel.get("body").as_string();
        r.asset_name = name;
        r.asset_url = a.get("browser_download_url").as_string();
        for (auto& c : rel.get("assets").items()) {
          std::string cn = c.get("name").as_string();
          if (cn == name + ".sha256" || (r.checksum_name.empty() && (ends_with(cn, "checksums.txt") ||
                                                                    cn == "SHA256SUMS" || cn == "sha256sums.txt"))) {
            r.checksum_name = cn;
            r.checksum_url = c.get("browser_download_url").as_string();
          }
        }
        best = r;
      }
      break;
    }
  }
  return best;
}

std::string check_for_newer_version(const std::string& current) {
  if (release_repo().empty()) return "";
  auto latest = detect_latest();
  if (!latest || compare_versions(latest->version, current) <= 0) return "";
  return latest->version;
}

std::string extract_binary(const std::string& asset_name, const std::string& data) {
  if (ends_with(asset_name, ".tar.gz") || ends_with(asset_name, ".tgz")) {
    std::string copy = data;
    GzipReader gz(string_source(&copy));
    TarReader tr([&](char* b, size_t n) { return gz.read(b, n); });
    TarEntry e;
    while (tr.next(&e)) {
      std::string base = fs::basename(e.name);
      std::string os = plat::release_target().substr(0, plat::release_target().find('-'));
      if ((e.type == '0' || e.type == '7') && (base == "devspace" || starts_with(base, "devspace-" + os) ||
                                               starts_with(base, "devspace_" + os)))
        return tr.read_all();
      tr.skip();
    }
    throw std::runtime_error("no devspace binary inside " + asset_name);
  }
  if (ends_with(asset_name, ".gz")) return gzip_decompress(data);
  return data;
}

void install_release(const Release& r, const std::string& exe) {
  if (r.checksum_url.empty())
    throw std::runtime_error("release " + r.tag + " publishes no SHA-256 for " + r.asset_name +
                             " (<asset>.sha256 or checksums.txt): refusing an unverifiable binary");
  std::string want = published_sha256(http_get(r.checksum_url, "application/octet-stream"), r.asset_name);
  if (want.empty()) throw std::runtime_error(r.checksum_name + " has no SHA-256 for " + r.asset_name);
  std::string asset = http_get(r.asset_url, "application/octet-stream");
  std::string got = sha256_hex(asset);
  if (got != want)
    throw std::runtime_error("checksum mismatch for " + r.asset_name + ": got " + got + ", published " + want);
  std::string bin = extract_binary(r.asset_name, asset);
  if (bin.size() < 4 || bin.compare(0, 4, "\x7f" "ELF") != 0)
    throw std::runtime_error("downloaded asset " + r.asset_name + " is not an executable");
  if (!is_this_product(bin))
    throw std::runtime_error("release " + r.tag + " is not a " + std::string(kProductId) + " build (e.g. an upstream "
                             "devspace binary): refusing to replace this one with it");
  // go-github-selfupdate's update.Apply: new file next to the target, old one kept until the
  // swap succeeded, then removed
  std::string staged = exe + ".new", old = exe + ".old";
  fs::write_file(staged, bin, 0755);
  ::chmod(staged.c_str(), 0755);
  fs::remove(old);
  if (!fs::rename(exe, old)) {
    fs::remove(staged);
    throw std::runtime_error("cannot move " + exe + " aside");
  }
  if (!fs::rename(staged, exe)) {
    fs::rename(old, exe);  // roll back
    fs::remove(staged);
    throw std::runtime_error("cannot replace " + exe);
  }
  fs::remove(old);
}

}  // namespace upgrade
}  // namespace ds

#include "build/docker.h"

#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <regex>
#include <cstdlib>
#include <set>
#include <stdexcept>

#include "core/codec.h"
#include "core/fs.h"
#include "core/log.h"
#include "core/match.h"
#include "core/proc.h"
#include "core/strutil.h"

namespace ds {
namespace build {

const char* const kDefaultIndexServer = "https://index.docker.io/v1/";

// ------------------------------------------------------------------------------ image names

static bool is_registry_component(const std::string& c) {
  return c == "localhost" || contains(c, ".") || contains(c, ":");
}

std::string registry_from_image(const std::string& image) {
  size_t slash = image.find('/');
  if (slash == std::string::npos) return "";
  std::string first = image.substr(0, slash);
  if (!is_registry_component(first)) return "";
  std::string host = to_lower(first);
  // docker.io / index.docker.io are the official index (repoInfo.Index.Official)
  if (host == "docker.io" || host == "index.docker.io" || host == "registry-1.docker.io") return "";
  return first;
}

std::pair<std::string, std::string> split_image_tag(const std::string& ref) {
  size_t at = ref.find('@');
  std::string name = at == std::string::npos ? ref : ref.substr(0, at);
  size_t slash = name.rfind('/');
  size_t colon = name.rfind(':');
  if (colon != std::string::npos && (slash == std::string::npos || colon > slash))
    return {name.substr(0, colon) + (at == std::string::npos ? "" : ref.substr(at)), name.substr(colon + 1)};
  return {ref, ""};
}

std::string image_reference_problem(const std::string& ref) {
  static const std::regex kComponent("[a-z0-9]+((\\.|_|__|-+)[a-z0-9]+)*");
  static const std::regex kDomain("([a-zA-Z0-9]|[a-zA-Z0-9][a-zA-Z0-9-]*[a-zA-Z0-9])(\\.([a-zA-Z0-9]|[a-zA-Z0-9][a-zA-Z0-9-]*"
                                  "[a-zA-Z0-9]))*(:[0-9]+)?");
  static const std::regex kTag("[\\w][\\w.-]{0,127}");
  static const std::regex kDigest("[A-Za-z][A-Za-z0-9]*([-_+.][A-Za-z][A-Za-z0-9]*)*:[0-9a-fA-F]{32,}");
  if (ref.empty()) return "the image name is empty";
  if (ref.size() > 255 + 128 + 80) return "the image reference is too long";
  std::string rest = ref;
  size_t at = rest.find('@');
  if (at != std::string::npos) {
    if (!std::regex_match(rest.substr(at + 1), kDigest)) return "invalid digest \"" + rest.substr(at + 1) + "\"";
    rest = rest.substr(0, at);
  }
  auto nt = split_image_tag(rest);
  if (!nt.second.empty() && !std::regex_match(nt.second, kTag)) return "invalid tag \"" + nt.second + "\"";
  if (rest.size() > 0 && rest.back() == ':') return "empty tag";
  std::vector<std::string> parts = split(nt.first, "/");
  size_t first = 0;
  if (parts.size() > 1 && (contains(parts[0], ".") || contains(parts[0], ":") || parts[0] == "localhost")) {
    if (!std::regex_match(parts[0], kDomain)) return "invalid registry host \"" + parts[0] + "\"";
    first = 1;
  }
  if (first >= parts.size()) return "no repository name after the registry";
  for (size_t i = first; i < parts.size(); ++i) {
    if (parts[i].empty()) return "empty path component in \"" + nt.first + "\" (leading, trailing or double '/')";
    if (!std::regex_match(parts[i], kComponent))
      return "invalid path component \"" + parts[i] + "\" (lower-case letters, digits and . _ __ - separators only)";
  }
  if (nt.first.size() > 255) return "the repository name is longer than 255 characters";
  return "";
}

std::string pull_secret_name(const std::string& registry) {
  if (registry.empty()) return "devspace-auth-docker";
  std::string out = "devspace-auth-";
  for (char c : to_lower(registry)) out.push_back((std::isalnum((unsigned char)c) || c == '-') ? c : '-');
  return out;
}

std::string registry_hostname(const std::string& url) {
  std::string s = url;
  if (starts_with(s, "http://")) s = s.substr(7);
  if (starts_with(s, "https://")) s = s.substr(8);
  return split(s, "/")[0];
}

// ------------------------------------------------------------------------------ credentials

Value AuthConfig::to_json() const {
  Value v = Value::map();
  if (!username.empty()) v["username"] = username;
  if (!password.empty()) v["password"] = password;
  if (!auth.empty()) v["auth"] = auth;
  if (!email.empty()) v["email"] = email;
  if (!server_address.empty()) v["serveraddress"] = server_address;
  if (!identity_token.empty()) v["identitytoken"] = identity_token;
  if (!registry_token.empty()) v["registrytoken"] = registry_token;
  return v;
}

AuthConfig AuthConfig::from_json(const Value& v) {
  AuthConfig a;
  auto pick = [&](const char* k1, const char* k2) {
    std::string s = v.get(k1).as_string();
    return s.empty() ? v.get(k2).as_string() : s;
  };
  a.username = pick("username", "Username");
  a.password = pick("password", "Password");
  a.auth = pick("auth", "Auth");
  a.email = pick("email", "Email");
  a.server_address = pick("serveraddress", "ServerAddress");
  a.identity_token = pick("identitytoken", "IdentityToken");
  a.registry_token = pick("registrytoken", "RegistryToken");
  if (!a.auth.empty() && a.username.empty()) {
    std::string dec = base64_decode(a.auth);
    size_t c = dec.find(':');
    if (c != std::string::npos) {
      a.username = dec.substr(0, c);
      a.password = dec.substr(c + 1);
    }
  }
  return a;
}

std::string DockerConfigFile::config_dir() {
  const char* d = std::getenv("DOCKER_CONFIG");
  if (d && *d) return d;
  return fs::join(fs::home_dir(), ".docker");
}

DockerConfigFile DockerConfigFile::load() {
  DockerConfigFile f;
  f.path = fs::join(config_dir(), "config.json");
  std::string text;
  if (fs::read_file(f.path, &text) && !trim(text).empty()) {
    try {
      f.raw = json_parse(text);
    } catch (const std::exception& e) {
      throw std::runtime_error("Error loading docker config " + f.path + ": " + e.what());
    }
    if (!f.raw.is_map()) f.raw = Value::map();
  }
  return f;
}

std::string DockerConfigFile::helper_for(const std::string& server) const {
  std::string host = registry_hostname(server);
  for (auto& e : raw.get("credHelpers").entries())
    if (e.first == server || registry_hostname(e.first) == host) return e.second.as_string();
  return raw.get("credsStore").as_string();
}

static std::optional<AuthConfig> helper_get(const std::string& helper, const std::string& server) {
  std::string bin = "docker-credential-" + helper;
  if (which(bin).empty()) return std::nullopt;
  RunResult r = run({bin, "get"}, server, {}, 10000);
  if (r.code != 0) return std::nullopt;
  try {
    Value v = json_parse(r.out);
    AuthConfig a;
    a.server_address = server;
    std::string user = v.get("Username").as_string();
    if (user == "<token>") {
      a.identity_token = v.get("Secret").as_string();
    } else {
      a.username = user;
      a.password = v.get("Secret").as_string();
    }
    return a;
  } catch (...) {
    return std::nullopt;
  }
}

AuthConfig DockerConfigFile::get(const std::string& server) const {
  std::string helper = helper_for(server);
  if (!helper.empty()) {
    if (auto a = helper_get(helper, server)) return *a;
  }
  const Value& auths = raw.get("auths");
  AuthConfig a;
  if (const Value* e = auths.find(server)) {
    a = AuthConfig::from_json(*e);
  } else {
    std::string host = registry_hostname(server);
    for (auto& kv : auths.entries()) {
      if (registry_hostname(kv.first) == host) {
        a = AuthConfig::from_json(kv.second);
        break;
      }
    }
  }
  a.server_address = server;
  return a;
}

std::map<std::string, AuthConfig> DockerConfigFile::all() const {
  std::map<std::string, AuthConfig> out;
  for (auto& kv : raw.get("auths").entries()) out[kv.first] = get(kv.first);
  for (auto& kv : raw.get("credHelpers").entries()) out[kv.first] = get(kv.first);
  return out;
}

void DockerConfigFile::store(const AuthConfig& a) {
  std::string helper = helper_for(a.server_address);
  if (!helper.empty() && !which("docker-credential-" + helper).empty()) {
    Value v = Value::map();
    v["ServerURL"] = a.server_address;
    v["Username"] = a.identity_token.empty() ? a.username : "<token>";
    v["Secret"] = a.identity_token.empty() ? a.password : a.identity_token;
    RunResult r = run({"docker-credential-" + helper, "store"}, json_dump(v), {}, 10000);
    if (r.code != 0) throw std::runtime_error("Error saving auth info in credentials store: " + trim(r.out + r.err));
    raw["auths"][a.server_address] = Value::map();
    return;
  }
  Value e = Value::map();
  e["auth"] = a.auth.empty() ? base64_encode(a.username + ":" + a.password) : a.auth;
  if (!a.email.empty()) e["email"] = a.email;
  if (!a.identity_token.empty()) e["identitytoken"] = a.identity_token;
  raw["auths"][a.server_address] = e;
}

void DockerConfigFile::save() const {
  fs::mkdirs(fs::dirname(path), 0700);
  fs::write_file_atomic(path, json_dump(raw, 1) + "\n", 0600);
}

// ------------------------------------------------------------------------------ Engine API

static std::map<std::string, std::string> minikube_docker_env() {
  std::map<std::string, std::string> env;
  RunResult r = run({"minikube", "docker-env", "--shell", "none"}, "", {}, 30000);
  if (r.spawn_failed || r.code != 0) throw std::runtime_error("minikube docker-env failed");
  for (auto& line : split(r.out, "\n")) {
    auto kv = split(trim(line), "=");
    if (kv.size() == 2) env[kv[0]] = kv[1];
  }
  return env;
}

std::unique_ptr<DockerClient> DockerClient::from_env(bool prefer_minikube, bool is_minikube) {
  std::map<std::string, std::string> env;
  bool from_minikube = false;
  if (prefer_minikube && is_minikube) {
    try {
      env = minikube_docker_env();
      from_minikube = true;
    } catch (...) {
    }
  }
  auto getenv_s = [&](const char* k) -> std::string {
    if (from_minikube) {
      auto it = env.find(k);
      return it == env.end() ? "" : it->second;
    }
    const char* v = std::getenv(k);
    return v ? v : "";
  };
  std::string host = getenv_s("DOCKER_HOST");
  if (host.empty()) host = "unix:///var/run/docker.sock";
  net::TlsOptions tls;
  std::string cert_path = getenv_s("DOCKER_CERT_PATH");
  if (!cert_path.empty() && !starts_with(host, "unix://")) {
    tls.enabled = true;
    fs::read_file(fs::join(cert_path, "ca.pem"), &tls.ca_pem);
    fs::read_file(fs::join(cert_path, "cert.pem"), &tls.cert_pem);
    fs::read_file(fs::join(cert_path, "key.pem"), &tls.key_pem);
    tls.insecure = getenv_s("DOCKER_TLS_VERIFY").empty();
  }
  return std::make_unique<DockerClient>(host, tls, getenv_s("DOCKER_API_VERSION"));
}

DockerClient::DockerClient(const std::string& host, net::TlsOptions tls, std::string api_version)
    : host_(host), version_(std::move(api_version)) {
  std::string url = host;
  if (starts_with(url, "tcp://")) url = (tls.enabled ? "https://" : "http://") + url.substr(6);
  http_ = net::HttpClient(url, tls);
}

std::string DockerClient::api(const std::string& path) const {
  return version_.empty() ? path : "/v" + version_ + path;
}

net::Response DockerClient::call(net::Request r) {
  r.path = api(r.path);
  return http_.request(std::move(r));
}

bool DockerClient::ping() {
  try {
    net::Request r;
    r.path = "/_ping";
    r.timeout_ms = 5000;
    return call(r).status == 200;
  } catch (const std::exception&) {
    return false;
  }
}

Value DockerClient::info() {
  net::Request r;
  r.path = "/info";
  r.timeout_ms = 10000;
  net::Response resp = call(r);
  if (resp.status != 200) throw std::runtime_error("docker info: HTTP " + std::to_string(resp.status));
  return json_parse(resp.body);
}

std::string DockerClient::official_server() {
  try {
    std::string s = info().get("IndexServerAddress").as_string();
    if (!s.empty()) return s;
  } catch (const std::exception&) {
  }
  return kDefaultIndexServer;
}

std::pair<bool, std::string> DockerClient::registry_endpoint(const std::string& registry) {
  std::string official = official_server();
  std::string url = registry.empty() || registry == "hub.docker.com" ? official : registry;
  return {url == official, url};
}

AuthConfig DockerClient::auth_config(const std::string& registry, bool check_store) {
  auto ep = registry_endpoint(registry);
  std::string server = ep.first ? ep.second : registry_hostname(ep.second);
  AuthConfig a;
  if (check_store) {
    try {
      a = DockerConfigFile::load().get(server);
    } catch (const std::exception& e) {
      log::warn(e.what());
    }
  }
  a.server_address = server;
  return a;
}

AuthConfig DockerClient::login(const std::string& registry, const std::string& user, const std::string& password,
                               bool check_store, bool save, bool relogin) {
  AuthConfig a = auth_config(registry, check_store);
  a.identity_token.clear();
  if (a.username.empty() || a.password.empty() || relogin) {
    a.username = trim(user);
    a.password = trim(password);
  }
  if (ping()) {
    net::Request r;
    r.method = "POST";
    r.path = "/auth";
    r.headers.push_back({"Content-Type", "application/json"});
    r.body = json_dump(a.to_json());
    net::Response resp = call(r);
    if (resp.status != 200) {
      std::string msg = resp.body;
      try {
        msg = json_parse(resp.body).get("message").as_string(resp.body);
      } catch (...) {
      }
      throw std::runtime_error("Error response from daemon: " + trim(msg));
    }
    try {
      std::string tok = json_parse(resp.body).get("IdentityToken").as_string();
      if (!tok.empty()) {
        a.password.clear();
        a.identity_token = tok;
      }
    } catch (...) {
    }
  }
  // (no daemon: the reference authenticates against the registry directly; this host has no
  // network, so the stored credentials are used as they are)
  if (save) {
    DockerConfigFile f = DockerConfigFile::load();
    f.store(a);
    f.save();
  }
  return a;
}

std::string render_json_message(const Value& m) {
  if (!m.is_map()) return "";
  if (m.has("errorDetail") || m.has("error")) {
    std::string msg = m.at_path("errorDetail.message").as_string();
    if (msg.empty()) msg = m.get("error").as_string();
    throw std::runtime_error(msg);
  }
  if (m.has("stream")) return m.get("stream").as_string();
  if (m.has("status")) {
    std::string out;
    if (!m.get("id").as_string().empty()) out += m.get("id").as_string() + ": ";
    out += m.get("status").as_string();
    if (!m.get("progress").as_string().empty()) out += " " + m.get("progress").as_string();
    return out + "\n";
  }
  return "";
}

// Feeds a JSON-lines message stream (messages may be split across chunks).
class JsonMessageStream {
 public:
  explicit JsonMessageStream(std::function<void(const Value&)> fn) : fn_(std::move(fn)) {}
  void feed(const std::string& d) {
    buf_ += d;
    size_t nl;
    while ((nl = buf_.find('\n')) != std::string::npos) {
      line(buf_.substr(0, nl));
      buf_.erase(0, nl + 1);
    }
  }
  void finish() {
    if (!trim(buf_).empty()) line(buf_);
    buf_.clear();
  }

 private:
  void line(const std::string& l) {
    std::string t = trim(l);
    if (t.empty()) return;
    Value v;
    try {
      v = json_parse(t);
    } catch (...) {
      v = Value::map();
      v["stream"] = t + "\n";
    }
    fn_(v);
  }
  std::function<void(const Value&)> fn_;
  std::string buf_;
};

std::string DockerClient::build(const std::string& context_tar, const BuildRequest& req,
                                const std::function<void(const std::string&)>& out) {
  return build_stream([&](const Sink& sink) { return sink(context_tar.data(), context_tar.size()); }, req, out);
}

std::string DockerClient::build_stream(const std::function<bool(const Sink&)>& write_context, const BuildRequest& req,
                                       const std::function<void(const std::string&)>& out) {
  std::string q = "/build?t=" + net::url_encode(req.tag) + "&dockerfile=" + net::url_encode(req.dockerfile) + "&rm=1";
  if (!req.build_args.empty()) {
    Value ba = Value::map();
    for (auto& kv : req.build_args) ba[kv.first] = kv.second;
    q += "&buildargs=" + net::url_encode(json_dump(ba));
  }
  if (!req.target.empty()) q += "&target=" + net::url_encode(req.target);
  if (!req.network_mode.empty()) q += "&networkmode=" + net::url_encode(req.network_mode);
  net::Request r;
  r.method = "POST";
  r.path = api(q);
  r.headers.push_back({"Content-Type", "application/x-tar"});
  if (!req.auth_configs.empty()) {
    Value ac = Value::map();
    for (auto& kv : req.auth_configs) ac[kv.first] = kv.second.to_json();
    r.headers.push_back({"X-Registry-Config", base64_encode(json_dump(ac), true)});
  }
  r.timeout_ms = 3600 * 1000;
  uint64_t sent = 0;
  auto t0 = std::chrono::steady_clock::now(), last = t0;
  r.body_writer = [&](const std::function<bool(const char*, size_t)>& to_daemon) {
    return write_context([&](const char* d, size_t n) {
      sent += n;
      auto now = std::chrono::steady_clock::now();
      if (now - last > std::chrono::seconds(5)) {  // big contexts: show that it moves
        last = now;
        out(strfmt("Sending build context to Docker daemon  %.2fMB\n", (double)sent / 1e6));
      }
      return to_daemon(d, n);
    });
  };
  out("Sending build context to Docker daemon\n");
  std::string image_id, err;
  JsonMessageStream js([&](const Value& m) {
    if (!err.empty()) return;
    try {
      if (m.at_path("aux.ID").is_string()) image_id = m.at_path("aux.ID").as_string();
      std::string s = render_json_message(m);
      if (!s.empty()) out(s);
    } catch (const std::exception& e) {
      err = e.what();
    }
  });
  std::string body;
  net::Response resp = http_.stream(r, [&](const std::string& d) {
    if (body.size() < 65536) body += d;
    js.feed(d);
    return true;
  });
  js.finish();
  out(strfmt("Sent build context: %.2fkB in %.2fs\n", (double)sent / 1000.0,
             std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count()));
  if (resp.status != 200) {
    std::string msg = body;
    try {
      msg = json_parse(body).get("message").as_string(body);
    } catch (...) {
    }
    throw std::runtime_error("Error response from daemon: " + trim(msg));
  }
  if (!err.empty()) throw std::runtime_error(err);
  return image_id;
}

void DockerClient::push(const std::string& image_with_tag, const AuthConfig& auth,
                        const std::function<void(const std::string&)>& out) {
  auto nt = split_image_tag(image_with_tag);
  std::string name = nt.first;
  // reference.FamiliarString: drop the implicit docker.io/library/ prefixes
  for (const char* p : {"docker.io/library/", "docker.io/"})
    if (starts_with(name, p)) name = name.substr(std::string(p).size());
  net::Request r;
  r.method = "POST";
  r.path = api("/images/" + name + "/push?tag=" + net::url_encode(nt.second.empty() ? "latest" : nt.second));
  r.headers.push_back({"X-Registry-Auth", base64_encode(json_dump(auth.to_json()), true)});
  r.timeout_ms = 3600 * 1000;
  std::string err, body;
  JsonMessageStream js([&](const Value& m) {
    if (!err.empty()) return;
    try {
      std::string s = render_json_message(m);
      if (!s.empty()) out(s);
    } catch (const std::exception& e) {
      err = e.what();
    }
  });
  net::Response resp = http_.stream(r, [&](const std::string& d) {
    if (body.size() < 65536) body += d;
    js.feed(d);
    return true;
  });
  js.finish();
  if (resp.status != 200) {
    std::string msg = body;
    try {
      msg = json_parse(body).get("message").as_string(body);
    } catch (...) {
    }
    throw std::runtime_error("Error response from daemon: " + trim(msg));
  }
  if (!err.empty()) throw std::runtime_error(err);
}

// ------------------------------------------------------------------------------ build context

std::vector<std::string> context_excludes(const std::string& context_dir, const std::string& rel_dockerfile) {
  std::vector<std::string> ex = read_dockerignore(fs::join(context_dir, ".dockerignore"));
  // build.TrimBuildFilesFromExcludes: the daemon always needs .dockerignore and the Dockerfile
  DockerIgnore m(ex);
  if (m.matches(".dockerignore")) ex.push_back("!.dockerignore");
  if (!rel_dockerfile.empty() && m.matches(rel_dockerfile)) ex.push_back("!" + rel_dockerfile);
  return ex;
}

static std::string read_link(const std::string& p) {
  char buf[4096];
  ssize_t n = ::readlink(p.c_str(), buf, sizeof(buf));
  return n < 0 ? "" : std::string(buf, (size_t)n);
}

// Shared walk of the docker context with .dockerignore semantics (archive.TarWithOptions /
// hash.DirectoryExcludes skip rules). fn(abs, rel, lstat) for every included entry.
static void walk_context(const std::string& root, const DockerIgnore& m,
                         const std::function<void(const std::string&, const std::string&, const fs::StatInfo&)>& fn) {
  std::string croot = fs::clean(root);
  fs::walk(croot, [&](const std::string& abs, const fs::StatInfo& st) {
    std::string rel = fs::relative(croot, abs);
    if (!rel.empty() && m.matches(rel)) {
      if (!st.is_dir) return false;
      // an excluded dir is still walked when a "!" exception may re-include something below
      if (!m.has_exclusions() || !m.dir_may_contain_exception(rel)) return false;
      return true;  // descend without emitting the dir itself
    }
    fn(abs, rel, st);
    return true;
  });
}

std::string context_tar(const std::string& context_dir, const std::vector<std::string>& excludes,
                        const std::string& rel_dockerfile, const std::optional<std::string>& dockerfile_override) {
  std::string out;
  write_context_tar(string_sink(&out), context_dir, excludes, rel_dockerfile, dockerfile_override);
  return out;
}

bool write_context_tar(const Sink& out, const std::string& context_dir, const std::vector<std::string>& excludes,
                       const std::string& rel_dockerfile, const std::optional<std::string>& dockerfile_override,
                       const std::vector<std::pair<std::string, std::string>>& extra) {
  bool ok = true;
  Sink guarded = [&](const char* d, size_t n) { return ok = ok && out(d, n); };
  TarWriter tw(guarded);
  DockerIgnore m(excludes);
  bool replaced = false;
  walk_context(context_dir, m, [&](const std::string& abs, const std::string& rel, const fs::StatInfo& st) {
    if (rel.empty()) return;
    TarEntry e;
    e.name = rel;
    e.mode = st.mode & 07777;
    e.mtime = st.mtime_sec;
    e.uid = e.gid = 0;  // ChownOpts{0,0}
    if (st.is_dir) {
      e.name += "/";
      e.type = '5';
      tw.add_dir(e);
    } else if (st.is_symlink) {
      e.type = '2';
      e.linkname = read_link(abs);
      e.size = 0;
      tw.write_header(e);
      tw.end_entry();
    } else if (st.is_reg) {
      if (dockerfile_override && rel == rel_dockerfile) {
        e.mode = 0600;
        e.size = (int64_t)dockerfile_override->size();
        tw.add_file(e, *dockerfile_override);
        replaced = true;
        return;
      }
      e.size = st.size;
      tw.add_file_from_path(e, abs);
    }
  });
  for (auto& f : extra) {
    if (fs::exists(fs::join(context_dir, f.first))) continue;
    TarEntry e;
    e.name = f.first;
    e.mode = 0644;
    e.mtime = time(nullptr);
    e.size = (int64_t)f.second.size();
    tw.add_file(e, f.second);
  }
  if (dockerfile_override && !replaced) {
    TarEntry e;
    e.name = rel_dockerfile;
    e.mode = 0600;
    e.mtime = time(nullptr);
    e.size = (int64_t)dockerfile_override->size();
    tw.add_file(e, *dockerfile_override);
  }
  tw.finish();
  return ok;
}

std::vector<int> dockerfile_ports(const std::string& content) {
  std::string d = replace_all(replace_all(content, "\r\n", "\n"), "\r", "\n");
  std::vector<int> ports;
  for (auto& line : split(d, "\n")) {
    // ^EXPOSE\s(.*)$ — case-sensitive, at line start, like the reference's regex
    if (line.size() < 7 || line.compare(0, 6, "EXPOSE") != 0 || !std::isspace((unsigned char)line[6])) continue;
    for (auto& tok : split(line.substr(7), " ")) {
      if (tok.empty()) continue;
      std::string num = tok.substr(0, tok.find('/'));
      int64_t p;
      if (!parse_int64(num, &p)) throw std::runtime_error("strconv.Atoi: parsing \"" + num + "\": invalid syntax");
      if (std::find(ports.begin(), ports.end(), (int)p) == ports.end()) ports.push_back((int)p);
    }
  }
  return ports;
}

std::string dockerfile_with_entrypoint(const std::string& content, const std::vector<std::string>& entrypoint) {
  if (entrypoint.empty()) throw std::runtime_error("Entrypoint is empty");
  auto q = [](const std::string& s) { return json_escape(s); };
  std::string out = content + "\n\nENTRYPOINT [\"" + q(entrypoint[0]) + "\"]";
  std::vector<std::string> rest;
  for (size_t i = 1; i < entrypoint.size(); ++i) rest.push_back(q(entrypoint[i]));
  // (the reference writes CMD [""] for a one-element entrypoint; an empty list is the intent)
  out += rest.empty() ? "\nCMD []" : "\nCMD [\"" + join(rest, "\",\"") + "\"]";
  return out;
}

// ------------------------------------------------------------------------------ hashes

std::string hash_directory(const std::string& path) {
  Sha256 h;
  fs::walk(fs::clean(path), [&](const std::string& abs, const fs::StatInfo& st) {
    int64_t ns = st.mtime_sec * 1000000000LL + st.mtime_nsec;
    h.update(abs + ";" + std::to_string(st.size) + ";" + std::to_string(ns));
    return true;
  });
  return h.hex();
}

namespace {

struct CrcCache {
  struct Entry {
    int64_t size = 0, mtime_ns = 0;
    std::string crc;
  };
  std::map<std::string, Entry> files;
  int64_t written_ns = 0;

  static int64_t now_ns() {
    struct timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    return (int64_t)ts.tv_sec * 1000000000LL + ts.tv_nsec;
  }

  void load(const std::string& path, const std::string& root) {
    std::string text;
    if (path.empty() || !fs::read_file(path, &text)) return;
    try {
      Value v = json_parse(text);
      if (v.get("root").as_string() != root || v.get("version").as_int() != 1) return;
      written_ns = v.get("written_ns").as_int();
      for (auto& kv : v.get("files").entries()) {
        Entry e;
        e.size = kv.second.get("size").as_int();
        e.mtime_ns = kv.second.get("mtime_ns").as_int();
        e.crc = kv.second.get("crc").as_string();
        if (!e.crc.empty()) files[kv.first] = e;
      }
    } catch (...) {
      files.clear();  // stale or corrupt: recompute everything
    }
  }

  void save(const std::string& path, const std::string& root) const {
    if (path.empty()) return;
    Value v = Value::map();
    v["version"] = 1;
    v["root"] = root;
    v["written_ns"] = now_ns();
    Value& f = v["files"];
    f = Value::map();
    for (auto& kv : files) {
      Value e = Value::map();
      e["size"] = kv.second.size;
      e["mtime_ns"] = kv.second.mtime_ns;
      e["crc"] = kv.second.crc;
      f[kv.first] = e;
    }
    try {
      fs::mkdirs(fs::dirname(path));
      fs::write_file_atomic(path, json_dump(v));
    } catch (const std::exception& e) {
      log::debug(std::string("context hash cache not saved: ") + e.what());
    }
  }
};

}  // namespace

std::string hash_directory_excludes(const std::string& path, const std::vector<std::string>& excludes,
                                    const std::string& cache_path) {
  fs::StatInfo rs = fs::lstat(path);
  if (!rs.exists) throw std::runtime_error("lstat " + path + ": no such file or directory");
  if (!rs.is_dir) throw std::runtime_error("Path " + path + " is not a directory");
  std::string root = fs::clean(path);
  CrcCache old, now;
  old.load(cache_path, root);
  Sha256 h;
  DockerIgnore m(excludes);
  walk_context(root, m, [&](const std::string& abs, const std::string&, const fs::StatInfo& st) {
    if (st.is_dir) {
      h.update(abs);
      return;
    }
    // files (and symlinks, whose target is read like the reference's os.Open)
    fs::StatInfo fst = st.is_symlink ? fs::stat(abs) : st;
    if (!fst.exists || fst.is_dir) return;
    int64_t mns = fst.mtime_sec * 1000000000LL + fst.mtime_nsec;
    std::string crc;
    auto it = old.files.find(abs);
    // entries modified within 1 s of the cache write may have changed again in the same
    // mtime tick: re-read those ("racy" entries, as git does for its index)
    if (it != old.files.end() && it->second.size == fst.size && it->second.mtime_ns == mns &&
        mns < old.written_ns - 1000000000LL) {
      crc = it->second.crc;
    } else {
      crc = crc32_file_hex(abs);
    }
    if (crc.empty()) return;  // unreadable: skipped like the reference
    h.update(abs + ";" + crc);
    if (!cache_path.empty() && !st.is_symlink) now.files[abs] = {fst.size, mns, crc};
  });
  if (!cache_path.empty()) now.save(cache_path, root);
  return h.hex();
}

}  // namespace build
}  // namespace ds

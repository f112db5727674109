// Docker side of the image pipeline: Engine API client (unix socket / tcp / TLS, minikube
// docker-env), registry credentials (~/.docker/config.json, credential helpers), image-name
// helpers, build-context tar with .dockerignore semantics, and the directory hashes behind the
// rebuild / redeploy skip caches.
//
// Reference equivalents: docker/client.go:19 NewClient (+ minikube docker-env :47-111),
// docker/auth.go:24 GetAuthConfig / :34 Login / :99 getOfficialServer, docker/config.go:16,27,
// registry/util.go:9 GetRegistryFromImageName, registry/registry.go:80 GetRegistryAuthSecretName,
// builder/util.go:43 CreateTempDockerfile, builder/docker/docker.go:55-216 (context tar, build,
// push with base64url X-Registry-Auth), util/hash/hash.go:20 Directory, :43 DirectoryExcludes.
//
// The reference links the docker/docker + docker/cli Go libraries; none of that exists here, so
// the Engine API is spoken directly over ds::net::HttpClient.
#pragma once

#include <functional>
#include <map>
#include <memory>
#include <optional>
#include <string>
#include <utility>
#include <vector>

#include "core/net.h"
#include "core/codec.h"
#include "core/value.h"

namespace ds {
namespace build {

extern const char* const kDefaultIndexServer;  // "https://index.docker.io/v1/"

// ---------------------------------------------------------------- image names

// Registry host of an image reference, "" for Docker Hub (registry/util.go:9). A first path
// component is a registry when it contains '.' or ':' or is "localhost".
std::string registry_from_image(const std::string& image);
// Splits "reg:5000/a/b:tag" into ("reg:5000/a/b", "tag"); digests are kept with the name.
std::pair<std::string, std::string> split_image_tag(const std::string& ref);
// Checks an image reference against the distribution reference grammar
// ([domain[:port]/]component(/component)*[:tag][@digest]; components lower-case alphanumerics
// joined by '.', '_', '__' or '-'s). Returns "" when valid, else why not.
std::string image_reference_problem(const std::string& ref);
// "devspace-auth-" + registry lower-cased with [^a-z0-9-] -> '-' ("docker" for Docker Hub).
std::string pull_secret_name(const std::string& registry);
// Hostname form used as credential key for non-default registries (registry.ConvertToHostname).
std::string registry_hostname(const std::string& url);

// ---------------------------------------------------------------- credentials

struct AuthConfig {
  std::string username, password, auth, email, server_address, identity_token, registry_token;
  Value to_json() const;  // Engine API AuthConfig (lower-case keys)
  static AuthConfig from_json(const Value& v);
  bool empty() const { return username.empty() && password.empty() && identity_token.empty(); }
};

// ~/.docker/config.json (or $DOCKER_CONFIG/config.json): `auths`, `credsStore`, `credHelpers`.
class DockerConfigFile {
 public:
  static DockerConfigFile load();
  static std::string config_dir();
  // Credentials for a server (credential helper first, then `auths`; basic auth decoded).
  AuthConfig get(const std::string& server) const;
  std::map<std::string, AuthConfig> all() const;
  void store(const AuthConfig& a);  // into the helper when one is configured, else `auths`
  void save() const;
  std::string path;
  Value raw = Value::map();

 private:
  std::string helper_for(const std::string& server) const;
};

// ---------------------------------------------------------------- Engine API

struct BuildRequest {
  std::string tag;              // image:tag
  std::string dockerfile;       // path of the Dockerfile inside the context tar
  std::map<std::string, std::string> build_args;
  std::string target, network_mode;
  std::map<std::string, AuthConfig> auth_configs;  // X-Registry-Config
};

class DockerClient {
 public:
  // NewClient(preferMinikube): minikube docker-env when preferred and the kube context is
  // minikube, else DOCKER_HOST / DOCKER_TLS_VERIFY / DOCKER_CERT_PATH / DOCKER_API_VERSION.
  static std::unique_ptr<DockerClient> from_env(bool prefer_minikube, bool is_minikube);
  explicit DockerClient(const std::string& host, net::TlsOptions tls = {}, std::string api_version = "");

  bool ping();
  Value info();
  // Default index server reported by the daemon (getOfficialServer).
  std::string official_server();
  // GetRegistryEndpoint: ("" | hub.docker.com) -> official server; returns (is_default, url).
  std::pair<bool, std::string> registry_endpoint(const std::string& registry);
  // GetAuthConfig (docker/auth.go:24).
  AuthConfig auth_config(const std::string& registry, bool check_store = true);
  // Login (docker/auth.go:34): stored credentials, verified by POST /auth when the daemon is up.
  AuthConfig login(const std::string& registry, const std::string& user, const std::string& password,
                   bool check_store, bool save, bool relogin);

  // POST /build with a (possibly gzip'ed) tar context. Output lines go to `out`; throws on a
  // daemon error message. Returns the image id when reported.
  std::string build(const std::string& context_tar, const BuildRequest& req,
                    const std::function<void(const std::string&)>& out);
  // Same with a streamed context: `write_context` produces the tar into the sink while it is
  // sent (chunked transfer encoding), so the context is never held in memory
  // (builder/docker/docker.go:94-158 streams a tar reader the same way).
  std::string build_stream(const std::function<bool(const Sink&)>& write_context, const BuildRequest& req,
                           const std::function<void(const std::string&)>& out);
  // POST /images/{name}/push?tag=  (X-Registry-Auth: base64url(JSON)).
  void push(const std::string& image_with_tag, const AuthConfig& auth,
            const std::function<void(const std::string&)>& out);
  const std::string& host() const { return host_; }

 private:
  net::Response call(net::Request r);
  std::string api(const std::string& path) const;
  std::string host_;
  std::string version_;
  net::HttpClient http_;
};

// Renders one Engine API JSON message like jsonmessage.DisplayJSONMessagesStream (non-TTY).
// Returns "" for messages that print nothing; throws on {"error": ...}.
std::string render_json_message(const Value& m);

// ---------------------------------------------------------------- build context

// Dockerfile + .dockerignore handling of `docker build` (build.GetContextFromLocalDir,
// ReadDockerignore, TrimBuildFilesFromExcludes): excludes for a context dir.
std::vector<std::string> context_excludes(const std::string& context_dir, const std::string& rel_dockerfile);

// Tar of the context (uid/gid 0, lexical order, .dockerignore applied with "!" exceptions).
// When `dockerfile_override` is set, the entry `rel_dockerfile` gets that content (or is added
// when absent, e.g. a Dockerfile outside the context).
std::string context_tar(const std::string& context_dir, const std::vector<std::string>& excludes,
                        const std::string& rel_dockerfile = "",
                        const std::optional<std::string>& dockerfile_override = std::nullopt);
// Streaming form: the tar goes to `out` while the context is walked. false when `out` failed.
// `extra`: files (relative path, content) added to the context where it has no such entry.
bool write_context_tar(const Sink& out, const std::string& context_dir, const std::vector<std::string>& excludes,
                       const std::string& rel_dockerfile = "",
                       const std::optional<std::string>& dockerfile_override = std::nullopt,
                       const std::vector<std::pair<std::string, std::string>>& extra = {});

// builder/util.go:43: Dockerfile content + ENTRYPOINT/CMD override (dev.overrideImages).
std::string dockerfile_with_entrypoint(const std::string& dockerfile_content, const std::vector<std::string>& entrypoint);

// util/dockerfile.GetPorts (pkg/util/dockerfile/get.go:14): the ports a Dockerfile EXPOSEs, in
// order, deduplicated ("8080/tcp" -> 8080; CRLF / CR newlines normalised). Throws on a
// non-numeric port, as the reference does. `devspace init` offers the first one as the default.
std::vector<int> dockerfile_ports(const std::string& dockerfile_content);

// ---------------------------------------------------------------- hashes

// util/hash/hash.go:20 — sha256 over "path;size;mtimeNs" of every walked entry (chart skip cache).
std::string hash_directory(const std::string& path);
// util/hash/hash.go:43 — sha256 over dirs' paths and "path;crc32" of every non-excluded file.
// With `cache_path`, per-file CRCs are reused when (size, mtime) are unchanged (entries younger
// than the cache's own write time are always re-read), so a warm deploy costs one stat walk
// instead of reading the whole build context. Same result as the uncached hash.
std::string hash_directory_excludes(const std::string& path, const std::vector<std::string>& excludes,
                                    const std::string& cache_path = "");

}  // namespace build
}  // namespace ds

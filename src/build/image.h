// Image pipeline: rebuild-skip cache, tags, docker / kaniko builders, push, pull secrets.
//
// Reference equivalents: image/build.go:24 BuildAll, :48 Build, :189 shouldRebuild;
// image/create_builder.go:18 CreateBuilder; builder/interface.go:6; builder/docker/docker.go;
// builder/kaniko/kaniko.go:53 Authenticate, :84 BuildImage; builder/kaniko/util.go:18
// formatKanikoOutput; registry/init.go:15 InitRegistries, :25 CreatePullSecrets;
// registry/registry.go:26 CreatePullSecret, :89 GetImageWithTag, :113 GetPullSecretNames.
//
// Differences by design: the kaniko build pod is watched (100 ms polls instead of 5 s sleeps)
// and deleted on every exit path; the build-context hash reuses per-file CRCs across runs
// (.devspace/cache/), so an unchanged project costs one stat walk instead of a full read.
#pragma once

#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "build/docker.h"
#include "config/config.h"
#include "kube/client.h"

namespace ds {
namespace build {

struct BuildOptions {
  bool is_dev = false;
  bool force_rebuild = false;
  std::string docker_target;            // --docker-target (overrides build.options.target)
  std::function<bool()> interrupted;    // Ctrl-C check while waiting on the kaniko pod
};

// Builder interface (builder/interface.go:6).
class Builder {
 public:
  virtual ~Builder() = default;
  virtual std::string engine() const = 0;
  virtual void authenticate() = 0;
  // context_dir / dockerfile are absolute; entrypoint empty = no override.
  virtual void build_image(const std::string& context_dir, const std::string& dockerfile,
                           const std::vector<std::string>& entrypoint) = 0;
  virtual void push_image() = 0;
};

struct ImageBuildSettings {
  std::string image, tag, last_tag;
  std::map<std::string, std::string> build_args;
  std::string target, network;
  bool insecure = false;
  bool no_cache = false;
  std::string kaniko_namespace, kaniko_pull_secret;
  // the executor image (images.*.build.kaniko.image, DEVSPACE_KANIKO_IMAGE; default: the
  // reference's pinned debug build). It needs the debug variant's /busybox: the build runs by exec.
  std::string kaniko_image;
  bool prefer_minikube = true;
};

// CreateBuilder (image/create_builder.go:18): kaniko when build.kaniko is set, else docker.
std::unique_ptr<Builder> create_builder(const Value& cfg, const Value& image_conf, const ImageBuildSettings& s,
                                        std::shared_ptr<kube::Client> kube, const BuildOptions& o);

// shouldRebuild (image/build.go:189); updates the cache's Dockerfile timestamp + context hash.
bool should_rebuild(config::Generated& gen, const Value& image_conf, const std::string& context_path,
                    const std::string& dockerfile_path, bool force, bool is_dev);

// Build one image (image/build.go:48). Returns true when it was (re)built.
bool build_image(const Value& cfg, config::Generated& gen, const std::string& image_config_name,
                 const Value& image_conf, std::shared_ptr<kube::Client> kube, const BuildOptions& o);
// BuildAll (image/build.go:24). Returns true if any image was rebuilt.
bool build_all(const Value& cfg, config::Generated& gen, std::shared_ptr<kube::Client> kube, const BuildOptions& o);

// registry: pull secrets (dockerconfigjson) per registry / deployment namespace.
void create_pull_secret(kube::Client& k, const std::string& ns, const std::string& registry,
                        const std::string& username, const std::string& password_or_token, const std::string& email);
void init_registries(const Value& cfg, std::shared_ptr<kube::Client> kube, const std::string& default_ns);
// Names of the pull secrets created by this process (injected into Helm values).
std::vector<std::string> pull_secret_names();
// registry.GetImageWithTag: image:tag (explicit tag or the generated.yaml cache).
std::string image_with_tag(config::Generated& gen, const Value& image_conf, bool is_dev);

// formatKanikoOutput line rewriting (exposed for tests): returns ("done"|"info"|"", text).
std::pair<std::string, std::string> format_kaniko_line(const std::string& line);

}  // namespace build
}  // namespace ds

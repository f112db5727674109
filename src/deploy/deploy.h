// Deployers (deploy/interface.go:8 Interface{Delete, Status, Deploy}, deploy/util.go:15 All).
//   HelmDeployer    — deploy/helm/*.go: chart-hash/override-mtime skip cache, values.yaml +
//                     overrides + overrideValues, image tag injection (images/containers),
//                     pull secrets, native Helm engine (deploy/helm.h).
//   KubectlDeployer — deploy/kubectl/*.go: manifest globs (.yaml/.yml), `image:` tag rewrite,
//                     applied natively through the API (or via `cmdPath`/kubectl when set).
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "config/config.h"
#include "kube/client.h"

namespace ds {
namespace deploy {

class Deployer {
 public:
  virtual ~Deployer() = default;
  virtual void deploy(config::Generated& gen, bool is_dev, bool force) = 0;
  virtual void remove() = 0;
  // rows: [name, status, namespace, details]
  virtual std::vector<std::vector<std::string>> status() = 0;
};

std::unique_ptr<Deployer> make_deployer(const Value& cfg, const Value& deployment, std::shared_ptr<kube::Client> kube);

// Deploy every configured deployment in order (deploy/util.go:15).
void deploy_all(const Value& cfg, config::Generated& gen, std::shared_ptr<kube::Client> kube, bool is_dev, bool force);
// Delete deployments in reverse order, optionally filtered by name (cmd/purge.go:104).
void purge(const Value& cfg, std::shared_ptr<kube::Client> kube, const std::vector<std::string>& only);

// Helm values for a deployment (exposed for tests): values.yaml + overrides + overrideValues
// + images/containers/pullSecrets injection.
Value helm_values(const Value& cfg, const Value& deployment, config::Generated& gen, bool is_dev);
// kubectl manifests with image tags substituted (exposed for tests).
std::vector<Value> kubectl_manifests(const Value& deployment, config::Generated& gen, bool is_dev);

}  // namespace deploy
}  // namespace ds

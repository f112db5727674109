// Config editing used by `devspace add/remove ...` and `devspace init`
// (pkg/devspace/configure/*.go). All functions edit the *base* config of the context (no
// overrides applied) and save it, like configutil.SaveBaseConfig.
#pragma once

#include <map>
#include <string>
#include <vector>

#include "config/config.h"
#include "core/value.h"

namespace ds {
namespace configure {

// "a=b, c=d" -> ordered map; throws "Wrong selector format: ..." (sync.go:150).
Value parse_selectors(const std::string& s);
bool label_maps_equal(const Value& a, const Value& b);
// "8080", "8080:80,9000" -> [{localPort, remotePort}] (port.go:163).
Value parse_port_mappings(const std::string& s);

void add_deployment(config::Context& ctx, const std::string& name, const std::string& ns,
                    const std::string& manifests, const std::string& chart);
void remove_deployment(config::Context& ctx, bool all, const std::string& name);

void add_image(config::Context& ctx, const std::string& name_in_config, const std::string& image,
               const std::string& tag, const std::string& context_path, const std::string& dockerfile,
               const std::string& build_engine);
void remove_image(config::Context& ctx, bool all, const std::vector<std::string>& names);

void add_selector(config::Context& ctx, const std::string& name, const std::string& label_selector,
                  const std::string& ns, bool save = true);
void remove_selector(config::Context& ctx, bool all, const std::string& name, const std::string& label_selector,
                     const std::string& ns);

void add_port(config::Context& ctx, const std::string& ns, const std::string& label_selector,
              const std::string& selector_name, const std::string& mappings);
void remove_port(config::Context& ctx, bool all, const std::string& label_selector, const std::string& ports);

void add_sync(config::Context& ctx, const std::string& local_path, const std::string& container_path,
              const std::string& ns, const std::string& label_selector, const std::string& excluded,
              const std::string& selector_name);
void remove_sync(config::Context& ctx, bool all, const std::string& local_path, const std::string& container_path,
                 const std::string& label_selector);

// Helm chart packages as dependencies of a deployment's chart (package.go).
void add_package(config::Context& ctx, const std::string& name, const std::string& chart_version,
                 const std::string& app_version, const std::string& deployment, bool skip_question);
void remove_package(config::Context& ctx, bool all, const std::string& deployment, const std::string& name);
// Default values / selectors for well-known packages (packagedefaults.go).
std::string package_default_values(const std::string& name);
Value package_default_selector(const std::string& name, const std::string& deployment);

// One member of a .tgz as a string ("" if absent) — util/tar/tar.go:64.
std::string extract_from_tgz(const std::string& tgz_path, const std::string& member);

// Image name + pull secret configuration during init (init_image.go:18).
void init_image(config::Context& ctx, const std::string& docker_username, bool is_cloud);

}  // namespace configure
}  // namespace ds

// Shared CLI plumbing: project root discovery, config loading, kube client creation,
// cloud configuration and the command registration entry points (cmd/*.go).
#pragma once

#include <atomic>
#include <memory>
#include <string>
#include <vector>

#include "config/config.h"
#include "core/cli.h"
#include "kube/client.h"

namespace ds {
namespace cmd {

extern const char* const kVersion;

// Process-wide interrupt flag (Ctrl-C / SIGTERM). Outside a GracefulInterrupt scope a signal
// ends the process right away (exit 128+signal), like a Go binary without a handler; inside
// one (dev loop, logs -f, enter, sync, kaniko build wait) the first signal only sets the flag
// so the command can clean up, and a second one ends the process.
std::atomic<bool>& interrupted();
void install_signal_handlers();
struct GracefulInterrupt {
  GracefulInterrupt();
  ~GracefulInterrupt();
  GracefulInterrupt(const GracefulInterrupt&) = delete;
  GracefulInterrupt& operator=(const GracefulInterrupt&) = delete;
};

// Finds the project root (SetDevSpaceRoot) or fails with the reference's message.
void require_devspace_root();

struct Session {
  config::Context ctx;
  std::shared_ptr<kube::Client> kube;
  const Value& cfg() { return ctx.get(true); }
};

// --config flag handling (configutil.ConfigPath override).
void apply_config_flag(config::Context& ctx, const cli::Command& c);
// Creates the kube client from the loaded config; `switch_context` writes ~/.kube/config.
std::shared_ptr<kube::Client> make_kube(const Value& cfg, bool switch_context);
// Path of the static in-container helper next to the running binary.
std::string helper_path();

// cloud.Configure / ConfigureWithSpaceName (cloud/configure.go:79,121).
void cloud_configure(config::Context& ctx, const std::string& space_name = "");

// Registration of command groups.
void register_core(cli::Command& root);     // deploy dev up enter logs analyze purge down reset
void register_init(cli::Command& root);     // init
void register_config(cli::Command& root);   // add list remove status update use create
void register_misc(cli::Command& root);     // install upgrade login version sync
// Prints the cached "newer version" notice and refreshes the cache in the background (root.go:38).
void notify_newer_version(const std::vector<std::string>& args);

std::unique_ptr<cli::Command> make_root();

}  // namespace cmd
}  // namespace ds

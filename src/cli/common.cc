#include "cli/common.h"

#include <limits.h>
#include <signal.h>
#include <unistd.h>

#include "cloud/cloud.h"
#include "core/fs.h"
#include "core/log.h"
#include "core/prompt.h"
#include "platform/platform.h"

namespace ds {
namespace cmd {

const char* const kVersion = "0.1.0-mi355x";

std::atomic<bool>& interrupted() {
  static std::atomic<bool> f{false};
  return f;
}

static std::atomic<int> g_graceful{0};

GracefulInterrupt::GracefulInterrupt() { g_graceful.fetch_add(1); }
GracefulInterrupt::~GracefulInterrupt() { g_graceful.fetch_sub(1); }

void install_signal_handlers() {
  signal(SIGPIPE, SIG_IGN);
  struct sigaction sa{};
  sa.sa_handler = [](int sig) {
    // async-signal-safe: atomics, write(2), _exit(2)
    bool again = interrupted().exchange(true);
    if (g_graceful.load() == 0 || again) {
      prompt::restore_cooked_tty_from_signal();
      const char nl = '\n';
      (void)!::write(2, &nl, 1);
      ::_exit(128 + sig);
    }
  };
  sigemptyset(&sa.sa_mask);
  sigaction(SIGINT, &sa, nullptr);
  sigaction(SIGTERM, &sa, nullptr);
}

void require_devspace_root() {
  if (!config::set_devspace_root()) log::fatal("Couldn't find a DevSpace configuration. Please run `devspace init`");
}

void apply_config_flag(config::Context& ctx, const cli::Command& c) {
  const cli::Flag* f = c.flag("config");
  if (f && !f->s.empty()) ctx.config_path = f->s;
}

std::shared_ptr<kube::Client> make_kube(const Value& cfg, bool switch_context) {
  try {
    return kube::Client::from_devspace_config(cfg, switch_context);
  } catch (const std::exception& e) {
    log::fatal(std::string("Unable to create new kubectl client: ") + e.what());
  }
}

std::string helper_path() {
  const char* env = getenv("DEVSPACE_HELPER");
  if (env && *env) return env;
  std::string exe = plat::self_exe();
  if (exe.empty()) return "";
  return fs::join(fs::dirname(exe), "devspace-helper");
}

void cloud_configure(config::Context& ctx, const std::string& space_name) {
  try {
    cloud::configure(ctx, space_name);
  } catch (const std::exception& e) {
    log::fatal(std::string("Unable to configure cloud provider: ") + e.what());
  }
}

std::unique_ptr<cli::Command> make_root() {
  auto root = std::make_unique<cli::Command>(
      "devspace", "Welcome to the DevSpace CLI!",
      "DevSpace accelerates developing, deploying and debugging applications with Docker and Kubernetes.\n"
      "This build targets Kubernetes nodes with AMD Instinct MI355X GPUs (amd.com/gpu).\n"
      "Get started by running the init command in one of your projects:\n\n    devspace init");
  root->persistent_bool("debug", "", false, "Prints the stack trace if an error occurs");
  register_core(*root);
  register_init(*root);
  register_config(*root);
  register_misc(*root);
  return root;
}

}  // namespace cmd
}  // namespace ds

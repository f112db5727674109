// devspace CLI entry point (main.go / cmd/root.go:35 Execute).
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "cli/common.h"
#include "core/log.h"
#include "core/net.h"
#include "core/trace.h"
#include "platform/platform.h"

// One span per CLI run with the transport counters: how many TCP dials / TLS handshakes the
// command cost and how many requests rode a pooled keep-alive connection.
static void emit_net_stats() {
  auto& s = ds::net::stats();
  if (s.requests.load() == 0 && s.tcp_dials.load() == 0) return;
  ds::trace::emit("net", ds::trace::now_us(), 0,
                  {{"tcp_dials", std::to_string(s.tcp_dials.load())},
                   {"tls_handshakes", std::to_string(s.tls_handshakes.load())},
                   {"tls_resumed", std::to_string(s.tls_resumed.load())},
                   {"requests", std::to_string(s.requests.load())},
                   {"reused", std::to_string(s.reused.load())},
                   {"proxied", std::to_string(s.proxied.load())}});
}

int main(int argc, char** argv) {
  ds::plat::set_argv0(argc > 0 ? argv[0] : nullptr);
  // a harness that wants its devspace children to end with it (tests/conftest.py) says so
  if (const char* p = std::getenv("DEVSPACE_PARENT_PID")) ds::plat::tie_to_parent(std::atol(p));
  ds::cmd::install_signal_handlers();
  ds::log::logdir();  // construct the function-local statics the handler uses before registering it
  ds::trace::enabled();
  std::atexit(emit_net_stats);
  std::vector<std::string> args(argv + 1, argv + argc);
  if (args.size() == 1 && (args[0] == "--version" || args[0] == "-v")) args[0] = "version";
  auto root = ds::cmd::make_root();
  ds::cmd::notify_newer_version(args);
  try {
    return root->execute(args);
  } catch (const ds::log::FatalError& e) {
    return 1;
  } catch (const std::exception& e) {
    // Any error that escaped a command is reported like log.Fatal does.
    ds::log::get().error(e.what());
    return 1;
  }
}

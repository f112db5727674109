// devspace CLI entry point (main.go / cmd/root.go:35 Execute).
#include <cstring>
#include <string>
#include <vector>

#include "cli/common.h"
#include "core/log.h"

int main(int argc, char** argv) {
  ds::cmd::install_signal_handlers();
  std::vector<std::string> args(argv + 1, argv + argc);
  if (args.size() == 1 && (args[0] == "--version" || args[0] == "-v")) args[0] = "version";
  auto root = ds::cmd::make_root();
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

// Tree-watcher factory of the portable build: the stat-diff scanner is the native backend
// (a kqueue or FSEvents backend replaces it per OS; docs/platforms.md).
#include <cstdlib>
#include <string>

#include "platform/watch.h"

namespace ds {

std::unique_ptr<TreeWatcher> make_tree_watcher() { return make_scan_watcher(scan_options_from_env()); }

}  // namespace ds

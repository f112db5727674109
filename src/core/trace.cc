#include "core/trace.h"

#include <unistd.h>

#include <cstdlib>
#include <mutex>

#include "core/fs.h"
#include "core/log.h"
#include "core/value.h"

namespace ds {
namespace trace {

// namespace scope: outlives atexit handlers registered from main() (the net.stats span)
static std::mutex g_mu;

bool enabled() {
  static const bool on = [] {
    const char* e = getenv("DEVSPACE_TRACE");
    return !(e && std::string(e) == "0");
  }();
  return on;
}

int64_t now_us() {
  return std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

void emit(const std::string& name, int64_t start_us, int64_t dur_us, const std::map<std::string, std::string>& fields) {
  if (!enabled()) return;
  // Only inside a project (.devspace/ exists): library users (bench, python module) that run
  // outside a project do not get stray log directories.
  std::string dir = log::logdir();
  if (!fs::is_dir(fs::dirname(fs::clean(dir)))) return;
  Value v = Value::map();
  v["span"] = name;
  v["start_us"] = start_us;
  v["dur_us"] = dur_us;
  v["pid"] = (int64_t)getpid();
  for (auto& kv : fields) v[kv.first] = kv.second;
  std::lock_guard<std::mutex> g(g_mu);
  try {
    fs::append_file(fs::join(dir, "trace.jsonl"), json_dump(v) + "\n");
  } catch (...) {
  }
}

}  // namespace trace
}  // namespace ds

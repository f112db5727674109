// File watching.
//  * TreeWatcher (platform/watch.h): recursive, event-driven where the OS allows it (the
//    reference uses rjeczalik/notify for the sync upstream, sync/sync_config.go:235).
//  * PollWatcher: glob-based size+mtime polling (watch/watch.go) — used for auto-reload paths
//    and symlink targets where a tree watcher cannot follow.
#pragma once

#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "platform/watch.h"

namespace ds {

class PollWatcher {
 public:
  // changed/deleted relative-or-absolute paths as matched by the patterns.
  using Callback = std::function<void(const std::vector<std::string>& changed, const std::vector<std::string>& deleted)>;
  PollWatcher(std::vector<std::string> patterns, Callback cb, int interval_ms = 1000);
  ~PollWatcher();
  void start();
  void stop();
  void update_patterns(std::vector<std::string> patterns);
  // One poll cycle (exposed for tests); returns true if anything changed.
  bool poll_once();

 private:
  struct Stamp {
    int64_t size, mtime_ns;
  };
  std::map<std::string, Stamp> gather();
  std::vector<std::string> patterns_;
  Callback cb_;
  int interval_ms_;
  std::map<std::string, Stamp> state_;
  bool primed_ = false;
  std::thread th_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool stop_ = false;
  bool started_ = false;
};

}  // namespace ds

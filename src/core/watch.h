// File watching.
//  * InotifyWatcher: recursive, event-driven (the reference uses rjeczalik/notify for the sync
//    upstream, sync/sync_config.go:235).
//  * PollWatcher: glob-based size+mtime polling (watch/watch.go) — used for auto-reload paths
//    and symlink targets where inotify cannot follow.
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

namespace ds {

class InotifyWatcher {
 public:
  // Callback receives absolute paths of changed entries (created/modified/removed/moved).
  // `overflow` is signalled with an empty path: the consumer should rescan. `settled` is true
  // for events that mark a finished write (close-after-write, rename-into, delete, mkdir).
  using Callback = std::function<void(const std::string& path, bool settled)>;
  InotifyWatcher() = default;
  ~InotifyWatcher();
  bool start(const std::string& root, Callback cb, std::string* err = nullptr);
  void stop();
  size_t watch_count();

 private:
  void add_recursive(const std::string& dir, bool emit_existing);
  void loop();
  int fd_ = -1;
  int wake_[2] = {-1, -1};
  std::string root_;
  Callback cb_;
  std::thread th_;
  std::atomic<bool> stop_{false};
  std::mutex mu_;
  std::unordered_map<int, std::string> wd_path_;
  std::unordered_map<std::string, int> path_wd_;
};

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

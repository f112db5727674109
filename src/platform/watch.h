// Recursive directory watching behind one event contract, the seam between the sync engine and
// the operating system's change notification.
//
// The reference watches sync paths with rjeczalik/notify (/root/reference/pkg/devspace/sync/
// sync_config.go:235): inotify on Linux, FSEvents on macOS, ReadDirectoryChangesW on Windows.
// Here:
//   * platform/linux_watch.cc — inotify, event-driven (the default build);
//   * platform/watch_scan.cc  — a stat-diff scanner, plain POSIX, with an interval that adapts
//                               to what a scan costs. It is the native backend of the portable
//                               build and the fallback anywhere (DEVSPACE_WATCHER=scan). A
//                               kqueue/FSEvents backend implements the same interface.
//
// Contract, whatever the backend:
//   * cb(path, settled) gets absolute paths of entries created, modified, removed or moved
//     below the root (not the root's existing entries at start);
//   * the entries of a directory that appears are reported too;
//   * an empty path means "events were lost: rescan";
//   * cb(root, true) means the root itself went away;
//   * `settled` marks a finished write (close after write, rename, delete, mkdir); an unsettled
//     change may be followed by more.
#pragma once

#include <functional>
#include <memory>
#include <string>

namespace ds {

class TreeWatcher {
 public:
  using Callback = std::function<void(const std::string& path, bool settled)>;
  virtual ~TreeWatcher() = default;
  virtual bool start(const std::string& root, Callback cb, std::string* err = nullptr) = 0;
  virtual void stop() = 0;
  // directories under watch
  virtual size_t watch_count() = 0;
  // "inotify", "scan", ...
  virtual const char* backend() const = 0;
};

// The platform's event-driven backend (scan where it has none). DEVSPACE_WATCHER=scan picks the
// scanner anywhere; DEVSPACE_WATCHER=native the event backend.
std::unique_ptr<TreeWatcher> make_tree_watcher();

struct ScanOptions {
  int min_interval_ms = 20;    // never scan more often than this
  int max_interval_ms = 1000;  // nor less often than this
  int cost_factor = 20;        // interval >= factor x the last scan's duration (<= 5 % of a core)
};
std::unique_ptr<TreeWatcher> make_scan_watcher(ScanOptions o = ScanOptions());
// Defaults, with DEVSPACE_SCAN_MIN_MS / DEVSPACE_SCAN_MAX_MS applied.
ScanOptions scan_options_from_env();

}  // namespace ds

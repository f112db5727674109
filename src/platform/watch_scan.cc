// Stat-diff tree watcher (platform/watch.h): plain POSIX, no change notification needed.
//
// Each scan lstat()s the tree and diffs it against the previous scan by (size, mtime, mode,
// inode): an inode change catches an editor's write-temp-and-rename that kept size and mtime.
// The interval adapts to the tree: a scan never takes more than 1/cost_factor of the time (5 %
// of one core by default), within [min_interval_ms, max_interval_ms]. A small project is
// scanned every 20 ms, a 10k-file tree every few hundred. Symlinks are not followed (the sync
// engine polls link targets itself, like the reference's sync/symlink.go).
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include "core/fs.h"
#include "platform/watch.h"

namespace ds {

namespace {

struct Stamp {
  int64_t size = 0;
  int64_t mtime_ns = 0;
  uint32_t mode = 0;
  uint64_t ino = 0;
  bool operator!=(const Stamp& o) const {
    return size != o.size || mtime_ns != o.mtime_ns || mode != o.mode || ino != o.ino;
  }
};

using Tree = std::map<std::string, Stamp>;

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::system_clock::now().time_since_epoch())
      .count();
}

class ScanWatcher : public TreeWatcher {
 public:
  explicit ScanWatcher(ScanOptions o) : o_(o) {}
  ~ScanWatcher() override { stop(); }

  bool start(const std::string& root, Callback cb, std::string* err) override {
    root_ = root;
    cb_ = std::move(cb);
    if (!fs::is_dir(root_)) {
      if (err) *err = "cannot watch " + root_ + ": not a directory";
      return false;
    }
    int64_t cost = scan(&tree_);
    interval_ms_ = next_interval(cost);
    th_ = std::thread([this] { loop(); });
    return true;
  }

  void stop() override {
    {
      std::lock_guard<std::mutex> g(mu_);  // no lost wake-up between the loop's check and wait
      if (stop_.exchange(true)) return;
    }
    cv_.notify_all();
    if (th_.joinable()) th_.join();
  }

  size_t watch_count() override { return dirs_.load(); }
  const char* backend() const override { return "scan"; }

 private:
  // Fills *out with the tree below root_; returns the scan's duration in ms.
  int64_t scan(Tree* out) {
    auto t0 = std::chrono::steady_clock::now();
    size_t dirs = 1;
    std::vector<std::string> stack{root_};
    while (!stack.empty()) {
      std::string dir = std::move(stack.back());
      stack.pop_back();
      for (auto& e : fs::list_dir(dir)) {
        std::string p = fs::join(dir, e.name);
        fs::StatInfo st = fs::lstat(p);
        if (!st.exists) continue;  // removed while listing
        (*out)[p] = {st.size, st.mtime_sec * 1000000000LL + st.mtime_nsec, st.mode, st.ino};
        if (st.is_dir && !st.is_symlink) {
          stack.push_back(p);
          ++dirs;
        }
      }
    }
    dirs_ = dirs;
    return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
  }

  int next_interval(int64_t cost_ms) const {
    int64_t iv = cost_ms * o_.cost_factor;
    if (iv < o_.min_interval_ms) iv = o_.min_interval_ms;
    if (iv > o_.max_interval_ms) iv = o_.max_interval_ms;
    return (int)iv;
  }

  void loop() {
    while (true) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        if (cv_.wait_for(lk, std::chrono::milliseconds(interval_ms_), [this] { return stop_.load(); })) return;
      }
      if (!fs::is_dir(root_)) {
        cb_(root_, true);
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return stop_.load(); });  // nothing left to watch
        return;
      }
      Tree now;
      int64_t cost = scan(&now);
      interval_ms_ = next_interval(cost);
      diff(now);
      tree_ = std::move(now);
    }
  }

  void diff(const Tree& now) {
    // a write that ended within two intervals may still be going on: unsettled
    int64_t recent = now_ns() - 2LL * interval_ms_ * 1000000LL;
    for (auto& kv : now) {  // path order: a new directory before its entries
      if (stop_) return;
      auto it = tree_.find(kv.first);
      if (it != tree_.end() && !(it->second != kv.second)) continue;
      bool is_dir = S_ISDIR(kv.second.mode);
      cb_(kv.first, is_dir || kv.second.mtime_ns < recent);
    }
    for (auto it = tree_.rbegin(); it != tree_.rend(); ++it) {  // entries before their directory
      if (stop_) return;
      if (!now.count(it->first)) cb_(it->first, true);
    }
  }

  ScanOptions o_;
  std::string root_;
  Callback cb_;
  Tree tree_;  // only the scan thread touches it after start()
  int interval_ms_ = 20;
  std::atomic<size_t> dirs_{0};
  std::thread th_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::atomic<bool> stop_{false};
};

}  // namespace

std::unique_ptr<TreeWatcher> make_scan_watcher(ScanOptions o) { return std::make_unique<ScanWatcher>(o); }

ScanOptions scan_options_from_env() {
  ScanOptions o;
  auto num = [](const char* name, int* out) {
    const char* v = getenv(name);
    if (!v || !*v) return;
    char* end = nullptr;
    long n = strtol(v, &end, 10);
    if (end && !*end && n > 0 && n < 600000) *out = (int)n;
  };
  num("DEVSPACE_SCAN_MIN_MS", &o.min_interval_ms);
  num("DEVSPACE_SCAN_MAX_MS", &o.max_interval_ms);
  if (o.max_interval_ms < o.min_interval_ms) o.max_interval_ms = o.min_interval_ms;
  return o;
}

}  // namespace ds

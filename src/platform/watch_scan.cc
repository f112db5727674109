// Stat-diff tree watcher (platform/watch.h): plain POSIX, no change notification needed.
//
// Two passes over the tree's lstat()s, diffed by (size, mtime, mode, inode) — an inode change
// catches an editor's write-temp-and-rename that kept size and mtime:
//   * the quick pass, every min_interval_ms: every directory, and the files changed lately
//     (the "hot" set, the files being edited). A directory whose stamp changed had entries
//     created, removed or renamed (an editor's atomic save among them): its entries are listed
//     again. Cost: one lstat per directory plus the hot files, so in a 10k-file tree of 100
//     directories a new file, a save by rename or a re-edit shows within tens of milliseconds;
//   * the full pass: every entry, compared in place (fstatat against the open directory, no
//     second tree built), at an interval that follows what it costs (at most 1/cost_factor of
//     the time, 5 % of one core by default, within [min, max]): it finds in-place writes to
//     files nobody touched lately.
// Symlinks are not followed (the sync engine polls link targets itself, like the reference's
// sync/symlink.go).
#include <dirent.h>
#include <fcntl.h>
#include <sys/stat.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include "core/fs.h"
#include "platform/platform.h"
#include "platform/watch.h"

namespace ds {

namespace {

struct Stamp {
  int64_t size = 0;
  int64_t mtime_ns = 0;
  uint32_t mode = 0;
  uint64_t ino = 0;
  uint32_t seen = 0;  // the full pass that last listed it (not part of the comparison)
  bool operator!=(const Stamp& o) const {
    return size != o.size || mtime_ns != o.mtime_ns || mode != o.mode || ino != o.ino;
  }
  bool is_dir() const { return S_ISDIR(mode); }
};

using Tree = std::map<std::string, Stamp>;

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::system_clock::now().time_since_epoch())
      .count();
}

int64_t mono_us() {
  return std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

Stamp to_stamp(const struct stat& st) {
  Stamp s;
  s.size = st.st_size;
  s.mtime_ns = plat::mtime_ns(st);
  s.mode = st.st_mode;
  s.ino = st.st_ino;
  return s;
}

bool stamp_of(const std::string& p, Stamp* out) {
  struct stat st;
  if (::lstat(p.c_str(), &st) != 0) return false;
  *out = to_stamp(st);
  return true;
}

// The entries of dir with their stamps (fstatat against the open directory: no path walk per
// entry). Entries removed while listing are left out; false if dir cannot be opened.
bool list_stamps(const std::string& dir, std::vector<std::pair<std::string, Stamp>>* out) {
  out->clear();
  DIR* d = ::opendir(dir.c_str());
  if (!d) return false;
  const int fd = ::dirfd(d);
  while (struct dirent* e = ::readdir(d)) {
    const char* n = e->d_name;
    if (n[0] == '.' && (n[1] == 0 || (n[1] == '.' && n[2] == 0))) continue;
    struct stat st;
    if (::fstatat(fd, n, &st, AT_SYMLINK_NOFOLLOW) != 0) continue;
    out->emplace_back(fs::join(dir, n), to_stamp(st));
  }
  ::closedir(d);
  return true;
}

constexpr size_t kHotMax = 512;              // files re-checked by every quick pass
constexpr int64_t kHotKeepUs = 600000000;  // a file stays hot for 10 minutes after its last change

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
    full_pass(false);
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
  int64_t clamp_interval_us(int64_t cost_us) const {
    int64_t iv = cost_us * o_.cost_factor;
    if (iv < o_.min_interval_ms * 1000LL) iv = o_.min_interval_ms * 1000LL;
    if (iv > o_.max_interval_ms * 1000LL) iv = o_.max_interval_ms * 1000LL;
    return iv;
  }

  bool settled(const Stamp& s, int64_t interval_us) const {
    // a write that ended within two intervals may still be going on: unsettled
    return s.is_dir() || s.mtime_ns < now_ns() - 2LL * interval_us * 1000LL;
  }

  void emit_change(const std::string& p, const Stamp& s, int64_t interval_us) {
    cb_(p, settled(s, interval_us));
    if (!s.is_dir()) hot(p);
  }

  void hot(const std::string& p) {
    hot_[p] = mono_us();
    if (hot_.size() <= kHotMax) return;
    auto oldest = hot_.begin();
    for (auto it = hot_.begin(); it != hot_.end(); ++it)
      if (it->second < oldest->second) oldest = it;
    hot_.erase(oldest);
  }

  void forget(const std::string& p) {
    tree_.erase(p);
    hot_.erase(p);
  }

  // Removes p and everything below it from tree_, reporting each (entries before their dirs).
  void remove_subtree(const std::string& p, bool report_p) {
    auto lo = tree_.lower_bound(p + "/"), hi = tree_.lower_bound(p + "0");  // '0' follows '/'
    std::vector<std::string> gone;
    for (auto it = lo; it != hi; ++it) gone.push_back(it->first);
    for (auto it = gone.rbegin(); it != gone.rend(); ++it) {
      cb_(*it, true);
      forget(*it);
    }
    if (report_p) {
      cb_(p, true);
      forget(p);
    }
  }

  // Adds a new directory's whole subtree to tree_, reporting each entry (a directory before
  // its entries).
  void add_subtree(const std::string& dir, int64_t interval_us) {
    std::vector<std::string> stack{dir};
    std::vector<std::pair<std::string, Stamp>> entries;
    while (!stack.empty()) {
      std::string d = std::move(stack.back());
      stack.pop_back();
      list_stamps(d, &entries);
      for (auto& kv : entries) {
        kv.second.seen = gen_;
        tree_[kv.first] = kv.second;
        emit_change(kv.first, kv.second, interval_us);
        if (kv.second.is_dir()) stack.push_back(kv.first);
      }
    }
  }

  // The direct entries of a directory whose stamp changed, against tree_.
  void rescan_dir(const std::string& dir, int64_t interval_us) {
    std::vector<std::pair<std::string, Stamp>> entries;
    list_stamps(dir, &entries);
    std::map<std::string, Stamp> now(entries.begin(), entries.end());
    const std::string prefix = dir + "/";
    std::vector<std::string> gone;
    for (auto it = tree_.lower_bound(prefix); it != tree_.end() && it->first.compare(0, prefix.size(), prefix) == 0;
         ++it)
      if (it->first.find('/', prefix.size()) == std::string::npos && !now.count(it->first)) gone.push_back(it->first);
    for (auto& p : gone) remove_subtree(p, true);
    for (auto& kv : now) {
      kv.second.seen = gen_;
      auto it = tree_.find(kv.first);
      if (it == tree_.end()) {
        tree_[kv.first] = kv.second;
        emit_change(kv.first, kv.second, interval_us);
        if (kv.second.is_dir()) add_subtree(kv.first, interval_us);
        continue;
      }
      if (!(it->second != kv.second)) continue;
      const bool was_dir = it->second.is_dir();
      it->second = kv.second;
      if (was_dir && !kv.second.is_dir()) remove_subtree(kv.first, false);  // a directory replaced
      if (!kv.second.is_dir()) {
        emit_change(kv.first, kv.second, interval_us);
      } else if (!was_dir) {
        emit_change(kv.first, kv.second, interval_us);  // a file replaced by a directory
        add_subtree(kv.first, interval_us);
      }
      // (a directory's own stamp change is handled when it is visited: its entries changed)
    }
  }

  // Directories and hot files; returns its duration in us.
  int64_t quick_pass() {
    const int64_t t0 = mono_us();
    const int64_t iv = o_.min_interval_ms * 1000LL;
    Stamp rs;
    if (!stamp_of(root_, &rs) || !rs.is_dir()) {
      root_gone_ = true;
      return 0;
    }
    std::vector<std::string> changed_dirs;
    if (rs != root_stamp_) changed_dirs.push_back(root_);
    root_stamp_ = rs;
    size_t dirs = 1;
    for (auto& kv : tree_) {
      if (!kv.second.is_dir()) continue;
      ++dirs;
      Stamp s;
      if (!stamp_of(kv.first, &s) || s != kv.second) changed_dirs.push_back(kv.first);
    }
    dirs_ = dirs;
    for (auto& d : changed_dirs) {
      if (stop_) break;
      if (d != root_) {
        auto it = tree_.find(d);
        if (it == tree_.end()) continue;  // went with a parent's rescan
        Stamp s;
        if (!stamp_of(d, &s) || !s.is_dir()) continue;  // gone or replaced: its parent's rescan says so
        it->second.size = s.size;
        it->second.mtime_ns = s.mtime_ns;
        it->second.mode = s.mode;
        it->second.ino = s.ino;
      }
      rescan_dir(d, iv);
    }
    const int64_t now = mono_us();
    std::vector<std::string> cold;
    for (auto& kv : hot_) {
      if (now - kv.second > kHotKeepUs) {
        cold.push_back(kv.first);
        continue;
      }
      auto it = tree_.find(kv.first);
      if (it == tree_.end()) continue;
      Stamp s;
      if (stamp_of(kv.first, &s) && s != it->second && !s.is_dir() && !it->second.is_dir()) {
        s.seen = it->second.seen;
        it->second = s;
        cb_(kv.first, settled(s, iv));
        kv.second = now;
      }
    }
    for (auto& p : cold) hot_.erase(p);
    return mono_us() - t0;
  }

  // Every entry, compared in place against tree_; report=false fills tree_ silently (start()).
  void full_pass(bool report) {
    const int64_t t0 = mono_us();
    const uint32_t gen = ++gen_;
    const int64_t iv = full_interval_us_;
    size_t dirs = 1;
    std::vector<std::string> stack{root_};
    std::vector<std::pair<std::string, Stamp>> entries;
    while (!stack.empty() && !stop_) {
      std::string dir = std::move(stack.back());
      stack.pop_back();
      list_stamps(dir, &entries);
      for (auto& kv : entries) {
        kv.second.seen = gen;
        auto ins = tree_.emplace(kv.first, kv.second);
        if (ins.second) {  // new (a directory is listed before its entries)
          if (report) emit_change(kv.first, kv.second, iv);
        } else {
          Stamp& old = ins.first->second;
          const bool changed = old != kv.second, was_dir = old.is_dir();
          old = kv.second;
          if (changed && report && !(was_dir && kv.second.is_dir())) emit_change(kv.first, kv.second, iv);
        }
        if (kv.second.is_dir()) {
          stack.push_back(kv.first);
          ++dirs;
        }
      }
    }
    if (stop_) return;
    std::vector<std::string> gone;
    for (auto it = tree_.rbegin(); it != tree_.rend(); ++it)  // entries before their directory
      if (it->second.seen != gen) gone.push_back(it->first);
    for (auto& p : gone) {
      if (report) cb_(p, true);
      forget(p);
    }
    stamp_of(root_, &root_stamp_);
    dirs_ = dirs;
    full_interval_us_ = clamp_interval_us(mono_us() - t0);
  }

  void loop() {
    int64_t next_full = mono_us() + full_interval_us_;
    int64_t quick_us = o_.min_interval_ms * 1000LL;
    while (true) {
      int64_t wait = std::min<int64_t>(quick_us, std::max<int64_t>(0, next_full - mono_us()));
      {
        std::unique_lock<std::mutex> lk(mu_);
        if (cv_.wait_for(lk, std::chrono::microseconds(wait), [this] { return stop_.load(); })) return;
      }
      if (mono_us() >= next_full) {
        if (!fs::is_dir(root_)) {
          root_gone_ = true;
        } else {
          full_pass(true);
          next_full = mono_us() + full_interval_us_;
        }
      } else {
        // the quick pass keeps within the same CPU budget as the full one
        quick_us = clamp_interval_us(quick_pass());
      }
      if (root_gone_) {
        cb_(root_, true);
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return stop_.load(); });  // nothing left to watch
        return;
      }
    }
  }

  ScanOptions o_;
  std::string root_;
  Callback cb_;
  Tree tree_;  // only the scan thread touches these after start()
  Stamp root_stamp_;
  std::map<std::string, int64_t> hot_;  // path -> last change (monotonic us)
  uint32_t gen_ = 0;
  int64_t full_interval_us_ = 20000;
  bool root_gone_ = false;
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

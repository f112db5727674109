#include "core/watch.h"

#include <fcntl.h>
#include <poll.h>
#include <sys/inotify.h>
#include <unistd.h>

#include <cstring>

#include "core/fs.h"
#include "core/match.h"
#include "core/strutil.h"

namespace ds {

static const uint32_t kMask = IN_CREATE | IN_DELETE | IN_MODIFY | IN_CLOSE_WRITE | IN_MOVED_FROM | IN_MOVED_TO |
                              IN_ATTRIB | IN_DELETE_SELF | IN_MOVE_SELF | IN_ONLYDIR * 0;

InotifyWatcher::~InotifyWatcher() { stop(); }

bool InotifyWatcher::start(const std::string& root, Callback cb, std::string* err) {
  root_ = root;
  cb_ = std::move(cb);
  fd_ = inotify_init1(IN_NONBLOCK | IN_CLOEXEC);
  if (fd_ < 0) {
    if (err) *err = std::string("inotify_init1: ") + std::strerror(errno);
    return false;
  }
  if (::pipe2(wake_, O_CLOEXEC | O_NONBLOCK) != 0) {
    if (err) *err = "pipe2 failed";
    return false;
  }
  add_recursive(root_, false);
  if (path_wd_.empty()) {
    if (err) *err = "cannot watch " + root_;
    return false;
  }
  th_ = std::thread([this] { loop(); });
  return true;
}

void InotifyWatcher::stop() {
  if (stop_.exchange(true)) return;
  if (wake_[1] >= 0) {
    char c = 1;
    ssize_t ignored = ::write(wake_[1], &c, 1);
    (void)ignored;
  }
  if (th_.joinable()) th_.join();
  if (fd_ >= 0) ::close(fd_);
  if (wake_[0] >= 0) ::close(wake_[0]);
  if (wake_[1] >= 0) ::close(wake_[1]);
  fd_ = wake_[0] = wake_[1] = -1;
}

size_t InotifyWatcher::watch_count() {
  std::lock_guard<std::mutex> g(mu_);
  return path_wd_.size();
}

void InotifyWatcher::add_recursive(const std::string& dir, bool emit_existing) {
  int wd = inotify_add_watch(fd_, dir.c_str(), kMask);
  if (wd < 0) return;
  {
    std::lock_guard<std::mutex> g(mu_);
    wd_path_[wd] = dir;
    path_wd_[dir] = wd;
  }
  for (auto& e : fs::list_dir(dir)) {
    std::string p = fs::join(dir, e.name);
    // Entries created between mkdir and add_watch would otherwise be missed.
    if (emit_existing && cb_) cb_(p, true);
    if (e.is_dir && !e.is_symlink) add_recursive(p, emit_existing);
  }
}

void InotifyWatcher::loop() {
  alignas(struct inotify_event) char buf[1 << 16];
  while (!stop_) {
    struct pollfd pf[2] = {{fd_, POLLIN, 0}, {wake_[0], POLLIN, 0}};
    int r = ::poll(pf, 2, 1000);
    if (r < 0) {
      if (errno == EINTR) continue;
      break;
    }
    if (stop_) break;
    if (!(pf[0].revents & POLLIN)) continue;
    while (true) {
      ssize_t n = ::read(fd_, buf, sizeof(buf));
      if (n <= 0) break;
      for (char* p = buf; p < buf + n;) {
        auto* ev = (struct inotify_event*)p;
        p += sizeof(struct inotify_event) + ev->len;
        if (ev->mask & IN_Q_OVERFLOW) {
          if (cb_) cb_("", true);
          continue;
        }
        std::string dir;
        {
          std::lock_guard<std::mutex> g(mu_);
          auto it = wd_path_.find(ev->wd);
          if (it == wd_path_.end()) continue;
          dir = it->second;
        }
        if (ev->mask & IN_IGNORED) {
          std::lock_guard<std::mutex> g(mu_);
          path_wd_.erase(dir);
          wd_path_.erase(ev->wd);
          continue;
        }
        std::string path = ev->len ? fs::join(dir, std::string(ev->name)) : dir;
        if ((ev->mask & (IN_DELETE_SELF | IN_MOVE_SELF)) && path == root_) {
          if (cb_) cb_(path, true);
          continue;
        }
        if ((ev->mask & IN_ISDIR) && (ev->mask & (IN_CREATE | IN_MOVED_TO))) {
          if (cb_) cb_(path, true);
          add_recursive(path, true);
          continue;
        }
        if ((ev->mask & IN_ISDIR) && (ev->mask & (IN_DELETE | IN_MOVED_FROM))) {
          std::lock_guard<std::mutex> g(mu_);
          // watches below a moved-away directory are stale
          for (auto it = path_wd_.begin(); it != path_wd_.end();) {
            if (it->first == path || starts_with(it->first, path + "/")) {
              inotify_rm_watch(fd_, it->second);
              wd_path_.erase(it->second);
              it = path_wd_.erase(it);
            } else {
              ++it;
            }
          }
        }
        if (ev->mask & (IN_DELETE_SELF | IN_MOVE_SELF)) continue;
        bool settled = (ev->mask & (IN_CLOSE_WRITE | IN_MOVED_TO | IN_MOVED_FROM | IN_DELETE)) != 0;
        if (cb_) cb_(path, settled);
      }
    }
  }
}

// ---------------------------------------------------------------- poll watcher

PollWatcher::PollWatcher(std::vector<std::string> patterns, Callback cb, int interval_ms)
    : patterns_(std::move(patterns)), cb_(std::move(cb)), interval_ms_(interval_ms) {}

PollWatcher::~PollWatcher() { stop(); }

std::map<std::string, PollWatcher::Stamp> PollWatcher::gather() {
  std::vector<std::string> pats;
  {
    std::lock_guard<std::mutex> g(mu_);
    pats = patterns_;
  }
  std::map<std::string, Stamp> out;
  for (auto& p : pats) {
    for (auto& f : glob_expand(p)) {
      // the reference ignores .devspace* paths (watch/watch.go:140)
      if (contains(f, ".devspace")) continue;
      fs::StatInfo st = fs::stat(f);
      if (!st.exists) continue;
      out[f] = {st.size, st.mtime_sec * 1000000000LL + st.mtime_nsec};
    }
  }
  return out;
}

bool PollWatcher::poll_once() {
  auto now = gather();
  if (!primed_) {
    state_ = now;
    primed_ = true;
    return false;
  }
  std::vector<std::string> changed, deleted;
  for (auto& kv : now) {
    auto it = state_.find(kv.first);
    if (it == state_.end() || it->second.size != kv.second.size || it->second.mtime_ns != kv.second.mtime_ns)
      changed.push_back(kv.first);
  }
  for (auto& kv : state_)
    if (!now.count(kv.first)) deleted.push_back(kv.first);
  state_ = std::move(now);
  if ((!changed.empty() || !deleted.empty()) && cb_) cb_(changed, deleted);
  return !changed.empty() || !deleted.empty();
}

void PollWatcher::start() {
  std::lock_guard<std::mutex> g(mu_);
  if (started_) return;  // (watch/watch.go:50 checks-then-sets under two locks; one here)
  started_ = true;
  stop_ = false;
  th_ = std::thread([this] {
    poll_once();
    while (true) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        if (cv_.wait_for(lk, std::chrono::milliseconds(interval_ms_), [this] { return stop_; })) return;
      }
      poll_once();
    }
  });
}

void PollWatcher::stop() {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (!started_) return;
    stop_ = true;
    started_ = false;
  }
  cv_.notify_all();
  if (th_.joinable()) th_.join();
}

void PollWatcher::update_patterns(std::vector<std::string> patterns) {
  std::lock_guard<std::mutex> g(mu_);
  patterns_ = std::move(patterns);
}

}  // namespace ds

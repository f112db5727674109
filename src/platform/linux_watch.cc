// inotify backend of platform/watch.h (the default Linux build), plus the factory that picks
// the backend.
#include <fcntl.h>
#include <poll.h>
#include <sys/inotify.h>
#include <unistd.h>

#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <unordered_map>

#include "core/fs.h"
#include "core/strutil.h"
#include "platform/platform.h"
#include "platform/watch.h"

namespace ds {

namespace {

class InotifyWatcher : public TreeWatcher {
 public:
  InotifyWatcher() = default;
  ~InotifyWatcher() override;
  bool start(const std::string& root, Callback cb, std::string* err) override;
  void stop() override;
  size_t watch_count() override;
  const char* backend() const override { return "inotify"; }

 private:
  void add_recursive(const std::string& dir, bool emit_existing);
  void loop();
  int fd_ = -1;
  plat::Waker wake_;
  std::string root_;
  Callback cb_;
  std::thread th_;
  std::atomic<bool> stop_{false};
  std::mutex mu_;
  std::unordered_map<int, std::string> wd_path_;
  std::unordered_map<std::string, int> path_wd_;
};

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
  if (!wake_.ok()) {
    if (err) *err = std::string("cannot create the wake-up descriptor: ") + std::strerror(errno);
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
  wake_.poke();
  if (th_.joinable()) th_.join();
  if (fd_ >= 0) ::close(fd_);
  fd_ = -1;
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
    struct pollfd pf[2] = {{fd_, POLLIN, 0}, {wake_.fd(), POLLIN, 0}};
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

}  // namespace

std::unique_ptr<TreeWatcher> make_tree_watcher() {
  const char* w = getenv("DEVSPACE_WATCHER");
  if (w && std::string(w) == "scan") return make_scan_watcher(scan_options_from_env());
  return std::make_unique<InotifyWatcher>();
}

}  // namespace ds

// The OS seam (src/platform/): the contracts both implementations keep, and the tree-watcher
// event contract run against every backend this build has (inotify and the stat-diff scanner
// in the default build; the scanner alone in -DDEVSPACE_PORTABLE=ON).
#include <fcntl.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <set>
#include <thread>

#include "core/fs.h"
#include "platform/platform.h"
#include "platform/watch.h"
#include "testing.h"

using namespace ds;

namespace {

bool cloexec(int fd) { return (fcntl(fd, F_GETFD) & FD_CLOEXEC) != 0; }

// Collects watcher events; wait_for(path) blocks until that path was reported.
struct Events {
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::pair<std::string, bool>> got;
  TreeWatcher::Callback cb() {
    return [this](const std::string& p, bool settled) {
      std::lock_guard<std::mutex> g(mu);
      got.push_back({p, settled});
      cv.notify_all();
    };
  }
  bool wait_for(const std::string& path, int ms = 3000) {
    std::unique_lock<std::mutex> lk(mu);
    return cv.wait_for(lk, std::chrono::milliseconds(ms), [&] {
      for (auto& e : got)
        if (e.first == path) return true;
      return false;
    });
  }
  void clear() {
    std::lock_guard<std::mutex> g(mu);
    got.clear();
  }
  std::set<std::string> paths() {
    std::lock_guard<std::mutex> g(mu);
    std::set<std::string> s;
    for (auto& e : got) s.insert(e.first);
    return s;
  }
};

void check_watcher_contract(std::unique_ptr<TreeWatcher> w) {
  std::string root = fs::make_temp_dir("ds-watch-");
  fs::write_file(root + "/old.txt", "x");
  fs::mkdirs(root + "/sub");
  Events ev;
  std::string err;
  EXPECT_TRUE(w->start(root, ev.cb(), &err));
  EXPECT_TRUE(w->watch_count() >= 2);  // the root and sub/
  std::this_thread::sleep_for(std::chrono::milliseconds(50));
  EXPECT_TRUE(ev.paths().empty());  // what existed at start is not reported

  fs::write_file(root + "/sub/new.txt", "hello");
  EXPECT_TRUE(ev.wait_for(root + "/sub/new.txt"));

  // a directory that appears with entries: all of them
  std::string stage = fs::make_temp_dir("ds-watch-stage-");
  fs::write_file(stage + "/inner/a.txt", "a");
  EXPECT_TRUE(fs::rename(stage, root + "/moved"));
  EXPECT_TRUE(ev.wait_for(root + "/moved"));
  // inotify reports the moved-in directory's entries from its rescan, the scanner from the diff
  EXPECT_TRUE(ev.wait_for(root + "/moved/inner/a.txt"));

  // an editor's atomic save: write a temp, rename it over the file (same size)
  ev.clear();
  fs::write_file(root + "/old.txt.tmp", "y");
  EXPECT_TRUE(fs::rename(root + "/old.txt.tmp", root + "/old.txt"));
  EXPECT_TRUE(ev.wait_for(root + "/old.txt"));

  ev.clear();
  EXPECT_TRUE(fs::remove(root + "/sub/new.txt"));
  EXPECT_TRUE(ev.wait_for(root + "/sub/new.txt"));
  {
    std::lock_guard<std::mutex> g(ev.mu);
    bool settled = false;
    for (auto& e : ev.got)
      if (e.first == root + "/sub/new.txt") settled = settled || e.second;
    EXPECT_TRUE(settled);  // a removal is a finished change
  }
  w->stop();
  fs::remove_all(root);
}

}  // namespace

TEST(platform_descriptors_are_close_on_exec) {
  int p[2];
  EXPECT_EQ(plat::pipe_cloexec(p, true), 0);
  EXPECT_TRUE(cloexec(p[0]) && cloexec(p[1]));
  EXPECT_TRUE((fcntl(p[0], F_GETFL) & O_NONBLOCK) != 0);
  close(p[0]);
  close(p[1]);
  int s = plat::socket_cloexec(AF_INET, SOCK_STREAM);
  EXPECT_TRUE(s >= 0 && cloexec(s));
  close(s);
  std::string d = fs::make_temp_dir("ds-plat-");
  int t = plat::open_unlinked_tmp(d);
  EXPECT_TRUE(t >= 0 && cloexec(t));
  EXPECT_EQ(::write(t, "abc", 3), (ssize_t)3);
  EXPECT_TRUE(fs::list_dir(d).empty());  // nameless: nothing to clean up
  close(t);
  fs::remove_all(d);
}

TEST(platform_accept_is_close_on_exec_and_send_never_raises_sigpipe) {
  int l = plat::socket_cloexec(AF_INET, SOCK_STREAM);
  struct sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  EXPECT_EQ(::bind(l, (struct sockaddr*)&a, sizeof(a)), 0);
  EXPECT_EQ(::listen(l, 4), 0);
  socklen_t len = sizeof(a);
  getsockname(l, (struct sockaddr*)&a, &len);
  int c = plat::socket_cloexec(AF_INET, SOCK_STREAM);
  EXPECT_EQ(::connect(c, (struct sockaddr*)&a, sizeof(a)), 0);
  int s = plat::accept_cloexec(l);
  EXPECT_TRUE(s >= 0 && cloexec(s));
  close(s);
  // the peer is gone: an error return (EPIPE or ECONNRESET). The Linux build passes
  // MSG_NOSIGNAL; the POSIX one relies on SIGPIPE being ignored, as the CLI's main() and this
  // harness do.
  ssize_t r = 0;
  for (int i = 0; i < 50 && r >= 0; ++i) r = plat::send_nosignal(c, "x", 1), usleep(1000);
  EXPECT_TRUE(r < 0);
  close(c);
  close(l);
}

TEST(platform_waker_wakes_a_poll_and_drains) {
  plat::Waker w;
  EXPECT_TRUE(w.ok());
  struct pollfd pf{w.fd(), POLLIN, 0};
  EXPECT_EQ(::poll(&pf, 1, 0), 0);
  std::thread t([&] { w.poke(); });
  EXPECT_EQ(::poll(&pf, 1, 2000), 1);
  t.join();
  w.poke();
  w.poke();
  w.drain();
  EXPECT_EQ(::poll(&pf, 1, 0), 0);
}

TEST(platform_self_exe_is_this_test_binary) {
  // the POSIX build learns it from argv[0]; give it what main() would
  plat::set_argv0(DEVSPACE_SOURCE_DIR "/bin/devspace_tests");
  std::string exe = plat::self_exe();
  EXPECT_TRUE(!exe.empty());
  EXPECT_EQ(fs::basename(exe), std::string("devspace_tests"));
  EXPECT_TRUE(fs::is_abs(exe));
}

TEST(platform_mtime_has_nanoseconds) {
  std::string d = fs::make_temp_dir("ds-plat-");
  fs::write_file(d + "/f", "x");
  EXPECT_TRUE(fs::set_mtime(d + "/f", 1500000000, 123456789));
  struct stat st;
  EXPECT_EQ(::stat((d + "/f").c_str(), &st), 0);
  EXPECT_EQ(plat::mtime_ns(st), (int64_t)1500000000 * 1000000000LL + 123456789);
  fs::StatInfo si = fs::stat(d + "/f");
  EXPECT_EQ(si.mtime_sec, (int64_t)1500000000);
  EXPECT_EQ(si.mtime_nsec, (int64_t)123456789);
  fs::remove_all(d);
}

TEST(platform_native_tree_watcher_keeps_the_contract) { check_watcher_contract(make_tree_watcher()); }

TEST(platform_scan_tree_watcher_keeps_the_contract) {
  ScanOptions o;
  o.min_interval_ms = 10;
  auto w = make_scan_watcher(o);
  EXPECT_EQ(std::string(w->backend()), std::string("scan"));
  check_watcher_contract(std::move(w));
}

TEST(platform_scan_watcher_reports_a_vanished_root) {
  std::string root = fs::make_temp_dir("ds-watch-");
  ScanOptions o;
  o.min_interval_ms = 10;
  auto w = make_scan_watcher(o);
  Events ev;
  EXPECT_TRUE(w->start(root, ev.cb(), nullptr));
  fs::remove_all(root);
  EXPECT_TRUE(ev.wait_for(root));
  w->stop();
}

TEST(platform_scan_watcher_interval_follows_the_scan_cost) {
  // 3000 files: a scan costs a few ms, so the scanner must slow down below its minimum, yet still
  // see an edit within its maximum
  std::string root = fs::make_temp_dir("ds-watch-");
  for (int d = 0; d < 30; ++d)
    for (int f = 0; f < 100; ++f) fs::write_file(root + "/d" + std::to_string(d) + "/f" + std::to_string(f), "x");
  ScanOptions o;
  o.min_interval_ms = 1;
  o.max_interval_ms = 400;
  auto w = make_scan_watcher(o);
  Events ev;
  EXPECT_TRUE(w->start(root, ev.cb(), nullptr));
  EXPECT_EQ(w->watch_count(), (size_t)31);
  auto t0 = std::chrono::steady_clock::now();
  fs::write_file(root + "/d7/f7", "changed");
  EXPECT_TRUE(ev.wait_for(root + "/d7/f7", 2000));
  auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
  EXPECT_TRUE(ms < 1000);
  EXPECT_EQ(ev.paths().size(), (size_t)1);
  w->stop();
  fs::remove_all(root);
}

TEST(platform_scan_watcher_quick_pass_sees_new_and_hot_files_between_full_scans) {
  // a CPU budget of 0.1 %: full scans of the 1000 files every 2 s (the maximum), quick passes
  // over the 21 directories and the hot files every few tens of ms. Creations, atomic saves and
  // re-edits of a file being worked on come through the quick pass, an in-place edit of a cold
  // file through the next full scan
  std::string root = fs::make_temp_dir("ds-watch-");
  for (int d = 0; d < 20; ++d)
    for (int f = 0; f < 50; ++f) fs::write_file(root + "/d" + std::to_string(d) + "/f" + std::to_string(f), "x");
  ScanOptions o;
  o.min_interval_ms = 20;
  o.max_interval_ms = 2000;
  o.cost_factor = 1000;
  auto w = make_scan_watcher(o);
  Events ev;
  EXPECT_TRUE(w->start(root, ev.cb(), nullptr));
  auto since = [](std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
  };
  auto t0 = std::chrono::steady_clock::now();
  fs::write_file(root + "/d3/new.py", "a");  // a new entry: d3's mtime moves
  EXPECT_TRUE(ev.wait_for(root + "/d3/new.py", 3000));
  EXPECT_TRUE(since(t0) < 1000);
  ev.clear();
  std::this_thread::sleep_for(std::chrono::milliseconds(30));
  t0 = std::chrono::steady_clock::now();
  fs::append_file(root + "/d3/new.py", "more");  // in place, but hot
  EXPECT_TRUE(ev.wait_for(root + "/d3/new.py", 3000));
  EXPECT_TRUE(since(t0) < 1000);
  ev.clear();
  t0 = std::chrono::steady_clock::now();
  fs::write_file_atomic(root + "/d5/f5", "saved");  // an editor's save: rename over the file
  EXPECT_TRUE(ev.wait_for(root + "/d5/f5", 3000));
  EXPECT_TRUE(since(t0) < 1000);
  ev.clear();
  fs::mkdirs(root + "/d9/sub/deeper");
  fs::write_file(root + "/d9/sub/deeper/x", "1");
  EXPECT_TRUE(ev.wait_for(root + "/d9/sub/deeper/x", 3000));
  fs::remove_all(root + "/d9");
  EXPECT_TRUE(ev.wait_for(root + "/d9/f0", 3000));  // entries below a removed directory
  EXPECT_TRUE(ev.wait_for(root + "/d9", 3000));
  ev.clear();
  fs::append_file(root + "/d11/f11", "cold edit");  // in place, cold: the full scan finds it
  EXPECT_TRUE(ev.wait_for(root + "/d11/f11", 5000));
  auto p = ev.paths();
  EXPECT_EQ(p.count(root + "/d11/f11"), (size_t)1);
  EXPECT_EQ(p.count(root + "/d9"), (size_t)0);  // reported once, not again by the full scan
  w->stop();
  fs::remove_all(root);
}

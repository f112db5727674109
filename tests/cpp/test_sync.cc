// Sync engine behaviour matrix — port of sync/sync_config_test.go (TestInitialSync,
// TestNormalSync incl. remove/rename matrix) and sync/util_test.go (TestCopyToContainerTestable),
// run over the local-shell transport in every protocol mode, and over the Kubernetes exec
// WebSocket transport (kube::ExecTransport) when tests/test_sync_matrix_kube.py points it at a pod.
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <chrono>
#include <regex>
#include <thread>

#include "core/fs.h"
#include "core/log.h"
#include "core/proc.h"
#include "core/strutil.h"
#include "kube/client.h"
#include "sync/frame.h"
#include "sync/sync.h"
#include "testing.h"

using namespace ds;
using namespace ds::sync;

namespace {

enum Edit { InRemote = 0, InLocal = 1, Outside = 2 };
struct Case {
  std::string path;
  bool in_local;
  bool in_remote;
  Edit edit;
};
using Cases = std::vector<Case>;
const char* kContents = "TestContents";

// Over the kube exec transport (DS_SYNC_KUBE_POD set by tests/test_sync_matrix_kube.py, which
// runs a pod on the bundled cluster): `remote` is the host directory behind the container path
// `dest` (the local kubelet's container root), so the matrix checks both sides directly.
struct KubeTarget {
  std::string ns, pod, container, root;  // root: host dir of the container's "/"
  bool enabled() const { return !pod.empty(); }
};

KubeTarget kube_target() {
  KubeTarget t;
  auto env = [](const char* k) { return std::string(getenv(k) ? getenv(k) : ""); };
  t.ns = env("DS_SYNC_KUBE_NS");
  t.pod = env("DS_SYNC_KUBE_POD");
  t.container = env("DS_SYNC_KUBE_CONTAINER");
  t.root = env("DS_SYNC_KUBE_ROOT");
  return t;
}

struct Dirs {
  std::string remote, local, outside;
  std::string dest;  // container path (== remote for the local-shell transport)
  Dirs() {
    KubeTarget k = kube_target();
    if (k.enabled()) {
      dest = "/matrix/" + fs::basename(fs::make_temp_dir("remote-"));
      remote = k.root + dest;
      fs::mkdirs(remote);
    } else {
      remote = fs::realpath(fs::make_temp_dir("remote-"));
      dest = remote;
    }
    local = fs::realpath(fs::make_temp_dir("local-"));
    outside = fs::realpath(fs::make_temp_dir("outside-"));
  }
  ~Dirs() {
    fs::remove_all(remote);
    fs::remove_all(local);
    fs::remove_all(outside);
  }
  std::string parent(Edit e) const { return e == InLocal ? local : e == InRemote ? remote : outside; }
};

Cases make_remote(Cases c) {
  Cases out = c;
  for (auto f : c) {
    if (contains(f.path, "Upload"))
      f.path = replace_all(f.path, "Upload", "Download");
    else if (contains(f.path, "Download"))
      f.path = replace_all(f.path, "Download", "Upload");
    out.push_back({replace_all(f.path, "Local", "Remote"), f.in_remote, f.in_local, InRemote});
  }
  return out;
}

Cases make_deep(Cases c) {
  Cases out = c;
  for (auto& f : c) {
    if (f.path == "testFolder") continue;
    out.push_back({"testFolder/" + f.path, f.in_local, f.in_remote, f.edit});
  }
  return out;
}

void basic(Cases* files, Cases* folders) {
  *files = {{"testFileLocal", true, true, InLocal},
            {"ignoreFileLocal", true, false, InLocal},
            {"noDownloadFileLocal", true, true, InLocal},
            {"noUploadFileLocal", true, false, InLocal}};
  *folders = {{"testFolder", true, true, InLocal},
              {"testFolderLocal", true, true, InLocal},
              {"ignoreFolderLocal", true, false, InLocal},
              {"noDownloadFolderLocal", true, true, InLocal},
              {"noUploadFolderLocal", true, false, InLocal}};
  *files = make_deep(make_remote(*files));
  *folders = make_deep(make_remote(*folders));
}

void remove_and_rename(Cases* files, Cases* folders) {
  static const std::regex fully("(testFolder/)?(testFile|testFolder)(Local|Remote)$");
  for (Cases* arr : {files, folders}) {
    Cases out = *arr;
    for (auto& f : *arr) {
      if (f.path == "testFolder") continue;
      out.push_back({f.path + "_Remove", f.in_local, f.in_remote, f.edit});
      out.push_back({f.path + "_RenameToFullContext", f.in_local, f.in_remote, f.edit});
      if (std::regex_search(f.path, fully)) {
        for (const char* s : {"_RenameToOutside", "_RenameToIgnore", "_RenameToNoDownload", "_RenameToNoUpload"})
          out.push_back({f.path + s, f.in_local, f.in_remote, f.edit});
      }
    }
    *arr = out;
  }
  Cases rf = {{"testFileOutsideToLocal_RenameToFullContext", false, false, Outside},
              {"testFileOutsideToRemote_RenameToFullContext", false, false, Outside}};
  Cases rd = {{"testFolderOutsideToLocal_RenameToFullContext", false, false, Outside},
              {"testFolderOutsideToRemote_RenameToFullContext", false, false, Outside},
              {"testFolder", true, true, Outside}};
  for (auto& c : make_deep(rf)) files->push_back(c);
  for (auto& c : make_deep(rd)) folders->push_back(c);
}

void set_excludes(Options* o, const Cases& all) {
  o->exclude_paths.clear();
  o->download_exclude_paths.clear();
  o->upload_exclude_paths.clear();
  for (auto& c : all) {
    if (contains(c.path, "ignore"))
      o->exclude_paths.push_back(c.path);
    else if (contains(c.path, "noDownload"))
      o->download_exclude_paths.push_back(c.path);
    else if (contains(c.path, "noUpload"))
      o->upload_exclude_paths.push_back(c.path);
    else if (ends_with(c.path, "_RenameToIgnore"))
      o->exclude_paths.push_back(c.path + "After");
    else if (ends_with(c.path, "_RenameToNoDownload"))
      o->download_exclude_paths.push_back(c.path + "After");
    else if (ends_with(c.path, "_RenameToNoUpload"))
      o->upload_exclude_paths.push_back(c.path + "After");
  }
}

void create_all(const Dirs& d, const Cases& files, const Cases& folders) {
  for (auto& f : folders) fs::mkdirs(fs::join(d.parent(f.edit), f.path));
  for (auto& f : files) fs::write_file(fs::join(d.parent(f.edit), f.path), kContents, 0666);
}

void remove_some(const Dirs& d, Cases* files, Cases* folders) {
  for (auto& pair : {std::make_pair(d.remote, std::string("Remote_Remove")),
                     std::make_pair(d.local, std::string("Local_Remove"))}) {
    std::vector<std::string> victims;
    fs::walk(pair.first, [&](const std::string& p, const fs::StatInfo&) {
      if (ends_with(p, pair.second)) victims.push_back(p);
      return true;
    });
    for (auto& v : victims) fs::remove_all(v);
  }
  for (Cases* arr : {files, folders})
    for (auto& f : *arr)
      if (ends_with(f.path, "_Remove")) f.in_local = f.in_remote = false;
}

void rename_some(const Dirs& d, Cases* files, Cases* folders) {
  for (Cases* arr : {files, folders}) {
    for (auto& f : *arr) {
      if (!contains(f.path, "_Rename")) continue;
      std::string from = fs::join(d.parent(f.edit), f.path);
      std::string to_parent;
      if (ends_with(f.path, "_RenameToOutside"))
        to_parent = d.outside;
      else if (contains(f.path, "Local_Rename"))
        to_parent = d.local;
      else if (contains(f.path, "Remote_Rename"))
        to_parent = d.remote;
      f.path += "After";
      std::string to = fs::join(to_parent, f.path);
      if (!fs::rename(from, to)) throw std::runtime_error("rename failed " + from + " -> " + to);
      if (ends_with(f.path, "_RenameToFullContextAfter")) {
        f.in_local = f.in_remote = true;
      } else if (ends_with(f.path, "_RenameToNoDownloadAfter")) {
        f.in_remote = true;
        f.in_local = f.edit == InLocal;
      } else if (ends_with(f.path, "_RenameToNoUploadAfter")) {
        f.in_local = true;
        f.in_remote = f.edit == InRemote;
      } else if (ends_with(f.path, "_RenameToIgnoreAfter")) {
        f.in_local = f.edit == InLocal;
        f.in_remote = f.edit == InRemote;
      } else if (ends_with(f.path, "_RenameToOutsideAfter")) {
        f.in_local = f.in_remote = false;
      }
    }
  }
}

std::string check_once(const Dirs& d, const Cases& files, const Cases& folders) {
  std::string errs;
  auto chk = [&](const Case& c, bool dir) {
    for (int side = 0; side < 2; ++side) {
      std::string root = side == 0 ? d.local : d.remote;
      bool want = side == 0 ? c.in_local : c.in_remote;
      std::string p = fs::join(root, c.path);
      fs::StatInfo st = fs::stat(p);
      if (want && !st.exists) errs += (side ? "remote missing " : "local missing ") + c.path + "\n";
      if (!want && st.exists) errs += (side ? "remote unexpected " : "local unexpected ") + c.path + "\n";
      if (want && st.exists && !dir) {
        std::string data;
        fs::read_file(p, &data);
        if (data != kContents) errs += "bad contents " + p + "\n";
      }
      if (want && st.exists && dir != st.is_dir) errs += "wrong type " + p + "\n";
    }
  };
  for (auto& f : files) chk(f, false);
  for (auto& f : folders) chk(f, true);
  return errs;
}

void check_eventually(const Dirs& d, const Cases& files, const Cases& folders, int timeout_ms) {
  auto t0 = std::chrono::steady_clock::now();
  std::string errs;
  while (true) {
    errs = check_once(d, files, folders);
    if (errs.empty()) return;
    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms)) break;
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
  throw dstest::Failure{"sync matrix mismatch:\n" + errs};
}

Options base_options(const Dirs& d, Mode m) {
  Options o;
  o.watch_path = d.local;
  o.dest_path = d.dest;
  o.verbose = true;
  o.mode = m;
  o.helper_path = fs::join(fs::dirname(fs::realpath("/proc/self/exe")), "devspace-helper");
  o.sync_log_name = "sync-test";
  return o;
}

std::shared_ptr<Transport> matrix_transport() {
  KubeTarget k = kube_target();
  if (!k.enabled()) return std::make_shared<LocalShellTransport>();
  auto client = kube::Client::from_devspace_config(Value::map(), false);
  Value pod = client->get("/api/v1/namespaces/" + k.ns + "/pods/" + k.pod);
  return std::make_shared<kube::ExecTransport>(client, pod, k.container);
}

void run_initial(Mode m) {
  log::logdir() = fs::make_temp_dir("synclogs-");
  Dirs d;
  Cases files, folders;
  basic(&files, &folders);
  Options o = base_options(d, m);
  Cases all = files;
  all.insert(all.end(), folders.begin(), folders.end());
  set_excludes(&o, all);
  Session s(o, matrix_transport());
  s.setup();
  s.open_shells();
  create_all(d, files, folders);
  s.start_watcher();
  s.start_loops(true, false);
  s.initial_sync();
  check_eventually(d, files, folders, 10000);
  s.stop();
}

void run_normal(Mode m) {
  log::logdir() = fs::make_temp_dir("synclogs-");
  Dirs d;
  Cases files, folders;
  basic(&files, &folders);
  remove_and_rename(&files, &folders);
  std::stable_sort(folders.begin(), folders.end(),
                   [](const Case& a, const Case& b) { return a.path.size() < b.path.size(); });
  Options o = base_options(d, m);
  Cases all = files;
  all.insert(all.end(), folders.begin(), folders.end());
  set_excludes(&o, all);
  Session s(o, matrix_transport());
  s.start();
  EXPECT_TRUE(s.wait_initial_sync(15000));
  create_all(d, files, folders);
  check_eventually(d, files, folders, 15000);
  remove_some(d, &files, &folders);
  check_eventually(d, files, folders, 15000);
  rename_some(d, &files, &folders);
  check_eventually(d, files, folders, 25000);
  EXPECT_TRUE(s.running());
  s.stop();
}

}  // namespace

TEST(sync_file_index) {
  // TestCreateDirInFileMap / TestRemoveDirInFileMap
  FileIndex idx;
  idx.create_dir("/TestDir1/TestDir2/TestDir3/TestDir4");
  EXPECT_EQ(idx.files.size(), (size_t)4);
  FileIndex idx2;
  FileInfo a;
  a.name = "/TestDir";
  a.is_dir = true;
  idx2.files[a.name] = a;
  FileInfo b;
  b.name = "/TestDir/File1";
  b.size = 1234;
  b.mtime = 1234;
  idx2.files[b.name] = b;
  FileInfo c;
  c.name = "/TestDir2";
  c.is_dir = true;
  idx2.files[c.name] = c;
  idx2.remove_dir("/TestDir");
  EXPECT_EQ(idx2.files.size(), (size_t)1);
}

TEST(sync_parse_file_line) {
  auto f = parse_file_line("/app/src/a.js///12,1500000000,81a4,644,0,0", "/app");
  EXPECT_TRUE(f.has_value());
  EXPECT_EQ(f->name, std::string("/src/a.js"));
  EXPECT_EQ(f->size, (int64_t)12);
  EXPECT_TRUE(!f->is_dir);
  EXPECT_EQ(f->remote_mode, (int64_t)0644);
  auto d = parse_file_line("/app/src///4096,1500000000,41ed,755,1000,1000", "/app");
  EXPECT_TRUE(d->is_dir);
  EXPECT_TRUE(!parse_file_line("/app///4096,1,41ed,755,0,0", "/app").has_value());
  EXPECT_THROWS(parse_file_line("garbage", "/app"));
}

TEST(sync_copy_to_container) {
  Dirs d;
  fs::write_file(fs::join(d.local, "testFile1"), kContents);
  fs::write_file(fs::join(d.local, "testFile2"), kContents);
  fs::write_file(fs::join(d.local, "ignoredFile"), kContents);
  fs::mkdirs(fs::join(d.local, "testFolder"));
  fs::mkdirs(fs::join(d.local, "testFolder2"));
  fs::mkdirs(fs::join(d.local, "ignoredFolder"));
  fs::write_file(fs::join(d.local, "testFolder/testFile1"), kContents);
  fs::write_file(fs::join(d.local, "testFolder/testFile2"), kContents);
  fs::write_file(fs::join(d.local, "testFolder/ignoredFile"), kContents);
  fs::write_file(fs::join(d.local, "ignoredFolder/testFile1"), kContents);
  for (Mode m : {Mode::Compat, Mode::Fast}) {
    fs::remove_all(d.remote);
    fs::mkdirs(d.remote);
    Session::copy_to_container(std::make_shared<LocalShellTransport>(), d.local, d.remote,
                               {"ignoredFile", "ignoredFolder", "testFolder/ignoredFile"}, m);
    Cases files = {{"testFile1", true, true, InLocal},         {"testFile2", true, true, InLocal},
                   {"ignoredFile", true, false, InLocal},      {"testFolder/testFile1", true, true, InLocal},
                   {"testFolder/testFile2", true, true, InLocal}, {"testFolder/ignoredFile", true, false, InLocal},
                   {"ignoredFolder/testFile1", true, false, InLocal}};
    Cases folders = {{"testFolder", true, true, InLocal},
                     {"testFolder2", true, true, InLocal},
                     {"ignoredFolder", true, false, InLocal}};
    check_eventually(d, files, folders, 10000);
  }
}

TEST(sync_initial_fast) { run_initial(Mode::Fast); }
TEST(sync_initial_compat) { run_initial(Mode::Compat); }
TEST(sync_initial_helper) { run_initial(Mode::Helper); }
TEST(sync_normal_fast) { run_normal(Mode::Fast); }
TEST(sync_normal_helper) { run_normal(Mode::Helper); }
TEST(sync_normal_compat) { run_normal(Mode::Compat); }

TEST(sync_reconnect_after_stream_drop) {
  log::logdir() = fs::make_temp_dir("synclogs-");
  Dirs d;
  Options o = base_options(d, Mode::Fast);
  FaultPlan plan;
  plan.kill_after_stdin_bytes = 400;  // first upstream shell dies mid-upload (after its setup command)
  plan.only_shell = 1;
  auto faulty = std::make_shared<FaultInjectingTransport>(std::make_shared<LocalShellTransport>(), plan);
  o.reconnect = [] { return std::make_shared<LocalShellTransport>(); };
  Session s(o, faulty);
  s.start();
  fs::write_file(fs::join(d.local, "a.txt"), kContents);
  Cases files = {{"a.txt", true, true, InLocal}};
  check_eventually(d, files, {}, 15000);
  EXPECT_TRUE(s.stats().reconnects >= 1);
  EXPECT_TRUE(s.running());
  s.stop();
}

TEST(sync_corrupt_ack_is_fatal_without_reconnect) {
  log::logdir() = fs::make_temp_dir("synclogs-");
  Dirs d;
  Options o = base_options(d, Mode::Fast);
  FaultPlan plan;
  plan.corrupt_from = "DONE";
  plan.corrupt_to = "DXNE";
  plan.only_shell = 2;  // downstream shell: scan ack never matches -> stream ends in error
  plan.kill_after_stdin_bytes = 0;
  auto faulty = std::make_shared<FaultInjectingTransport>(std::make_shared<LocalShellTransport>(), plan);
  std::string err;
  o.on_error = [&](const std::string& e) { err = e; };
  Session s(o, faulty);
  s.start();
  // the corrupted ack turns into a parse failure of the scan
  auto t0 = std::chrono::steady_clock::now();
  while (s.running() && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(10))
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  EXPECT_TRUE(!s.running());
  EXPECT_TRUE(!err.empty());
  s.stop();
}

namespace {
// A shell whose close() takes 600 ms: stop() outlives a short DEVSPACE_SYNC_STOP_WARN_MS.
class SlowCloseShell : public Shell {
 public:
  std::unique_ptr<Shell> inner;
  int in() override { return inner->in(); }
  int out() override { return inner->out(); }
  int err() override { return inner->err(); }
  bool alive() override { return inner->alive(); }
  void terminate() override { inner->terminate(); }
  void close() override {
    std::this_thread::sleep_for(std::chrono::milliseconds(600));
    inner->close();
  }
};

class SlowCloseTransport : public Transport {
 public:
  std::unique_ptr<Shell> open(const std::vector<std::string>& argv) override {
    auto s = std::make_unique<SlowCloseShell>();
    s->inner = inner_.open(argv);
    return s;
  }
  std::string describe() const override { return "slow-close(local-shell)"; }

 private:
  LocalShellTransport inner_;
};
}  // namespace

// A stop that takes longer than DEVSPACE_SYNC_STOP_WARN_MS says, in sync.log, where it waits:
// the step of stop() and the loops still running (the diagnosis a stop that never ends needs).
TEST(sync_slow_stop_is_logged_with_its_step) {
  log::logdir() = fs::make_temp_dir("synclogs-");
  ::setenv("DEVSPACE_SYNC_STOP_WARN_MS", "150", 1);
  Dirs d;
  Options o = base_options(d, Mode::Fast);
  {
    Session s(o, std::make_shared<SlowCloseTransport>());
    s.start();
    EXPECT_TRUE(s.wait_initial_sync(15000));
    s.stop();
  }
  ::unsetenv("DEVSPACE_SYNC_STOP_WARN_MS");
  std::string text = fs::read_file(fs::join(log::logdir(), "sync-test.log"));
  EXPECT_TRUE(contains(text, "Stop still waiting after"));
  EXPECT_TRUE(contains(text, "at 'stop_loops: closing shells'; loops still running: none"));
  EXPECT_TRUE(contains(text, "Sync stopped"));
}

// archive entries from the container must never be written outside the synced
// folder (the reference's untar has the same gap; sync/tar.go:44).
TEST(sync_downstream_archive_rejects_parent_segments) {
  Dirs d;
  std::string tar;
  {
    TarWriter tw(string_sink(&tar));
    TarEntry ok;
    ok.name = "ok.txt";
    ok.mtime = 1500000000;
    tw.add_file(ok, "fine");
    TarEntry evil;
    evil.name = "../" + fs::basename(d.outside) + "/escaped.txt";
    evil.mtime = 1500000000;
    tw.add_file(evil, "pwned");
    TarEntry deep;
    deep.name = "sub/../../escaped2.txt";
    deep.mtime = 1500000000;
    tw.add_file(deep, "pwned");
    tw.finish();
  }
  Options o;
  o.watch_path = d.local;
  o.dest_path = d.remote;
  o.mode = Mode::Fast;
  Session s(o, std::make_shared<LocalShellTransport>());
  s.setup();
  s.apply_downstream_archive(gzip_compress(tar));
  EXPECT_EQ(fs::read_file(fs::join(d.local, "ok.txt")), std::string("fine"));
  EXPECT_TRUE(!fs::exists(fs::join(d.outside, "escaped.txt")));
  EXPECT_TRUE(!fs::exists(fs::join(fs::dirname(d.local), "escaped2.txt")));
  EXPECT_TRUE(has_dotdot_segment("/a/../b"));
  EXPECT_TRUE(!has_dotdot_segment("/a/..b/c.."));
}

// ---------------------------------------------------------------- streaming (bounded memory)

TEST(sync_frame_header_is_64_bit) {
  for (uint64_t n : {0ull, 1ull, 0xffffffffull, 0x100000000ull, (5ull << 30) + 7, (1ull << 63) + 3}) {
    std::string h = sync::frame::header('D', n);
    EXPECT_EQ(h.size(), sync::frame::kHeaderSize);
    char op = 0;
    uint64_t len = 0;
    sync::frame::parse_header((const unsigned char*)h.data(), &op, &len);
    EXPECT_EQ(op, 'D');
    EXPECT_EQ(len, n);
  }
}

// 4.5 GiB of generated data through ChunkWriter -> pipe of chunks -> ChunkReader, never held in
// memory: the archive stream of the helper protocol has no 32-bit limit anywhere.
TEST(sync_chunk_stream_over_4gib) {
  const uint64_t total = (9ull << 29) + 12345;  // 4.5 GiB + change
  auto gen = [](uint64_t off) { return (char)((off >> 16) * 2654435761ull >> 7); };  // per 64 KiB block
  // the writer's output is consumed by the reader through a bounded ring (no real pipe needed)
  std::string ring;
  size_t ring_pos = 0;
  uint64_t produced = 0;
  sync::frame::ChunkWriter cw([&](const char* d, size_t n) {
    ring.append(d, n);
    return true;
  });
  Source raw = [&](char* b, size_t n) -> ssize_t {
    while (ring_pos >= ring.size()) {
      ring.clear();
      ring_pos = 0;
      if (produced == total) {
        if (!cw.finish()) return -1;
        if (ring.empty()) return 0;
        break;
      }
      char buf[1 << 16];
      size_t k = (size_t)std::min<uint64_t>(sizeof(buf), total - produced);
      std::memset(buf, gen(produced), k);  // produced is 64 KiB-aligned here
      produced += k;
      if (!cw.write(buf, k)) return -1;
    }
    size_t c = std::min(n, ring.size() - ring_pos);
    std::memcpy(b, ring.data() + ring_pos, c);
    ring_pos += c;
    return (ssize_t)c;
  };
  sync::frame::ChunkReader cr(raw);
  uint64_t got = 0;
  bool ok = true;
  char buf[1 << 16];
  while (true) {
    ssize_t r = cr.read(buf, sizeof(buf));
    if (r == 0) break;
    for (ssize_t i = 0; i < r; i += 4093) ok = ok && buf[i] == gen(got + (uint64_t)i);
    got += (uint64_t)r;
  }
  EXPECT_TRUE(ok);
  EXPECT_EQ(got, total);
  EXPECT_EQ(cr.bytes(), total);
  EXPECT_TRUE(ring.size() < (4u << 20));  // bounded buffering
}

TEST(sync_chunk_reader_rejects_truncation) {
  std::string wire;
  sync::frame::ChunkWriter cw(string_sink(&wire), 1000);
  std::string data(2500, 'x');
  cw.write(data.data(), data.size());
  cw.finish();
  std::string cut = wire.substr(0, wire.size() - 600);  // inside the last chunk, no end marker
  sync::frame::ChunkReader cr(string_source(&cut));
  EXPECT_THROWS(cr.drain());
}

TEST(sync_adaptive_gzip_stream_matches_oneshot) {
  std::string data;
  for (int i = 0; i < 3000000; ++i) data.push_back((char)(i % 7 == 0 ? (i * 131) : 'a' + i % 13));
  std::string rnd = random_string(3 << 20);
  data += rnd;
  std::string out;
  AdaptiveGzipWriter w(string_sink(&out), 1);
  for (size_t off = 0; off < data.size(); off += 77777) w.write(data.data() + off, std::min<size_t>(77777, data.size() - off));
  EXPECT_TRUE(w.finish());
  EXPECT_EQ(gzip_decompress(out), data);
  EXPECT_EQ(gzip_decompress(gzip_compress_adaptive(data, 1)), data);
}

TEST(sync_gzip_single_member_returns_leftover) {
  std::string member = gzip_compress(std::string(100000, 'q'));
  std::string wire = member + "\nDSEND 0\n";
  GzipReader gz(string_source(&wire));
  gz.set_single_member(true);
  std::string out;
  char buf[4096];
  while (true) {
    ssize_t n = gz.read(buf, sizeof(buf));
    EXPECT_TRUE(n >= 0);
    if (n == 0) break;
    out.append(buf, (size_t)n);
  }
  EXPECT_EQ(out.size(), (size_t)100000);
  EXPECT_EQ(gz.leftover(), std::string("\nDSEND 0\n"));
}

TEST(sync_spill_buffer_spills_and_replays) {
  SpillBuffer sb(1000);
  std::string want;
  for (int i = 0; i < 5000; ++i) {
    std::string piece = std::to_string(i) + ",";
    want += piece;
    EXPECT_TRUE(sb.append(piece.data(), piece.size()));
  }
  EXPECT_TRUE(sb.spilled());
  EXPECT_EQ(sb.size(), (uint64_t)want.size());
  std::string got;
  EXPECT_TRUE(sb.replay(string_sink(&got)));
  EXPECT_EQ(got, want);
  EXPECT_EQ(sb.head(6), want.substr(0, 6));
  SpillBuffer small(1000);
  small.append("abc", 3);
  EXPECT_TRUE(!small.spilled());
  got.clear();
  EXPECT_TRUE(small.replay(string_sink(&got)));
  EXPECT_EQ(got, std::string("abc"));
}

TEST(sync_tar_reader_rejects_bad_checksum) {
  std::string raw;
  TarWriter tw(string_sink(&raw));
  TarEntry e;
  e.name = "a.txt";
  tw.add_file(e, "hello");
  tw.finish();
  raw[10] ^= 0x5a;  // corrupt the name: the header checksum no longer matches
  TarReader tr(string_source(&raw));
  TarEntry got;
  EXPECT_THROWS(tr.next(&got));
}

TEST(sync_chunk_stream_codes_chunks_by_entropy) {
  std::string text, rnd = random_string(1);
  for (int i = 0; i < 200000; ++i) text += "line " + std::to_string(i % 977) + " of a log\n";
  std::string noise;
  for (int i = 0; i < (3 << 20); ++i) noise.push_back((char)(std::rand() & 0xff));
  std::string data = text + noise + text;
  std::string wire;
  sync::frame::ChunkWriter cw(string_sink(&wire), sync::frame::kMaxChunk, 1);
  for (size_t off = 0; off < data.size(); off += 100000) cw.write(data.data() + off, std::min<size_t>(100000, data.size() - off));
  EXPECT_TRUE(cw.finish());
  EXPECT_TRUE(cw.deflated_chunks() >= 4);                 // the text chunks
  EXPECT_TRUE(wire.size() < noise.size() + text.size());  // text compressed, noise stored as-is
  sync::frame::ChunkReader cr(string_source(&wire));
  std::string back;
  char buf[70000];
  while (true) {
    ssize_t r = cr.read(buf, sizeof(buf));
    if (r == 0) break;
    back.append(buf, (size_t)r);
  }
  EXPECT_EQ(back.size(), data.size());
  EXPECT_TRUE(back == data);
  std::string bad = wire;
  bad[10] ^= 0x55;  // inside the first (deflated) chunk
  sync::frame::ChunkReader cr2(string_source(&bad));
  EXPECT_THROWS(cr2.drain());
}

// The helper's directory probe (hardened pods mount /tmp noexec): the first candidate that
// already holds the helper wins, else the first writable one where a file can execute.
TEST(sync_helper_probe_picks_a_usable_directory) {
  auto run = [](const std::string& script) {
    std::string path = "/tmp/ds-probe-" + std::to_string(getpid()) + ".sh";
    fs::write_file(path, script);
    RunResult r = ds::run({"sh", path}, "", {}, 20000);
    ::unlink(path.c_str());
    return trim(r.out);
  };
  std::string base = "/tmp/ds-helper-probe-" + std::to_string(getpid());
  fs::remove_all(base);
  fs::mkdirs(base + "/b");
  // /proc refuses a new directory: skipped; the next candidate is created and usable
  std::string out = run(sync::helper_probe_script("devspace-helper-x", {"/proc/ds-no-such", base + "/a", base + "/b"}));
  EXPECT_TRUE(out == "NEED " + base + "/a" || out == "NEEDZ " + base + "/a");
  // an executable helper already in a later candidate is reused before uploading anew
  fs::write_file(base + "/b/devspace-helper-x", "#!/bin/sh\n");
  ::chmod((base + "/b/devspace-helper-x").c_str(), 0755);
  out = run(sync::helper_probe_script("devspace-helper-x", {base + "/a", base + "/b"}));
  EXPECT_EQ(out, "HAVE " + base + "/b");
  EXPECT_TRUE(!fs::exists(base + "/a/.devspace-x"));
  // a helper that is there starts in the probe's round trip; one still to upload does not
  out = run(sync::helper_probe_script("devspace-helper-x", {base + "/a", base + "/b"}, "echo STARTED \"$dsd\""));
  EXPECT_EQ(out, "HAVE " + base + "/b\nSTARTED " + base + "/b");
  out = run(sync::helper_probe_script("devspace-helper-y", {base + "/a"}, "echo STARTED \"$dsd\""));
  EXPECT_TRUE(out == "NEED " + base + "/a" || out == "NEEDZ " + base + "/a");
  out = run(sync::helper_probe_script("devspace-helper-x", {"/proc/ds-no-such"}));
  EXPECT_EQ(out, "NOHELPER");
  fs::remove_all(base);
}

// Helper-mode upload lanes under concurrency (TSan covers this in scripts/sanitize.sh): a bulk
// file on its lane, edits on theirs while it travels, a pod-side write coming back meanwhile;
// everything lands with the right bytes and the edits are not overwritten by older ones.
TEST(sync_helper_lanes_concurrent_uploads) {
  log::logdir() = fs::make_temp_dir("synclogs-");
  Dirs d;
  if (d.dest != d.remote) return;  // local-shell transport only (no kube target needed)
  Options o = base_options(d, Mode::Helper);
  Session s(o, std::make_shared<LocalShellTransport>());
  s.start();
  EXPECT_TRUE(s.wait_initial_sync(15000));
  EXPECT_TRUE(s.effective_mode() == Mode::Helper);
  std::string big(48u << 20, '\0');
  uint64_t x = 0x9e3779b97f4a7c15ull;
  for (size_t i = 0; i < big.size(); i += 8) {  // incompressible: chunks go out stored
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    std::memcpy(&big[i], &x, 8);
  }
  fs::write_file(fs::join(d.local, "ckpt.bin"), big);
  for (int i = 0; i < 20; ++i) {
    fs::write_file(fs::join(d.local, "edit.py"), "v = " + std::to_string(i) + "\n");
    if (i == 5) fs::write_file(fs::join(d.remote, "from_pod.txt"), "pod\n");
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  }
  auto t0 = std::chrono::steady_clock::now();
  auto waited = [&] { return std::chrono::steady_clock::now() - t0 < std::chrono::seconds(60); };
  std::string got;
  while (waited() && !(fs::read_file(fs::join(d.remote, "ckpt.bin"), &got) && got.size() == big.size()))
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  EXPECT_TRUE(got == big);
  while (waited() && !(fs::read_file(fs::join(d.remote, "edit.py"), &got) && got == "v = 19\n"))
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  EXPECT_EQ(got, std::string("v = 19\n"));
  while (waited() && !(fs::read_file(fs::join(d.local, "from_pod.txt"), &got) && got == "pod\n"))
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  EXPECT_EQ(got, std::string("pod\n"));
  std::this_thread::sleep_for(std::chrono::milliseconds(300));
  EXPECT_TRUE(fs::read_file(fs::join(d.remote, "edit.py"), &got) && got == "v = 19\n");
  EXPECT_TRUE(s.running());
  s.stop();
}

// Helper-mode bulk download channel under concurrency (TSan covers this in scripts/sanitize.sh):
// a big pod-side file comes down on its own channel while small pod-side writes keep arriving on
// the main one and a local edit goes up; a stop in the middle of a second big download ends
// cleanly (the channel's shell and thread are torn down with the session).
TEST(sync_helper_bulk_download_channel) {
  log::logdir() = fs::make_temp_dir("synclogs-");
  Dirs d;
  if (d.dest != d.remote) return;  // local-shell transport only (no kube target needed)
  Options o = base_options(d, Mode::Helper);
  Session s(o, std::make_shared<LocalShellTransport>());
  s.start();
  EXPECT_TRUE(s.wait_initial_sync(15000));
  EXPECT_TRUE(s.effective_mode() == Mode::Helper);
  auto noise = [](size_t n, uint64_t x) {
    std::string b(n, '\0');
    for (size_t i = 0; i < b.size(); i += 8) {
      x ^= x << 13;
      x ^= x >> 7;
      x ^= x << 17;
      std::memcpy(&b[i], &x, 8);
    }
    return b;
  };
  std::string big = noise(40u << 20, 0x9e3779b97f4a7c15ull);
  fs::write_file(fs::join(d.remote, "ckpt.bin.partial"), big);
  ::rename(fs::join(d.remote, "ckpt.bin.partial").c_str(), fs::join(d.remote, "ckpt.bin").c_str());
  for (int i = 0; i < 10; ++i) {
    fs::write_file(fs::join(d.remote, "metrics.json"), "{\"step\": " + std::to_string(i) + "}\n");
    if (i == 3) fs::write_file(fs::join(d.local, "edit.py"), "v = 1\n");
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  }
  auto t0 = std::chrono::steady_clock::now();
  auto waited = [&] { return std::chrono::steady_clock::now() - t0 < std::chrono::seconds(60); };
  std::string got;
  while (waited() && !(fs::read_file(fs::join(d.local, "ckpt.bin"), &got) && got.size() == big.size()))
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  EXPECT_TRUE(got == big);
  while (waited() && !(fs::read_file(fs::join(d.local, "metrics.json"), &got) && got == "{\"step\": 9}\n"))
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  EXPECT_EQ(got, std::string("{\"step\": 9}\n"));
  while (waited() && !(fs::read_file(fs::join(d.remote, "edit.py"), &got) && got == "v = 1\n"))
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  EXPECT_EQ(got, std::string("v = 1\n"));
  EXPECT_TRUE(s.running());
  // a second big file, and stop while it may still be coming down
  fs::write_file(fs::join(d.remote, "ckpt2.bin"), noise(24u << 20, 0x2545f4914f6cdd1dull));
  std::this_thread::sleep_for(std::chrono::milliseconds(150));
  s.stop();
  EXPECT_TRUE(!s.running());
}

// A pod process that rewrites a file at the same size within the second (a metrics or status
// file) is downloaded every time: the helper's listing carries the mtime's nanoseconds. And a
// rewrite that even keeps the nanoseconds (a coarse filesystem clock gives two writes in one
// tick the same stamp; here forced with utimensat) is caught by content once the file is still:
// its stamp was fresh when it was downloaded, so the copy is checked by CRC-32.
TEST(sync_helper_same_size_rewrites_within_a_second_come_down) {
  log::logdir() = fs::make_temp_dir("synclogs-");
  Dirs d;
  if (d.dest != d.remote) return;  // local-shell transport only
  Options o = base_options(d, Mode::Helper);
  Session s(o, std::make_shared<LocalShellTransport>());
  s.start();
  EXPECT_TRUE(s.wait_initial_sync(15000));
  const std::string rf = fs::join(d.remote, "status.txt"), lf = fs::join(d.local, "status.txt");
  auto wait_local = [&](const std::string& want, int ms) {
    auto t0 = std::chrono::steady_clock::now();
    std::string got;
    while (std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(ms)) {
      if (fs::read_file(lf, &got) && got == want) return true;
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
    return false;
  };
  for (int i = 0; i < 6; ++i) {  // same size, a few ms apart: the last one must land
    fs::write_file(rf, "step " + std::to_string(i) + "\n");
    std::this_thread::sleep_for(std::chrono::milliseconds(3));
  }
  EXPECT_TRUE(wait_local("step 5\n", 10000));
  // same size and the very same stamp as the version already downloaded
  struct stat st;
  EXPECT_EQ(::stat(rf.c_str(), &st), 0);
  fs::write_file(rf, "step X\n");
  struct timespec ts[2] = {st.st_atim, st.st_mtim};
  EXPECT_EQ(::utimensat(AT_FDCWD, rf.c_str(), ts, 0), 0);
  EXPECT_TRUE(wait_local("step X\n", 10000));
  EXPECT_TRUE(s.running());
  s.stop();
}

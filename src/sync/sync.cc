#include "sync/sync.h"

#include <fcntl.h>
#include <poll.h>
#include <signal.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <chrono>
#include <cstdlib>
#include <cstring>

#include "core/strutil.h"
#include "core/trace.h"
#include "sync/frame.h"

namespace ds {
namespace sync {

static const char* kStart = "START";
static const char* kDone = "DONE";
static const char* kError = "ERROR";
static const char* kTmpSuffix = ".devspace-tmp";  // in-flight files (helper and local untar)
// a stamp younger than this (on the container's clock) may be shared by the next write: a
// filesystem's coarse clock ticks every few ms, and the same-size rewrite it hides is only
// seen by content
static const int64_t kUnsettledNs = 1000000000LL;
static const int64_t kVerifyMaxBytes = 8LL << 20;
static const size_t kInitialUpstreamBatch = 1000;  // sync_config.go:20

static long mono_us() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1000000L + ts.tv_nsec / 1000;
}

static void sleep_ms(int ms) { std::this_thread::sleep_for(std::chrono::milliseconds(ms)); }

Mode parse_mode(const std::string& s_in) {
  std::string s = to_lower(s_in);
  if (s.empty()) {
    const char* e = getenv("DEVSPACE_SYNC_MODE");
    if (e && *e) s = to_lower(e);
  }
  if (s == "compat" || s == "reference") return Mode::Compat;
  if (s == "fast" || s == "posix") return Mode::Fast;
  return Mode::Helper;  // default: helper with automatic fallback to fast POSIX
}

const char* mode_name(Mode m) {
  switch (m) {
    case Mode::Compat: return "compat";
    case Mode::Fast: return "fast";
    case Mode::Helper: return "helper";
  }
  return "?";
}

struct SyncError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// ============================================================ file info / index

std::optional<FileInfo> parse_file_line(const std::string& line, const std::string& dest) {
  auto t = split(line, "///");
  if (t.size() != 2) throw SyncError("[Downstream] Wrong fileline: " + line);
  if (t[0].size() <= dest.size()) return std::nullopt;
  FileInfo f;
  f.name = t[0].substr(dest.size());
  auto p = split(t[1], ",");
  if (p.size() != 6 && p.size() != 7) throw SyncError("[Downstream] Wrong fileline: " + line);
  int64_t v;
  if (!parse_int64(p[0], &v)) throw SyncError("[Downstream] Wrong fileline: " + line);
  f.size = v;
  if (!parse_int64(p[1], &v)) throw SyncError("[Downstream] Wrong fileline: " + line);
  f.mtime = v;
  unsigned long raw = std::strtoul(p[2].c_str(), nullptr, 16);
  f.is_symlink = (raw & 0120000) == 0120000;
  f.is_dir = (raw & 040000) == 040000 && !f.is_symlink;
  f.remote_mode = std::strtol(p[3].c_str(), nullptr, 8);
  f.remote_uid = std::atoi(p[4].c_str());
  f.remote_gid = std::atoi(p[5].c_str());
  f.has_remote_attrs = true;
  if (p.size() == 7) {
    if (!parse_int64(p[6], &v) || v < 0 || v >= 1000000000) throw SyncError("[Downstream] Wrong fileline: " + line);
    f.remote_mtime_ns = f.mtime * 1000000000LL + v;
  }
  return f;
}

void FileIndex::create_dir(const std::string& dirpath) {
  if (dirpath == "/" || dirpath.empty() || dirpath == ".") return;
  auto parts = split(dirpath, "/");
  for (size_t i = parts.size(); i > 1; --i) {
    std::vector<std::string> sub(parts.begin(), parts.begin() + i);
    std::string p = join(sub, "/");
    if (p.empty()) continue;
    if (!files.count(p)) {
      FileInfo f;
      f.name = p;
      f.is_dir = true;
      files[p] = f;
    }
  }
}

void FileIndex::remove_dir(const std::string& dirpath) {
  auto it = files.find(dirpath);
  if (it == files.end()) return;
  files.erase(it);
  std::string prefix = dirpath + "/";
  auto lo = files.lower_bound(prefix);
  auto hi = lo;
  while (hi != files.end() && starts_with(hi->first, prefix)) ++hi;
  files.erase(lo, hi);
}

// ============================================================ session setup

Session::Session(Options opts, std::shared_ptr<Transport> transport)
    : o_(std::move(opts)), transport_(std::move(transport)), mode_(o_.mode) {}

Session::~Session() { stop(); }

std::string Session::pod_name() {
  std::lock_guard<std::mutex> g(pod_mu_);
  return o_.pod_name;
}

void Session::logf(const std::string& msg) {
  if (o_.silent || !log_) return;
  std::map<std::string, std::string> f{{"local", o_.watch_path}, {"container", o_.dest_path}};
  std::string pod = pod_name();
  if (!pod.empty()) f["pod"] = pod;
  log_->emit("info", msg, f);
}

void Session::log_error(const std::string& msg) {
  if (!log_) return;
  std::map<std::string, std::string> f{{"local", o_.watch_path}, {"container", o_.dest_path}};
  std::string pod = pod_name();
  if (!pod.empty()) f["pod"] = pod;
  log_->emit("error", msg, f);
}

std::string Session::remote(const std::string& p) const {
  std::string pre = transport_ ? transport_->path_prefix() : "";
  if (pre.empty()) return p;
  return fs::clean(pre + "/" + p);
}

void Session::setup() {
  std::string real = fs::realpath(o_.watch_path);
  if (real.empty()) throw SyncError("lstat " + o_.watch_path + ": no such file or directory");
  o_.watch_path = real;
  // exclude the sync log to prevent an endless upstream loop (sync_config.go:116)
  o_.exclude_paths.push_back("/.devspace/logs");
  ignore_ = GitIgnore(o_.exclude_paths);
  has_ignore_ = !ignore_.empty();
  download_ignore_ = GitIgnore(o_.download_exclude_paths);
  has_download_ignore_ = !download_ignore_.empty();
  upload_ignore_ = GitIgnore(o_.upload_exclude_paths);
  has_upload_ignore_ = !upload_ignore_.empty();
  if (!o_.silent) {
    // rotate sync.log into sync.log.old once per process (sync/util.go:305)
    static std::once_flag rotated;
    std::string logfile = fs::join(log::logdir(), o_.sync_log_name + ".log");
    std::call_once(rotated, [&] {
      std::string data;
      if (fs::read_file(logfile, &data)) {
        fs::append_file(logfile + ".old", data);
        fs::remove(logfile);
      }
    });
    log_ = log::file_logger(o_.sync_log_name);
  }
  switch (mode_) {
    case Mode::Compat:
      window_ms_ = 600;
      poll_ms_ = 1300;
      break;
    case Mode::Fast:
      window_ms_ = 15;
      poll_ms_ = 250;
      break;
    case Mode::Helper:
      window_ms_ = 10;
      // fallback listing only: the helper's inotify events (its own writes filtered out by
      // path, queue overflows reported) drive downstream
      poll_ms_ = 10000;
      break;
  }
  if (o_.large_file_warn_bytes >= 0) {
    large_warn_bytes_ = o_.large_file_warn_bytes;
  } else if (const char* mb = getenv("DEVSPACE_SYNC_WARN_FILE_MB")) {
    large_warn_bytes_ = std::atoll(mb) << 20;
  }
  if (o_.upstream_window_ms >= 0) window_ms_ = o_.upstream_window_ms;
  if (o_.downstream_poll_ms >= 0) poll_ms_ = o_.downstream_poll_ms;
  dest_ = remote(o_.dest_path);
}

// ============================================================ helper bootstrap

using frame::request;

// Sniffs gzip (0x1f 0x8b) vs plain tar.
static bool is_gzip_magic(const std::string& m) {
  return m.size() >= 2 && (unsigned char)m[0] == 0x1f && (unsigned char)m[1] == 0x8b;
}

// tar bytes -> wire bytes for the shell protocols (`tar x` / `tar xz` in the container): plain
// tar while the archive is small (latency-bound edits: no gzip on either side) or when its
// first MiB is incompressible (checkpoints: gzip would only add CRC + framing work on both
// ends), gzip otherwise — adaptive, so incompressible chunks later in the stream go out as
// stored blocks. plain_limit 0 = always gzip (the reference's protocol).
class ArchiveEncoder {
 public:
  ArchiveEncoder(Sink out, size_t plain_limit, int level) : out_(std::move(out)), limit_(plain_limit), level_(level) {}
  bool write(const char* d, size_t n) {
    if (gz_) return gz_->write(d, n);
    if (plain_) return out_(d, n);
    pending_.append(d, n);
    if (limit_ == 0 || pending_.size() >= kDecideBytes) return decide();
    return true;
  }
  Sink sink() {
    return [this](const char* d, size_t n) { return write(d, n); };
  }
  bool finish() {
    if (!gz_ && !plain_) {
      if (limit_ > 0 && pending_.size() <= limit_) {
        plain_ = true;
        return pending_.empty() || out_(pending_.data(), pending_.size());
      }
      if (!decide()) return false;
    }
    return gz_ ? gz_->finish() : true;
  }
  bool gzipped() const { return gz_ != nullptr; }

 private:
  static const size_t kDecideBytes = 1 << 20;
  bool decide() {
    if (limit_ > 0 && entropy(pending_) > 7.2) {
      plain_ = true;
    } else {
      gz_ = std::make_unique<AdaptiveGzipWriter>(out_, level_);
    }
    bool ok = gz_ ? gz_->write(pending_) : out_(pending_.data(), pending_.size());
    std::string().swap(pending_);
    return ok;
  }
  static double entropy(const std::string& d) {
    uint32_t hist[256] = {0};
    for (unsigned char c : d) hist[c]++;
    double h = 0;
    for (uint32_t c : hist)
      if (c) h -= (double)c / (double)d.size() * std::log2((double)c / (double)d.size());
    return h;
  }
  Sink out_;
  size_t limit_;
  int level_;
  bool plain_ = false;
  std::string pending_;
  std::unique_ptr<AdaptiveGzipWriter> gz_;
};

static const size_t kPlainTarLimit = 256 * 1024;
static const uint64_t kProgressMin = 64ull << 20;

static std::string human_bytes(uint64_t b) {
  if (b >= (1ull << 30)) return strfmt("%.2f GiB", (double)b / (double)(1ull << 30));
  if (b >= (1ull << 20)) return strfmt("%.1f MiB", (double)b / (double)(1ull << 20));
  if (b >= 1024) return strfmt("%.1f KiB", (double)b / 1024.0);
  return strfmt("%llu B", (unsigned long long)b);
}

// Progress lines in sync.log for big transfers (every 5 s, and a summary at the end).
struct Session::Progress {
  Session* s;
  std::string what;
  uint64_t total;  // 0 = unknown
  uint64_t done = 0;
  long start_us, last_us;
  Progress(Session* sess, std::string w, uint64_t t) : s(sess), what(std::move(w)), total(t) {
    start_us = last_us = mono_us();
  }
  void add(size_t n) {
    done += n;
    long now = mono_us();
    if (now - last_us < 5000000 || done < kProgressMin) return;
    last_us = now;
    double mbps = (double)done / 1e6 / ((double)(now - start_us) / 1e6);
    if (total)
      s->logf(strfmt("%s: %s / %s (%.0f%%, %.0f MB/s)", what.c_str(), human_bytes(done).c_str(),
                     human_bytes(total).c_str(), 100.0 * (double)done / (double)total, mbps));
    else
      s->logf(strfmt("%s: %s (%.0f MB/s)", what.c_str(), human_bytes(done).c_str(), mbps));
  }
  void finish() {
    if (done < kProgressMin) return;
    double secs = (double)(mono_us() - start_us) / 1e6;
    s->logf(strfmt("%s: %s in %.1f s (%.0f MB/s)", what.c_str(), human_bytes(done).c_str(), secs,
                   (double)done / 1e6 / std::max(secs, 1e-6)));
  }
};

const std::vector<std::string>& helper_dirs() {
  static const std::vector<std::string> dirs = {"/tmp", "/dev/shm", "/var/tmp", "$HOME"};
  return dirs;
}

std::string helper_probe_script(const std::string& file, const std::vector<std::string>& dirs,
                                const std::string& when_present) {
  std::string list;
  for (auto& d : dirs) list += (d[0] == '$' ? "\"" + d + "\"" : shell_quote(d)) + " ";
  // a one-line `#!/bin/sh` script run from the directory tells a noexec mount apart
  return "dsd=; dss=; if [ \"$(uname -m 2>/dev/null)\" = x86_64 ]; then for d in " + list +
         "; do if [ -n \"$d\" ] && [ -x \"$d/" + file + "\" ]; then dsd=$d; dss=HAVE; break; fi; done; fi; "
         "if [ -z \"$dsd\" ] && [ \"$(uname -m 2>/dev/null)\" = x86_64 ]; then for d in " + list +
         "; do [ -n \"$d\" ] || continue; if mkdir -p \"$d\" 2>/dev/null && [ -w \"$d\" ] && printf '#!/bin/sh\\nexit 0\\n' > \"$d/.devspace-x$$\" "
         "2>/dev/null && chmod +x \"$d/.devspace-x$$\" 2>/dev/null && \"$d/.devspace-x$$\" 2>/dev/null; then "
         "rm -f \"$d/.devspace-x$$\"; dsd=$d; dss=NEED; break; fi; rm -f \"$d/.devspace-x$$\" 2>/dev/null; done; fi; "
         "if [ \"$dss\" = HAVE ]; then echo \"HAVE $dsd\"; " + (when_present.empty() ? std::string(":") : when_present) +
         "; elif [ -n \"$dsd\" ]; then if command -v gzip >/dev/null 2>&1; then echo \"NEEDZ $dsd\"; "
         "else echo \"NEED $dsd\"; fi; else echo NOHELPER; fi\n";
}

// The helper gzip-compressed for the upload (0.53 MB for 1.1 MB, in about 35 ms), made once per
// machine: cached under ~/.cache/devspace by its content hash.
static std::string packed_helper(const std::string& file, const std::string& bin) {
  static std::mutex mu;
  static std::map<std::string, std::string> mem;
  std::lock_guard<std::mutex> g(mu);
  auto& z = mem[file];
  if (!z.empty()) return z;
  std::string dir = fs::join(fs::home_dir(), ".cache/devspace");
  std::string path = fs::join(dir, file + ".gz");
  std::string cached;
  if (fs::read_file(path, &cached) && !cached.empty()) {
    try {
      if (gzip_decompress(cached) == bin) return z = cached;
    } catch (const std::exception&) {
    }
  }
  z = gzip_compress(bin, 1);  // level 9 saves 40 KB more and takes 0.27 s
  try {
    fs::mkdirs(dir);
    fs::write_file_atomic(path, z);
  } catch (const std::exception&) {  // a read-only home: compressed again next time
  }
  return z;
}

bool Session::start_helper(std::unique_ptr<Shell>& sh, LineReader& out, HelperRole role) {
  // Probe architecture + a writable directory that allows exec, upload the static helper once
  // (content-addressed), then exec it in place of the shell.
  // The uploader tells a waiting shell whether the helper is in the container (on every return
  // before that is known: it is not)
  struct Announce {
    Session* s;
    bool on;
    int state = 2;
    void set(int st) {
      if (!on) return;
      on = false;
      {
        std::lock_guard<std::mutex> g(s->helper_mu_);
        s->helper_state_ = st;
      }
      s->helper_cv_.notify_all();
    }
    ~Announce() { set(2); }
  } announce{this, role == kUploader};
  if (o_.helper_path.empty() || !fs::is_file(o_.helper_path)) return false;
  std::string bin;
  if (!fs::read_file(o_.helper_path, &bin)) return false;
  std::string file = "devspace-helper-" + sha256_hex(bin).substr(0, 16);
  // stdout carries replies, stderr the change events: exec with the shell's fds as-is
  auto start = [&](const std::string& path) {
    return "mkdir -p " + shell_quote(dest_) + " && exec " + path + " serve " + shell_quote(dest_) + " || echo HELPERFAIL";
  };
  // a helper already in the container starts in the probe's round trip
  const auto t_probe = std::chrono::steady_clock::now();
  if (!write_all(sh->in(), helper_probe_script(file, helper_dirs(), start("\"$dsd/" + file + "\"")))) return false;
  std::string line;
  if (!out.read_line(&line, 15000)) return false;
  const long probe_ms = (long)std::chrono::duration_cast<std::chrono::milliseconds>(
                            std::chrono::steady_clock::now() - t_probe).count();
  if (line == "NOHELPER" || line.size() < 6 ||
      (!starts_with(line, "HAVE ") && !starts_with(line, "NEED ") && !starts_with(line, "NEEDZ "))) {
    logf("[Sync] No directory in the container can hold and run the helper (" + line + ")");
    return false;
  }
  if (starts_with(line, "HAVE ")) announce.set(1);
  if (starts_with(line, "NEED")) {
    // "NEEDZ <dir>": the container has gzip. On a remote cluster (the probe took 5 ms or more)
    // the helper then travels compressed: a first `dev` on a slow uplink waits for half the
    // bytes. Next to the cluster, sending 1.1 MB costs less than compressing it.
    const bool gz = starts_with(line, "NEEDZ ") && probe_ms >= 5;
    const std::string dir = line.substr(starts_with(line, "NEEDZ ") ? 6 : 5);
    std::string name = shell_quote(dir + "/" + file);
    bool there = false;
    if (role == kWaiter) {  // the other shell is uploading it: wait for that, not the bytes again
      std::unique_lock<std::mutex> lk(helper_mu_);
      helper_cv_.wait_for(lk, std::chrono::seconds(60), [this] { return helper_state_ != 0; });
      there = helper_state_ == 1;
    }
    if (!there) {
      // a temporary name per shell: shells may upload at the same time
      std::string tmp = shell_quote(dir + "/" + file) + ".tmp.$$";
      std::string payload = gz ? packed_helper(file, bin) : bin;
      std::string up = "echo " + std::string(kStart) + "; head -c " + std::to_string(payload.size()) +
                       (gz ? " | gzip -dc" : "") + " > " + tmp + " && chmod +x " + tmp + " && mv " + tmp + " " + name +
                       "; echo " + kDone + "\n";
      if (!write_all(sh->in(), up)) return false;
      if (!out.wait_for(kStart, 15000)) return false;
      if (!write_all(sh->in(), payload)) return false;
      if (!out.wait_for(kDone, 30000)) return false;
      announce.set(1);
    }
    if (!write_all(sh->in(), start(name) + "\n")) return false;
  }
  if (!out.read_line(&line, 15000)) return false;
  return line == "HELPER READY";
}

void Session::open_up_shell(std::unique_ptr<Shell> opened) {
  std::lock_guard<std::mutex> g(up_shell_mu_);
  up_shell_ = opened ? std::move(opened) : transport_->open({"sh"});
  up_out_.reset(up_shell_->out());
  up_helper_ = false;
  if (mode_ == Mode::Helper) {
    up_helper_ = start_helper(up_shell_, up_out_, concurrent_open_ ? kUploader : kAlone);
    if (!up_helper_) {
      logf("[Sync] Helper unavailable, falling back to fast POSIX protocol");
      up_shell_->close();
      up_shell_ = transport_->open({"sh"});
      up_out_.reset(up_shell_->out());
    }
  }
  up_has_head_ = false;
  if (up_helper_) up_err_.reset(up_shell_->err());  // the watch's events, once open_down_shell asks
  set_nonblocking(up_shell_->in(), true);
  if (up_helper_) start_up_reader();
  if (mode_ != Mode::Compat && !up_helper_) {
    // create the destination once instead of per upload, and check for `head` (the streamed
    // upload needs `head -c`; without it uploads use the reference's cat + stat protocol)
    write_all(up_shell_->in(), "mkdir -p " + shell_quote(dest_) + " " + shell_quote(remote("/tmp")) +
                                   "; if command -v head >/dev/null 2>&1; then echo HAVEHEAD; fi; echo " + kDone + "\n");
    std::string before;
    wait_ack(up_out_, kDone, false, &before, 30000);
    up_has_head_ = contains(before, "HAVEHEAD");
    if (!up_has_head_) logf("[Sync] `head` not found in the container: uploads use the POSIX cat/stat protocol");
  }
}

void Session::open_down_shell() {
  std::lock_guard<std::mutex> g(down_shell_mu_);
  down_shell_ = transport_->open({"sh"});
  down_out_.reset(down_shell_->out());
  down_err_.reset(down_shell_->err());
  down_helper_ = false;
  if (mode_ == Mode::Helper) {
    down_helper_ = start_helper(down_shell_, down_out_, concurrent_open_ ? kWaiter : kAlone);
    if (!down_helper_) {
      down_shell_->close();
      down_shell_ = transport_->open({"sh"});
      down_out_.reset(down_shell_->out());
      down_err_.reset(down_shell_->err());
    }
  }
}

void Session::request_watch() {
  if (!down_helper_) return;  // the downstream side probes instead
  if (up_helper_) {
    // The change watch runs in the upstream helper (the echo of its own writes is filtered
    // where they are recorded, src/helper/helper.cc is_own), and only now that the downstream
    // side is known to read its events (a watch whose stderr nobody drains fills the
    // channel and stalls the exec stream that carries the upload replies).
    std::lock_guard<std::mutex> ug(up_shell_mu_);
    write_all(up_shell_->in(), request('W', ""));
  } else {
    // no upstream helper: container-side change events come from this one (no echo filter)
    std::lock_guard<std::mutex> dg(down_shell_mu_);
    write_all(down_shell_->in(), request('W', ""));
  }
}

void Session::open_shells() {
  // The opens keep their order (upstream, then downstream: fault injection counts on it), and
  // the upstream helper's start overlaps the downstream shell's open and helper start: on a
  // remote cluster that is a round trip less before the sync runs.
  std::unique_ptr<Shell> up = transport_->open({"sh"});
  {
    std::lock_guard<std::mutex> g(helper_mu_);
    helper_state_ = 0;
  }
  concurrent_open_ = true;
  struct Reset {
    bool& f;
    ~Reset() { f = false; }
  } reset{concurrent_open_};
  std::exception_ptr down_error;
  std::thread down([this, &down_error] {
    try {
      open_down_shell();
    } catch (...) {
      down_error = std::current_exception();
    }
  });
  try {
    open_up_shell(std::move(up));
  } catch (...) {
    down.join();
    throw;
  }
  down.join();
  if (down_error) std::rethrow_exception(down_error);
  request_watch();
}

// ============================================================ rules (evaluater.go)

bool Session::should_remove_remote(const std::string& rel) {
  if (has_ignore_ && ignore_.matches(rel)) return false;
  if (has_upload_ignore_ && upload_ignore_.matches(rel)) return false;
  FileInfo* f = index_.find(rel);
  if (!f) return false;
  if (f->is_symlink) return false;
  return true;
}

bool Session::should_upload(const std::string& rel, const fs::StatInfo& st, bool initial) {
  if (!st.exists) return false;
  if (has_ignore_ && ignore_.matches(rel)) return false;
  if (st.is_symlink) return false;
  FileInfo* f = index_.find(rel);
  if (f) {
    if (st.is_dir) return false;
    if (f->is_symlink) return false;
    if (initial) {
      if (st.mtime_rounded() <= f->mtime) return false;
    } else {
      if (mode_ != Mode::Compat && f->local_mtime_ns) {
        if (st.mtime_sec * 1000000000LL + st.mtime_nsec == f->local_mtime_ns && st.size == f->size) return false;
      } else if (st.mtime_rounded() == f->mtime && st.size == f->size) {
        return false;
      }
    }
  }
  return true;
}

bool Session::should_download(const FileInfo& fi) {
  if (has_ignore_ && ignore_.matches(fi.name)) return false;
  if (has_download_ignore_ && download_ignore_.matches(fi.name)) return false;
  if (fi.is_symlink) return false;
  FileInfo* f = index_.find(fi.name);
  if (f) {
    if (!fi.is_dir) {
      if (fi.mtime > f->mtime) return true;
      if (fi.mtime == f->mtime && fi.size != f->size) return true;
      // helper listings: a same-size rewrite within the second moved the nanoseconds
      if (fi.mtime == f->mtime && fi.remote_mtime_ns && f->remote_mtime_ns && fi.remote_mtime_ns != f->remote_mtime_ns)
        return true;
    }
    return false;
  }
  return true;
}

bool Session::should_remove_local(const std::string& abs, const FileInfo& fi) {
  if (has_download_ignore_ && download_ignore_.matches(fi.name)) return false;
  fs::StatInfo st = fs::stat(abs);
  if (!st.exists) return false;
  FileInfo* f = index_.find(fi.name);
  if (!f) return false;
  if (st.is_dir != f->is_dir || st.is_dir != fi.is_dir) {
    logf("Skip " + abs + " because stat returned unequal isdir with fileMap");
    return false;
  }
  if (!fi.is_dir) {
    if (fi.mtime == f->mtime && fi.size == f->size) {
      if (st.mtime_rounded() <= fi.mtime) return true;
      logf(strfmt("Skip %s because stat.ModTime() %lld is greater than fileInformation.Mtime %lld", abs.c_str(),
                  (long long)st.mtime_rounded(), (long long)fi.mtime));
    } else {
      logf("Skip " + abs + " because Mtime or Size is unequal between fileInformation and fileMap");
    }
    return false;
  }
  return true;
}

// ============================================================ symlinks

std::optional<fs::StatInfo> Session::add_symlink(const std::string& rel, const std::string& abs) {
  std::string target = fs::realpath(abs);
  if (target.empty()) {
    logf("Warning: resolving symlink of " + abs);
    return std::nullopt;
  }
  fs::StatInfo st = fs::stat(target);
  if (!st.exists) {
    logf("Warning: stating symlink " + target);
    return std::nullopt;
  }
  std::lock_guard<std::mutex> g(symlink_mu_);
  if (symlinks_.count(abs)) return st;
  if (has_ignore_ && ignore_.matches(rel)) return std::nullopt;
  std::string pattern = st.is_dir ? target + "/**" : target;
  std::string link = abs;
  auto w = std::make_unique<PollWatcher>(
      std::vector<std::string>{pattern},
      [this, link, target](const std::vector<std::string>& changed, const std::vector<std::string>& deleted) {
        for (auto& p : changed) {
          UpEvent e;
          e.abs_path = link + p.substr(target.size());
          push_event(e);
        }
        for (auto& p : deleted) {
          UpEvent e;
          e.abs_path = link + p.substr(target.size());
          push_event(e);
        }
      },
      500);
  w->start();
  symlinks_[abs] = std::move(w);
  symlink_targets_[abs] = target;
  return st;
}

void Session::remove_symlinks(const std::string& abs) {
  std::lock_guard<std::mutex> g(symlink_mu_);
  for (auto it = symlinks_.begin(); it != symlinks_.end();) {
    if (it->first == abs || starts_with(it->first, abs + "/")) {
      it->second->stop();
      symlink_targets_.erase(it->first);
      it = symlinks_.erase(it);
    } else {
      ++it;
    }
  }
}

// ============================================================ upstream

void Session::push_event(UpEvent e) {
  if (!e.t_us) e.t_us = mono_us();
  {
    std::lock_guard<std::mutex> g(q_mu_);
    queue_.push_back(std::move(e));
  }
  // all: q_cv_ also has the bulk upload/download loops waiting on other predicates; a
  // notify_one that lands on one of those leaves the upstream loop asleep for its whole quiet
  // window (10 ms per edit in helper mode, measured on the MI355X box)
  q_cv_.notify_all();
}

void Session::start_watcher() {
  watcher_ = make_tree_watcher();
  std::string err;
  bool ok = watcher_->start(
      o_.watch_path,
      [this](const std::string& path, bool settled) {
        if (path.empty()) {
          // queue overflow: rescan everything
          UpEvent e;
          e.abs_path = o_.watch_path;
          push_event(e);
          return;
        }
        UpEvent e;
        e.abs_path = path;
        e.settled = settled;
        push_event(e);
      },
      &err);
  if (!ok) throw SyncError("cannot watch " + o_.watch_path + ": " + err);
}

std::optional<FileInfo> Session::evaluate_change(const std::string& rel, const std::string& abs) {
  if (ends_with(rel, kTmpSuffix)) return std::nullopt;  // a download in progress
  fs::StatInfo st = fs::stat(abs);
  if (st.exists) {
    if (has_upload_ignore_ && upload_ignore_.matches(rel)) {
      FileInfo* f = index_.find(rel);
      if (f && f->mtime < st.mtime_rounded()) {
        FileInfo n;
        n.name = rel;
        n.mtime = st.mtime_rounded();
        n.size = st.size;
        n.is_dir = st.is_dir;
        index_.files[rel] = n;
      }
      return std::nullopt;
    }
    fs::StatInfo lst = fs::lstat(abs);
    if (lst.is_symlink) {
      bool existed;
      {
        std::lock_guard<std::mutex> g(symlink_mu_);
        existed = symlinks_.count(abs) > 0;
      }
      auto s2 = add_symlink(rel, abs);
      if (!s2) return std::nullopt;
      st = *s2;
      if (!existed && st.is_dir) {
        // crawl linked tree (symlink.go:96)
        std::string target = fs::realpath(abs);
        fs::walk(target, [&](const std::string& p, const fs::StatInfo&) {
          UpEvent e;
          e.abs_path = abs + p.substr(target.size());
          push_event(e);
          return true;
        });
      }
    }
    if (should_upload(rel, st, false)) {
      FileInfo f;
      f.name = rel;
      f.mtime = st.mtime_rounded();
      f.size = st.size;
      f.is_dir = st.is_dir;
      return f;
    }
    return std::nullopt;
  }
  remove_symlinks(abs);
  if (should_remove_remote(rel)) {
    FileInfo f;
    f.name = rel;
    return f;
  }
  return std::nullopt;
}

void Session::upstream_loop() {
  while (!stopping_ && !failed_) {
    std::vector<UpEvent> batch;
    {
      std::unique_lock<std::mutex> lk(q_mu_);
      q_cv_.wait_for(lk, std::chrono::milliseconds(200), [this] { return !queue_.empty() || stopping_ || failed_; });
      if (queue_.empty()) continue;
      up_busy_ = true;  // a batch is being gathered / uploaded (see wait_upstream_idle)
    }
    struct Idle {  // cleared on every way out of this iteration
      Session* s;
      ~Idle() {
        {
          std::lock_guard<std::mutex> g(s->q_mu_);
          s->up_busy_ = false;
        }
        s->q_cv_.notify_all();
      }
    } idle{this};
    std::vector<FileInfo> changes;
    std::map<std::string, size_t> pos;
    long first_us = 0;
    long batch_start_us = mono_us();
    size_t last_count = 0;
    bool first = true;
    bool last_settled = false;
    while (!stopping_ && !failed_) {
      std::vector<UpEvent> evs;
      {
        std::unique_lock<std::mutex> lk(q_mu_);
        if (!first) {
          // Fast modes: a finished write (close/rename/delete) only needs a short grace period to
          // absorb its sibling events (an editor's write-temp + rename arrive in the same inotify
          // read, well inside 250 us); partial writes wait the full quiet window.
          long w_us = (mode_ != Mode::Compat && last_settled) ? std::min<long>(window_ms_ * 1000L, 250)
                                                               : window_ms_ * 1000L;
          q_cv_.wait_for(lk, std::chrono::microseconds(w_us), [this] { return !queue_.empty() || stopping_ || failed_; });
        }
        evs.assign(std::make_move_iterator(queue_.begin()), std::make_move_iterator(queue_.end()));
        queue_.clear();
      }
      first = false;
      if (evs.empty()) {
        if (!changes.empty()) break;  // quiet window elapsed
        break;
      }
      if (!first_us) first_us = evs.front().t_us;
      last_settled = evs.back().settled || evs.back().has_info;
      {
        std::lock_guard<std::mutex> g(index_.mu);
        for (auto& ev : evs) {
          std::optional<FileInfo> fi;
          if (ev.has_info) {
            fi = ev.info;
          } else {
            if (!starts_with(ev.abs_path, o_.watch_path)) continue;
            std::string rel = ev.abs_path.substr(o_.watch_path.size());
            rel = replace_all(rel, "//", "/");
            if (rel.empty()) {
              // root itself (rescan request): diff the whole tree
              continue;
            }
            fi = evaluate_change(rel, ev.abs_path);
          }
          if (!fi) continue;
          auto it = pos.find(fi->name);
          if (mode_ == Mode::Compat) {
            changes.push_back(*fi);  // the reference appends duplicates (upstream.go:140)
          } else if (it != pos.end()) {
            changes[it->second] = *fi;
          } else {
            pos[fi->name] = changes.size();
            changes.push_back(*fi);
          }
        }
      }
      // compat: stop gathering when a window passed without new changes (upstream.go:148)
      if (mode_ == Mode::Compat) {
        if (!changes.empty() && changes.size() == last_count) break;
        last_count = changes.size();
      } else if (mono_us() - batch_start_us > 500000) {
        break;  // cap coalescing under continuous writes
      }
    }
    if (changes.empty() || stopping_ || failed_) continue;
    try {
      if (up_helper_)
        dispatch_upstream(changes, first_us);
      else
        apply_upstream(changes, first_us);
    } catch (const std::exception& e) {
      fail(e.what());
      return;
    }
  }
}

// A file at least this big goes to the bulk lane; so does a whole batch whose small files
// together pass kBulkBatchBytes (an edit-sized upload stays interactive).
static const int64_t kBulkFileBytes = 4ll << 20;
static const uint64_t kBulkBatchBytes = 32ull << 20;

void Session::dispatch_upstream(std::vector<FileInfo>& changes, long first_event_us) {
  std::vector<FileInfo> now, bulk;
  std::vector<std::string> later;
  uint64_t small_bytes = 0;
  for (auto& c : changes) {
    if (in_flight(c.name, true)) {  // the bulk upload carries this path: after it, re-evaluated
      later.push_back(o_.watch_path + c.name);
      continue;
    }
    if (c.mtime > 0 && !c.is_dir && c.size >= kBulkFileBytes) {
      bulk.push_back(c);
    } else {
      if (c.mtime > 0 && !c.is_dir) small_bytes += (uint64_t)std::max<int64_t>(0, c.size);
      now.push_back(c);
    }
  }
  if (small_bytes >= kBulkBatchBytes) {  // a big tree of small files (a dataset copied in): all bulk
    std::vector<FileInfo> keep;
    for (auto& c : now) (c.mtime > 0 ? bulk : keep).push_back(c);
    now.swap(keep);
  }
  if (!later.empty()) {
    std::lock_guard<std::mutex> g(q_mu_);
    deferred_.insert(deferred_.end(), later.begin(), later.end());
  }
  if (!bulk.empty()) {
    mark_inflight(bulk, true, true);
    {
      std::lock_guard<std::mutex> g(q_mu_);
      bulk_q_.push_back(std::move(bulk));
    }
    q_cv_.notify_all();
  }
  if (!now.empty()) apply_upstream(now, first_event_us);
}

void Session::bulk_loop() {
  while (!stopping_ && !failed_) {
    std::vector<FileInfo> batch;
    {
      std::unique_lock<std::mutex> lk(q_mu_);
      q_cv_.wait_for(lk, std::chrono::milliseconds(200), [this] { return !bulk_q_.empty() || stopping_ || failed_; });
      if (bulk_q_.empty()) continue;
      batch = std::move(bulk_q_.front());
      bulk_q_.pop_front();
      bulk_busy_ = true;
    }
    struct Done {  // on every way out: the paths are no longer in flight, deferred edits go again
      Session* s;
      const std::vector<FileInfo>& b;
      ~Done() {
        s->mark_inflight(b, true, false);
        {
          std::lock_guard<std::mutex> g(s->q_mu_);
          s->bulk_busy_ = false;
          for (auto& p : s->deferred_) {
            UpEvent e;
            e.abs_path = p;
            e.settled = true;
            e.t_us = mono_us();
            s->queue_.push_back(std::move(e));
          }
          s->deferred_.clear();
        }
        s->q_cv_.notify_all();
      }
    } done{this, batch};
    try {
      apply_upstream(batch, 0, true);
    } catch (const std::exception& e) {
      fail(e.what());
      return;
    }
  }
}

void Session::mark_inflight(const std::vector<FileInfo>& files, bool bulk, bool on) {
  std::lock_guard<std::mutex> g(inflight_mu_);
  auto& m = bulk ? inflight_bulk_ : inflight_;
  for (auto& f : files) {
    if (on) {
      ++m[f.name];
    } else {
      auto it = m.find(f.name);
      if (it != m.end() && --it->second <= 0) m.erase(it);
    }
  }
}

bool Session::in_flight(const std::string& rel, bool bulk_only) {
  std::lock_guard<std::mutex> g(inflight_mu_);
  if (inflight_bulk_.empty() && (bulk_only || inflight_.empty())) return false;
  // the path itself or a directory above it (a directory upload carries its tree)
  for (std::string q = rel; !q.empty() && q != "/"; q = fs::dirname(q)) {
    if (inflight_bulk_.count(q) || (!bulk_only && inflight_.count(q))) return true;
    if (q.find('/') == std::string::npos) break;
  }
  return false;
}

// Lane ids of the upstream helper: one upload at a time per lane (edits come from the upstream
// loop, bulk transfers from the bulk loop), removes only tag their reply.
static const int kEditLane = 1, kBulkLane = 2, kRemoveTag = 3;

void Session::up_frame(const std::string& head, const char* d, size_t n) {
  std::lock_guard<std::mutex> g(up_wmu_);
  int fd = up_shell_->in();
  send(fd, head.data(), head.size());
  if (n) send(fd, d, n);
}

void Session::wait_no_priority() {
  if (up_prio_.load() == 0) return;
  std::unique_lock<std::mutex> lk(up_pmu_);
  up_pcv_.wait_for(lk, std::chrono::milliseconds(o_.idle_timeout_ms),
                   [this] { return up_prio_.load() == 0 || stopping_ || failed_; });
}

void Session::start_up_reader() {
  std::lock_guard<std::mutex> g(up_rmu_);
  up_replies_.clear();
  up_reader_eof_ = false;
  up_reading_ = false;
}

// Replies of the upstream helper, read by whichever waiter gets there first (leader/follower):
// with one upload in flight — an edit — its own thread reads its reply, no hand-off; a reply for
// another lane is parked in up_replies_ for its waiter.
std::string Session::up_wait(int lane, int idle_ms, const char* what) {
  std::unique_lock<std::mutex> lk(up_rmu_);
  long start = mono_us();
  while (true) {
    auto it = up_replies_.find(lane);
    if (it != up_replies_.end()) {
      std::string r = it->second;
      up_replies_.erase(it);
      return r;
    }
    if (up_reader_eof_) throw SyncError(std::string(what) + ": stream closed");
    if (stopping_) throw SyncError("sync stopped");
    if (mono_us() - start > (long)idle_ms * 1000)
      throw SyncError(strfmt("%s: no reply for %d s", what, idle_ms / 1000));
    if (up_reading_) {
      up_rcv_.wait_for(lk, std::chrono::milliseconds(50));
      continue;
    }
    up_reading_ = true;
    lk.unlock();
    std::string line;
    bool got = up_out_.read_line(&line, 50);
    bool eof = !got && up_out_.eof();
    lk.lock();
    up_reading_ = false;
    if (got) {
      if (line.size() > 1 && line[0] == '@') {
        size_t sp = line.find(' ');
        int l = std::atoi(line.substr(1, sp == std::string::npos ? std::string::npos : sp - 1).c_str());
        up_replies_[l] = sp == std::string::npos ? "" : line.substr(sp + 1);
      } else if (!line.empty()) {
        logf("[Upstream] Helper: " + line);
      }
    }
    if (eof) up_reader_eof_ = true;
    up_rcv_.notify_all();
  }
}

void Session::apply_upstream(std::vector<FileInfo>& changes, long first_event_us, bool bulk) {
  trace::Span span(bulk ? "sync.upstream_bulk" : "sync.upstream_batch",
                   {{"changes", std::to_string(changes.size())}, {"dest", o_.dest_path}});
  std::vector<FileInfo> creates, removes;
  for (auto& c : changes) (c.mtime > 0 ? creates : removes).push_back(c);
  if (!removes.empty()) apply_removes(removes);
  if (!creates.empty()) apply_creates(creates, bulk);
  logf(strfmt("[Upstream] Successfully processed %zu change(s)", changes.size()));
  std::lock_guard<std::mutex> g(stats_mu_);
  stats_.upstream_batches++;
  stats_.upstream_changes += changes.size();
  if (first_event_us) stats_.last_upload_ms = (double)(mono_us() - first_event_us) / 1000.0;
}

bool Session::wait_ack(LineReader& r, const std::string& keyword, bool partial, std::string* before,
                       int timeout_ms) {
  // idle timeout: any byte received (e.g. listing lines before the keyword) restarts it
  long start = mono_us();
  while (!stopping_) {
    if (r.wait_for(keyword, 200, before, partial)) return true;
    if (r.eof()) throw SyncError("stream closed unexpectedly while waiting for " + keyword);
    if (mono_us() - std::max(start, r.last_activity_us()) > (long)timeout_ms * 1000)
      throw SyncError(strfmt("no data for %d s while waiting for %s", timeout_ms / 1000, keyword.c_str()));
  }
  throw SyncError("sync stopped");
}

void Session::send(int fd, const char* d, size_t n) {
  // the shell's stdin is non-blocking on our side (open_*_shell): a container that stops
  // reading is detected after the idle timeout instead of blocking this thread for ever
  long last = mono_us();
  while (n > 0) {
    ssize_t w = ::write(fd, d, n);
    if (w > 0) {
      d += w;
      n -= (size_t)w;
      last = mono_us();
      continue;
    }
    if (w < 0 && errno == EINTR) continue;
    if (w < 0 && errno != EAGAIN) throw SyncError(std::string("stream closed while sending: ") + std::strerror(errno));
    if (stopping_) throw SyncError("sync stopped");
    if (mono_us() - last > (long)o_.idle_timeout_ms * 1000)
      throw SyncError(strfmt("the container accepted no data for %d s", o_.idle_timeout_ms / 1000));
    struct pollfd pf{fd, POLLOUT, 0};
    ::poll(&pf, 1, 200);
  }
}

std::string Session::read_line_idle(LineReader& r, int idle_ms, const char* what) {
  long start = mono_us();
  std::string line;
  while (true) {
    if (r.read_line(&line, 200)) return line;
    if (r.eof()) throw SyncError(std::string(what) + ": stream closed");
    if (stopping_) throw SyncError("sync stopped");
    if (mono_us() - std::max(start, r.last_activity_us()) > (long)idle_ms * 1000)
      throw SyncError(strfmt("%s: no data for %d s", what, idle_ms / 1000));
  }
}

Source Session::reader_source(LineReader& r, int idle_ms, const char* what) {
  std::string w = what;
  return [this, &r, idle_ms, w](char* b, size_t n) -> ssize_t {
    long start = mono_us();
    while (true) {
      ssize_t got = r.read_some(b, n, 200);
      if (got > 0) return got;
      if (got == 0 || got == -1) throw SyncError(w + ": stream closed");
      if (stopping_) throw SyncError("sync stopped");
      if (mono_us() - std::max(start, r.last_activity_us()) > (long)idle_ms * 1000)
        throw SyncError(strfmt("%s: no data for %d s", w.c_str(), idle_ms / 1000));
    }
  };
}

void Session::warn_large(const std::string& rel, int64_t size) {
  if (large_warn_bytes_ <= 0 || size < large_warn_bytes_ || !warned_large_.insert(rel).second) return;
  std::string msg = strfmt(
      "[Sync] Large file %s (%s) is being synced; if it should stay on one side, add it to excludePaths "
      "(or uploadExcludePaths / downloadExcludePaths) of this sync path",
      rel.c_str(), human_bytes((uint64_t)size).c_str());
  logf(msg);
  if (!o_.silent) log::warn(msg);
}

void Session::apply_removes(const std::vector<FileInfo>& files) {
  logf(strfmt("[Upstream] Handling %zu removes", files.size()));
  // the index entries go first (under the lock), the container's copies after (without it); the
  // paths stay in flight meanwhile so a downstream scan does not fetch them back
  std::vector<std::pair<std::vector<std::string>, std::string>> groups;  // (shell args, helper payload)
  mark_inflight(files, false, true);  // before the index forgets them
  struct Unmark {
    Session* s;
    const std::vector<FileInfo>& g;
    ~Unmark() { s->mark_inflight(g, false, false); }
  } unmark{this, files};
  {
    std::lock_guard<std::mutex> ig(index_.mu);
    for (size_t i = 0; i < files.size(); i += 50) {
      std::vector<std::string> args;
      std::string helper_payload;
      for (size_t j = 0; j < 50 && i + j < files.size(); ++j) {
        const std::string& rel = files[i + j].name;
        FileInfo* f = index_.find(rel);
        if (!f) continue;
        args.push_back(shell_quote(dest_ + rel));
        helper_payload += rel + "\n";
        if (f->is_dir)
          index_.remove_dir(rel);
        else
          index_.files.erase(rel);
        if (o_.verbose || files.size() <= 3) logf("[Upstream] Remove " + rel);
      }
      if (!args.empty()) groups.emplace_back(std::move(args), std::move(helper_payload));
    }
  }
  if (groups.empty()) return;
  if (up_helper_) {
    for (auto& grp : groups) {
      int lane = kRemoveTag;
      up_frame(request('X', std::string(1, (char)lane) + grp.second), nullptr, 0);
      std::string r = up_wait(lane, o_.idle_timeout_ms, "upstream: helper reply");
      if (r != "OK") throw SyncError("upstream: helper error: " + r);
    }
    return;
  }
  std::lock_guard<std::mutex> sg(up_shell_mu_);
  for (auto& grp : groups) {
    const auto& args = grp.first;
    if (mode_ == Mode::Compat) {
      std::string cmd = "rm -R " + join(args, " ") + "  >/dev/null 2>/dev/null && printf \"" + kDone +
                        "\" || printf \"" + kDone + "\"\n";
      send(up_shell_->in(), cmd);
      wait_ack(up_out_, kDone, true);
    } else {
      std::string cmd = "rm -R " + join(args, " ") + " >/dev/null 2>&1; echo " + kDone + "\n";
      send(up_shell_->in(), cmd);
      wait_ack(up_out_, kDone, false);
    }
  }
}

void Session::recursive_tar(const std::string& rel, std::map<std::string, FileInfo>* written, TarWriter* tw,
                            int depth) {
  // the index lock is taken per lookup (the upload runs without it)
  if (depth > 64 || written->count(rel)) return;
  if (has_ignore_ && ignore_.matches(rel)) return;
  if (has_upload_ignore_ && upload_ignore_.matches(rel)) return;
  if (ends_with(rel, kTmpSuffix)) return;
  std::string abs = o_.watch_path + rel;
  fs::StatInfo st = fs::stat(abs);  // follows symlinks like the reference (os.Stat)
  if (!st.exists) {
    logf("[Upstream] Couldn't stat file " + abs);
    return;
  }
  FileInfo fi;
  fi.name = rel;
  fi.size = st.size;
  fi.mtime = st.mtime_rounded();
  fi.is_dir = st.is_dir;
  if (mode_ != Mode::Compat) fi.local_mtime_ns = st.mtime_sec * 1000000000LL + st.mtime_nsec;
  uint32_t mode = st.mode & 07777;
  uint32_t uid = st.uid, gid = st.gid;
  {
    std::lock_guard<std::mutex> ig(index_.mu);
    if (FileInfo* known = index_.find(rel)) {
      fi.remote_mode = known->remote_mode;
      fi.remote_uid = known->remote_uid;
      fi.remote_gid = known->remote_gid;
      fi.has_remote_attrs = known->has_remote_attrs;
      if (known->has_remote_attrs) {
        mode = (uint32_t)known->remote_mode;
        uid = (uint32_t)known->remote_uid;
        gid = (uint32_t)known->remote_gid;
      }
    }
  }
  std::string name = rel.empty() ? "" : rel.substr(1);
  if (st.is_dir) {
    auto entries = fs::list_dir(abs);
    if (entries.empty() && !rel.empty()) {
      TarEntry e;
      e.name = name;
      e.mode = mode;
      e.uid = uid;
      e.gid = gid;
      e.mtime = st.mtime_sec;
      tw->add_dir(e);
      (*written)[rel] = fi;
    }
    for (auto& e : entries) recursive_tar(rel + "/" + e.name, written, tw, depth + 1);
    return;
  }
  TarEntry e;
  e.name = name;
  e.mode = mode;
  e.uid = uid;
  e.gid = gid;
  e.size = st.size;
  e.mtime = st.mtime_sec;
  {
    std::lock_guard<std::mutex> ig(index_.mu);
    warn_large(rel, st.size);
  }
  if (!tw->add_file_from_path(e, abs)) {
    logf("[Upstream] Couldn't read file " + abs);
    return;
  }
  (*written)[rel] = fi;
}

uint64_t Session::stream_upload(const std::vector<FileInfo>& files, std::map<std::string, FileInfo>* written,
                                bool bulk) {
  int fd = up_shell_->in();
  RateLimiter rl(o_.upstream_limit);
  Progress prog(this, "[Upstream] Upload", 0);
  Sink to_shell = [&](const char* d, size_t n) {
    if (o_.upstream_limit > 0) rl.take(n);
    prog.add(n);
    send(fd, d, n);
    return true;
  };
  auto tar_all = [&](TarWriter& tw) {
    for (auto& f : files)
      if (!written->count(f.name)) recursive_tar(f.name, written, &tw, 0);
    return tw.finish();
  };
  if (up_helper_) {
    // chunk-framed stream on a lane of its own: tar -> chunks (per-chunk deflate where it pays)
    // -> 'C' frames, no length announced, nothing staged (the container extracts while we read
    // the files). An interactive upload holds the priority while it sends: bulk frames wait.
    int lane = bulk ? kBulkLane : kEditLane;
    struct Prio {
      Session* s;
      bool on;
      ~Prio() {
        if (on && s->up_prio_.fetch_sub(1) == 1) {
          std::lock_guard<std::mutex> g(s->up_pmu_);
          s->up_pcv_.notify_all();
        }
      }
    } prio{this, !bulk};
    if (!bulk) up_prio_.fetch_add(1);
    const std::string lane_byte(1, (char)lane);
    // lane bytes are coalesced into frames of up to kMaxChunk: an edit travels as one write
    // (lane open + its whole chunk stream), a bulk stream as one frame per chunk
    std::string pend;
    bool opened = false;
    auto flush = [&] {
      std::string head;
      if (!opened) {
        head = request('U', lane_byte);
        opened = true;
      }
      if (!pend.empty()) head += frame::header('C', pend.size() + 1) + lane_byte;
      if (head.empty()) return;
      if (bulk) wait_no_priority();
      up_frame(head, pend.data(), pend.size());
      pend.clear();
    };
    Sink to_lane = [&](const char* d, size_t n) {
      if (o_.upstream_limit > 0) rl.take(n);
      prog.add(n);
      if (!pend.empty() && pend.size() + n > frame::kMaxChunk) flush();
      pend.append(d, n);
      if (pend.size() >= frame::kMaxChunk) flush();
      return true;
    };
    frame::ChunkWriter cw(to_lane, frame::kMaxChunk, 1);
    TarWriter tw(cw.sink());
    if (!tar_all(tw) || !cw.finish()) throw SyncError("upstream: write failed");
    flush();
    if (prio.on) {  // sent: bulk frames may go while we wait for the reply
      prio.on = false;
      if (up_prio_.fetch_sub(1) == 1) {
        std::lock_guard<std::mutex> g(up_pmu_);
        up_pcv_.notify_all();
      }
    }
    std::string r = up_wait(lane, o_.idle_timeout_ms, "upstream: helper reply");
    if (r != "OK") throw SyncError("upstream: helper error: " + r);
    prog.finish();
    return prog.done;
  }
  // The shell protocols announce the length first (`head -c N`, the reference's fileSize=N
  // script): the archive is staged in a SpillBuffer — memory up to 8 MiB, an unlinked temp
  // file beyond — instead of a string (the reference always used a temp file, tar.go:146).
  // The reference always gzips; fast modes ship small edits as plain tar.
  SpillBuffer spill;
  ArchiveEncoder enc(spill.sink(), mode_ == Mode::Compat ? 0 : kPlainTarLimit, mode_ == Mode::Compat ? 6 : 1);
  TarWriter tw(enc.sink());
  if (!tar_all(tw) || !enc.finish()) throw SyncError("upstream: cannot stage the archive (temp space?)");
  if (written->empty()) return 0;
  const std::string size = std::to_string(spill.size());
  const char* xflags = enc.gzipped() ? "xzpf" : "xpf";
  // the container cannot start extracting before the whole archive arrived (compat) or after
  // the last byte only finishes the last file (fast); allow for it beyond the idle timeout
  int done_ms = o_.idle_timeout_ms + (int)std::min<uint64_t>(spill.size() / 20000, 3600000);
  auto send_payload = [&] {
    if (!spill.replay(to_shell)) throw SyncError("upstream: write failed");
  };
  if (mode_ == Mode::Compat || !up_has_head_) {
    // the reference protocol (sync/upstream.go:387-411); compat archives are always gzip, the
    // fast mode's cat/stat fallback may ship a small edit as plain tar. Its fixed temp file
    // lives in the container's /tmp (remote(): under the pod root for local-pod backends, whose
    // pods share the host's /tmp).
    std::string cmd = "fileSize=" + size + R"(;
					tmpFile=")" + remote("/tmp/devspace-upstream") + R"(";
					mkdir -p )" + remote("/tmp") + R"(;
					mkdir -p ')" + dest_ + R"(';

					pid=$$;
					cat </proc/$pid/fd/0 >"$tmpFile" &
					ddPid=$!;

					echo "START";

					while true; do
							bytesRead=$(stat -c "%s" "$tmpFile" 2>/dev/null || printf "0");

							if [ "$bytesRead" = "$fileSize" ]; then
									kill $ddPid;
									break;
							fi;

							sleep 0.1;
					done;

					tar )" + std::string(xflags) + R"( "$tmpFile" -C ')" + dest_ + R"(/.' 2>)" + remote("/tmp/devspace-upstream-error") + R"(;
					echo "DONE";
		)";
    send(fd, cmd);
    wait_ack(up_out_, kStart, false, nullptr, o_.idle_timeout_ms);
    send_payload();
    wait_ack(up_out_, kDone, false, nullptr, done_ms);
    prog.finish();
    return spill.size();
  }
  // dest is created once when the shell opens; `head -c N | tar x` streams (no temp file, no
  // polling in the container)
  std::string cmd = "echo " + std::string(kStart) + " && head -c " + size + " | tar " + xflags + " - -C " +
                    shell_quote(dest_ + "/.") + " 2>" + remote("/tmp/devspace-upstream-error") + "; echo " + kDone + "\n";
  send(fd, cmd);
  wait_ack(up_out_, kStart, false, nullptr, o_.idle_timeout_ms);
  send_payload();
  wait_ack(up_out_, kDone, false, nullptr, done_ms);
  prog.finish();
  return spill.size();
}

void Session::apply_creates(const std::vector<FileInfo>& files, bool bulk) {
  std::map<std::string, FileInfo> written;
  uint64_t sent = 0;
  // No index lock while the bytes travel (a multi-GB upload must not stall the upstream event
  // batching or the downstream loop); the paths are in flight instead, which the downstream
  // loop leaves alone until they are committed below.
  mark_inflight(files, false, true);
  struct Unmark {
    Session* s;
    const std::vector<FileInfo>& f;
    ~Unmark() { s->mark_inflight(f, false, false); }
  } unmark{this, files};
  try {
    if (up_helper_) {
      sent = stream_upload(files, &written, bulk);  // lanes: concurrent uploads share the helper
    } else {
      std::lock_guard<std::mutex> sg(up_shell_mu_);
      sent = stream_upload(files, &written, bulk);
    }
  } catch (...) {
    // whatever was in flight may sit half-written in the container with a fresh mtime; the
    // initial sync after the reconnect must send it again instead of trusting that mtime
    std::lock_guard<std::mutex> ig(index_.mu);
    for (auto& kv : written) force_up_.insert(kv.first);
    for (auto& f : files) force_up_.insert(f.name);
    throw;
  }
  if (written.empty()) return;
  std::lock_guard<std::mutex> ig(index_.mu);
  if (o_.verbose || written.size() <= 3) {
    for (auto& kv : written) logf((kv.second.is_dir ? "[Upstream] Create Folder " : "[Upstream] Create File ") + kv.first);
  }
  logf(strfmt("[Upstream] Upload %zu create changes (size %llu)", written.size(), (unsigned long long)sent));
  for (auto& kv : written) {
    index_.create_dir(fs::dirname(kv.first));
    FileInfo f = kv.second;
    // the container's copy carries the archive's whole-second mtime (recursive_tar)
    if (!f.is_dir && f.local_mtime_ns) f.remote_mtime_ns = f.local_mtime_ns / 1000000000LL * 1000000000LL;
    if (FileInfo* old = index_.find(kv.first)) {
      if (!f.has_remote_attrs && old->has_remote_attrs) {
        f.remote_mode = old->remote_mode;
        f.remote_uid = old->remote_uid;
        f.remote_gid = old->remote_gid;
        f.has_remote_attrs = true;
      }
    }
    index_.files[kv.first] = f;
  }
  std::lock_guard<std::mutex> g(stats_mu_);
  stats_.bytes_up += sent;
}

void Session::send_changes_to_upstream(std::vector<FileInfo> changes) {
  for (size_t j = 0; j < changes.size(); j += kInitialUpstreamBatch) {
    while (!stopping_) {
      {
        std::lock_guard<std::mutex> g(q_mu_);
        if (queue_.empty()) break;
      }
      sleep_ms(mode_ == Mode::Compat ? 1000 : 20);
    }
    std::vector<FileInfo> batch;
    {
      std::lock_guard<std::mutex> g(index_.mu);
      for (size_t i = j; i < j + kInitialUpstreamBatch && i < changes.size(); ++i) {
        FileInfo* f = index_.find(changes[i].name);
        if (!f || changes[i].mtime > f->mtime) batch.push_back(changes[i]);
      }
    }
    for (auto& c : batch) {
      UpEvent e;
      e.has_info = true;
      e.info = c;
      e.abs_path = o_.watch_path + c.name;
      push_event(e);
    }
  }
}

// ============================================================ initial sync

void Session::diff_server_client(const std::string& abs, std::vector<FileInfo>* send,
                                 std::map<std::string, FileInfo>* download, bool dont_send) {
  std::string rel = abs.substr(o_.watch_path.size());
  if (ends_with(rel, kTmpSuffix)) return;
  fs::StatInfo st = fs::stat(abs);
  if (!st.exists) return;
  download->erase(rel);
  if (has_upload_ignore_ && upload_ignore_.matches(rel)) {
    std::lock_guard<std::mutex> g(index_.mu);
    FileInfo* f = index_.find(rel);
    if (f && f->mtime < st.mtime_rounded()) {
      FileInfo n;
      n.name = rel;
      n.mtime = st.mtime_rounded();
      n.size = st.size;
      n.is_dir = st.is_dir;
      index_.files[rel] = n;
    }
    dont_send = true;
  }
  if (!dont_send) {
    fs::StatInfo lst = fs::lstat(abs);
    if (lst.is_symlink) {
      auto s2 = add_symlink(rel, abs);
      if (!s2) return;
      st = *s2;
      logf("Symlink at " + abs);
    }
  }
  if (st.is_dir) {
    auto entries = fs::list_dir(abs);
    if (entries.empty() && !rel.empty() && !dont_send) {
      bool up;
      {
        std::lock_guard<std::mutex> g(index_.mu);
        up = should_upload(rel, st, true);
      }
      if (up) {
        FileInfo f;
        f.name = rel;
        f.mtime = st.mtime_rounded();
        f.size = st.size;
        f.is_dir = true;
        send->push_back(f);
      }
    }
    for (auto& e : entries) diff_server_client(abs + "/" + e.name, send, download, dont_send);
    return;
  }
  if (!dont_send) {
    bool up;
    {
      std::lock_guard<std::mutex> g(index_.mu);
      up = should_upload(rel, st, true);
    }
    if (up) {
      FileInfo f;
      f.name = rel;
      f.mtime = st.mtime_rounded();
      f.size = st.size;
      send->push_back(f);
    }
  }
}

std::map<std::string, FileInfo> Session::clone_index() {
  std::lock_guard<std::mutex> g(index_.mu);
  std::map<std::string, FileInfo> out;
  for (auto& kv : index_.files) {
    if (kv.second.is_symlink) continue;
    FileInfo f;
    f.name = kv.second.name;
    f.size = kv.second.size;
    f.mtime = kv.second.mtime;
    f.is_dir = kv.second.is_dir;
    out[kv.first] = f;
  }
  return out;
}

void Session::initial_sync() {
  trace::Span span("sync.initial", {{"dest", o_.dest_path}});
  // populate the index from the remote tree (downstream.go:84)
  auto creates = collect_changes(nullptr);
  {
    std::lock_guard<std::mutex> g(index_.mu);
    for (auto& f : creates)
      if (!index_.files.count(f.name)) index_.files[f.name] = f;
    // uploads cut off by a broken stream: whatever the container holds there now (a partial
    // file with a fresh mtime in the shell protocols) must not win the mtime comparison
    for (auto& p : force_up_) {
      FileInfo* f = index_.find(p);
      if (f && !f->is_dir) index_.files.erase(p);
    }
  }
  std::vector<FileInfo> local_changes;
  auto remote_only = clone_index();
  diff_server_client(o_.watch_path, &local_changes, &remote_only, false);
  {
    std::lock_guard<std::mutex> g(index_.mu);
    force_up_.clear();
  }
  if (down_helper_ && mode_ != Mode::Compat && !local_changes.empty()) drop_identical_copies(local_changes);
  if (!local_changes.empty()) send_changes_to_upstream(std::move(local_changes));
  if (!remote_only.empty()) {
    std::vector<FileInfo> dl;
    for (auto& kv : remote_only) dl.push_back(kv.second);
    std::map<std::string, FileInfo> none;
    apply_downstream(dl, none);
  }
  // "initial sync done" means the container has the files, not that they are queued (and the
  // files only the container had are here)
  wait_upstream_idle();
  wait_bulk_down_idle();
}

// Initial sync against a pod whose image already holds the project (`COPY . .`): the copies
// carry whole-second mtimes (tar), so a local file whose mtime has a sub-second part >= 0.5
// rounds past its remote copy and the reference re-uploads it (roundMtime vs %Y). Files whose
// remote mtime is the local mtime truncated and whose size matches are compared by CRC-32 in
// the container (helper 'H') instead; identical ones are recorded as synced, not re-sent.
void Session::drop_identical_copies(std::vector<FileInfo>& changes) {
  std::vector<size_t> cand;
  {
    std::lock_guard<std::mutex> g(index_.mu);
    for (size_t i = 0; i < changes.size(); ++i) {
      const FileInfo& c = changes[i];
      if (c.is_dir) continue;
      FileInfo* f = index_.find(c.name);
      if (!f || f->is_dir || f->is_symlink || f->size != c.size || f->mtime != c.mtime - 1) continue;
      cand.push_back(i);
    }
  }
  if (cand.empty()) return;
  std::vector<bool> same(changes.size(), false);
  size_t dropped = 0;
  for (size_t b = 0; b < cand.size(); b += 2000) {
    size_t e = std::min(cand.size(), b + 2000);
    std::string list;
    for (size_t k = b; k < e; ++k) list += changes[cand[k]].name + "\n";
    std::vector<std::string> remote;
    {
      std::lock_guard<std::mutex> sg(down_shell_mu_);
      send(down_shell_->in(), request('H', list));
      long deadline = mono_us() + 300000000L;
      while (true) {
        std::string line;
        if (!down_out_.read_line(&line, 200)) {
          if (down_out_.eof()) throw SyncError("\n[Downstream] Stream closed unexpectedly");
          if (stopping_) throw SyncError("sync stopped");
          if (mono_us() > deadline) throw SyncError("downstream: hash timeout");
          continue;
        }
        if (line == kDone) break;
        remote.push_back(line);
      }
    }
    if (remote.size() != e - b) throw SyncError("downstream: hash reply size mismatch");
    for (size_t k = b; k < e; ++k) {
      const FileInfo& c = changes[cand[k]];
      std::string abs = o_.watch_path + c.name;
      fs::StatInfo st = fs::stat(abs);
      if (!st.exists || st.size != c.size) continue;
      if (remote[k - b] != "-" && remote[k - b] == crc32_file_hex(abs)) {
        same[cand[k]] = true;
        ++dropped;
        std::lock_guard<std::mutex> g(index_.mu);
        FileInfo* f = index_.find(c.name);
        if (f) {
          f->mtime = st.mtime_rounded();
          f->local_mtime_ns = st.mtime_sec * 1000000000LL + st.mtime_nsec;
        }
      }
    }
  }
  if (!dropped) return;
  std::vector<FileInfo> keep;
  keep.reserve(changes.size() - dropped);
  for (size_t i = 0; i < changes.size(); ++i)
    if (!same[i]) keep.push_back(std::move(changes[i]));
  changes.swap(keep);
  logf(strfmt("[Sync] %zu file(s) already identical in the container (CRC-32), not re-uploaded", dropped));
}

void Session::wait_upstream_idle() {
  std::unique_lock<std::mutex> lk(q_mu_);
  while (!stopping_ && !failed_ && (up_busy_ || !queue_.empty() || bulk_busy_ || !bulk_q_.empty()))
    q_cv_.wait_for(lk, std::chrono::milliseconds(50));
}

// ============================================================ downstream

std::vector<FileInfo> Session::collect_changes(std::map<std::string, FileInfo>* removes) {
  std::vector<FileInfo> creates;
  bool dest_found = false;
  std::lock_guard<std::mutex> sg(down_shell_mu_);
  std::string qd = shell_quote(dest_);
  if (down_helper_) {
    send(down_shell_->in(), request('S', ""));
  } else if (mode_ == Mode::Compat) {
    std::string cmd = "mkdir -p '" + dest_ + "' && find -L '" + dest_ +
                      "' -exec stat -c \"%n///%s,%Y,%f,%a,%u,%g\" {} + 2>/dev/null && echo -n \"" + kDone +
                      "\" || echo -n \"" + kError + "\"\n";
    send(down_shell_->in(), cmd);
  } else {
    std::string cmd = "mkdir -p " + qd + " && find -L " + qd +
                      " -exec stat -c '%n///%s,%Y,%f,%a,%u,%g' {} + 2>/dev/null && echo " + kDone + " || echo " +
                      kError + "\n";
    send(down_shell_->in(), cmd);
  }
  RateLimiter rl(o_.downstream_limit);
  long deadline = mono_us() + 300000000L;
  bool partial_ok = mode_ == Mode::Compat && !down_helper_;
  uint64_t scan_bytes = 0;
  int64_t pod_now_ns = 0;           // the helper's clock, first line of its listing
  std::vector<FileInfo> verify;     // downloaded while unsettled, still since: check the content
  struct Count {  // recorded on every exit path
    Session* s;
    uint64_t* bytes;
    ~Count() {
      std::lock_guard<std::mutex> g(s->stats_mu_);
      s->stats_.full_scans++;
      s->stats_.scan_bytes += *bytes;
    }
  } count{this, &scan_bytes};
  while (true) {
    std::string line;
    if (!down_out_.read_line(&line, 200)) {
      if (down_out_.eof()) throw SyncError("\n[Downstream] Stream closed unexpectedly");
      if (stopping_) throw SyncError("sync stopped");
      if (partial_ok) {
        std::string rest = down_out_.take_buffer();
        if (rest == kDone) break;
        if (rest == kError) {
          sleep_ms(4000);
          return collect_changes(removes);
        }
        // put back partial data
        if (!rest.empty()) {
          // no-op: the remaining buffer is an incomplete line; re-append by reading more
          std::string more;
          while (!down_out_.read_line(&more, 200)) {
            if (down_out_.eof()) throw SyncError("\n[Downstream] Stream closed unexpectedly");
            // (a stream that stops inside a line: the stop and the scan deadline still apply;
            // without them a stop waited here for ever, seen by the stop watchdog)
            if (stopping_) throw SyncError("sync stopped");
            if (mono_us() > deadline) throw SyncError("downstream: scan timeout");
            std::string r2 = down_out_.take_buffer();
            rest += r2;
            if (rest == kDone || rest == kError) break;
          }
          if (rest == kDone) break;
          if (rest == kError) {
            sleep_ms(4000);
            return collect_changes(removes);
          }
          line = rest + more;
        } else {
          if (mono_us() > deadline) throw SyncError("downstream: scan timeout");
          continue;
        }
      } else {
        if (mono_us() > deadline) throw SyncError("downstream: scan timeout");
        continue;
      }
    }
    if (o_.downstream_limit > 0) rl.take(line.size() + 1);
    scan_bytes += line.size() + 1;
    if (line == kDone) break;
    if (line == kError) {
      sleep_ms(4000);
      return collect_changes(removes);
    }
    if (line.empty()) continue;
    if (down_helper_ && starts_with(line, "#NOW ")) {
      int64_t v;
      if (parse_int64(line.substr(5), &v)) pod_now_ns = v;
      continue;
    }
    // compat acks have no newline: a "DONE" may be glued to nothing else, handled above
    std::optional<FileInfo> fi;
    try {
      fi = parse_file_line(line, dest_);
    } catch (const SyncError&) {
      if (ends_with(line, kDone) && line.find("///") == std::string::npos) break;
      throw;
    }
    if (!fi) {
      dest_found = true;
      continue;
    }
    if (ends_with(fi->name, kTmpSuffix)) continue;
    if (fi->remote_mtime_ns && pod_now_ns && !fi->is_dir && !fi->is_symlink) fi->remote_unsettled = pod_now_ns - fi->remote_mtime_ns < kUnsettledNs;
    std::lock_guard<std::mutex> ig(index_.mu);
    if (removes) removes->erase(fi->name);
    FileInfo* known = index_.find(fi->name);
    if (known) {
      known->remote_mode = fi->remote_mode;
      known->remote_uid = fi->remote_uid;
      known->remote_gid = fi->remote_gid;
      known->has_remote_attrs = true;
    }
    if (fi->is_symlink) index_.files[fi->name] = *fi;
    bool busy = in_flight(fi->name, false) || downloading(fi->name);
    if (should_download(*fi)) {
      if (!busy) creates.push_back(*fi);
    } else if (known && known->remote_unsettled && !fi->remote_unsettled && !busy &&
               known->remote_mtime_ns == fi->remote_mtime_ns) {
      if (fi->size <= kVerifyMaxBytes)
        verify.push_back(*fi);
      else
        known->remote_unsettled = false;  // a big file is not rewritten within a clock tick
    }
  }
  if (!verify.empty()) verify_unsettled(verify, &creates);
  if (!dest_found) throw SyncError("DestPath not found, find command did not execute correctly");
  if (removes) {  // an upload or remove in flight: the index is about to change, not the pod
    for (auto it = removes->begin(); it != removes->end();) {
      if (in_flight(it->first, false) || downloading(it->first))
        it = removes->erase(it);
      else
        ++it;
    }
  }
  return creates;
}

void Session::verify_unsettled(const std::vector<FileInfo>& files, std::vector<FileInfo>* creates) {
  std::string list;
  for (auto& f : files) list += f.name + "\n";
  send(down_shell_->in(), request('H', list));
  std::vector<std::string> remote;
  long deadline = mono_us() + 300000000L;
  while (true) {
    std::string line;
    if (!down_out_.read_line(&line, 200)) {
      if (down_out_.eof()) throw SyncError("\n[Downstream] Stream closed unexpectedly");
      if (stopping_) throw SyncError("sync stopped");
      if (mono_us() > deadline) throw SyncError("downstream: hash timeout");
      continue;
    }
    if (line == kDone) break;
    remote.push_back(line);
  }
  if (remote.size() != files.size()) throw SyncError("downstream: hash reply size mismatch");
  size_t differ = 0;
  for (size_t i = 0; i < files.size(); ++i) {
    const FileInfo& f = files[i];
    std::string local = crc32_file_hex(o_.watch_path + f.name);
    fs::StatInfo st = fs::stat(o_.watch_path + f.name);
    std::lock_guard<std::mutex> ig(index_.mu);
    FileInfo* known = index_.find(f.name);
    if (!known || known->remote_mtime_ns != f.remote_mtime_ns) continue;  // moved on meanwhile
    known->remote_unsettled = false;
    // edited here since it came down: that edit goes up, nothing comes down over it
    if (!st.exists || st.size != known->size ||
        (known->local_mtime_ns && st.mtime_sec * 1000000000LL + st.mtime_nsec != known->local_mtime_ns))
      continue;
    if (remote[i] != "-" && remote[i] != local) {
      known->remote_mtime_ns = 0;  // this stamp is not the content we hold
      creates->push_back(f);
      ++differ;
    }
  }
  if (differ) logf(strfmt("[Downstream] %zu file(s) rewritten within a clock tick of their download (CRC-32)", differ));
}

// Fast mode: instead of listing the whole tree every poll, ask the container whether anything
// under the destination changed since the stamp written two probes ago (`find -cnewer`, one
// word back). Comparing against the stamp from two probes back (not the last one) keeps files
// written in the same coarse timestamp tick as a stamp from being missed. Only tools of the
// reference's POSIX set are used (sh builtins, find, rm): stamps are created with a shell
// redirect and numbered instead of renamed, and the first match is taken with `read`. No
// writable /tmp reports a change, i.e. falls back to full listings.
bool Session::probe_changes() {
  std::lock_guard<std::mutex> sg(down_shell_mu_);
  if (probe_id_.empty()) probe_id_ = hex_encode(random_string(6));
  std::string st = "/tmp/.devspace-sync-" + probe_id_ + ".";
  long k = probe_seq_++;
  std::string qd = shell_quote(dest_);
  std::string cur = st + std::to_string(k), old = st + std::to_string(k - 2);
  // -cnewer (inode change time: every write and chmod bumps it, no tool can preserve it) where
  // find has it (GNU); busybox find falls back to -newer (mtime)
  std::string cmd = ": > " + cur + " 2>/dev/null || echo NOSTAMP; if [ -e " + old + " ]; then { find -L " + qd +
                    " -cnewer " + old + " 2>/dev/null || find -L " + qd + " -newer " + old +
                    " 2>/dev/null; } | { IFS= read -r l && echo CHANGED; }; else echo FIRST; fi; rm -f " + st +
                    std::to_string(k - 3) + "; echo " + kDone + "\n";
  send(down_shell_->in(), cmd);
  long deadline = mono_us() + 60000000L;
  bool hit = false;
  while (true) {
    std::string line;
    if (!down_out_.read_line(&line, 200)) {
      if (down_out_.eof()) throw SyncError("\n[Downstream] Stream closed unexpectedly");
      if (stopping_) throw SyncError("sync stopped");
      if (mono_us() > deadline) throw SyncError("downstream: probe timeout");
      continue;
    }
    if (line == kDone) break;
    if (!line.empty()) hit = true;
  }
  std::lock_guard<std::mutex> g(stats_mu_);
  stats_.probes++;
  if (hit) stats_.probe_hits++;
  return hit;
}

bool Session::downloading(const std::string& rel) {
  std::lock_guard<std::mutex> g(inflight_mu_);
  return !downloading_.empty() && downloading_.count(rel) > 0;
}

bool Session::open_bulk_down_shell() {
  if (bulk_down_shell_ && bulk_down_shell_->alive()) return true;
  std::unique_ptr<Shell> sh;
  try {
    sh = transport_->open({"sh"});
    bulk_down_out_.reset(sh->out());
    if (start_helper(sh, bulk_down_out_)) {
      std::lock_guard<std::mutex> g(bulk_down_ptr_mu_);
      bulk_down_shell_ = std::move(sh);
      return true;
    }
  } catch (const std::exception& e) {
    logf(std::string("[Downstream] No bulk download channel: ") + e.what());
  }
  if (sh) sh->close();
  std::lock_guard<std::mutex> g(bulk_down_ptr_mu_);
  bulk_down_shell_.reset();
  return false;
}

void Session::bulk_down_loop() {
  while (!stopping_ && !failed_) {
    std::vector<FileInfo> batch;
    {
      std::unique_lock<std::mutex> lk(q_mu_);
      q_cv_.wait_for(lk, std::chrono::milliseconds(200),
                     [this] { return !bulk_down_q_.empty() || stopping_ || failed_; });
      if (bulk_down_q_.empty()) continue;
      batch = std::move(bulk_down_q_.front());
      bulk_down_q_.pop_front();
      bulk_down_busy_ = true;
    }
    struct Done {
      Session* s;
      const std::vector<FileInfo>& b;
      ~Done() {
        {
          std::lock_guard<std::mutex> g(s->inflight_mu_);
          for (auto& f : b) s->downloading_.erase(f.name);
        }
        {
          std::lock_guard<std::mutex> g(s->q_mu_);
          s->bulk_down_busy_ = false;
        }
        s->q_cv_.notify_all();
      }
    } done{this, batch};
    try {
      bool own;
      {
        std::lock_guard<std::mutex> g(bulk_down_mu_);
        own = open_bulk_down_shell();
      }
      download_and_apply(batch, own);  // no second channel: the main one, as before
      std::lock_guard<std::mutex> g(stats_mu_);
      stats_.downstream_batches++;
      stats_.downstream_changes += batch.size();
    } catch (const std::exception& e) {
      fail(e.what());
      return;
    }
  }
}

void Session::wait_bulk_down_idle() {
  std::unique_lock<std::mutex> lk(q_mu_);
  while (!stopping_ && !failed_ && (bulk_down_busy_ || !bulk_down_q_.empty()))
    q_cv_.wait_for(lk, std::chrono::milliseconds(50));
}

void Session::download_and_apply(const std::vector<FileInfo>& files, bool bulk) {
  uint64_t total = 0;
  for (auto& f : files) total += (uint64_t)std::max<int64_t>(0, f.size);
  if (files.size() > 3) logf(strfmt("[Downstream] Download %zu files (size: %llu)", files.size(), (unsigned long long)total));
  {
    std::lock_guard<std::mutex> ig(index_.mu);
    for (auto& f : files) {
      if (files.size() <= 3 || o_.verbose)
        logf(strfmt("[Downstream] Download file %s, size: %lld", f.name.c_str(), (long long)f.size));
      warn_large(f.name, f.size);
    }
  }
  std::lock_guard<std::mutex> sg(bulk ? bulk_down_mu_ : down_shell_mu_);
  Shell* shell = bulk ? bulk_down_shell_.get() : down_shell_.get();
  LineReader& reply = bulk ? bulk_down_out_ : down_out_;
  int fd = shell->in();
  const int idle = o_.idle_timeout_ms;
  Progress prog(this, "[Downstream] Download", total);
  RateLimiter rl(o_.downstream_limit);
  auto counted = [&](Source inner) -> Source {
    return [&, inner](char* b, size_t n) -> ssize_t {
      ssize_t r = inner(b, n);
      if (r > 0) {
        if (o_.downstream_limit > 0) rl.take((size_t)r);
        prog.add((size_t)r);
      }
      return r;
    };
  };
  struct Count {  // wire bytes, recorded however the transfer ends
    Session* s;
    Progress* p;
    ~Count() {
      std::lock_guard<std::mutex> g(s->stats_mu_);
      s->stats_.bytes_down += p->done;
    }
  } count{this, &prog};
  // Smallest first (not in compat mode): files land one by one as the stream is extracted, so a
  // log or metrics file written next to a multi-GB checkpoint arrives before the checkpoint
  // instead of after it.
  std::vector<const FileInfo*> order;
  for (auto& f : files) order.push_back(&f);
  if (mode_ != Mode::Compat)
    std::stable_sort(order.begin(), order.end(), [](const FileInfo* a, const FileInfo* b) { return a->size < b->size; });
  if (down_helper_ || bulk) {
    std::string rels;
    for (auto* f : order) rels += f->name + "\n";
    send(fd, request('D', rels));
    std::string line = read_line_idle(reply, idle, "downstream: helper reply");
    if (line != "STREAM") throw SyncError("downstream: helper error: " + line);
    frame::ChunkReader cr(counted(reader_source(reply, idle, "downstream: helper stream")));
    untar_stream(cr.source(), nullptr);
    cr.drain();
    line = read_line_idle(reply, idle, "downstream: helper reply");
    if (line != "OK") throw SyncError("downstream: helper error: " + line);
    {
      // the container's stamp of what was listed: what came down is that version or a newer one
      // (read after the listing), so a stamp that moves again is always downloaded again
      std::lock_guard<std::mutex> ig(index_.mu);
      for (auto& f : files) {
        FileInfo* x = index_.find(f.name);
        if (!x || x->is_dir || x->mtime != f.mtime || x->size != f.size) continue;
        x->remote_mtime_ns = f.remote_mtime_ns;
        x->remote_unsettled = f.remote_unsettled;
      }
    }
    prog.finish();
    return;
  }
  std::string list;
  for (auto* f : order) list += dest_ + f->name + "\n";
  if (mode_ == Mode::Compat) {
    std::string cmd = "fileSize=" + std::to_string(list.size()) + R"(;
					tmpFileInput=")" + remote("/tmp/devspace-downstream-input") + R"(";
					tmpFileOutput=")" + remote("/tmp/devspace-downstream-output") + R"(";
					mkdir -p )" + remote("/tmp") + R"(;

					pid=$$;
					cat </proc/$pid/fd/0 >"$tmpFileInput" &
					ddPid=$!;

					echo "START";

					while true; do
							bytesRead=$(stat -c "%s" "$tmpFileInput" 2>/dev/null || printf "0");

							if [ "$bytesRead" = "$fileSize" ]; then
									kill $ddPid;
									break;
							fi;

							sleep 0.1;
					done;
					tar -czf "$tmpFileOutput" -T "$tmpFileInput" 2>)" + remote("/tmp/devspace-downstream-error") + R"(;
					(>&2 echo "START");
					(>&2 echo $(stat -c "%s" "$tmpFileOutput"));
					(>&2 echo "DONE");
					cat "$tmpFileOutput";
		)";
    send(fd, cmd);
    wait_ack(down_out_, kStart, false, nullptr, idle);
    send(fd, list);
    // the container gzips everything into its temp file before the size line: silent for a
    // while on big files (gzip -6 runs ~20 MB/s on incompressible data)
    std::string before;
    wait_ack(down_err_, kDone, false, &before, idle + (int)std::min<uint64_t>(total / 5000, 3600000));
    auto lines = split(trim(before), "\n");
    if (lines.empty()) throw SyncError("[Downstream] Cannot find size");
    int64_t n = std::atoll(lines.back().c_str());
    if (n == 0) throw SyncError("[Downstream] Empty tar");
    Source body = limited_source(counted(reader_source(down_out_, idle, "[Downstream] tar stream")), (uint64_t)n);
    untar_stream(body, nullptr);
    char sink[1 << 15];
    while (true) {  // the rest of the announced bytes (tar padding)
      ssize_t r = body(sink, sizeof(sink));
      if (r == 0) break;
      if (r < 0) throw SyncError("[Downstream] Downloaded tar has wrong filesize");
    }
    prog.finish();
    return;
  }
  // fast POSIX: the container streams `tar -c` straight to stdout between two marker lines (no
  // temp file in the pod, no size needed up front). Small sets are gzipped; big ones go as
  // plain tar, which is link-bound instead of gzip-bound (~20 MB/s on checkpoints).
  bool gz = total <= (8ull << 20);
  std::vector<std::string> args;
  for (auto& f : files) args.push_back(shell_quote("." + f.name));
  std::string cmd = "mkdir -p " + shell_quote(remote("/tmp")) + " 2>/dev/null; echo DSSTART; tar -c" +
                    std::string(gz ? "z" : "") + "f - -C " + shell_quote(dest_) + " -- " +
                    join(args, " ") + " 2>" + remote("/tmp/devspace-downstream-error") + "; echo; echo \"DSEND $?\"\n";
  send(fd, cmd);
  while (read_line_idle(down_out_, idle, "downstream") != "DSSTART") {
  }
  std::string leftover;
  untar_stream(counted(reader_source(down_out_, idle, "downstream: tar stream")), &leftover);
  down_out_.unread(leftover);
  // plain tar: zero blocks up to the end of tar's last record, then the marker line
  char zb[4096];
  while (true) {
    ssize_t r = down_out_.read_some(zb, sizeof(zb), 200);
    if (r == -2) {
      if (stopping_) throw SyncError("sync stopped");
      if (mono_us() - down_out_.last_activity_us() > (long)idle * 1000) throw SyncError("downstream: no end marker");
      continue;
    }
    if (r <= 0) throw SyncError("downstream: stream closed");
    ssize_t i = 0;
    while (i < r && zb[i] == 0) ++i;
    if (i < r) {
      down_out_.unread(std::string(zb + i, (size_t)(r - i)));
      break;
    }
  }
  while (true) {
    std::string line = read_line_idle(down_out_, idle, "downstream");
    if (starts_with(line, "DSEND")) break;
  }
  prog.finish();
}

bool has_dotdot_segment(const std::string& rel) {
  for (auto& seg : split(rel, "/"))
    if (seg == "..") return true;
  return false;
}

void Session::untar_stream(Source raw, std::string* leftover) {
  std::string magic;
  {
    char m[2];
    while (magic.size() < 2) {
      ssize_t n = raw(m, 2 - magic.size());
      if (n <= 0) break;
      magic.append(m, (size_t)n);
    }
  }
  if (magic.empty()) return;
  if (leftover && magic[0] == '\n') {  // fast protocol: tar wrote nothing, the end marker follows
    *leftover = magic;
    return;
  }
  bool gz = is_gzip_magic(magic);
  Source src = prefixed_source(magic, raw);
  std::unique_ptr<GzipReader> gzr;
  if (gz) {
    gzr = std::make_unique<GzipReader>(src);
    gzr->set_single_member(leftover != nullptr);
  }
  TarReader tr([&](char* b, size_t n) -> ssize_t {
    if (!gzr) return src(b, n);
    ssize_t r = gzr->read(b, n);
    if (r < 0) throw SyncError("[Downstream] corrupt gzip stream");
    return r;
  });
  TarEntry e;
  int count = 0;
  std::vector<char> buf(1 << 20);
  while (tr.next(&e)) {
    std::string name = e.name;
    if (starts_with(name, "./")) name = name.substr(1);
    if (!starts_with(name, "/")) name = "/" + name;
    std::string rel = name;
    // compat archives carry absolute container paths (tar strips the leading "/")
    if (starts_with(rel, dest_ + "/") || rel == dest_) rel = rel.substr(dest_.size());
    if (!rel.empty() && rel.back() == '/') rel.pop_back();
    if (rel.empty()) continue;
    if (has_dotdot_segment(rel)) {
      // the archive comes from the container: never let it write outside the synced folder
      logf("[Downstream] Skipping archive entry " + e.name + ": path escapes the sync directory");
      tr.skip();
      continue;
    }
    std::string out = o_.watch_path + rel;
    fs::StatInfo before;
    {
      std::lock_guard<std::mutex> ig(index_.mu);
      before = fs::stat(out);
      if (before.exists && before.mtime_rounded() > e.mtime) {
        FileInfo f;
        f.name = rel;
        f.mtime = before.mtime_rounded();
        f.size = before.size;
        f.is_dir = before.is_dir;
        index_.files[rel] = f;
        logf("[Downstream] Don't override " + rel + " because file has newer mTime timestamp");
        tr.skip();
        continue;
      }
      fs::mkdirs(fs::dirname(out));
      if (e.type == '5') {
        fs::mkdirs(out);
        index_.create_dir(rel);
        continue;
      }
      if (e.type != '0' && e.type != '7') {
        tr.skip();
        continue;
      }
    }
    // stream the contents to a temp name next to the target (the upstream watcher ignores the
    // suffix) without holding the index: a big file must not stall local edits meanwhile
    std::string tmp = out + kTmpSuffix;
    int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0600);
    if (fd < 0) {
      sleep_ms(mode_ == Mode::Compat ? 5000 : 200);  // retry once (tar.go:97)
      fs::mkdirs(fs::dirname(out));
      fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0600);
    }
    if (fd < 0) {
      logf("[Downstream] Cannot create " + out + ": " + std::strerror(errno));
      tr.skip();
      continue;
    }
    int64_t written = 0;
    try {
      while (true) {
        ssize_t n = tr.read(buf.data(), buf.size());
        if (n <= 0) break;
        if (!write_all(fd, buf.data(), (size_t)n)) throw SyncError("[Downstream] write " + out + ": " + std::strerror(errno));
        written += n;
      }
    } catch (...) {
      ::close(fd);
      ::unlink(tmp.c_str());  // an interrupted transfer leaves no partial file behind
      throw;
    }
    ::fchmod(fd, (mode_t)(before.exists ? (before.mode & 07777) : (e.mode & 07777 ? e.mode & 07777 : 0644)));
    ::close(fd);
    fs::set_mtime(tmp, e.mtime, 0);
    std::lock_guard<std::mutex> ig(index_.mu);
    fs::StatInfo now = fs::stat(out);
    if (now.exists != before.exists ||
        (now.exists && (now.mtime_sec != before.mtime_sec || now.mtime_nsec != before.mtime_nsec ||
                        now.size != before.size || now.ino != before.ino))) {
      // edited locally while it was downloading: the local edit wins (it is uploaded next)
      ::unlink(tmp.c_str());
      logf("[Downstream] Don't override " + rel + " because it changed locally during the download");
      continue;
    }
    if (::rename(tmp.c_str(), out.c_str()) != 0) {
      ::unlink(tmp.c_str());
      logf("[Downstream] Cannot write " + out + ": " + std::strerror(errno));
      continue;
    }
    index_.create_dir(fs::dirname(rel));
    FileInfo f;
    f.name = rel;
    f.mtime = e.mtime;
    f.size = written;
    if (mode_ != Mode::Compat) f.local_mtime_ns = e.mtime * 1000000000LL;
    index_.files[rel] = f;
    if (++count % 500 == 0) logf(strfmt("[Downstream] Untared %d files...", count));
  }
  if (gzr && leftover) {
    // the rest of the member (tar's zero records), then whatever followed it on the stream
    while (gzr->read(buf.data(), buf.size()) > 0) {
    }
    *leftover = gzr->leftover();
  }
}

void Session::delete_safe_recursive(const std::string& rel, std::map<std::string, FileInfo>& removes) {
  std::string abs = o_.watch_path + rel;
  if (!index_.find(rel) || !removes.count(rel)) {
    logf("[Downstream] Skip delete directory " + rel);
    return;
  }
  for (auto& e : fs::list_dir(abs)) {
    std::string child = rel + "/" + e.name;
    FileInfo* f = index_.find(child);
    if (f) {
      FileInfo copy = *f;
      if (should_remove_local(abs + "/" + e.name, copy)) {
        if (e.is_dir && !e.is_symlink)
          delete_safe_recursive(child, removes);
        else if (!fs::remove(abs + "/" + e.name))
          logf("[Downstream] Skip file delete " + child);
      } else {
        logf("[Downstream] Skip delete " + child);
      }
    } else {
      logf("[Downstream] Skip delete " + child);
    }
    index_.files.erase(child);
  }
  if (::rmdir(abs.c_str()) != 0) logf("[Downstream] Skip delete directory " + rel + ", because it is not empty");
  index_.files.erase(rel);
}

void Session::remove_files_and_folders(std::map<std::string, FileInfo>& removes) {
  std::lock_guard<std::mutex> ig(index_.mu);
  if (removes.size() > 3) logf(strfmt("[Downstream] Remove %zu files", removes.size()));
  for (auto& kv : removes) {
    std::string abs = o_.watch_path + kv.first;
    if (should_remove_local(abs, kv.second)) {
      if (removes.size() <= 3 || o_.verbose) logf("[Downstream] Remove " + kv.first);
      if (kv.second.is_dir)
        delete_safe_recursive(kv.first, removes);
      else if (!fs::remove(abs) && fs::exists(abs))
        logf("[Downstream] Skip file delete " + kv.first);
    }
    index_.files.erase(kv.first);
  }
}

void Session::create_folders(const std::vector<FileInfo>& dirs) {
  std::lock_guard<std::mutex> ig(index_.mu);
  if (dirs.size() > 3) logf(strfmt("[Downstream] Create %zu folders", dirs.size()));
  for (auto& d : dirs) {
    if (dirs.size() <= 3 || o_.verbose) logf("[Downstream] Create folder: " + d.name);
    fs::mkdirs(o_.watch_path + d.name);
    if (!index_.find(d.name)) index_.create_dir(d.name);
  }
}

void Session::apply_downstream(const std::vector<FileInfo>& creates, std::map<std::string, FileInfo>& removes) {
  trace::Span span("sync.downstream_batch",
                   {{"changes", std::to_string(creates.size() + removes.size())}, {"dest", o_.dest_path}});
  std::vector<FileInfo> files, dirs;
  for (auto& c : creates) (c.is_dir ? dirs : files).push_back(c);
  remove_files_and_folders(removes);
  create_folders(dirs);
  if (down_helper_ && bulk_down_on_ && !files.empty()) {
    // big files come down on the bulk channel: the next pod-side changes do not wait for them
    std::vector<FileInfo> small, big;
    for (auto& f : files) (f.size >= kBulkFileBytes ? big : small).push_back(f);
    if (!big.empty()) {
      {
        std::lock_guard<std::mutex> g(inflight_mu_);
        for (auto& f : big) downloading_.insert(f.name);
      }
      {
        std::lock_guard<std::mutex> g(q_mu_);
        bulk_down_q_.push_back(std::move(big));
      }
      q_cv_.notify_all();
    }
    files.swap(small);
  }
  if (!files.empty()) {
    // batch very long lists (argv limits in fast mode); every batch streams into the tree
    size_t step = mode_ != Mode::Compat && !down_helper_ ? 500 : files.size();
    for (size_t i = 0; i < files.size(); i += step) {
      std::vector<FileInfo> part(files.begin() + i, files.begin() + std::min(files.size(), i + step));
      download_and_apply(part);
    }
  }
  logf(strfmt("[Downstream] Successfully processed %zu change(s)", creates.size() + removes.size()));
  std::lock_guard<std::mutex> g(stats_mu_);
  stats_.downstream_batches++;
  stats_.downstream_changes += creates.size() + removes.size();
}

void Session::downstream_loop() {
  size_t last_amount = 0;
  // fast mode without the helper: cheap change probes while idle, full listings only after a
  // probe saw a change and until the stability rule has applied it
  bool probing = mode_ == Mode::Fast && !down_helper_ && o_.downstream_probe;
  bool scanned = false;
  // Adaptive probe interval (fast mode): every probe walks the remote tree (`find -cnewer`), so
  // poll at poll_ms_ (250 ms) only while something moves — a probe hit, a pending change, an
  // upload — and back off by doubling to the reference's 1.3 s walk rate when idle.
  bool adaptive = probing && o_.downstream_poll_ms < 0;
  const int idle_ms = std::max(poll_ms_, 1300);
  int wait_ms = poll_ms_;
  uint64_t seen_up = 0;
  while (!stopping_ && !failed_) {
    bool skip = false;
    bool active = false;
    try {
      if (probing && scanned && last_amount == 0) skip = !probe_changes();
      active = probing && scanned && !skip;
    } catch (const std::exception& e) {
      fail(e.what());
      return;
    }
    if (!skip) try {
      auto removes = clone_index();
      std::vector<FileInfo> creates = collect_changes(&removes);
      scanned = true;
      size_t amount = creates.size() + removes.size();
      bool apply;
      if (down_helper_)
        apply = amount > 0;  // event-driven: the helper only signals after writes settle
      else
        apply = last_amount > 0 && amount == last_amount;  // stability rule (downstream.go:117)
      if (apply) apply_downstream(creates, removes);
      last_amount = amount;
      active = active || amount > 0;
    } catch (const std::exception& e) {
      fail(e.what());
      return;
    }
    if (adaptive) {
      {
        std::lock_guard<std::mutex> g(stats_mu_);
        if (stats_.upstream_batches != seen_up) active = true;
        seen_up = stats_.upstream_batches;
        wait_ms = active ? poll_ms_ : std::min(idle_ms, wait_ms * 2);
        stats_.probe_interval_ms = wait_ms;
      }
    } else {
      wait_ms = poll_ms_;
    }
    if (down_helper_) {
      // a file downloaded while its stamp was fresh is checked once it is still (collect_changes):
      // look again shortly after instead of at the next event
      std::lock_guard<std::mutex> ig(index_.mu);
      for (auto& kv : index_.files)
        if (kv.second.remote_unsettled) {
          wait_ms = std::min(wait_ms, (int)(kUnsettledNs / 1000000) + 100);
          break;
        }
    }
    // wait for the next poll (or a container-side event in helper mode)
    long until = mono_us() + (long)wait_ms * 1000;
    while (!stopping_ && !failed_ && mono_us() < until) {
      if (down_helper_) {
        LineReader& events = up_helper_ ? up_err_ : down_err_;
        std::string ev;
        if (events.read_line(&ev, 50)) {
          if (ev == "E") {
            // coalesce bursts of events
            while (events.read_line(&ev, 15)) {
            }
            break;
          }
        } else if (events.eof()) {
          fail("downstream: helper event stream closed");
          return;
        }
      } else {
        sleep_ms(std::min<int>(50, wait_ms));
      }
    }
  }
}

// ============================================================ lifecycle

std::thread Session::spawn_loop(LoopBit bit, std::function<void()> body) {
  live_loops_ |= bit;
  return std::thread([this, bit, body = std::move(body)] {
    struct Done {
      Session* s;
      LoopBit b;
      ~Done() { s->live_loops_ &= ~(unsigned)b; }
    } done{this, bit};
    body();
  });
}

std::string Session::describe_stop_state() {
  static const std::pair<unsigned, const char*> names[] = {{kUpLoop, "upstream"},
                                                           {kBulkLoop, "bulk upload"},
                                                           {kBulkDownLoop, "bulk download"},
                                                           {kDownLoop, "downstream"},
                                                           {kSupervisor, "supervisor"}};
  unsigned live = live_loops_.load();
  std::string loops;
  for (auto& n : names)
    if (live & n.first) loops += std::string(loops.empty() ? "" : ", ") + n.second;
  return strfmt("at '%s'; loops still running: %s", stop_step_.load(), loops.empty() ? "none" : loops.c_str());
}

void Session::start_loops(bool upstream, bool downstream) {
  if (upstream) up_thread_ = spawn_loop(kUpLoop, [this] { upstream_loop(); });
  if (upstream) bulk_thread_ = spawn_loop(kBulkLoop, [this] { bulk_loop(); });
  if (downstream) {
    bulk_down_on_ = true;
    bulk_down_thread_ = spawn_loop(kBulkDownLoop, [this] { bulk_down_loop(); });
  }
  if (downstream) down_thread_ = spawn_loop(kDownLoop, [this] { downstream_loop(); });
}

void Session::fail(const std::string& err) {
  if (stopping_) return;
  {
    std::lock_guard<std::mutex> g(state_mu_);
    if (failed_) return;
    failed_ = true;
    pending_failure_ = err;
  }
  state_cv_.notify_all();
  q_cv_.notify_all();
}

void Session::stop_loops() {
  q_cv_.notify_all();
  stop_step_ = "stop_loops: terminating shells";
  if (up_shell_) up_shell_->terminate();
  if (down_shell_) down_shell_->terminate();
  {
    // (bulk_down_mu_ may be held by a download for minutes: the pointer has a lock of its own)
    std::lock_guard<std::mutex> g(bulk_down_ptr_mu_);
    if (bulk_down_shell_) bulk_down_shell_->terminate();
  }
  {
    std::lock_guard<std::mutex> g(up_pmu_);
    up_pcv_.notify_all();
  }
  up_rcv_.notify_all();
  stop_step_ = "stop_loops: joining the upload loops";
  if (up_thread_.joinable() && up_thread_.get_id() != std::this_thread::get_id()) up_thread_.join();
  if (bulk_thread_.joinable() && bulk_thread_.get_id() != std::this_thread::get_id()) bulk_thread_.join();
  stop_step_ = "stop_loops: joining the bulk download loop";
  if (bulk_down_thread_.joinable() && bulk_down_thread_.get_id() != std::this_thread::get_id())
    bulk_down_thread_.join();
  bulk_down_on_ = false;
  {
    stop_step_ = "stop_loops: closing the bulk download shell";
    std::lock_guard<std::mutex> g(bulk_down_ptr_mu_);
    if (bulk_down_shell_) {
      bulk_down_shell_->close();
      bulk_down_shell_.reset();
    }
  }
  stop_step_ = "stop_loops: joining the downstream loop";
  if (down_thread_.joinable() && down_thread_.get_id() != std::this_thread::get_id()) down_thread_.join();
  stop_step_ = "stop_loops: closing shells";
  {
    // a reconnect starts over from an initial sync: nothing is in flight or queued for the bulk lane
    std::lock_guard<std::mutex> g(q_mu_);
    bulk_q_.clear();
    deferred_.clear();
    bulk_busy_ = false;
    bulk_down_q_.clear();
    bulk_down_busy_ = false;
  }
  {
    std::lock_guard<std::mutex> g(inflight_mu_);
    inflight_.clear();
    inflight_bulk_.clear();
    downloading_.clear();
  }
  if (up_shell_) up_shell_->close();
  if (down_shell_) down_shell_->close();
}

void Session::supervise() {
  // initial sync + downstream run on their own thread; the supervisor handles failures.
  auto run_initial = [this]() -> bool {
    try {
      initial_sync();
      logf("[Sync] Initial sync completed");
      {
        std::lock_guard<std::mutex> g(state_mu_);
        initial_done_ = true;
      }
      state_cv_.notify_all();
      if (o_.on_initial_sync_done) o_.on_initial_sync_done();
      return true;
    } catch (const std::exception& e) {
      fail(e.what());
      return false;
    }
  };
  logf("[Sync] Start syncing");
  up_thread_ = spawn_loop(kUpLoop, [this] { upstream_loop(); });
  bulk_thread_ = spawn_loop(kBulkLoop, [this] { bulk_loop(); });
  bulk_down_on_ = true;
  bulk_down_thread_ = spawn_loop(kBulkDownLoop, [this] { bulk_down_loop(); });
  down_thread_ = spawn_loop(kDownLoop, [this, run_initial] {
    if (run_initial()) downstream_loop();
  });
  while (true) {
    std::string err;
    {
      std::unique_lock<std::mutex> lk(state_mu_);
      state_cv_.wait(lk, [this] { return stopping_ || failed_; });
      if (stopping_) return;
      err = pending_failure_;
    }
    log_error("Error: " + err);
    bool can_reconnect = mode_ != Mode::Compat && o_.reconnect && reconnects_ < o_.max_reconnects;
    if (!can_reconnect) {
      {
        std::lock_guard<std::mutex> g(state_mu_);
        error_ = err;
      }
      running_ = false;
      if (o_.on_error) o_.on_error(err);
      state_cv_.notify_all();
      return;
    }
    ++reconnects_;
    {
      std::lock_guard<std::mutex> g(stats_mu_);
      stats_.reconnects++;
    }
    logf(strfmt("[Sync] Stream failed (%s), reconnecting (attempt %d)", err.c_str(), reconnects_));
    stop_loops();
    sleep_ms(std::min(200 * reconnects_, 2000));
    try {
      auto t = o_.reconnect();
      if (!t) throw SyncError("no pod available");
      transport_ = t;
      dest_ = remote(o_.dest_path);
      if (!t->pod_name().empty()) {
        std::lock_guard<std::mutex> g(pod_mu_);
        o_.pod_name = t->pod_name();  // `status sync` shows the pod the sync now talks to
      }
      open_shells();
      logf("[Sync] Reconnected to " + t->describe());
    } catch (const std::exception& e) {
      std::lock_guard<std::mutex> g(state_mu_);
      pending_failure_ = e.what();
      failed_ = true;
      continue;
    }
    {
      std::lock_guard<std::mutex> g(state_mu_);
      failed_ = false;
      pending_failure_.clear();
    }
    up_thread_ = spawn_loop(kUpLoop, [this] { upstream_loop(); });
    bulk_thread_ = spawn_loop(kBulkLoop, [this] { bulk_loop(); });
    bulk_down_on_ = true;
    bulk_down_thread_ = spawn_loop(kBulkDownLoop, [this] { bulk_down_loop(); });
    down_thread_ = spawn_loop(kDownLoop, [this, run_initial] {
      if (run_initial()) downstream_loop();
    });
  }
}

void Session::start() {
  setup();
  open_shells();
  start_watcher();
  running_ = true;
  supervisor_ = spawn_loop(kSupervisor, [this] { supervise(); });
}

bool Session::wait_initial_sync(int timeout_ms) {
  std::unique_lock<std::mutex> lk(state_mu_);
  auto ready = [this] { return initial_done_ || !error_.empty() || stopping_; };
  if (timeout_ms < 0)
    state_cv_.wait(lk, ready);
  else if (!state_cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), ready))
    return false;
  return initial_done_;
}

std::string Session::error() {
  std::lock_guard<std::mutex> g(state_mu_);
  return error_;
}

Stats Session::stats() {
  std::lock_guard<std::mutex> g(stats_mu_);
  return stats_;
}

void Session::stop(const std::string& fatal_error) {
  if (stopping_.exchange(true)) return;
  {
    std::lock_guard<std::mutex> g(state_mu_);
    if (!fatal_error.empty()) error_ = fatal_error;
  }
  state_cv_.notify_all();
  q_cv_.notify_all();
  // watchdog: a stop is normally done within a few hundred ms (every loop checks stopping_ at
  // least every 200 ms and every shell is killed before the joins)
  std::mutex wd_mu;
  std::condition_variable wd_cv;
  bool stopped = false;
  int warn_ms = 20000;
  if (const char* v = std::getenv("DEVSPACE_SYNC_STOP_WARN_MS")) warn_ms = std::max(10, std::atoi(v));
  std::thread watchdog([&] {
    long t0 = mono_us();
    std::unique_lock<std::mutex> lk(wd_mu);
    while (!wd_cv.wait_for(lk, std::chrono::milliseconds(warn_ms), [&] { return stopped; })) {
      std::string msg = strfmt("[Sync] Stop still waiting after %.1fs %s", (mono_us() - t0) / 1e6,
                               describe_stop_state().c_str());
      logf(msg);
      std::fprintf(stderr, "%s\n", msg.c_str());
    }
  });
  stop_step_ = "stopping the symlink watchers";
  {
    std::lock_guard<std::mutex> g(symlink_mu_);
    for (auto& kv : symlinks_) kv.second->stop();
    symlinks_.clear();
  }
  stop_step_ = "stopping the file watcher";
  if (watcher_) watcher_->stop();
  stop_step_ = "joining the supervisor";
  if (supervisor_.joinable()) supervisor_.join();
  stop_loops();
  stop_step_ = "stopped";
  {
    std::lock_guard<std::mutex> g(wd_mu);
    stopped = true;
  }
  wd_cv.notify_all();
  watchdog.join();
  running_ = false;
  logf("[Sync] Sync stopped");
  if (!fatal_error.empty()) log_error("Error: " + fatal_error);
}

// ============================================================ one-shot copy

void Session::copy_to_container(std::shared_ptr<Transport> t, const std::string& local_path,
                                const std::string& container_path, std::vector<std::string> excludes, Mode mode) {
  fs::StatInfo st = fs::lstat(local_path);
  if (!st.exists) throw SyncError("lstat " + local_path + ": no such file or directory");
  std::string root = local_path;
  if (!st.is_dir) {
    root = fs::dirname(local_path);
    for (auto& e : fs::list_dir(root))
      if (fs::join(root, e.name) != local_path) excludes.push_back("/" + e.name);
  }
  Options o;
  o.watch_path = root;
  o.dest_path = container_path;
  o.exclude_paths = excludes;
  o.silent = true;
  o.mode = mode == Mode::Helper ? Mode::Fast : mode;
  Session s(o, t);
  s.setup();
  s.open_up_shell();
  FileInfo rootinfo;
  rootinfo.name = "";
  rootinfo.is_dir = true;
  rootinfo.mtime = 1;
  s.apply_creates({rootinfo});
  s.stopping_ = true;
  if (s.up_shell_) s.up_shell_->close();
}

}  // namespace sync
}  // namespace ds

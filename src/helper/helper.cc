// devspace-helper — static in-container sync agent (SURVEY.md §7.6 "optional static helper").
//
// Replaces the reference's per-operation shell scripts (sync/upstream.go:387, downstream.go:373)
// and the 1.3 s full `find` poll with a persistent process speaking a framed protocol on
// stdin/stdout and pushing inotify change notifications on stderr (framing: src/sync/frame.h):
//
//   request := op:u8 len:u64be payload[len]
//   'U' (len 0) + chunk stream of a tar (or tar.gz) -> extract under <dest>   reply "OK\n" | "ERR msg\n"
//   'U' payload=lane:u8         -> an upload on lane `lane` (the lane is created on first use): its
//                                  chunk stream arrives in 'C' frames and is extracted on the lane's
//                                  thread                                  reply "@lane OK\n" | "@lane ERR msg\n"
//   'C' payload=lane:u8 bytes   -> the next bytes of lane `lane`'s chunk stream (no reply)
//   'X' payload=lane:u8 rel\n.. -> rm -rf <dest><rel>                          reply "@lane OK\n"
//   'R' payload=rel\n...        -> rm -rf <dest><rel>                          reply "OK\n"
//   'S' (empty)                 -> "<abs>///size,mtime,hexmode,perm,uid,gid\n"... then "DONE\n"
//   'D' payload=rel\n...        -> "STREAM\n" + chunk stream of a tar (relative member names)
//                                  + "OK\n"
//   'H' payload=rel\n...        -> one crc32 hex (or "-") per path, then "DONE\n"
//   'W' (empty)                 -> start watching; "E\n" on stderr after foreign changes settle
//   'Q'                          -> exit
//
// `devspace-helper forward` serves port-forwarded connections instead (src/helper/forward.cc).
//
// Lanes: the upstream session interleaves several uploads frame by frame on one stdin — a bulk
// transfer (a multi-GB checkpoint) in one lane, a code edit in another — so an edit never waits
// behind a bulk archive for more than one frame. Each lane extracts on its own thread, fed through
// a pipe by the frame reader; extraction writes through temp names and renames as before.
//
// Archives are streamed through fixed-size buffers in both directions, so memory stays bounded
// for files of any size (a multi-GB checkpoint written in a training pod is read and sent in
// 1 MiB pieces; the helper shares the pod's memory cgroup). Extraction writes each file to a
// temp name and renames it into place, so an interrupted transfer never leaves a truncated
// file at the real path. Built with -static so it runs in any x86_64 container image.
#include <fcntl.h>
#include <poll.h>
#include <signal.h>
#include <sys/inotify.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>
#include <zlib.h>

#include <atomic>
#include <climits>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "core/codec.h"
#include "core/fs.h"
#include "core/proc.h"
#include "core/strutil.h"
#include "helper/forward.h"
#include "sync/frame.h"

using namespace ds;
namespace frame = ds::sync::frame;

static std::string g_dest;
static const char* kTmpSuffix = ".devspace-tmp";

static long now_us() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1000000L + ts.tv_nsec / 1000;
}

// What this helper itself wrote or removed (upstream ops), so the inotify echo of its own
// writes does not trigger a downstream scan. An event counts as our own only while the path
// still holds exactly what we left there (same kind, size and mtime for files; absent for
// removals): a pod process that rewrites a file it just received — a formatter, a code
// generator — changes size or mtime and is reported at once. Records live while an op runs
// and for kOwnEchoUs after the last one finished (the echo of a write arrives within
// milliseconds). The session runs its watch ('W') in this same process, the upstream one, so
// the records of its own writes are where the watcher looks.
struct OwnRecord {
  enum Kind { File, Dir, Link, Gone } kind = File;
  int64_t size = 0;
  int64_t mtime = 0;  // seconds; written files carry nsec 0 (tar resolution)
};
static std::mutex g_own_mu;
static std::map<std::string, OwnRecord> g_own;
static std::set<std::string> g_gone_trees;  // removed subtrees: anything absent below is ours
static int g_own_active = 0;  // upstream ops running (lanes run concurrently)
static long g_own_until = 0;  // monotonic us: records expire after this once no op runs
static const long kOwnEchoUs = 2000000;

static void own_begin() {
  std::lock_guard<std::mutex> g(g_own_mu);
  ++g_own_active;
}

static void own_end() {
  std::lock_guard<std::mutex> g(g_own_mu);
  --g_own_active;
  g_own_until = now_us() + kOwnEchoUs;
}

struct OwnOp {  // own_begin/own_end around one upstream op, exceptions included
  OwnOp() { own_begin(); }
  ~OwnOp() { own_end(); }
};

static void own_record(const std::string& p, OwnRecord r) {
  std::lock_guard<std::mutex> g(g_own_mu);
  if (!starts_with(p, g_dest)) return;
  g_own[p] = r;
  // ancestors get IN_ATTRIB / IN_CREATE echoes while we write below them
  for (std::string q = fs::dirname(p); q.size() >= g_dest.size() && starts_with(q, g_dest); q = fs::dirname(q)) {
    auto it = g_own.find(q);
    if (it != g_own.end() && it->second.kind == OwnRecord::Dir) break;
    OwnRecord d;
    d.kind = OwnRecord::Dir;
    g_own[q] = d;
    if (q.size() == g_dest.size()) break;
  }
}

static void own_gone_tree(const std::string& p) {
  OwnRecord r;
  r.kind = OwnRecord::Gone;
  own_record(p, r);
  std::lock_guard<std::mutex> g(g_own_mu);
  g_gone_trees.insert(p);
}

static bool matches(const OwnRecord& r, const std::string& p) {
  struct stat st;
  bool exists = ::lstat(p.c_str(), &st) == 0;
  switch (r.kind) {
    case OwnRecord::Gone: return !exists;
    case OwnRecord::Dir: return exists && S_ISDIR(st.st_mode);
    case OwnRecord::Link: return exists && S_ISLNK(st.st_mode);
    case OwnRecord::File:
      return exists && S_ISREG(st.st_mode) && st.st_size == r.size && st.st_mtim.tv_sec == r.mtime &&
             st.st_mtim.tv_nsec == 0;
  }
  return false;
}

static bool is_own(const std::string& p) {
  std::lock_guard<std::mutex> g(g_own_mu);
  if (g_own_active == 0 && now_us() > g_own_until) {
    g_own.clear();
    g_gone_trees.clear();
    return false;
  }
  auto it = g_own.find(p);
  if (it != g_own.end()) return matches(it->second, p);
  for (std::string q = p; q.size() > g_dest.size(); q = fs::dirname(q))
    if (g_gone_trees.count(q)) {
      struct stat st;
      return ::lstat(p.c_str(), &st) != 0;
    }
  return false;
}

static std::mutex g_reply_mu;  // lane threads reply concurrently with the main loop
static bool reply(const std::string& s) {
  std::lock_guard<std::mutex> g(g_reply_mu);
  return write_all(1, s);
}

static std::string safe_join(const std::string& rel_in) {
  std::string rel = rel_in;
  while (starts_with(rel, "./")) rel = rel.substr(2);
  std::string c = fs::clean("/" + rel);  // strips any ".." escaping the root
  return c == "/" ? g_dest : g_dest + c;
}

// Extracts a (gzip-or-plain) tar stream under g_dest with `tar xpf` semantics.
static std::string op_extract(Source src) {
  // sniff gzip vs plain tar (small edits are shipped uncompressed)
  std::string magic;
  char m[2];
  while (magic.size() < 2) {
    ssize_t n = src(m, 2 - magic.size());
    if (n <= 0) break;
    magic.append(m, (size_t)n);
  }
  if (magic.empty()) return "OK";
  bool gzipped = magic.size() == 2 && (unsigned char)magic[0] == 0x1f && (unsigned char)magic[1] == 0x8b;
  Source raw = prefixed_source(magic, src);
  GzipReader gz(raw);
  TarReader tr([&](char* b, size_t n) { return gzipped ? gz.read(b, n) : raw(b, n); });
  TarEntry e;
  bool root = ::geteuid() == 0;
  std::string tmp;
  std::vector<char> buf(1 << 20);
  try {
    while (tr.next(&e)) {
      std::string out = safe_join(e.name);
      if (e.type == '5') {
        fs::mkdirs(out, 0755);
        ::chmod(out.c_str(), e.mode & 07777);
        if (root) {
          int ignored = ::lchown(out.c_str(), e.uid, e.gid);
          (void)ignored;
        }
        fs::set_mtime(out, e.mtime);
        OwnRecord r;
        r.kind = OwnRecord::Dir;
        own_record(out, r);
        continue;
      }
      if (e.type == '2') {
        fs::mkdirs(fs::dirname(out));
        ::unlink(out.c_str());
        int ignored = ::symlink(e.linkname.c_str(), out.c_str());
        (void)ignored;
        OwnRecord r;
        r.kind = OwnRecord::Link;
        own_record(out, r);
        continue;
      }
      if (e.type != '0' && e.type != '7') {
        tr.skip();
        continue;
      }
      fs::mkdirs(fs::dirname(out));
      tmp = out + kTmpSuffix;
      int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0600);
      if (fd < 0) {
        std::string err = std::string("ERR open ") + out + ": " + std::strerror(errno);
        tmp.clear();
        return err;
      }
      while (true) {
        ssize_t n = tr.read(buf.data(), buf.size());
        if (n <= 0) break;
        if (!write_all(fd, buf.data(), (size_t)n)) {
          std::string err = std::string("ERR write ") + out + ": " + std::strerror(errno);
          ::close(fd);
          ::unlink(tmp.c_str());
          return err;
        }
      }
      ::fchmod(fd, e.mode & 07777);
      if (root) {
        int ignored = ::fchown(fd, e.uid, e.gid);
        (void)ignored;
      }
      ::close(fd);
      fs::set_mtime(tmp, e.mtime);
      OwnRecord r;
      r.size = e.size;
      r.mtime = e.mtime;
      own_record(out, r);  // before the rename: its IN_MOVED_TO echo must find the record
      if (::rename(tmp.c_str(), out.c_str()) != 0) {
        // target may be a directory being replaced by a file
        fs::remove_all(out);
        if (::rename(tmp.c_str(), out.c_str()) != 0) {
          ::unlink(tmp.c_str());
          return "ERR rename " + out;
        }
      }
      tmp.clear();
    }
  } catch (const std::exception& ex) {
    if (!tmp.empty()) ::unlink(tmp.c_str());  // never leave a partial file behind
    return std::string("ERR ") + ex.what();
  }
  return "OK";
}

// Buffered stdout writer for listings of any size.
struct OutBuf {
  std::string b;
  bool ok = true;
  void put(const std::string& s) {
    b += s;
    if (b.size() >= (256u << 10)) flush();
  }
  void flush() {
    if (ok && !b.empty()) ok = write_all(1, b);
    b.clear();
  }
};

static void scan_rec(const std::string& p, OutBuf& out, std::set<std::pair<uint64_t, uint64_t>>& seen, int depth) {
  struct stat lst;
  if (::lstat(p.c_str(), &lst) != 0) return;
  if (ends_with(p, kTmpSuffix)) {
    // a transfer in progress (its ctime moves with every write) or one cut off when a helper
    // was killed mid-upload: the latter is removed once it has been still for two minutes
    struct timespec now;
    clock_gettime(CLOCK_REALTIME, &now);
    if (S_ISREG(lst.st_mode) && now.tv_sec - lst.st_ctim.tv_sec > 120) ::unlink(p.c_str());
    return;
  }
  struct stat st = lst;
  if (S_ISLNK(lst.st_mode)) {
    if (::stat(p.c_str(), &st) != 0) st = lst;
  }
  // like `find -L ... -exec stat -c` : stat of the path itself (links reported as links), plus
  // the mtime's nanoseconds (a same-size rewrite within the second moves only those)
  out.put(p + "///" + std::to_string((long long)lst.st_size) + "," + std::to_string((long long)lst.st_mtim.tv_sec) +
          "," + strfmt("%x", (unsigned)lst.st_mode) + "," + strfmt("%o", (unsigned)(lst.st_mode & 07777)) + "," +
          std::to_string(lst.st_uid) + "," + std::to_string(lst.st_gid) + "," +
          std::to_string((long)lst.st_mtim.tv_nsec) + "\n");
  if (S_ISDIR(st.st_mode) && depth < 128) {
    auto key = std::make_pair((uint64_t)st.st_dev, (uint64_t)st.st_ino);
    if (seen.count(key)) return;
    seen.insert(key);
    for (auto& e : fs::list_dir(p)) scan_rec(p + "/" + e.name, out, seen, depth + 1);
  }
}

static void op_scan() {
  fs::mkdirs(g_dest);
  OutBuf out;
  struct timespec now;  // the clock file stamps come from: how fresh each one is
  clock_gettime(CLOCK_REALTIME, &now);
  out.put("#NOW " + std::to_string((long long)now.tv_sec * 1000000000LL + now.tv_nsec) + "\n");
  std::set<std::pair<uint64_t, uint64_t>> seen;
  scan_rec(g_dest, out, seen, 0);
  out.put("DONE\n");
  out.flush();
}

static void op_remove(const std::string& payload) {
  for (auto& rel : split(payload, "\n")) {
    if (rel.empty()) continue;
    std::string p = safe_join(rel);
    if (p == g_dest) continue;
    own_gone_tree(p);
    fs::remove_all(p);
  }
}

// 'D': streams the requested files as one tar.gz, chunk-framed, while reading them.
static void op_download(const std::string& payload) {
  if (!reply("STREAM\n")) return;
  // checkpoints and other binaries written in the pod are incompressible: those chunks go out
  // as they are, text chunks raw-deflated (frame::ChunkWriter), no gzip CRC pass
  frame::ChunkWriter cw(fd_sink(1), frame::kMaxChunk, 1);
  TarWriter tw(cw.sink());
  bool ok = true;
  for (auto& rel : split(payload, "\n")) {
    if (rel.empty() || !ok) continue;
    std::string p = safe_join(rel);
    fs::StatInfo st = fs::stat(p);
    if (!st.exists || st.is_dir) continue;
    TarEntry e;
    e.name = rel[0] == '/' ? rel.substr(1) : rel;
    e.mode = st.mode & 07777;
    e.uid = st.uid;
    e.gid = st.gid;
    e.size = st.size;
    e.mtime = st.mtime_sec;
    if (!tw.add_file_from_path(e, p)) {
      // unreadable or vanished before open: skip it (the header may already be out, padded
      // with zeros by add_file_from_path when the file shrank)
      continue;
    }
  }
  ok = tw.finish() && cw.finish();
  if (ok) reply("OK\n");
}

// 'H': CRC-32 of files (initial sync: tells identical copies from changed files when mtimes
// differ only by the sub-second part a seconds-resolution tar dropped). "-" = unreadable.
static std::string op_hash(const std::string& payload) {
  std::string out;
  std::vector<char> buf(1 << 20);
  for (auto& rel : split(payload, "\n")) {
    if (rel.empty()) continue;
    int fd = ::open(safe_join(rel).c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) {
      out += "-\n";
      continue;
    }
    uLong crc = crc32(0L, Z_NULL, 0);
    ssize_t n;
    while ((n = ::read(fd, buf.data(), buf.size())) > 0) crc = crc32(crc, (const Bytef*)buf.data(), (uInt)n);
    ::close(fd);
    out += n < 0 ? "-\n" : strfmt("%08lx\n", (unsigned long)crc);
  }
  return out + "DONE\n";
}

static void add_watch_rec(int fd, const std::string& dir, std::map<int, std::string>& wds, int depth) {
  int wd = inotify_add_watch(fd, dir.c_str(),
                             IN_CREATE | IN_DELETE | IN_CLOSE_WRITE | IN_MOVED_FROM | IN_MOVED_TO | IN_ATTRIB);
  if (wd < 0) return;
  wds[wd] = dir;
  if (depth > 64) return;
  for (auto& e : fs::list_dir(dir))
    if (e.is_dir && !e.is_symlink) add_watch_rec(fd, dir + "/" + e.name, wds, depth + 1);
}

static void watch_loop() {
  int fd = inotify_init1(IN_CLOEXEC);
  if (fd < 0) return;
  std::map<int, std::string> wds;
  fs::mkdirs(g_dest);
  add_watch_rec(fd, g_dest, wds, 0);
  alignas(struct inotify_event) char buf[1 << 16];
  while (true) {
    ssize_t n = ::read(fd, buf, sizeof(buf));
    if (n <= 0) {
      if (errno == EINTR) continue;
      break;
    }
    // true if the batch holds a change the pod made (not the echo of our own writes)
    auto process = [&](ssize_t len) {
      bool foreign = false;
      for (char* p = buf; p < buf + len;) {
        auto* ev = (struct inotify_event*)p;
        p += sizeof(struct inotify_event) + ev->len;
        if (ev->mask & IN_Q_OVERFLOW) {  // events were lost: rescan
          foreign = true;
          continue;
        }
        std::string name = ev->len ? std::string(ev->name) : "";
        auto it = wds.find(ev->wd);
        if (ev->mask & IN_IGNORED) {
          wds.erase(ev->wd);
          continue;
        }
        if (it == wds.end()) continue;
        std::string path = name.empty() ? it->second : it->second + "/" + name;
        if ((ev->mask & IN_ISDIR) && (ev->mask & (IN_CREATE | IN_MOVED_TO))) add_watch_rec(fd, path, wds, 0);
        if (ends_with(name, kTmpSuffix) || is_own(path)) continue;
        foreign = true;
      }
      return foreign;
    };
    bool changed = process(n);
    // settle: wait until no events for 20 ms, then notify once
    while (true) {
      struct pollfd pf{fd, POLLIN, 0};
      if (::poll(&pf, 1, 20) <= 0) break;
      ssize_t m = ::read(fd, buf, sizeof(buf));
      if (m <= 0) break;
      changed |= process(m);
    }
    if (!changed) continue;
    write_all(2, "E\n");
  }
}

// An upload lane: the frame reader writes the lane's chunk-stream bytes into `w`; the lane's
// thread extracts one chunk stream after the other from the other end and replies
// "@lane OK|ERR ..." after each. Lanes persist: an upload on a lane that exists costs no thread
// or pipe set-up (the session keeps one lane for edits and one for bulk transfers).
struct Lane {
  int w = -1;
  std::thread t;
};

static std::string lane_tag(int lane) { return "@" + std::to_string(lane) + " "; }

static void lane_loop(int r, int lane) {
  while (true) {
    struct pollfd pf{r, POLLIN, 0};
    if (::poll(&pf, 1, -1) < 0) {
      if (errno == EINTR) continue;
      break;
    }
    std::string res;
    {
      OwnOp own;  // from the first byte of a stream: its echo is ours while it runs and shortly after
      frame::ChunkReader cr(fd_source(r));
      try {
        res = op_extract(cr.source());
        cr.drain();  // an early error still consumes the whole stream: the lane stays in step
      } catch (const std::exception&) {
        std::_Exit(1);  // the stream itself is broken (sender gone): the session reconnects
      }
    }
    reply(lane_tag(lane) + res + "\n");
  }
}

static void open_lane(std::map<int, Lane>& lanes, int lane) {
  Lane& l = lanes[lane];
  if (l.w >= 0) return;  // persistent: the next stream follows the previous one in its pipe
  int fds[2];
  if (::pipe2(fds, O_CLOEXEC) != 0) {
    reply(lane_tag(lane) + "ERR pipe: " + std::strerror(errno) + "\n");
    std::_Exit(1);
  }
#ifdef F_SETPIPE_SZ
  ::fcntl(fds[1], F_SETPIPE_SZ, 1 << 20);  // one frame in flight per lane without blocking the reader
#endif
  l.w = fds[1];
  l.t = std::thread(lane_loop, fds[0], lane);
  l.t.detach();  // ends with the process (std::_Exit)
}

int main(int argc, char** argv) {
  if (argc >= 2 && std::string(argv[1]) == "forward") return ds::helper::forward_main();
  if (argc < 3 || std::string(argv[1]) != "serve") {
    std::fprintf(stderr, "usage: devspace-helper serve <dest> | devspace-helper forward\n");
    std::_Exit(2);
  }
  signal(SIGPIPE, SIG_IGN);
  g_dest = fs::clean(argv[2]);
  fs::mkdirs(g_dest);
  reply("HELPER READY\n");
  bool watching = false;
  Source in = fd_source(0);
  std::map<int, Lane> lanes;
  std::vector<char> cbuf;
  while (true) {
    unsigned char hdr[frame::kHeaderSize];
    if (!read_exact(0, hdr, sizeof(hdr))) break;
    char op;
    uint64_t len;
    frame::parse_header(hdr, &op, &len);
    if (op == 'C') {  // lane data: straight from stdin into the lane's pipe
      if (len < 1 || len > frame::kMaxChunk + 64) {
        std::fprintf(stderr, "devspace-helper: bad lane frame of %llu bytes\n", (unsigned long long)len);
        std::_Exit(1);
      }
      cbuf.resize((size_t)len);
      if (!read_exact(0, cbuf.data(), (size_t)len)) break;
      auto it = lanes.find((unsigned char)cbuf[0]);
      if (it == lanes.end() || it->second.w < 0 || !write_all(it->second.w, cbuf.data() + 1, (size_t)len - 1)) {
        std::fprintf(stderr, "devspace-helper: data for a lane that is not open\n");
        std::_Exit(1);
      }
      continue;
    }
    if (op == 'U' && len == 1) {
      unsigned char lane;
      if (!read_exact(0, &lane, 1)) break;
      open_lane(lanes, lane);
      continue;
    }
    if (op == 'U') {
      std::string r;
      {
        OwnOp own;  // the echo of our own extraction is ignored while it runs and shortly after
        frame::ChunkReader cr(in);
        try {
          r = op_extract(cr.source());
          cr.drain();  // an early error still consumes the whole stream: framing stays in step
        } catch (const std::exception& ex) {
          std::_Exit(1);  // the stream itself is broken (sender gone): nothing left to reply to
        }
      }
      reply(r + "\n");
      continue;
    }
    if (len > frame::kMaxListPayload) {
      std::fprintf(stderr, "devspace-helper: request payload of %llu bytes refused\n", (unsigned long long)len);
      std::_Exit(1);
    }
    std::string payload((size_t)len, '\0');
    if (len && !read_exact(0, &payload[0], (size_t)len)) break;
    switch (op) {
      case 'R': {
        {
          OwnOp own;
          try {
            op_remove(payload);
          } catch (const std::exception&) {
            // like the shell protocols' `rm -R ... || true`: a path that cannot be removed does
            // not stop the sync
          }
        }
        reply("OK\n");
        break;
      }
      case 'X': {  // tagged remove (lanes): payload = lane byte + rel list
        if (payload.empty()) std::_Exit(1);
        int lane = (unsigned char)payload[0];
        {
          OwnOp own;
          try {
            op_remove(payload.substr(1));
          } catch (const std::exception&) {
          }
        }
        reply(lane_tag(lane) + "OK\n");
        break;
      }
      case 'S': op_scan(); break;
      case 'H': reply(op_hash(payload)); break;
      case 'D': op_download(payload); break;
      case 'W':
        // one watch loop per helper process (a detached thread is never joinable again, so
        // joinable() cannot be the guard); it ends with the process
        if (!watching) {
          watching = true;
          std::thread(watch_loop).detach();
        }
        break;
      case 'Q':
        std::_Exit(0);  // lane threads may still be parked on their pipes
      default: reply("ERR unknown op\n");
    }
  }
  std::_Exit(0);
}

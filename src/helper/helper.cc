// devspace-helper — static in-container sync agent (SURVEY.md §7.6 "optional static helper").
//
// Replaces the reference's per-operation shell scripts (sync/upstream.go:387, downstream.go:373)
// and the 1.3 s full `find` poll with a persistent process speaking a framed protocol on
// stdin/stdout and pushing inotify change notifications on stderr:
//
//   request  := op:u8  len:u32be  payload[len]
//   'U' payload=tar.gz          -> extract under <dest> (tar xzpf semantics)   reply "OK\n" | "ERR msg\n"
//   'R' payload=rel\n...        -> rm -rf <dest><rel>                          reply "OK\n"
//   'S' (empty)                 -> "<abs>///size,mtime,hexmode,perm,uid,gid\n"... then "DONE\n"
//   'D' payload=rel\n...        -> "SIZE n\n" + n bytes tar.gz (relative member names)
//   'H' payload=rel\n...        -> one crc32 hex (or "-") per path, then "DONE\n"
//   'W' (empty)                 -> start watching; "E\n" on stderr after changes settle
//   'Q'                          -> exit
//
// Built with -static so it runs in any x86_64 container image (no libc/zlib dependency).
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

using namespace ds;

static std::string g_dest;

static long now_us() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1000000L + ts.tv_nsec / 1000;
}

// Paths this helper itself wrote or removed (upstream ops), so their inotify echo does not
// trigger a downstream scan, while changes the pod makes to any other path — even during an
// upload — still do. Entries live while an op runs and for kOwnEchoUs after it finished.
static std::mutex g_own_mu;
static std::set<std::string> g_own, g_own_trees;
static long g_own_until = 0;  // monotonic us; LONG_MAX while an op runs
static const long kOwnEchoUs = 2000000;

static void own_begin() {
  std::lock_guard<std::mutex> g(g_own_mu);
  g_own_until = LONG_MAX;
}

static void own_end() {
  std::lock_guard<std::mutex> g(g_own_mu);
  g_own_until = now_us() + kOwnEchoUs;
}

struct OwnOp {  // own_begin/own_end around one upstream op, exceptions included
  OwnOp() { own_begin(); }
  ~OwnOp() { own_end(); }
};

static void own_path(const std::string& p) {
  std::lock_guard<std::mutex> g(g_own_mu);
  if (!starts_with(p, g_dest)) return;
  for (std::string q = p;; q = fs::dirname(q)) {
    if (!g_own.insert(q).second) break;  // ancestors already recorded
    if (q.size() <= g_dest.size()) break;  // dest itself (its own IN_ATTRIB echo) included
  }
}

static void own_subtree(const std::string& p) {
  own_path(p);
  std::lock_guard<std::mutex> g(g_own_mu);
  g_own_trees.insert(p);
}

static bool is_own(const std::string& p) {
  std::lock_guard<std::mutex> g(g_own_mu);
  if (now_us() > g_own_until) {
    g_own.clear();
    g_own_trees.clear();
    return false;
  }
  if (g_own.count(p)) return true;
  for (std::string q = p; q.size() > g_dest.size(); q = fs::dirname(q))
    if (g_own_trees.count(q)) return true;
  return false;
}

static bool reply(const std::string& s) { return write_all(1, s); }

static std::string safe_join(const std::string& rel_in) {
  std::string rel = rel_in;
  while (starts_with(rel, "./")) rel = rel.substr(2);
  std::string c = fs::clean("/" + rel);  // strips any ".." escaping the root
  return c == "/" ? g_dest : g_dest + c;
}

static std::string op_extract(const std::string& payload) {
  // gzip or plain tar (small edits are shipped uncompressed)
  bool gzipped = payload.size() >= 2 && (unsigned char)payload[0] == 0x1f && (unsigned char)payload[1] == 0x8b;
  GzipReader gz(string_source(&payload));
  Source raw = string_source(&payload);
  TarReader tr([&](char* b, size_t n) { return gzipped ? gz.read(b, n) : raw(b, n); });
  TarEntry e;
  bool root = ::geteuid() == 0;
  try {
    while (tr.next(&e)) {
      std::string out = safe_join(e.name);
      own_path(out);
      if (e.type == '5') {
        fs::mkdirs(out, 0755);
        ::chmod(out.c_str(), e.mode & 07777);
        if (root) {
          int ignored = ::lchown(out.c_str(), e.uid, e.gid);
          (void)ignored;
        }
        fs::set_mtime(out, e.mtime);
        continue;
      }
      if (e.type == '2') {
        fs::mkdirs(fs::dirname(out));
        ::unlink(out.c_str());
        int ignored = ::symlink(e.linkname.c_str(), out.c_str());
        (void)ignored;
        continue;
      }
      if (e.type != '0' && e.type != '7') {
        tr.skip();
        continue;
      }
      fs::mkdirs(fs::dirname(out));
      std::string tmp = out + ".devspace-tmp";
      int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0600);
      if (fd < 0) return std::string("ERR open ") + out + ": " + std::strerror(errno);
      char buf[1 << 16];
      while (true) {
        ssize_t n = tr.read(buf, sizeof(buf));
        if (n <= 0) break;
        if (!write_all(fd, buf, (size_t)n)) {
          ::close(fd);
          return "ERR write " + out;
        }
      }
      ::fchmod(fd, e.mode & 07777);
      if (root) {
        int ignored = ::fchown(fd, e.uid, e.gid);
        (void)ignored;
      }
      ::close(fd);
      fs::set_mtime(tmp, e.mtime);
      if (::rename(tmp.c_str(), out.c_str()) != 0) {
        // target may be a directory being replaced by a file
        fs::remove_all(out);
        if (::rename(tmp.c_str(), out.c_str()) != 0) return "ERR rename " + out;
      }
    }
  } catch (const std::exception& ex) {
    return std::string("ERR ") + ex.what();
  }
  return "OK";
}

static void scan_rec(const std::string& p, std::string& out, std::set<std::pair<uint64_t, uint64_t>>& seen,
                     int depth) {
  struct stat lst;
  if (::lstat(p.c_str(), &lst) != 0) return;
  struct stat st = lst;
  if (S_ISLNK(lst.st_mode)) {
    if (::stat(p.c_str(), &st) != 0) st = lst;
  }
  // like `find -L ... -exec stat -c` : stat of the path itself (links reported as links)
  out += p + "///" + std::to_string((long long)lst.st_size) + "," + std::to_string((long long)lst.st_mtim.tv_sec) +
         "," + strfmt("%x", (unsigned)lst.st_mode) + "," + strfmt("%o", (unsigned)(lst.st_mode & 07777)) + "," +
         std::to_string(lst.st_uid) + "," + std::to_string(lst.st_gid) + "\n";
  if (S_ISDIR(st.st_mode) && depth < 128) {
    auto key = std::make_pair((uint64_t)st.st_dev, (uint64_t)st.st_ino);
    if (seen.count(key)) return;
    seen.insert(key);
    for (auto& e : fs::list_dir(p)) scan_rec(p + "/" + e.name, out, seen, depth + 1);
  }
}

static std::string op_scan() {
  fs::mkdirs(g_dest);
  std::string out;
  std::set<std::pair<uint64_t, uint64_t>> seen;
  scan_rec(g_dest, out, seen, 0);
  out += "DONE\n";
  return out;
}

static void op_remove(const std::string& payload) {
  for (auto& rel : split(payload, "\n")) {
    if (rel.empty()) continue;
    std::string p = safe_join(rel);
    if (p == g_dest) continue;
    own_subtree(p);
    fs::remove_all(p);
  }
}

static std::string op_download(const std::string& payload) {
  std::string raw;
  TarWriter tw(string_sink(&raw));
  for (auto& rel : split(payload, "\n")) {
    if (rel.empty()) continue;
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
    tw.add_file_from_path(e, p);
  }
  tw.finish();
  // checkpoints and other binaries written in the pod are incompressible: stored blocks for
  // those chunks instead of deflate at ~20 MB/s
  return gzip_compress_adaptive(raw, 1);
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
        if (ends_with(name, ".devspace-tmp") || is_own(path)) continue;
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

int main(int argc, char** argv) {
  if (argc < 3 || std::string(argv[1]) != "serve") {
    std::fprintf(stderr, "usage: devspace-helper serve <dest>\n");
    return 2;
  }
  signal(SIGPIPE, SIG_IGN);
  g_dest = fs::clean(argv[2]);
  fs::mkdirs(g_dest);
  reply("HELPER READY\n");
  bool watching = false;
  while (true) {
    unsigned char hdr[5];
    if (!read_exact(0, hdr, 5)) break;
    uint32_t len = ((uint32_t)hdr[1] << 24) | ((uint32_t)hdr[2] << 16) | ((uint32_t)hdr[3] << 8) | hdr[4];
    std::string payload(len, '\0');
    if (len && !read_exact(0, &payload[0], len)) break;
    switch (hdr[0]) {
      case 'U': {
        std::string r;
        {
          OwnOp op;  // the echo of our own extraction is ignored while it runs and shortly after
          r = op_extract(payload);
        }
        reply(r + "\n");
        break;
      }
      case 'R': {
        {
          OwnOp op;
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
      case 'S': reply(op_scan()); break;
      case 'H': reply(op_hash(payload)); break;
      case 'D': {
        std::string a = op_download(payload);
        reply("SIZE " + std::to_string(a.size()) + "\n");
        write_all(1, a);
        break;
      }
      case 'W':
        // one watch loop per helper process (a detached thread is never joinable again, so
        // joinable() cannot be the guard); it ends with the process
        if (!watching) {
          watching = true;
          std::thread(watch_loop).detach();
        }
        break;
      case 'Q': return 0;
      default: reply("ERR unknown op\n");
    }
  }
  return 0;
}

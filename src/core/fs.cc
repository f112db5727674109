#include "core/fs.h"

#include <dirent.h>
#include <fcntl.h>
#include <limits.h>
#include <stdlib.h>
#include <sys/time.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>

#include "core/strutil.h"
#include "platform/platform.h"

namespace ds {
namespace fs {

static StatInfo from_stat(const struct stat& st) {
  StatInfo s;
  s.exists = true;
  s.is_dir = S_ISDIR(st.st_mode);
  s.is_reg = S_ISREG(st.st_mode);
  s.is_symlink = S_ISLNK(st.st_mode);
  s.size = st.st_size;
  int64_t mt = plat::mtime_ns(st);
  s.mtime_sec = mt / 1000000000LL;
  s.mtime_nsec = mt % 1000000000LL;
  s.mode = st.st_mode;
  s.uid = st.st_uid;
  s.gid = st.st_gid;
  s.ino = st.st_ino;
  return s;
}

StatInfo stat(const std::string& path) {
  struct stat st;
  if (::stat(path.c_str(), &st) != 0) return StatInfo{};
  return from_stat(st);
}

StatInfo lstat(const std::string& path) {
  struct stat st;
  if (::lstat(path.c_str(), &st) != 0) return StatInfo{};
  return from_stat(st);
}

bool exists(const std::string& path) { return lstat(path).exists; }
bool is_dir(const std::string& path) { return stat(path).is_dir; }
bool is_file(const std::string& path) { return stat(path).is_reg; }

bool read_file(const std::string& path, std::string* out) {
  int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return false;
  std::string data;
  char buf[65536];
  while (true) {
    ssize_t n = ::read(fd, buf, sizeof(buf));
    if (n < 0) {
      if (errno == EINTR) continue;
      ::close(fd);
      return false;
    }
    if (n == 0) break;
    data.append(buf, (size_t)n);
  }
  ::close(fd);
  *out = std::move(data);
  return true;
}

std::string read_file(const std::string& path) {
  std::string out;
  if (!read_file(path, &out)) throw std::runtime_error("open " + path + ": " + std::strerror(errno));
  return out;
}

static void write_all(int fd, const std::string& data, const std::string& path) {
  size_t off = 0;
  while (off < data.size()) {
    ssize_t n = ::write(fd, data.data() + off, data.size() - off);
    if (n < 0) {
      if (errno == EINTR) continue;
      ::close(fd);
      throw std::runtime_error("write " + path + ": " + std::strerror(errno));
    }
    off += (size_t)n;
  }
}

void write_file(const std::string& path, const std::string& data, int mode) {
  std::string dir = dirname(path);
  if (!dir.empty()) mkdirs(dir);
  int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, mode);
  if (fd < 0) throw std::runtime_error("open " + path + ": " + std::strerror(errno));
  write_all(fd, data, path);
  ::close(fd);
}

void write_file_atomic(const std::string& path, const std::string& data, int mode) {
  std::string dir = dirname(path);
  if (!dir.empty()) mkdirs(dir);
  std::string tmp = path + ".tmp." + std::to_string(::getpid());
  write_file(tmp, data, mode);
  if (::rename(tmp.c_str(), path.c_str()) != 0) {
    ::unlink(tmp.c_str());
    throw std::runtime_error("rename " + tmp + ": " + std::strerror(errno));
  }
}

void append_file(const std::string& path, const std::string& data) {
  std::string dir = dirname(path);
  if (!dir.empty()) mkdirs(dir);
  int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_APPEND | O_CLOEXEC, 0644);
  if (fd < 0) throw std::runtime_error("open " + path + ": " + std::strerror(errno));
  write_all(fd, data, path);
  ::close(fd);
}

bool mkdirs(const std::string& path, int mode) {
  if (path.empty()) return true;
  if (is_dir(path)) return true;
  std::string parent = dirname(path);
  if (!parent.empty() && parent != path) mkdirs(parent, mode);
  if (::mkdir(path.c_str(), mode) != 0 && errno != EEXIST) return false;
  return true;
}

bool remove(const std::string& path) {
  if (::unlink(path.c_str()) == 0) return true;
  if (errno == EISDIR || errno == EPERM) return ::rmdir(path.c_str()) == 0;
  return false;
}

bool remove_all(const std::string& path) {
  StatInfo st = lstat(path);
  if (!st.exists) return true;
  if (st.is_dir) {
    for (auto& e : list_dir(path)) remove_all(join(path, e.name));
    return ::rmdir(path.c_str()) == 0;
  }
  return ::unlink(path.c_str()) == 0;
}

bool rename(const std::string& from, const std::string& to) { return ::rename(from.c_str(), to.c_str()) == 0; }

void copy(const std::string& from, const std::string& to, bool overwrite) {
  StatInfo st = stat(from);
  if (!st.exists) throw std::runtime_error("copy: " + from + " does not exist");
  if (st.is_dir) {
    mkdirs(to, st.mode & 07777);
    for (auto& e : list_dir(from)) copy(join(from, e.name), join(to, e.name), overwrite);
    return;
  }
  if (!overwrite && exists(to)) return;
  write_file(to, read_file(from), st.mode & 07777);
}

bool set_mtime(const std::string& path, int64_t sec, int64_t nsec) {
  struct timespec ts[2];
  ts[0].tv_sec = 0;
  ts[0].tv_nsec = UTIME_NOW;
  ts[1].tv_sec = sec;
  ts[1].tv_nsec = nsec;
  return ::utimensat(AT_FDCWD, path.c_str(), ts, 0) == 0;
}

std::vector<DirEntry> list_dir(const std::string& path) {
  std::vector<DirEntry> out;
  DIR* d = ::opendir(path.c_str());
  if (!d) return out;
  while (struct dirent* e = ::readdir(d)) {
    if (std::strcmp(e->d_name, ".") == 0 || std::strcmp(e->d_name, "..") == 0) continue;
    DirEntry de;
    de.name = e->d_name;
    if (e->d_type == DT_UNKNOWN) {
      StatInfo s = lstat(join(path, de.name));
      de.is_dir = s.is_dir;
      de.is_symlink = s.is_symlink;
    } else {
      de.is_dir = e->d_type == DT_DIR;
      de.is_symlink = e->d_type == DT_LNK;
    }
    out.push_back(de);
  }
  ::closedir(d);
  std::sort(out.begin(), out.end(), [](const DirEntry& a, const DirEntry& b) { return a.name < b.name; });
  return out;
}

static void walk_rec(const std::string& p, const std::function<bool(const std::string&, const StatInfo&)>& fn,
                     bool follow, int depth) {
  if (depth > 256) return;
  StatInfo st = follow ? stat(p) : lstat(p);
  if (!st.exists) return;
  bool descend = fn(p, st);
  if (st.is_dir && descend) {
    for (auto& e : list_dir(p)) walk_rec(join(p, e.name), fn, follow, depth + 1);
  }
}

void walk(const std::string& root, const std::function<bool(const std::string&, const StatInfo&)>& fn,
          bool follow_symlinks) {
  walk_rec(root, fn, follow_symlinks, 0);
}

std::string make_temp_dir(const std::string& prefix) {
  const char* t = getenv("TMPDIR");
  std::string base = t && *t ? t : "/tmp";
  std::string tmpl = join(base, prefix + "XXXXXX");
  std::vector<char> buf(tmpl.begin(), tmpl.end());
  buf.push_back(0);
  if (!::mkdtemp(buf.data())) throw std::runtime_error("mkdtemp failed: " + std::string(std::strerror(errno)));
  return std::string(buf.data());
}

std::string make_temp_file(const std::string& prefix) {
  const char* t = getenv("TMPDIR");
  std::string base = t && *t ? t : "/tmp";
  std::string tmpl = join(base, prefix + "XXXXXX");
  std::vector<char> buf(tmpl.begin(), tmpl.end());
  buf.push_back(0);
  int fd = ::mkstemp(buf.data());
  if (fd < 0) throw std::runtime_error("mkstemp failed: " + std::string(std::strerror(errno)));
  ::close(fd);
  return std::string(buf.data());
}

std::string cwd() {
  char buf[PATH_MAX];
  if (!::getcwd(buf, sizeof(buf))) return ".";
  return buf;
}

bool chdir(const std::string& path) { return ::chdir(path.c_str()) == 0; }

std::string home_dir() {
  const char* h = getenv("HOME");
  if (h && *h) return h;
  // /etc/passwd directly instead of getpwuid (NSS is unavailable to the static binary)
  std::string pw;
  if (read_file("/etc/passwd", &pw)) {
    std::string uid = std::to_string(getuid());
    size_t pos = 0;
    while (pos < pw.size()) {
      size_t nl = pw.find('\n', pos);
      std::string line = pw.substr(pos, nl == std::string::npos ? std::string::npos : nl - pos);
      pos = nl == std::string::npos ? pw.size() : nl + 1;
      std::vector<std::string> f;
      size_t a = 0, b;
      while ((b = line.find(':', a)) != std::string::npos) {
        f.push_back(line.substr(a, b - a));
        a = b + 1;
      }
      f.push_back(line.substr(a));
      if (f.size() >= 6 && f[2] == uid && !f[5].empty()) return f[5];
    }
  }
  return "/";
}

std::string realpath(const std::string& path) {
  char buf[PATH_MAX];
  if (!::realpath(path.c_str(), buf)) return "";
  return buf;
}

std::string abs_path(const std::string& path) {
  if (is_abs(path)) return clean(path);
  return clean(join(cwd(), path));
}

bool is_abs(const std::string& p) { return !p.empty() && p[0] == '/'; }

std::string join(const std::string& a, const std::string& b) {
  if (a.empty()) return b;
  if (b.empty()) return a;
  if (a.back() == '/' && b[0] == '/') return a + b.substr(1);
  if (a.back() == '/' || b[0] == '/') return a + b;
  return a + "/" + b;
}

std::string dirname(const std::string& p) {
  if (p.empty()) return ".";
  size_t e = p.size();
  while (e > 1 && p[e - 1] == '/') --e;
  size_t pos = p.rfind('/', e - 1);
  if (pos == std::string::npos) return ".";
  if (pos == 0) return "/";
  return p.substr(0, pos);
}

std::string basename(const std::string& p) {
  if (p.empty()) return ".";
  size_t e = p.size();
  while (e > 1 && p[e - 1] == '/') --e;
  size_t pos = p.rfind('/', e - 1);
  if (pos == std::string::npos) return p.substr(0, e);
  return p.substr(pos + 1, e - pos - 1);
}

std::string clean(const std::string& p) {
  if (p.empty()) return ".";
  bool abs = p[0] == '/';
  std::vector<std::string> parts;
  for (auto& seg : split(p, "/")) {
    if (seg.empty() || seg == ".") continue;
    if (seg == "..") {
      if (!parts.empty() && parts.back() != "..")
        parts.pop_back();
      else if (!abs)
        parts.push_back("..");
      continue;
    }
    parts.push_back(seg);
  }
  std::string out = (abs ? "/" : "") + ds::join(parts, "/");
  if (out.empty()) return ".";
  return out;
}

std::string extension(const std::string& p) {
  std::string b = basename(p);
  size_t pos = b.rfind('.');
  if (pos == std::string::npos || pos == 0) return "";
  return b.substr(pos);
}

std::string relative(const std::string& base, const std::string& path) {
  std::string b = clean(base), q = clean(path);
  if (b == q) return "";
  if (b == "/") return q.substr(1);
  if (starts_with(q, b + "/")) return q.substr(b.size() + 1);
  return path;
}

}  // namespace fs
}  // namespace ds

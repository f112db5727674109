// Filesystem + path helpers (util/fsutil/filesystem.go, path/filepath in the reference).
#pragma once

#include <sys/stat.h>

#include <cstdint>
#include <functional>
#include <optional>
#include <string>
#include <vector>

namespace ds {
namespace fs {

struct StatInfo {
  bool exists = false;
  bool is_dir = false;
  bool is_reg = false;
  bool is_symlink = false;  // only meaningful for lstat
  int64_t size = 0;
  int64_t mtime_sec = 0;   // whole seconds
  int64_t mtime_nsec = 0;  // nanoseconds part
  uint32_t mode = 0;       // full st_mode
  uint32_t uid = 0, gid = 0;
  uint64_t ino = 0;
  // Round-to-nearest-second mtime (sync/util.go:87 roundMtime).
  int64_t mtime_rounded() const { return mtime_sec + (mtime_nsec >= 500000000 ? 1 : 0); }
};

StatInfo stat(const std::string& path);
StatInfo lstat(const std::string& path);
bool exists(const std::string& path);
bool is_dir(const std::string& path);
bool is_file(const std::string& path);

std::string read_file(const std::string& path);                    // throws on error
bool read_file(const std::string& path, std::string* out);         // no-throw
void write_file(const std::string& path, const std::string& data, int mode = 0644);  // mkdir -p parent
void write_file_atomic(const std::string& path, const std::string& data, int mode = 0644);
void append_file(const std::string& path, const std::string& data);
bool mkdirs(const std::string& path, int mode = 0755);
bool remove(const std::string& path);      // file or empty dir
bool remove_all(const std::string& path);  // rm -rf
bool rename(const std::string& from, const std::string& to);
// Copies a file or a directory tree; existing files are left untouched when !overwrite
// (util/fsutil/filesystem.go:27 Copy does not overwrite).
void copy(const std::string& from, const std::string& to, bool overwrite = false);
bool set_mtime(const std::string& path, int64_t sec, int64_t nsec = 0);

struct DirEntry {
  std::string name;
  bool is_dir = false;
  bool is_symlink = false;
};
std::vector<DirEntry> list_dir(const std::string& path);  // sorted by name, no . / ..

// Recursive walk; callback gets (abs path, lstat); return false to skip descending.
void walk(const std::string& root, const std::function<bool(const std::string&, const StatInfo&)>& fn,
          bool follow_symlinks = false);

std::string make_temp_dir(const std::string& prefix = "devspace-");
std::string make_temp_file(const std::string& prefix = "devspace-");
std::string cwd();
bool chdir(const std::string& path);
std::string home_dir();
std::string realpath(const std::string& path);  // empty on failure
std::string abs_path(const std::string& path);

// Pure path helpers (forward slashes).
std::string join(const std::string& a, const std::string& b);
template <typename... R>
std::string join(const std::string& a, const std::string& b, const R&... rest) {
  return join(join(a, b), rest...);
}
std::string dirname(const std::string& p);
std::string basename(const std::string& p);
std::string clean(const std::string& p);
std::string extension(const std::string& p);
// Relative path of `path` inside `base` ("" when equal); returns path unchanged if not inside.
std::string relative(const std::string& base, const std::string& path);
bool is_abs(const std::string& p);

}  // namespace fs
}  // namespace ds

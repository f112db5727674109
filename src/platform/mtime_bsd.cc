// plat::mtime_ns where struct stat names it st_mtimespec (macOS / Darwin). CMake picks this file
// when the header has no st_mtim (CMakeLists.txt).
#include <sys/stat.h>

#include <cstdint>

#include "platform/platform.h"

namespace ds {
namespace plat {

int64_t mtime_ns(const struct stat& st) {
  return (int64_t)st.st_mtimespec.tv_sec * 1000000000LL + st.st_mtimespec.tv_nsec;
}

}  // namespace plat
}  // namespace ds

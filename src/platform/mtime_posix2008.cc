// plat::mtime_ns where struct stat has POSIX.1-2008's st_mtim (Linux, the BSDs' newer headers).
// CMake picks this file or mtime_bsd.cc by probing the header (CMakeLists.txt).
#include <sys/stat.h>

#include <cstdint>

#include "platform/platform.h"

namespace ds {
namespace plat {

int64_t mtime_ns(const struct stat& st) { return (int64_t)st.st_mtim.tv_sec * 1000000000LL + st.st_mtim.tv_nsec; }

}  // namespace plat
}  // namespace ds

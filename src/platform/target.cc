// plat::release_target (platform/platform.h): uname(2) is POSIX, so both builds share it.
#include <sys/utsname.h>

#include <cctype>
#include <string>

#include "platform/platform.h"

namespace ds {
namespace plat {

std::string release_target() {
  struct utsname u{};
  if (::uname(&u) != 0) return "linux-amd64";
  std::string os;
  for (const char* c = u.sysname; *c; ++c) os += (char)std::tolower((unsigned char)*c);
  std::string m = u.machine, arch = m;
  if (m == "x86_64" || m == "amd64") arch = "amd64";
  else if (m == "aarch64" || m == "arm64") arch = "arm64";
  else if (m == "i386" || m == "i686") arch = "386";
  return os + "-" + arch;
}

}  // namespace plat
}  // namespace ds

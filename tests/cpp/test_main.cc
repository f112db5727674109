#include <signal.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <exception>

#include "core/log.h"
#include "testing.h"

namespace dstest {
std::vector<Case>& registry() {
  static std::vector<Case> r;
  return r;
}
}  // namespace dstest

int main(int argc, char** argv) {
  std::string filter = argc > 1 ? argv[1] : "";
  signal(SIGPIPE, SIG_IGN);
  setvbuf(stdout, nullptr, _IOLBF, 0);
  ds::log::set_fatal_throws(true);
  int pass = 0, fail = 0;
  for (auto& c : dstest::registry()) {
    if (!filter.empty() && std::strstr(c.name, filter.c_str()) == nullptr) continue;
    auto t0 = std::chrono::steady_clock::now();
    try {
      c.fn();
      ++pass;
      auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
      std::cout << "PASS " << c.name << " (" << ms << " ms)\n";
    } catch (const dstest::Failure& f) {
      ++fail;
      std::cout << "FAIL " << c.name << "\n  " << f.msg << "\n";
    } catch (const std::exception& e) {
      ++fail;
      std::cout << "FAIL " << c.name << "\n  exception: " << e.what() << "\n";
    }
  }
  std::cout << pass << " passed, " << fail << " failed\n";
  return fail ? 1 : 0;
}

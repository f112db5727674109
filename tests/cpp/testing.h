// Tiny self-registering test harness (no gtest in the image). Run: bin/devspace_tests [filter]
#pragma once

#include <functional>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

namespace dstest {

struct Case {
  const char* name;
  std::function<void()> fn;
};
std::vector<Case>& registry();
struct Reg {
  Reg(const char* n, std::function<void()> f) { registry().push_back({n, std::move(f)}); }
};
struct Failure {
  std::string msg;
};

}  // namespace dstest

#define DS_CAT2(a, b) a##b
#define DS_CAT(a, b) DS_CAT2(a, b)
#define TEST(name)                                                          \
  static void name();                                                       \
  static dstest::Reg DS_CAT(reg_, name)(#name, name);                       \
  static void name()

#define EXPECT_TRUE(c)                                                                   \
  do {                                                                                   \
    if (!(c)) {                                                                          \
      std::ostringstream _os;                                                            \
      _os << __FILE__ << ":" << __LINE__ << ": expected true: " #c;                      \
      throw dstest::Failure{_os.str()};                                                  \
    }                                                                                    \
  } while (0)

#define EXPECT_EQ(a, b)                                                                  \
  do {                                                                                   \
    auto _a = (a);                                                                       \
    auto _b = (b);                                                                       \
    if (!(_a == _b)) {                                                                   \
      std::ostringstream _os;                                                            \
      _os << __FILE__ << ":" << __LINE__ << ": " #a " == " #b "\n  got: " << _a          \
          << "\n  want: " << _b;                                                         \
      throw dstest::Failure{_os.str()};                                                  \
    }                                                                                    \
  } while (0)

#define EXPECT_THROWS(stmt)                                                              \
  do {                                                                                   \
    bool _t = false;                                                                     \
    try {                                                                                \
      stmt;                                                                              \
    } catch (...) {                                                                      \
      _t = true;                                                                         \
    }                                                                                    \
    if (!_t) {                                                                           \
      std::ostringstream _os;                                                            \
      _os << __FILE__ << ":" << __LINE__ << ": expected exception from " #stmt;          \
      throw dstest::Failure{_os.str()};                                                  \
    }                                                                                    \
  } while (0)

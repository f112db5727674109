#include "core/safe_regex.h"

#include <pthread.h>

#include <algorithm>
#include <exception>
#include <functional>
#include <stdexcept>

namespace ds {

namespace {

// Inputs up to this size run inline (measured: 10 kB fine, 30 kB overflow on 8 MB).
constexpr size_t kInline = 4096;
#if defined(__SANITIZE_ADDRESS__) || defined(__SANITIZE_THREAD__)
constexpr size_t kSanitizerFactor = 4;
#elif defined(__has_feature)
#if __has_feature(thread_sanitizer) || __has_feature(address_sanitizer)
constexpr size_t kSanitizerFactor = 4;
#else
constexpr size_t kSanitizerFactor = 1;
#endif
#else
constexpr size_t kSanitizerFactor = 1;
#endif

struct Job {
  std::function<void()> fn;
  std::exception_ptr err;
};

void* trampoline(void* p) {
  auto* j = static_cast<Job*>(p);
  try {
    j->fn();
  } catch (...) {
    j->err = std::current_exception();
  }
  return nullptr;
}

void run(size_t input, const std::function<void()>& fn) {
  if (input <= kInline) {
    fn();
    return;
  }
  if (input > (size_t(1) << 20))
    throw std::runtime_error("regex: input of " + std::to_string(input) + " bytes is too long to match safely (max 1 MiB)");
  Job job{fn, nullptr};
  pthread_attr_t attr;
  pthread_attr_init(&attr);
  // libstdc++ needs ~280 B of stack per input byte (measured); 1 kB per byte leaves margin
  // (4 kB in sanitizer builds, whose frames are several times larger)
  size_t stack = std::max<size_t>(64u << 20, input * 1024 * kSanitizerFactor);
  pthread_attr_setstacksize(&attr, stack);
  pthread_t t;
  int rc = pthread_create(&t, &attr, trampoline, &job);
  pthread_attr_destroy(&attr);
  if (rc != 0) throw std::runtime_error("regex: cannot start a matcher thread");
  pthread_join(t, nullptr);
  if (job.err) std::rethrow_exception(job.err);
}

}  // namespace

void safe_regex_run(size_t input_bytes, const std::function<void()>& fn) { run(input_bytes, fn); }

bool safe_regex_search(const std::string& s, std::smatch* m, const std::regex& re) {
  bool r = false;
  run(s.size(), [&] { r = std::regex_search(s, *m, re); });
  return r;
}

bool safe_regex_search(const std::string& s, const std::regex& re) {
  bool r = false;
  run(s.size(), [&] { r = std::regex_search(s, re); });
  return r;
}

bool safe_regex_match(const std::string& s, std::smatch* m, const std::regex& re) {
  bool r = false;
  run(s.size(), [&] { r = std::regex_match(s, *m, re); });
  return r;
}

bool safe_regex_match(const std::string& s, const std::regex& re) {
  bool r = false;
  run(s.size(), [&] { r = std::regex_match(s, re); });
  return r;
}

std::string safe_regex_replace(const std::string& s, const std::regex& re, const std::string& fmt) {
  std::string r;
  run(s.size(), [&] { r = std::regex_replace(s, re, fmt); });
  return r;
}

}  // namespace ds

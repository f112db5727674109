// Phase spans: monotonic-clock timings of build / push / deploy / rollout wait /
// sync batches, appended as JSON lines to .devspace/logs/trace.jsonl:
//   {"span":"deploy.helm","start_us":..., "dur_us":..., "pid":..., <fields>}
// The reference has no instrumentation; these spans back the latency numbers in bench.py and
// `devspace status` style diagnostics. Disabled with DEVSPACE_TRACE=0.
#pragma once

#include <chrono>
#include <map>
#include <string>

namespace ds {
namespace trace {

bool enabled();
// Monotonic microseconds since an arbitrary epoch (steady_clock).
int64_t now_us();
void emit(const std::string& name, int64_t start_us, int64_t dur_us,
          const std::map<std::string, std::string>& fields = {});

class Span {
 public:
  explicit Span(std::string name, std::map<std::string, std::string> fields = {})
      : name_(std::move(name)), fields_(std::move(fields)), start_(now_us()) {}
  ~Span() { end(); }
  void set(const std::string& k, const std::string& v) { fields_[k] = v; }
  int64_t end() {
    if (done_) return dur_;
    done_ = true;
    dur_ = now_us() - start_;
    emit(name_, start_, dur_, fields_);
    return dur_;
  }

 private:
  std::string name_;
  std::map<std::string, std::string> fields_;
  int64_t start_;
  int64_t dur_ = 0;
  bool done_ = false;
};

}  // namespace trace
}  // namespace ds

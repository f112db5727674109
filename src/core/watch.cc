#include "core/watch.h"

#include "core/fs.h"
#include "core/match.h"
#include "core/strutil.h"

namespace ds {

// ---------------------------------------------------------------- poll watcher

PollWatcher::PollWatcher(std::vector<std::string> patterns, Callback cb, int interval_ms)
    : patterns_(std::move(patterns)), cb_(std::move(cb)), interval_ms_(interval_ms) {}

PollWatcher::~PollWatcher() { stop(); }

std::map<std::string, PollWatcher::Stamp> PollWatcher::gather() {
  std::vector<std::string> pats;
  {
    std::lock_guard<std::mutex> g(mu_);
    pats = patterns_;
  }
  std::map<std::string, Stamp> out;
  for (auto& p : pats) {
    for (auto& f : glob_expand(p)) {
      // the reference ignores .devspace* paths (watch/watch.go:140)
      if (contains(f, ".devspace")) continue;
      fs::StatInfo st = fs::stat(f);
      if (!st.exists) continue;
      out[f] = {st.size, st.mtime_sec * 1000000000LL + st.mtime_nsec};
    }
  }
  return out;
}

bool PollWatcher::poll_once() {
  auto now = gather();
  if (!primed_) {
    state_ = now;
    primed_ = true;
    return false;
  }
  std::vector<std::string> changed, deleted;
  for (auto& kv : now) {
    auto it = state_.find(kv.first);
    if (it == state_.end() || it->second.size != kv.second.size || it->second.mtime_ns != kv.second.mtime_ns)
      changed.push_back(kv.first);
  }
  for (auto& kv : state_)
    if (!now.count(kv.first)) deleted.push_back(kv.first);
  state_ = std::move(now);
  if ((!changed.empty() || !deleted.empty()) && cb_) cb_(changed, deleted);
  return !changed.empty() || !deleted.empty();
}

void PollWatcher::start() {
  std::lock_guard<std::mutex> g(mu_);
  if (started_) return;  // (watch/watch.go:50 checks-then-sets under two locks; one here)
  started_ = true;
  stop_ = false;
  th_ = std::thread([this] {
    poll_once();
    while (true) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        if (cv_.wait_for(lk, std::chrono::milliseconds(interval_ms_), [this] { return stop_; })) return;
      }
      poll_once();
    }
  });
}

void PollWatcher::stop() {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (!started_) return;
    stop_ = true;
    started_ = false;
  }
  cv_.notify_all();
  if (th_.joinable()) th_.join();
}

void PollWatcher::update_patterns(std::vector<std::string> patterns) {
  std::lock_guard<std::mutex> g(mu_);
  patterns_ = std::move(patterns);
}

}  // namespace ds

#include "core/log.h"

#include <sys/ioctl.h>
#include <time.h>
#include <unistd.h>

#include <cstdarg>
#include <cstdio>
#include <iostream>

#include "core/fs.h"
#include "core/value.h"

namespace ds {
namespace log {

static std::atomic<bool> g_fatal_throws{false};
void set_fatal_throws(bool t) { g_fatal_throws = t; }

[[noreturn]] static void die(const std::string& m) {
  if (g_fatal_throws) throw FatalError(m);
  std::fflush(stdout);
  std::fflush(stderr);
  std::exit(1);
}

void Logger::fatal(const std::string& m) {
  error(m);
  die(m);
}

void DiscardLogger::fatal(const std::string& m) { die(m); }

void Logger::print_table(const std::vector<std::string>& header, const std::vector<std::vector<std::string>>& rows) {
  std::string out = join(header, " | ") + "\n";
  for (auto& r : rows) out += join(r, " | ") + "\n";
  info(out);
}

std::string rfc3339_now() {
  time_t t = time(nullptr);
  struct tm tmv;
  localtime_r(&t, &tmv);
  char buf[64];
  strftime(buf, sizeof(buf), "%Y-%m-%dT%H:%M:%S", &tmv);
  long off = tmv.tm_gmtoff;
  std::string tz;
  if (off == 0) {
    tz = "Z";
  } else {
    char sign = off < 0 ? '-' : '+';
    off = off < 0 ? -off : off;
    tz = strfmt("%c%02ld:%02ld", sign, off / 3600, (off % 3600) / 60);
  }
  return std::string(buf) + tz;
}

FileLogger::FileLogger(const std::string& path) : path_(path) { fs::mkdirs(fs::dirname(path)); }

void FileLogger::emit(const std::string& level, const std::string& msg,
                      const std::map<std::string, std::string>& fields) {
  Value v = Value::map();
  for (auto& kv : fields) v[kv.first] = kv.second;
  v["level"] = level;
  v["msg"] = msg;
  v["time"] = rfc3339_now();
  std::string line = json_dump(v) + "\n";
  std::lock_guard<std::mutex> g(mu_);
  try {
    fs::append_file(path_, line);
  } catch (...) {
  }
}

std::string color(const std::string& text, const std::string& spec) {
  std::string code;
  bool bold = ends_with(spec, "+b");
  std::string c = bold ? spec.substr(0, spec.size() - 2) : spec;
  if (c == "red")
    code = "31";
  else if (c == "green")
    code = "32";
  else if (c == "yellow")
    code = "33";
  else if (c == "blue")
    code = "34";
  else if (c == "magenta")
    code = "35";
  else if (c == "cyan")
    code = "36";
  else if (c == "white")
    code = "37";
  else if (!c.empty() && std::isdigit((unsigned char)c[0]))
    code = "38;5;" + c;
  else
    return text;
  StdoutLogger* sl = stdout_logger();
  if (sl && !sl->use_color()) return text;
  return "\x1b[" + std::string(bold ? "1;" : "") + code + "m" + text + "\x1b[0m";
}

struct Kind {
  const char* tag;
  const char* color;
  Level level;
};
static const Kind kKinds[] = {
    {"[debug]  ", "green+b", Level::Debug}, {"[info]   ", "cyan+b", Level::Info},
    {"[warn]   ", "166+b", Level::Warn},    {"[error]  ", "red+b", Level::Error},
    {"[fatal]  ", "red+b", Level::Fatal},   {"[done] √ ", "green+b", Level::Info},
    {"[fail] X ", "red+b", Level::Error},
};

static long now_ms() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1000 + ts.tv_nsec / 1000000;
}

StdoutLogger::StdoutLogger() {
  tty_ = ::isatty(1);
  const char* nc = getenv("NO_COLOR");
  color_ = tty_ && !(nc && *nc);
  const char* fc = getenv("DEVSPACE_FORCE_COLOR");
  if (fc && *fc == '1') color_ = true;
}

StdoutLogger::~StdoutLogger() {
  spinner_stop_ = true;
  if (spinner_.joinable()) spinner_.join();
}

void StdoutLogger::clear_spinner_locked() {
  if (waiting_ && tty_ && shown_) {
    std::string blank(wait_msg_.size() + 24, ' ');
    std::fputs(("\r" + blank + "\r").c_str(), stdout);
    std::fflush(stdout);
    shown_ = false;
  }
}

void StdoutLogger::write_msg(int kind, const std::string& m) {
  const Kind& k = kKinds[kind];
  if ((int)level_ < (int)k.level) return;
  std::string msg = m;
  if (msg.empty() || msg.back() != '\n') msg.push_back('\n');
  {
    std::lock_guard<std::recursive_mutex> g(mu_);
    clear_spinner_locked();
    std::string line = log::color(k.tag, k.color) + msg;
    std::fputs(line.c_str(), stdout);
    std::fflush(stdout);
  }
  if (file_) {
    static const char* lv[] = {"debug", "info", "warning", "error", "fatal", "info", "error"};
    file_->emit(lv[kind], m, {});
    // errors and fatals also go to errors.log, as the reference's runtime error handler does
    // (util/log/file_logger.go OverrideRuntimeErrorHandler)
    if (kind == 3 || kind == 4 || kind == 6) file_logger("errors")->emit(lv[kind], m, {});
  }
}

void StdoutLogger::fatal(const std::string& m) {
  write_msg(4, m);
  die(m);
}

void StdoutLogger::spinner_loop() {
  static const char* runes[] = {"⠋", "⠙", "⠹", "⠸", "⠼", "⠴", "⠦", "⠧", "⠇", "⠏"};
  while (!spinner_stop_) {
    {
      std::lock_guard<std::recursive_mutex> g(mu_);
      if (waiting_ && tty_) {
        long el = (now_ms() - wait_start_ms_) / 1000;
        std::string line = "\r" + log::color("[wait] ", "red+b") + runes[rune_ % 10] + " " + wait_msg_ + " (" +
                           std::to_string(el) + "s)";
        rune_++;
        std::fputs(line.c_str(), stdout);
        std::fflush(stdout);
        shown_ = true;
      }
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(150));
  }
}

void StdoutLogger::start_wait(const std::string& m) {
  std::lock_guard<std::recursive_mutex> g(mu_);
  clear_spinner_locked();
  wait_msg_ = m;
  wait_start_ms_ = now_ms();
  waiting_ = true;
  if (!tty_) {
    std::fputs((log::color("[wait] ", "red+b") + m + "\n").c_str(), stdout);
    std::fflush(stdout);
  }
  if (tty_ && !spinner_.joinable()) spinner_ = std::thread([this] { spinner_loop(); });
}

void StdoutLogger::stop_wait() {
  std::lock_guard<std::recursive_mutex> g(mu_);
  clear_spinner_locked();
  waiting_ = false;
}

void StdoutLogger::write(const std::string& raw) {
  std::lock_guard<std::recursive_mutex> g(mu_);
  clear_spinner_locked();
  std::fwrite(raw.data(), 1, raw.size(), stdout);
  std::fflush(stdout);
}

void StdoutLogger::print_table(const std::vector<std::string>& header,
                               const std::vector<std::vector<std::string>>& rows) {
  // util/log/stdout_logger.go:186 layout
  std::vector<size_t> w(header.size());
  for (size_t i = 0; i < header.size(); ++i) w[i] = header[i].size();
  for (auto& r : rows)
    for (size_t i = 0; i < r.size() && i < w.size(); ++i) w[i] = std::max(w[i], r[i].size());
  std::string out = "\n";
  for (size_t i = 0; i < header.size(); ++i) {
    out += log::color(" " + header[i] + "  ", "green+b");
    out += std::string(w[i] - header[i].size(), ' ');
  }
  out += "\n";
  if (rows.empty()) out += " No entries found\n";
  for (auto& r : rows) {
    for (size_t i = 0; i < r.size() && i < w.size(); ++i) {
      out += " " + r[i] + "  ";
      out += std::string(w[i] - r[i].size(), ' ');
    }
    out += "\n";
  }
  out += "\n";
  write(out);
}

static std::mutex g_mu;
static std::shared_ptr<Logger>& g_logger() {
  static std::shared_ptr<Logger> l = std::make_shared<StdoutLogger>();
  return l;
}

Logger& get() {
  std::lock_guard<std::mutex> g(g_mu);
  return *g_logger();
}

void set(std::shared_ptr<Logger> l) {
  std::lock_guard<std::mutex> g(g_mu);
  g_logger() = std::move(l);
}

StdoutLogger* stdout_logger() { return dynamic_cast<StdoutLogger*>(g_logger().get()); }

std::string& logdir() {
  static std::string d = "./.devspace/logs/";
  return d;
}

std::shared_ptr<FileLogger> file_logger(const std::string& name) {
  static std::mutex mu;
  static std::map<std::string, std::shared_ptr<FileLogger>> loggers;
  std::lock_guard<std::mutex> g(mu);
  std::string path = fs::join(logdir(), name + ".log");
  auto it = loggers.find(path);
  if (it != loggers.end()) return it->second;
  auto l = std::make_shared<FileLogger>(path);
  loggers[path] = l;
  return l;
}

void start_file_logging() {
  if (auto* s = stdout_logger()) s->set_file_logger(file_logger("default"));
}

}  // namespace log
}  // namespace ds

namespace ds {
namespace log {

static std::string vformat(const char* fmt, va_list ap) {
  va_list ap2;
  va_copy(ap2, ap);
  int n = vsnprintf(nullptr, 0, fmt, ap2);
  va_end(ap2);
  std::string out(n > 0 ? n : 0, '\0');
  if (n > 0) vsnprintf(&out[0], n + 1, fmt, ap);
  return out;
}

void donef(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  std::string m = vformat(fmt, ap);
  va_end(ap);
  done(m);
}

void infof(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  std::string m = vformat(fmt, ap);
  va_end(ap);
  info(m);
}

}  // namespace log
}  // namespace ds

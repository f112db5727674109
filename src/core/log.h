// Console + JSON-file logging (util/log/*.go in the reference).
//
// Console: colored tags "[info]   ", "[done] √ ", spinner "[wait] ⠋ msg (Ns)", tables.
// Files: logrus-compatible JSON lines in .devspace/logs/<name>.log — `status sync` parses the
// exact message strings (cmd/status/sync.go:19-21), so those are kept verbatim.
#pragma once

#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "core/strutil.h"

namespace ds {
namespace log {

enum class Level { Panic = 0, Fatal = 1, Error = 2, Warn = 3, Info = 4, Debug = 5 };

class Logger {
 public:
  virtual ~Logger() = default;
  virtual void debug(const std::string& m) = 0;
  virtual void info(const std::string& m) = 0;
  virtual void warn(const std::string& m) = 0;
  virtual void error(const std::string& m) = 0;
  virtual void done(const std::string& m) = 0;
  virtual void fail(const std::string& m) = 0;
  [[noreturn]] virtual void fatal(const std::string& m);
  virtual void start_wait(const std::string& m) { (void)m; }
  virtual void stop_wait() {}
  virtual void print_table(const std::vector<std::string>& header, const std::vector<std::vector<std::string>>& rows);
  virtual void write(const std::string& raw) { (void)raw; }
  virtual void set_level(Level l) { level_ = l; }
  Level level() const { return level_; }

 protected:
  Level level_ = Level::Info;
};

// JSON-lines file logger with optional context fields (logrus WithKey).
class FileLogger : public Logger {
 public:
  explicit FileLogger(const std::string& path);
  void debug(const std::string& m) override { emit("debug", m, {}); }
  void info(const std::string& m) override { emit("info", m, {}); }
  void warn(const std::string& m) override { emit("warning", m, {}); }
  void error(const std::string& m) override { emit("error", m, {}); }
  void done(const std::string& m) override { emit("info", m, {}); }
  void fail(const std::string& m) override { emit("error", m, {}); }
  void emit(const std::string& level, const std::string& msg, const std::map<std::string, std::string>& fields);
  const std::string& path() const { return path_; }

 private:
  std::string path_;
  std::mutex mu_;
};

class DiscardLogger : public Logger {
 public:
  void debug(const std::string&) override {}
  void info(const std::string&) override {}
  void warn(const std::string&) override {}
  void error(const std::string&) override {}
  void done(const std::string&) override {}
  void fail(const std::string&) override {}
  void fatal(const std::string& m) override;
};

class StdoutLogger : public Logger {
 public:
  StdoutLogger();
  ~StdoutLogger() override;
  void debug(const std::string& m) override { write_msg(0, m); }
  void info(const std::string& m) override { write_msg(1, m); }
  void warn(const std::string& m) override { write_msg(2, m); }
  void error(const std::string& m) override { write_msg(3, m); }
  void done(const std::string& m) override { write_msg(5, m); }
  void fail(const std::string& m) override { write_msg(6, m); }
  [[noreturn]] void fatal(const std::string& m) override;
  void start_wait(const std::string& m) override;
  void stop_wait() override;
  void print_table(const std::vector<std::string>& header,
                   const std::vector<std::vector<std::string>>& rows) override;
  void write(const std::string& raw) override;
  void set_file_logger(std::shared_ptr<FileLogger> f) { file_ = std::move(f); }
  bool use_color() const { return color_; }

 private:
  void write_msg(int kind, const std::string& m);
  void spinner_loop();
  void clear_spinner_locked();
  std::recursive_mutex mu_;
  bool color_ = false;
  bool tty_ = false;
  std::shared_ptr<FileLogger> file_;
  std::string wait_msg_;
  std::atomic<bool> waiting_{false};
  long wait_start_ms_ = 0;
  std::thread spinner_;
  std::atomic<bool> spinner_stop_{false};
  int rune_ = 0;
  bool shown_ = false;
};

// Process-wide default logger (explicitly replaceable, e.g. by tests).
Logger& get();
void set(std::shared_ptr<Logger> l);
StdoutLogger* stdout_logger();  // nullptr if the default is not a StdoutLogger

// Directory for named file loggers (default ./.devspace/logs/).
std::string& logdir();
std::shared_ptr<FileLogger> file_logger(const std::string& name);
// Mirror console output into default.log (util/log/log.go:144).
void start_file_logging();

inline void debug(const std::string& m) { get().debug(m); }
inline void info(const std::string& m) { get().info(m); }
inline void warn(const std::string& m) { get().warn(m); }
inline void error(const std::string& m) { get().error(m); }
inline void done(const std::string& m) { get().done(m); }
inline void fail(const std::string& m) { get().fail(m); }
[[noreturn]] inline void fatal(const std::string& m) { get().fatal(m); }
inline void start_wait(const std::string& m) { get().start_wait(m); }
inline void stop_wait() { get().stop_wait(); }
inline void print_table(const std::vector<std::string>& h, const std::vector<std::vector<std::string>>& r) {
  get().print_table(h, r);
}
void donef(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
void infof(const char* fmt, ...) __attribute__((format(printf, 1, 2)));

// ANSI colouring helper ("green+b", "red+b", "cyan+b", "white+b", "166+b").
std::string color(const std::string& text, const std::string& spec);

// Thrown by fatal() when the process is configured not to exit (library / test use).
struct FatalError : std::runtime_error {
  using std::runtime_error::runtime_error;
};
void set_fatal_throws(bool t);

std::string rfc3339_now();

}  // namespace log
}  // namespace ds

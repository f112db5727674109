#include "core/prompt.h"

#include <termios.h>
#include <unistd.h>

#include <cstdio>
#include <atomic>
#include <deque>
#include <iostream>
#include <mutex>
#include <regex>

#include "core/log.h"
#include "core/strutil.h"

namespace ds {
namespace prompt {

static std::mutex g_mu;
static std::deque<std::string>& scripted() {
  static std::deque<std::string> q;
  return q;
}
static bool g_scripted = false;

void set_scripted_answers(const std::vector<std::string>& answers) {
  std::lock_guard<std::mutex> g(g_mu);
  scripted().assign(answers.begin(), answers.end());
  g_scripted = true;
}

bool interactive() {
  const char* ni = getenv("DEVSPACE_NONINTERACTIVE");
  if (ni && *ni && std::string(ni) != "0") return false;
  return ::isatty(0) && ::isatty(1);
}

static bool read_line(std::string* out, bool secret) {
  {
    std::lock_guard<std::mutex> g(g_mu);
    if (g_scripted) {
      if (scripted().empty()) return false;
      *out = scripted().front();
      scripted().pop_front();
      return true;
    }
  }
  struct termios old{};
  bool restore = false;
  if (secret && ::isatty(0) && tcgetattr(0, &old) == 0) {
    struct termios t = old;
    t.c_lflag &= ~(tcflag_t)ECHO;
    tcsetattr(0, TCSANOW, &t);
    restore = true;
  }
  std::string line;
  bool ok = (bool)std::getline(std::cin, line);
  if (restore) {
    tcsetattr(0, TCSANOW, &old);
    std::fputs("\n", stdout);
  }
  if (!ok) return false;
  *out = trim_right(line, "\r\n");
  return true;
}

std::string ask(const Params& p) {
  bool tty = interactive() && !g_scripted;
  std::string q = p.question;
  if (!p.options.empty()) {
    if (tty) {
      log::get().write(log::color("? ", "green+b") + q + "\n");
      for (size_t i = 0; i < p.options.size(); ++i)
        log::get().write(strfmt("  %zu) %s%s\n", i + 1, p.options[i].c_str(),
                                p.options[i] == p.default_value ? " (default)" : ""));
    }
    while (true) {
      if (tty) log::get().write("> ");
      std::string line;
      if (!read_line(&line, false)) {
        if (!p.default_value.empty()) return p.default_value;
        if (!p.options.empty()) return p.options[0];
        throw PromptError("no answer for: " + q);
      }
      line = trim(line);
      if (line.empty() && !p.default_value.empty()) return p.default_value;
      int64_t idx;
      if (parse_int64(line, &idx) && idx >= 1 && idx <= (int64_t)p.options.size()) return p.options[idx - 1];
      for (auto& o : p.options)
        if (o == line) return o;
      if (!tty) throw PromptError("invalid selection '" + line + "' for: " + q);
    }
  }
  while (true) {
    if (tty) {
      std::string shown = log::color("? ", "green+b") + q;
      if (!p.default_value.empty() && !p.is_password) shown += " (" + p.default_value + ")";
      log::get().write(shown + "\n> ");
    }
    std::string line;
    if (!read_line(&line, p.is_password)) {
      if (!p.default_value.empty()) return p.default_value;
      if (p.optional) return "";
      throw PromptError("cannot prompt for \"" + q +
                        "\" in non-interactive mode (set a default, an env var, or run interactively)");
    }
    std::string ans = trim(line);
    if (ans.empty()) ans = p.default_value;
    if (!p.validation_regex.empty()) {
      try {
        std::regex re("^(?:" + p.validation_regex + ")$");
        if (!std::regex_match(ans, re)) {
          if (!tty) throw PromptError("answer '" + ans + "' does not match " + p.validation_regex);
          log::get().write(log::color("X ", "red+b") + "Answer does not match " + p.validation_regex + "\n");
          continue;
        }
      } catch (const std::regex_error&) {
      }
    }
    // No validation pattern = "^.*$" (stdin.go:40): an empty answer is a valid answer.
    return ans;
  }
}

std::string ask(const std::string& question, const std::string& def) {
  Params p;
  p.question = question;
  p.default_value = def;
  return ask(p);
}

bool confirm(const std::string& question, bool def) {
  Params p;
  p.question = question;
  p.options = {"yes", "no"};
  p.default_value = def ? "yes" : "no";
  return ask(p) == "yes";
}

std::string select(const std::string& question, const std::vector<std::string>& options, const std::string& def) {
  Params p;
  p.question = question;
  p.options = options;
  p.default_value = def;
  return ask(p);
}

static struct termios g_cooked{};
static std::atomic<bool> g_cooked_set{false};

void remember_cooked_tty(const struct termios& saved) {
  g_cooked = saved;
  g_cooked_set = true;
}

void forget_cooked_tty() { g_cooked_set = false; }

void restore_cooked_tty_from_signal() {
  if (g_cooked_set.load()) tcsetattr(0, TCSANOW, &g_cooked);
}

}  // namespace prompt
}  // namespace ds

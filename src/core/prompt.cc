#include "core/prompt.h"

#include <termios.h>
#include <unistd.h>

#include <cstdio>
#include <atomic>
#include <deque>
#include <iostream>
#include <map>
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

static std::map<std::string, std::string>& answers() {
  static std::map<std::string, std::string> m;
  return m;
}

void set_answer(const std::string& key, const std::string& value) {
  std::lock_guard<std::mutex> g(g_mu);
  answers()[key] = value;
}

bool has_answer(const std::string& key) {
  std::lock_guard<std::mutex> g(g_mu);
  return answers().count(key) > 0;
}

bool noninteractive_env() {
  const char* ni = getenv("DEVSPACE_NONINTERACTIVE");
  return ni && *ni && std::string(ni) != "0";
}

bool interactive() {
  if (noninteractive_env()) return false;
  return ::isatty(0) && ::isatty(1);
}

static bool preset(const Params& p, std::string* out) {
  {
    std::lock_guard<std::mutex> g(g_mu);
    auto it = p.key.empty() ? answers().end() : answers().find(p.key);
    if (it != answers().end()) {
      *out = it->second;
      return true;
    }
  }
  const char* v = p.env.empty() ? nullptr : getenv(p.env.c_str());
  if (v && *v) {
    *out = v;
    return true;
  }
  return false;
}

static std::string hint(const Params& p) {
  std::string h;
  if (!p.key.empty()) h = "--" + p.key;
  if (!p.env.empty()) h += (h.empty() ? "" : " or ") + p.env;
  return h;
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
  // CI runners and `docker exec -i` leave stdin open with nobody writing: never wait on it
  if (noninteractive_env()) return false;
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

// A preset answer goes through the same checks as a typed one.
static std::string checked_preset(const Params& p, const std::string& v_in) {
  std::string v = trim(v_in);
  std::string from = hint(p);
  if (!p.options.empty()) {
    for (auto& o : p.options)
      if (o == v) return o;
    throw PromptError("invalid value '" + v + "' (" + from + ") for: " + p.question + " (one of: " + join(p.options, ", ") +
                      ")");
  }
  if (!p.validation_regex.empty()) {
    try {
      if (!std::regex_match(v, std::regex("^(?:" + p.validation_regex + ")$")))
        throw PromptError("invalid value '" + v + "' (" + from + ") for: " + p.question + " (must match " +
                          p.validation_regex + ")");
    } catch (const std::regex_error&) {
    }
  }
  return v;
}

std::string ask(const Params& p) {
  std::string pre;
  if (preset(p, &pre)) return checked_preset(p, pre);
  bool tty = interactive() && !g_scripted;
  std::string q = p.question;
  std::string set_it = hint(p).empty() ? "" : " (set " + hint(p) + ")";
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
        throw PromptError("no answer for: " + q + set_it);
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
      throw PromptError("cannot prompt for \"" + q + "\" in non-interactive mode" +
                        (set_it.empty() ? " (run interactively)" : set_it));
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

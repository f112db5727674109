// Interactive prompts (util/stdinutil/stdin.go:26 GetFromStdin, survey.v1 selects).
// Answer sources, first match wins:
//   1. a preset answer for the prompt's key (a command-line flag, or its environment variable);
//   2. DEVSPACE_NONINTERACTIVE=1: stdin is never read, whatever it is; the default answer, or
//      an error naming the flag / variable that answers the question;
//   3. otherwise the next line of stdin (a terminal, or scripted answers piped in), the
//      default at EOF.
#pragma once

#include <termios.h>

#include <functional>
#include <stdexcept>
#include <string>
#include <vector>

namespace ds {
namespace prompt {

struct Params {
  std::string question;
  std::string default_value;
  std::string validation_regex;  // anchored implicitly like the reference (^...$)
  bool is_password = false;
  std::vector<std::string> options;  // select prompt when non-empty
  bool optional = false;  // no answer available (non-interactive, stdin at EOF) = "" instead of an error
  // Preset answers: set_answer(key, ...) (a flag) or the environment variable `env`. `hint`
  // names them in errors ("--image or DEVSPACE_INIT_IMAGE").
  std::string key;
  std::string env;
};

struct PromptError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

std::string ask(const Params& p);
std::string ask(const std::string& question, const std::string& def = "");
bool confirm(const std::string& question, bool def);
std::string select(const std::string& question, const std::vector<std::string>& options,
                   const std::string& def = "");

bool interactive();
// DEVSPACE_NONINTERACTIVE is set (to anything but 0): prompts never read stdin.
bool noninteractive_env();
// A flag's value answers the prompt with this key.
void set_answer(const std::string& key, const std::string& value);
bool has_answer(const std::string& key);
// Test hook: answers consumed in order instead of reading stdin.
void set_scripted_answers(const std::vector<std::string>& answers);

// Terminal mode saved by whoever puts stdin into raw mode, so a signal handler that ends the
// process can put the user's terminal back (tcsetattr is async-signal-safe).
void remember_cooked_tty(const struct termios& saved);
void forget_cooked_tty();
void restore_cooked_tty_from_signal();

}  // namespace prompt
}  // namespace ds

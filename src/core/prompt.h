// Interactive prompts (util/stdinutil/stdin.go:26 GetFromStdin, survey.v1 selects).
// Non-interactive runs (stdin not a TTY, or DEVSPACE_NONINTERACTIVE=1) take the default
// answer, or the next line from stdin when one is piped in; a prompt with neither fails.
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
// Test hook: answers consumed in order instead of reading stdin.
void set_scripted_answers(const std::vector<std::string>& answers);

// Terminal mode saved by whoever puts stdin into raw mode, so a signal handler that ends the
// process can put the user's terminal back (tcsetattr is async-signal-safe).
void remember_cooked_tty(const struct termios& saved);
void forget_cooked_tty();
void restore_cooked_tty_from_signal();

}  // namespace prompt
}  // namespace ds

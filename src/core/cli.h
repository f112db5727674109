// Minimal cobra-compatible command tree + flag parser (cmd/root.go:24 uses spf13/cobra).
// Supports: nested subcommands, aliases, long/short flags, "--f=v", "--f v", "-abc" bool
// clusters, "--bool=false", string slices (comma split, repeatable), "--" terminator,
// required flags, hidden/deprecated commands and generated help.
#pragma once

#include <functional>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace ds {
namespace cli {

struct Flag {
  enum Kind { String, Bool, Int, StringSlice } kind = String;
  std::string name;
  std::string shorthand;
  std::string usage;
  std::string def;  // textual default
  bool required = false;
  bool hidden = false;
  // values
  std::string s;
  bool b = false;
  long long i = 0;
  std::vector<std::string> list;
  bool changed = false;
};

class Command;
using RunFn = std::function<int(Command&, const std::vector<std::string>&)>;

class Command {
 public:
  Command(std::string use, std::string short_desc, std::string long_desc = "");
  Command& add(std::unique_ptr<Command> sub);
  Command* sub(const std::string& name);

  // Flag registration (returns *this for chaining)
  Command& str(const std::string& name, const std::string& sh, const std::string& def, const std::string& usage);
  Command& boolean(const std::string& name, const std::string& sh, bool def, const std::string& usage);
  Command& integer(const std::string& name, const std::string& sh, long long def, const std::string& usage);
  Command& slice(const std::string& name, const std::string& sh, const std::string& usage);
  Command& required(const std::string& name);
  Command& persistent_str(const std::string& name, const std::string& sh, const std::string& def,
                          const std::string& usage);
  Command& persistent_bool(const std::string& name, const std::string& sh, bool def, const std::string& usage);

  // Flag access after parsing
  const std::string& get_str(const std::string& name) const;
  bool get_bool(const std::string& name) const;
  long long get_int(const std::string& name) const;
  const std::vector<std::string>& get_slice(const std::string& name) const;
  bool changed(const std::string& name) const;
  Flag* flag(const std::string& name);
  const Flag* flag(const std::string& name) const;

  std::string name() const;
  const std::string& use() const { return use_; }
  std::string path() const;
  std::vector<std::string> aliases;
  std::string deprecated;
  bool hidden = false;
  // Positional arg validation: -1 = any
  int min_args = 0, max_args = -1;
  RunFn run;
  Command* parent = nullptr;

  std::string help() const;
  // Full dispatch from argv (argv[0] excluded). Returns process exit code.
  int execute(const std::vector<std::string>& args);
  const std::vector<std::unique_ptr<Command>>& subs() const { return subs_; }

 private:
  Flag* lookup_long(const std::string& n);
  Flag* lookup_short(const std::string& n);
  int parse_and_run(const std::vector<std::string>& args);
  std::string use_, short_, long_;
  std::vector<std::unique_ptr<Command>> subs_;
  std::vector<Flag> flags_;
  std::vector<Flag> persistent_;
};

struct UsageError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

}  // namespace cli
}  // namespace ds

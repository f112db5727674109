#include "core/cli.h"

#include <cstdio>
#include <iostream>
#include <stdexcept>

#include "core/strutil.h"

namespace ds {
namespace cli {

Command::Command(std::string use, std::string short_desc, std::string long_desc)
    : use_(std::move(use)), short_(std::move(short_desc)), long_(std::move(long_desc)) {}

Command& Command::add(std::unique_ptr<Command> sub) {
  sub->parent = this;
  subs_.push_back(std::move(sub));
  return *subs_.back();
}

Command* Command::sub(const std::string& name) {
  for (auto& s : subs_) {
    if (s->name() == name) return s.get();
    for (auto& a : s->aliases)
      if (a == name) return s.get();
  }
  return nullptr;
}

std::string Command::name() const {
  size_t sp = use_.find(' ');
  return sp == std::string::npos ? use_ : use_.substr(0, sp);
}

std::string Command::path() const { return parent ? parent->path() + " " + name() : name(); }

static Flag make_flag(Flag::Kind k, const std::string& name, const std::string& sh, const std::string& usage) {
  Flag f;
  f.kind = k;
  f.name = name;
  f.shorthand = sh;
  f.usage = usage;
  return f;
}

Command& Command::str(const std::string& name, const std::string& sh, const std::string& def,
                      const std::string& usage) {
  Flag f = make_flag(Flag::String, name, sh, usage);
  f.def = def;
  f.s = def;
  flags_.push_back(f);
  return *this;
}

Command& Command::boolean(const std::string& name, const std::string& sh, bool def, const std::string& usage) {
  Flag f = make_flag(Flag::Bool, name, sh, usage);
  f.def = def ? "true" : "false";
  f.b = def;
  flags_.push_back(f);
  return *this;
}

Command& Command::integer(const std::string& name, const std::string& sh, long long def, const std::string& usage) {
  Flag f = make_flag(Flag::Int, name, sh, usage);
  f.def = std::to_string(def);
  f.i = def;
  flags_.push_back(f);
  return *this;
}

Command& Command::slice(const std::string& name, const std::string& sh, const std::string& usage) {
  Flag f = make_flag(Flag::StringSlice, name, sh, usage);
  f.def = "[]";
  flags_.push_back(f);
  return *this;
}

Command& Command::required(const std::string& name) {
  Flag* f = flag(name);
  if (f) f->required = true;
  return *this;
}

Command& Command::persistent_str(const std::string& name, const std::string& sh, const std::string& def,
                                 const std::string& usage) {
  Flag f = make_flag(Flag::String, name, sh, usage);
  f.def = def;
  f.s = def;
  persistent_.push_back(f);
  return *this;
}

Command& Command::persistent_bool(const std::string& name, const std::string& sh, bool def,
                                  const std::string& usage) {
  Flag f = make_flag(Flag::Bool, name, sh, usage);
  f.def = def ? "true" : "false";
  f.b = def;
  persistent_.push_back(f);
  return *this;
}

Flag* Command::flag(const std::string& name) {
  for (auto& f : flags_)
    if (f.name == name) return &f;
  for (Command* c = this; c; c = c->parent)
    for (auto& f : c->persistent_)
      if (f.name == name) return &f;
  return nullptr;
}

const Flag* Command::flag(const std::string& name) const { return const_cast<Command*>(this)->flag(name); }

Flag* Command::lookup_long(const std::string& n) { return flag(n); }

Flag* Command::lookup_short(const std::string& n) {
  for (auto& f : flags_)
    if (f.shorthand == n) return &f;
  for (Command* c = this; c; c = c->parent)
    for (auto& f : c->persistent_)
      if (f.shorthand == n) return &f;
  return nullptr;
}

static const std::string kEmpty;
static const std::vector<std::string> kEmptyList;

const std::string& Command::get_str(const std::string& name) const {
  const Flag* f = flag(name);
  return f ? f->s : kEmpty;
}
bool Command::get_bool(const std::string& name) const {
  const Flag* f = flag(name);
  return f ? f->b : false;
}
long long Command::get_int(const std::string& name) const {
  const Flag* f = flag(name);
  return f ? f->i : 0;
}
const std::vector<std::string>& Command::get_slice(const std::string& name) const {
  const Flag* f = flag(name);
  return f ? f->list : kEmptyList;
}
bool Command::changed(const std::string& name) const {
  const Flag* f = flag(name);
  return f && f->changed;
}

static void set_value(Flag* f, const std::string& v) {
  f->changed = true;
  switch (f->kind) {
    case Flag::String: f->s = v; break;
    case Flag::Bool: {
      std::string l = to_lower(v);
      if (l == "true" || l == "1" || l == "t")
        f->b = true;
      else if (l == "false" || l == "0" || l == "f")
        f->b = false;
      else
        throw UsageError("invalid argument \"" + v + "\" for \"--" + f->name + "\" flag: strconv.ParseBool: parsing");
      break;
    }
    case Flag::Int: {
      int64_t iv;
      if (!parse_int64(v, &iv))
        throw UsageError("invalid argument \"" + v + "\" for \"--" + f->name + "\" flag: strconv.ParseInt: parsing");
      f->i = iv;
      break;
    }
    case Flag::StringSlice:
      for (auto& p : split(v, ","))
        if (!p.empty()) f->list.push_back(p);
      break;
  }
}

std::string Command::help() const {
  std::string out;
  std::string desc = long_.empty() ? short_ : long_;
  if (!desc.empty()) out += trim(desc) + "\n\n";
  out += "Usage:\n";
  bool has_subs = false;
  for (auto& s : subs_)
    if (!s->hidden) has_subs = true;
  std::string full = parent ? parent->path() + " " + use_ : use_;
  if (run) out += "  " + full + " [flags]\n";
  if (has_subs) out += "  " + path() + " [command]\n";
  if (!aliases.empty()) out += "\nAliases:\n  " + name() + ", " + join(aliases, ", ") + "\n";
  if (has_subs) {
    out += "\nAvailable Commands:\n";
    size_t w = 0;
    for (auto& s : subs_)
      if (!s->hidden) w = std::max(w, s->name().size());
    for (auto& s : subs_) {
      if (s->hidden) continue;
      out += "  " + s->name() + std::string(w - s->name().size() + 3, ' ') + s->short_ + "\n";
    }
  }
  auto fmt_flags = [&](const std::vector<Flag>& fl, const std::string& title) {
    if (fl.empty()) return;
    out += "\n" + title + ":\n";
    std::vector<std::pair<std::string, std::string>> rows;
    size_t w = 0;
    for (auto& f : fl) {
      if (f.hidden) continue;
      std::string left = f.shorthand.empty() ? "      --" + f.name : "  -" + f.shorthand + ", --" + f.name;
      if (f.kind == Flag::String) left += " string";
      if (f.kind == Flag::Int) left += " int";
      if (f.kind == Flag::StringSlice) left += " strings";
      std::string right = f.usage;
      if (f.kind == Flag::Bool && f.def == "true") right += " (default true)";
      if (f.kind == Flag::String && !f.def.empty()) right += " (default \"" + f.def + "\")";
      if (f.kind == Flag::Int && f.def != "0") right += " (default " + f.def + ")";
      if (f.required) right += " (required)";
      w = std::max(w, left.size());
      rows.emplace_back(left, right);
    }
    for (auto& r : rows) out += r.first + std::string(w - r.first.size() + 3, ' ') + r.second + "\n";
  };
  fmt_flags(flags_, "Flags");
  std::vector<Flag> inherited;
  for (const Command* c = this; c; c = c->parent)
    for (auto& f : c->persistent_) inherited.push_back(f);
  fmt_flags(inherited, "Global Flags");
  if (has_subs) out += "\nUse \"" + path() + " [command] --help\" for more information about a command.\n";
  return out;
}

int Command::execute(const std::vector<std::string>& args) {
  // Walk down the subcommand tree using leading non-flag args.
  Command* cur = this;
  std::vector<std::string> rest;
  size_t i = 0;
  // Find subcommand path: first non-flag tokens that name subcommands
  std::vector<std::string> pre_flags;
  for (; i < args.size(); ++i) {
    const std::string& a = args[i];
    if (a == "--") break;
    if (starts_with(a, "-")) {
      pre_flags.push_back(a);
      // flag with separate value: peek if it takes a value
      Flag* f = nullptr;
      if (starts_with(a, "--") && a.find('=') == std::string::npos)
        f = cur->lookup_long(a.substr(2));
      else if (!starts_with(a, "--") && a.size() == 2)
        f = cur->lookup_short(a.substr(1));
      if (f && f->kind != Flag::Bool && i + 1 < args.size()) pre_flags.push_back(args[++i]);
      continue;
    }
    Command* s = cur->sub(a);
    if (!s) break;
    cur = s;
  }
  for (auto& p : pre_flags) rest.push_back(p);
  for (; i < args.size(); ++i) rest.push_back(args[i]);
  try {
    return cur->parse_and_run(rest);
  } catch (const UsageError& e) {
    std::fprintf(stderr, "Error: %s\n%s", e.what(), cur->help().c_str());
    return 1;
  }
}

int Command::parse_and_run(const std::vector<std::string>& args) {
  std::vector<std::string> positional;
  bool want_help = false;
  for (size_t i = 0; i < args.size(); ++i) {
    const std::string& a = args[i];
    if (a == "--") {
      for (size_t j = i + 1; j < args.size(); ++j) positional.push_back(args[j]);
      break;
    }
    if (a == "--help" || a == "-h") {
      want_help = true;
      continue;
    }
    if (starts_with(a, "--")) {
      std::string body = a.substr(2);
      std::string val;
      bool has_val = false;
      size_t eq = body.find('=');
      if (eq != std::string::npos) {
        val = body.substr(eq + 1);
        body = body.substr(0, eq);
        has_val = true;
      }
      Flag* f = lookup_long(body);
      if (!f) throw UsageError("unknown flag: --" + body);
      if (f->kind == Flag::Bool) {
        set_value(f, has_val ? val : "true");
      } else {
        if (!has_val) {
          if (i + 1 >= args.size()) throw UsageError("flag needs an argument: --" + body);
          val = args[++i];
        }
        set_value(f, val);
      }
      continue;
    }
    if (starts_with(a, "-") && a.size() > 1) {
      // cluster of shorthands
      for (size_t k = 1; k < a.size(); ++k) {
        std::string sh(1, a[k]);
        Flag* f = lookup_short(sh);
        if (!f) throw UsageError("unknown shorthand flag: '" + sh + "' in " + a);
        if (f->kind == Flag::Bool) {
          if (k + 1 < a.size() && a[k + 1] == '=') {
            set_value(f, a.substr(k + 2));
            break;
          }
          set_value(f, "true");
        } else {
          std::string val;
          if (k + 1 < a.size()) {
            val = a.substr(k + 1);
            if (starts_with(val, "=")) val = val.substr(1);
          } else {
            if (i + 1 >= args.size()) throw UsageError("flag needs an argument: '" + sh + "' in " + a);
            val = args[++i];
          }
          set_value(f, val);
          break;
        }
      }
      continue;
    }
    positional.push_back(a);
  }
  if (want_help || (!run && positional.empty())) {
    std::fputs(help().c_str(), stdout);
    return 0;
  }
  if (!run) {
    throw UsageError("unknown command \"" + positional[0] + "\" for \"" + path() + "\"");
  }
  for (auto& f : flags_)
    if (f.required && !f.changed) throw UsageError("required flag(s) \"" + f.name + "\" not set");
  if ((int)positional.size() < min_args)
    throw UsageError("requires at least " + std::to_string(min_args) + " arg(s), only received " +
                     std::to_string(positional.size()));
  if (max_args >= 0 && (int)positional.size() > max_args) {
    if (max_args == 0) throw UsageError("unknown command \"" + positional[0] + "\" for \"" + path() + "\"");
    throw UsageError("accepts at most " + std::to_string(max_args) + " arg(s), received " +
                     std::to_string(positional.size()));
  }
  if (!deprecated.empty()) std::fprintf(stderr, "Command \"%s\" is deprecated, %s\n", name().c_str(), deprecated.c_str());
  return run(*this, positional);
}

}  // namespace cli
}  // namespace ds

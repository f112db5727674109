#include "deploy/gotemplate.h"

#include "core/resolve.h"

#include <arpa/inet.h>
#include <netdb.h>

#include <algorithm>
#include <map>
#include <cmath>
#include <cstring>
#include <ctime>
#include <regex>
#include <sstream>
#include <vector>

#include <openssl/evp.h>
#include <zlib.h>

#include "core/codec.h"
#include "core/match.h"
#include "core/safe_regex.h"
#include "core/strutil.h"
#include "deploy/sprig_crypto.h"

namespace ds {
namespace tmpl {

// ============================================================== lexer for actions

namespace {

enum class T { Ident, Field, Var, Str, Num, Bool, Nil, LParen, RParen, Pipe, Declare, Assign, Comma, Dot, End };

struct Tok {
  T t;
  std::string s;
};

std::vector<Tok> lex_action(const std::string& a) {
  std::vector<Tok> out;
  size_t i = 0;
  auto is_id = [](char c) { return std::isalnum((unsigned char)c) || c == '_'; };
  while (i < a.size()) {
    char c = a[i];
    if (std::isspace((unsigned char)c)) {
      ++i;
      continue;
    }
    if (c == '(') {
      out.push_back({T::LParen, "("});
      ++i;
    } else if (c == ')') {
      out.push_back({T::RParen, ")"});
      ++i;
      // field chain after a paren: ").Foo"
    } else if (c == '|') {
      out.push_back({T::Pipe, "|"});
      ++i;
    } else if (c == ',') {
      out.push_back({T::Comma, ","});
      ++i;
    } else if (c == ':' && i + 1 < a.size() && a[i + 1] == '=') {
      out.push_back({T::Declare, ":="});
      i += 2;
    } else if (c == '=') {
      out.push_back({T::Assign, "="});
      ++i;
    } else if (c == '"') {
      std::string s;
      ++i;
      while (i < a.size() && a[i] != '"') {
        if (a[i] == '\\' && i + 1 < a.size()) {
          char e = a[++i];
          switch (e) {
            case 'n': s.push_back('\n'); break;
            case 't': s.push_back('\t'); break;
            case 'r': s.push_back('\r'); break;
            case '\\': s.push_back('\\'); break;
            case '"': s.push_back('"'); break;
            default: s.push_back('\\'); s.push_back(e);
          }
          ++i;
          continue;
        }
        s.push_back(a[i++]);
      }
      ++i;
      out.push_back({T::Str, s});
    } else if (c == '`') {
      size_t e = a.find('`', i + 1);
      if (e == std::string::npos) throw TemplateError("unterminated raw string");
      out.push_back({T::Str, a.substr(i + 1, e - i - 1)});
      i = e + 1;
    } else if (c == '\'') {
      // char constant -> number
      size_t e = a.find('\'', i + 1);
      out.push_back({T::Num, std::to_string((int)(unsigned char)a[i + 1])});
      i = e + 1;
    } else if (c == '.' ) {
      if (i + 1 < a.size() && is_id(a[i + 1]) && !std::isdigit((unsigned char)a[i + 1])) {
        size_t e = i + 1;
        while (e < a.size() && (is_id(a[e]) || (a[e] == '.' && e + 1 < a.size() && is_id(a[e + 1])))) ++e;
        out.push_back({T::Field, a.substr(i, e - i)});
        i = e;
      } else if (i + 1 < a.size() && std::isdigit((unsigned char)a[i + 1])) {
        size_t e = i + 1;
        while (e < a.size() && (std::isdigit((unsigned char)a[e]) || a[e] == 'e')) ++e;
        out.push_back({T::Num, "0" + a.substr(i, e - i)});
        i = e;
      } else {
        out.push_back({T::Dot, "."});
        ++i;
      }
    } else if (c == '$') {
      size_t e = i + 1;
      while (e < a.size() && (is_id(a[e]) || (a[e] == '.' && e + 1 < a.size() && is_id(a[e + 1])))) ++e;
      out.push_back({T::Var, a.substr(i, e - i)});
      i = e;
    } else if (std::isdigit((unsigned char)c) || ((c == '-' || c == '+') && i + 1 < a.size() && std::isdigit((unsigned char)a[i + 1]))) {
      size_t e = i + 1;
      while (e < a.size() && (std::isalnum((unsigned char)a[e]) || a[e] == '.' || a[e] == '_' ||
                              ((a[e] == '-' || a[e] == '+') && (a[e - 1] == 'e' || a[e - 1] == 'E'))))
        ++e;
      out.push_back({T::Num, a.substr(i, e - i)});
      i = e;
    } else if (is_id(c)) {
      size_t e = i;
      while (e < a.size() && is_id(a[e])) ++e;
      std::string id = a.substr(i, e - i);
      if (id == "true" || id == "false")
        out.push_back({T::Bool, id});
      else if (id == "nil")
        out.push_back({T::Nil, id});
      else
        out.push_back({T::Ident, id});
      i = e;
    } else {
      throw TemplateError(std::string("unexpected character '") + c + "' in action: " + a);
    }
  }
  out.push_back({T::End, ""});
  return out;
}

// ============================================================== AST

struct Pipeline;
struct Arg {
  enum Kind { Field, Var, Lit, Ident, Sub, Dot } kind;
  std::string name;  // field chain ".a.b", var "$x.a", ident
  Value lit;
  std::shared_ptr<Pipeline> sub;
  std::string chain;  // field chain applied after a sub-pipeline
};

struct Command {
  std::vector<Arg> args;
};

struct Pipeline {
  std::vector<std::string> decl;  // variable names
  bool assign = false;            // "=" instead of ":="
  std::vector<Command> cmds;
};

struct Node {
  enum Kind { Text, Action, If, Range, With, Template, List, Break, Continue } kind;
  std::string text;
  std::shared_ptr<Pipeline> pipe;
  std::vector<std::shared_ptr<Node>> body, else_body;
  std::string name;  // template name
};
using NodeP = std::shared_ptr<Node>;

class PipeParser {
 public:
  explicit PipeParser(std::vector<Tok> toks) : t_(std::move(toks)) {}
  std::shared_ptr<Pipeline> parse_pipeline(bool allow_decl = true) {
    auto p = std::make_shared<Pipeline>();
    if (allow_decl) {
      // lookahead: $a [, $b] := | =
      size_t save = i_;
      std::vector<std::string> vars;
      while (t_[i_].t == T::Var) {
        vars.push_back(t_[i_].s);
        ++i_;
        if (t_[i_].t == T::Comma) {
          ++i_;
          continue;
        }
        break;
      }
      if (!vars.empty() && (t_[i_].t == T::Declare || t_[i_].t == T::Assign)) {
        p->assign = t_[i_].t == T::Assign;
        p->decl = vars;
        ++i_;
      } else {
        i_ = save;
      }
    }
    while (true) {
      Command c;
      while (t_[i_].t != T::Pipe && t_[i_].t != T::End && t_[i_].t != T::RParen) c.args.push_back(parse_arg());
      if (c.args.empty()) throw TemplateError("missing value for command");
      p->cmds.push_back(std::move(c));
      if (t_[i_].t == T::Pipe) {
        ++i_;
        continue;
      }
      break;
    }
    return p;
  }
  bool at_end() const { return t_[i_].t == T::End; }
  const Tok& peek() const { return t_[i_]; }
  Tok next() { return t_[i_++]; }

 private:
  Arg parse_arg() {
    const Tok& k = t_[i_++];
    Arg a;
    switch (k.t) {
      case T::Field: a.kind = Arg::Field; a.name = k.s; break;
      case T::Var: a.kind = Arg::Var; a.name = k.s; break;
      case T::Dot: a.kind = Arg::Dot; break;
      case T::Ident: a.kind = Arg::Ident; a.name = k.s; break;
      case T::Str: {
        a.kind = Arg::Lit;
        a.lit = Value(k.s);
        a.lit.set_quoted(true);
        break;
      }
      case T::Num: {
        a.kind = Arg::Lit;
        int64_t iv;
        double dv;
        std::string s = k.s;
        if (parse_int64(s, &iv))
          a.lit = Value(iv);
        else if (starts_with(s, "0x") || starts_with(s, "0X"))
          a.lit = Value((int64_t)std::strtoll(s.c_str() + 2, nullptr, 16));
        else if (parse_double(s, &dv))
          a.lit = Value(dv);
        else
          throw TemplateError("bad number: " + s);
        break;
      }
      case T::Bool: a.kind = Arg::Lit; a.lit = Value(k.s == "true"); break;
      case T::Nil: a.kind = Arg::Lit; break;
      case T::LParen: {
        a.kind = Arg::Sub;
        a.sub = parse_pipeline(false);
        if (t_[i_].t != T::RParen) throw TemplateError("unclosed parenthesis");
        ++i_;
        if (t_[i_].t == T::Field) a.chain = t_[i_++].s;
        break;
      }
      default: throw TemplateError("unexpected token '" + k.s + "' in pipeline");
    }
    return a;
  }
  std::vector<Tok> t_;
  size_t i_ = 0;
};

struct Segment {
  bool action;
  std::string s;
};

std::vector<Segment> split_segments(const std::string& src) {
  std::vector<Segment> out;
  size_t i = 0;
  bool trim_next = false;
  while (i < src.size()) {
    size_t open = src.find("{{", i);
    std::string text = src.substr(i, open == std::string::npos ? std::string::npos : open - i);
    if (trim_next) text = trim_left(text, " \t\r\n");
    if (open == std::string::npos) {
      out.push_back({false, text});
      break;
    }
    size_t body_start = open + 2;
    bool trim_left_ws = body_start + 1 < src.size() && src[body_start] == '-' &&
                        (src[body_start + 1] == ' ' || src[body_start + 1] == '\t' || src[body_start + 1] == '\n');
    if (trim_left_ws) {
      text = trim_right(text, " \t\r\n");
      body_start += 1;
    }
    out.push_back({false, text});
    // find closing "}}" outside string literals
    size_t j = body_start;
    char q = 0;
    while (j + 1 < src.size()) {
      char c = src[j];
      if (q) {
        if (c == '\\' && q == '"') {
          j += 2;
          continue;
        }
        if (c == q) q = 0;
        ++j;
        continue;
      }
      if (c == '"' || c == '`') {
        q = c;
        ++j;
        continue;
      }
      if (c == '}' && src[j + 1] == '}') break;
      ++j;
    }
    if (j + 1 >= src.size()) throw TemplateError("unclosed action");
    size_t body_end = j;
    trim_next = false;
    if (body_end > body_start && src[body_end - 1] == '-' && body_end >= 2 &&
        (src[body_end - 2] == ' ' || src[body_end - 2] == '\t' || src[body_end - 2] == '\n')) {
      trim_next = true;
      body_end -= 1;
    }
    out.push_back({true, src.substr(body_start, body_end - body_start)});
    i = j + 2;
  }
  return out;
}

}  // namespace


// ============================================================== Helm objects with methods

namespace {

const char* const kObjTag = "\x01obj";
const char* const kObjData = "\x01" "data";

bool is_obj(const Value& v, const char* kind) {
  if (!v.is_map()) return false;
  const Value* t = v.find(kObjTag);
  return t && t->str() == kind;
}

std::string base_name(const std::string& p) {
  size_t s = p.rfind('/');
  return s == std::string::npos ? p : p.substr(s + 1);
}

// toYAML of a map[string]string (Files.AsConfig / AsSecrets): keys sorted like yaml.Marshal.
std::string yaml_string_map(std::vector<std::pair<std::string, std::string>> kv) {
  std::sort(kv.begin(), kv.end());
  Value m = Value::map();
  for (auto& e : kv) {
    Value v(e.second);
    v.set_quoted(true);
    m[e.first] = v;
  }
  if (kv.empty()) return "{}";
  std::string y = yaml_dump(m);
  if (ends_with(y, "\n")) y.pop_back();
  return y;
}

// Method call on a Helm object; *found=false when `recv` has no such method.
Value call_method(const Value& recv, const std::string& name, const std::vector<Value>& args, bool* found) {
  *found = true;
  auto need = [&](size_t n) {
    if (args.size() != n)
      throw TemplateError("wrong number of args for " + name + ": want " + std::to_string(n) + " got " +
                          std::to_string(args.size()));
  };
  if (is_obj(recv, "files")) {
    const Value& data = recv.get(kObjData);
    if (name == "Get" || name == "GetBytes") {
      need(1);
      return Value(data.get(args[0].as_string()).as_string());
    }
    if (name == "Lines") {
      need(1);
      const Value* f = data.find(args[0].as_string());
      if (!f || f->str().empty()) return Value::seq();
      std::string t = f->str();
      if (t.back() == '\n') t.pop_back();
      return Value::strings(split(t, "\n"));
    }
    if (name == "Glob") {
      need(1);
      std::vector<std::pair<std::string, std::string>> sel;
      for (auto& e : data.entries())
        if (glob_match(args[0].as_string(), e.first)) sel.emplace_back(e.first, e.second.str());
      return make_files_object(sel);
    }
    if (name == "AsConfig" || name == "AsSecrets") {
      need(0);
      std::vector<std::pair<std::string, std::string>> kv;
      for (auto& e : data.entries())
        kv.emplace_back(base_name(e.first), name == "AsConfig" ? e.second.str() : base64_encode(e.second.str()));
      return Value(yaml_string_map(std::move(kv)));
    }
  } else if (is_obj(recv, "apiversions")) {
    if (name == "Has") {
      need(1);
      for (auto& v : recv.get(kObjData).items())
        if (v.str() == args[0].as_string()) return Value(true);
      return Value(false);
    }
  }
  *found = false;
  return Value();
}

// "v1.2.3-rc.1+meta" -> (1, 2, 3, "rc.1"); missing / x components are 0
struct Semver {
  int64_t major = 0, minor = 0, patch = 0;
  std::string pre;
  bool ok = false;
};

Semver parse_semver(std::string v) {
  Semver s;
  v = trim(v);
  if (!v.empty() && (v[0] == 'v' || v[0] == 'V')) v.erase(0, 1);
  size_t plus = v.find('+');
  if (plus != std::string::npos) v = v.substr(0, plus);
  size_t dash = v.find('-');
  if (dash != std::string::npos) {
    s.pre = v.substr(dash + 1);
    v = v.substr(0, dash);
  }
  auto parts = split(v, ".");
  if (parts.empty() || parts.size() > 3) return s;
  int64_t* dst[3] = {&s.major, &s.minor, &s.patch};
  for (size_t i = 0; i < parts.size(); ++i) {
    if (parts[i] == "x" || parts[i] == "X" || parts[i] == "*") continue;
    if (!parse_int64(parts[i], dst[i])) return s;
  }
  s.ok = true;
  return s;
}

int semver_cmp(const Semver& a, const Semver& b) {
  if (a.major != b.major) return a.major < b.major ? -1 : 1;
  if (a.minor != b.minor) return a.minor < b.minor ? -1 : 1;
  if (a.patch != b.patch) return a.patch < b.patch ? -1 : 1;
  if (a.pre == b.pre) return 0;
  if (a.pre.empty()) return 1;  // 1.0.0 > 1.0.0-rc
  if (b.pre.empty()) return -1;
  return a.pre < b.pre ? -1 : 1;
}

// Masterminds/semver constraint check: comma (AND) and "||" (OR) lists of
// =, !=, >, <, >=, <=, ~ (patch-level), ^ (major-level), x-ranges and "a - b" ranges.
// As Helm does for Capabilities checks, a prerelease version satisfies only constraints
// that name a prerelease — except that the "-0" idiom (">=1.19-0") admits all prereleases.
bool semver_satisfies(const std::string& constraint, const std::string& version) {
  Semver v = parse_semver(version);
  if (!v.ok) throw TemplateError("invalid semantic version: " + version);
  for (auto& alt : split(constraint, "||")) {
    bool all = true;
    std::string a = trim(alt);
    // hyphen range "1.2 - 1.4.5"
    size_t hy = a.find(" - ");
    std::vector<std::string> terms;
    if (hy != std::string::npos) {
      terms.push_back(">=" + trim(a.substr(0, hy)));
      terms.push_back("<=" + trim(a.substr(hy + 3)));
    } else {
      for (auto& t : split(a, ",")) {
        // space-separated terms are ANDed too (">= 1.2 < 2")
        std::string cur;
        std::string tt = trim(t);
        for (size_t i = 0; i < tt.size(); ++i) {
          char c = tt[i];
          if (c == ' ' && !cur.empty() && !std::strchr("<>=!~^", cur.back())) {
            terms.push_back(cur);
            cur.clear();
          } else if (c != ' ') {
            cur.push_back(c);
          }
        }
        if (!cur.empty()) terms.push_back(cur);
      }
    }
    for (auto& term : terms) {
      std::string op;
      std::string t = term;
      while (!t.empty() && std::strchr("<>=!~^", t[0])) op.push_back(t[0]), t.erase(0, 1);
      Semver c = parse_semver(t);
      if (!c.ok) throw TemplateError("improper constraint: " + term);
      std::string tv = trim(t);
      if (!tv.empty() && (tv[0] == 'v' || tv[0] == 'V')) tv.erase(0, 1);
      int given = 0;  // how many components were spelled (x-ranges count as not given)
      for (auto& p : split(tv.substr(0, tv.find_first_of("-+")), ".")) {
        if (p == "x" || p == "X" || p == "*") break;
        ++given;
      }
      if (!v.pre.empty() && c.pre.empty()) {
        all = false;  // prerelease versions only match prerelease constraints
        break;
      }
      int r = semver_cmp(v, c);
      bool ok;
      if (op.empty() || op == "=" || op == "==") {
        if (given >= 3) ok = r == 0;
        else if (given == 2) ok = v.major == c.major && v.minor == c.minor;
        else if (given == 1) ok = v.major == c.major;
        else ok = true;
      } else if (op == "!=") ok = r != 0;
      else if (op == ">") {
        if (given == 2) ok = v.major > c.major || (v.major == c.major && v.minor > c.minor);
        else if (given == 1) ok = v.major > c.major;
        else ok = r > 0;
      } else if (op == ">=" || op == "=>") ok = r >= 0;
      else if (op == "<") ok = r < 0;
      else if (op == "<=" || op == "=<") {
        if (given == 2) ok = v.major < c.major || (v.major == c.major && v.minor <= c.minor);
        else if (given == 1) ok = v.major <= c.major;
        else ok = r <= 0;
      } else if (op == "~" || op == "~>") {
        ok = r >= 0 && v.major == c.major && (given <= 1 || v.minor == c.minor);
      } else if (op == "^") {
        if (c.major > 0) ok = r >= 0 && v.major == c.major;
        else if (c.minor > 0 || given < 3) ok = r >= 0 && v.major == 0 && (given < 2 || v.minor == c.minor);
        else ok = r >= 0 && v.major == 0 && v.minor == 0 && v.patch == c.patch;
      } else {
        throw TemplateError("improper constraint: " + term);
      }
      if (!ok) {
        all = false;
        break;
      }
    }
    if (all) return true;
  }
  return false;
}

std::string digest_hex(const EVP_MD* md, const std::string& data) {
  unsigned char out[EVP_MAX_MD_SIZE];
  unsigned int n = 0;
  EVP_Digest(data.data(), data.size(), out, &n, md, nullptr);
  return hex_encode(std::string((const char*)out, n));
}

std::string b32_encode(const std::string& in) {
  static const char* A = "ABCDEFGHIJKLMNOPQRSTUVWXYZ234567";
  std::string out;
  size_t i = 0;
  while (i < in.size()) {
    unsigned char b[5] = {0, 0, 0, 0, 0};
    size_t n = std::min<size_t>(5, in.size() - i);
    for (size_t k = 0; k < n; ++k) b[k] = (unsigned char)in[i + k];
    uint64_t x = 0;
    for (int k = 0; k < 5; ++k) x = (x << 8) | b[k];
    static const size_t chars_for[6] = {0, 2, 4, 5, 7, 8};
    for (size_t k = 0; k < 8; ++k) out.push_back(k < chars_for[n] ? A[(x >> (35 - 5 * k)) & 31] : '=');
    i += n;
  }
  return out;
}

std::string b32_decode(const std::string& in) {
  std::string out;
  uint64_t buf = 0;
  int bits = 0;
  for (char c : in) {
    int v;
    if (c >= 'A' && c <= 'Z') v = c - 'A';
    else if (c >= '2' && c <= '7') v = c - '2' + 26;
    else if (c == '=') break;
    else throw TemplateError("illegal base32 data");
    buf = (buf << 5) | (uint64_t)v;
    bits += 5;
    if (bits >= 8) {
      bits -= 8;
      out.push_back((char)((buf >> bits) & 0xff));
    }
  }
  return out;
}

// Sprig's word splitting for camelcase/snakecase/kebabcase.
std::vector<std::string> words_of(const std::string& s) {
  std::vector<std::string> w;
  std::string cur;
  for (size_t i = 0; i < s.size(); ++i) {
    char c = s[i];
    if (c == '_' || c == '-' || c == ' ' || c == '.') {
      if (!cur.empty()) w.push_back(cur), cur.clear();
      continue;
    }
    if (std::isupper((unsigned char)c) && !cur.empty() &&
        (std::islower((unsigned char)cur.back()) ||
         (i + 1 < s.size() && std::islower((unsigned char)s[i + 1]) && std::isupper((unsigned char)cur.back()))))
      w.push_back(cur), cur.clear();
    cur.push_back(c);
  }
  if (!cur.empty()) w.push_back(cur);
  return w;
}

std::string path_clean(const std::string& p) {
  if (p.empty()) return ".";
  bool abs = p[0] == '/';
  std::vector<std::string> out;
  for (auto& seg : split(p, "/")) {
    if (seg.empty() || seg == ".") continue;
    if (seg == "..") {
      if (!out.empty() && out.back() != "..") out.pop_back();
      else if (!abs) out.push_back("..");
      continue;
    }
    out.push_back(seg);
  }
  std::string r = (abs ? "/" : "") + join(out, "/");
  return r.empty() ? "." : r;
}

std::string toml_scalar(const Value& v) {
  if (v.is_string()) {
    std::string o = "\"";
    for (char c : v.str()) {
      if (c == '"' || c == '\\') o.push_back('\\');
      if (c == '\n') {
        o += "\\n";
        continue;
      }
      o.push_back(c);
    }
    return o + "\"";
  }
  if (v.is_seq()) {
    std::vector<std::string> parts;
    for (auto& it : v.items()) parts.push_back(toml_scalar(it));
    return "[" + join(parts, ", ") + "]";
  }
  return v.as_string();
}

void toml_table(const Value& m, const std::string& prefix, std::string& out) {
  std::vector<std::string> subs;
  for (auto& e : m.entries()) {
    if (e.second.is_map()) {
      subs.push_back(e.first);
      continue;
    }
    if (e.second.is_null()) continue;
    out += e.first + " = " + toml_scalar(e.second) + "\n";
  }
  for (auto& k : subs) {
    std::string name = prefix.empty() ? k : prefix + "." + k;
    out += "\n[" + name + "]\n";
    toml_table(m.get(k), name, out);
  }
}

}  // namespace

bool semver_match(const std::string& constraint, const std::string& version) {
  return semver_satisfies(constraint, version);
}

Value make_files_object(const std::vector<std::pair<std::string, std::string>>& files) {
  Value o = Value::map();
  o[kObjTag] = "files";
  Value d = Value::map();
  for (auto& f : files) d[f.first] = f.second;
  o[kObjData] = d;
  return o;
}

Value make_api_versions_object(const std::vector<std::string>& versions) {
  Value o = Value::map();
  o[kObjTag] = "apiversions";
  o[kObjData] = Value::strings(versions);
  return o;
}

// ============================================================== engine

struct LoopBreak {};
struct LoopContinue {};

struct Engine::Impl {
  std::map<std::string, std::vector<NodeP>> templates;
  Engine* owner = nullptr;

  // ---------------------------------------------------------- parse
  std::vector<NodeP> parse(const std::string& name, const std::string& src) {
    auto segs = split_segments(src);
    size_t pos = 0;
    std::string stop;
    auto body = parse_list(name, segs, pos, &stop);
    if (!stop.empty()) throw TemplateError(name + ": unexpected {{" + stop + "}}");
    return body;
  }

  // Parses until {{end}} / {{else ...}}; the terminating keyword action text goes to *stop.
  std::vector<NodeP> parse_list(const std::string& tname, const std::vector<Segment>& segs, size_t& pos,
                                std::string* stop) {
    std::vector<NodeP> out;
    while (pos < segs.size()) {
      const Segment& s = segs[pos++];
      if (!s.action) {
        if (!s.s.empty()) {
          auto n = std::make_shared<Node>();
          n->kind = Node::Text;
          n->text = s.s;
          out.push_back(n);
        }
        continue;
      }
      std::string a = trim(s.s);
      if (starts_with(a, "/*")) continue;  // comment
      std::string kw = a.substr(0, a.find_first_of(" \t\n("));
      if (kw == "end" || kw == "else") {
        *stop = a;
        return out;
      }
      if (a == "break" || a == "continue") {  // Go 1.18: only valid inside {{range}}
        auto n = std::make_shared<Node>();
        n->kind = a == "break" ? Node::Break : Node::Continue;
        out.push_back(n);
        continue;
      }
      if (kw == "if" || kw == "with" || kw == "range") {
        out.push_back(parse_control(tname, kw, a.substr(kw.size()), segs, pos));
        continue;
      }
      if (kw == "define" || kw == "block") {
        PipeParser pp(lex_action(a.substr(kw.size())));
        Tok nm = pp.next();
        if (nm.t != T::Str) throw TemplateError("define requires a name");
        std::string st;
        auto body = parse_list(tname, segs, pos, &st);
        if (trim(st) != "end") throw TemplateError("define " + nm.s + " missing end");
        templates[nm.s] = body;
        if (kw == "block") {
          auto n = std::make_shared<Node>();
          n->kind = Node::Template;
          n->name = nm.s;
          n->pipe = pp.at_end() ? nullptr : pp.parse_pipeline(false);
          out.push_back(n);
        }
        continue;
      }
      if (kw == "template") {
        PipeParser pp(lex_action(a.substr(kw.size())));
        Tok nm = pp.next();
        if (nm.t != T::Str) throw TemplateError("template requires a name");
        auto n = std::make_shared<Node>();
        n->kind = Node::Template;
        n->name = nm.s;
        n->pipe = pp.at_end() ? nullptr : pp.parse_pipeline(false);
        out.push_back(n);
        continue;
      }
      auto n = std::make_shared<Node>();
      n->kind = Node::Action;
      PipeParser pp(lex_action(a));
      n->pipe = pp.parse_pipeline(true);
      if (!pp.at_end()) throw TemplateError("unexpected '" + pp.peek().s + "' in action: " + a);
      out.push_back(n);
    }
    if (stop) stop->clear();
    return out;
  }

  NodeP parse_control(const std::string& tname, const std::string& kw, const std::string& rest,
                      const std::vector<Segment>& segs, size_t& pos) {
    auto n = std::make_shared<Node>();
    n->kind = kw == "if" ? Node::If : kw == "with" ? Node::With : Node::Range;
    PipeParser pp(lex_action(rest));
    n->pipe = pp.parse_pipeline(true);
    std::string st;
    n->body = parse_list(tname, segs, pos, &st);
    if (st.empty()) throw TemplateError(tname + ": unexpected EOF in " + kw);
    if (trim(st) == "end") return n;
    // else / else if / else with
    std::string after = trim(trim(st).substr(4));
    if (after.empty()) {
      std::string st2;
      n->else_body = parse_list(tname, segs, pos, &st2);
      if (trim(st2) != "end") throw TemplateError(tname + ": expected end after else");
      return n;
    }
    std::string kw2 = after.substr(0, after.find_first_of(" \t\n("));
    if (kw2 == "if" || kw2 == "with") {
      // "else if" chains share a single end
      n->else_body.push_back(parse_control(tname, kw2, after.substr(kw2.size()), segs, pos));
      return n;
    }
    throw TemplateError(tname + ": bad else clause: " + st);
  }

  // ---------------------------------------------------------- evaluation

  struct Scope {
    std::vector<std::pair<std::string, Value>> vars;
    Value dot;
  };

  static bool truth(const Value& v) {
    switch (v.type()) {
      case Value::Type::Null: return false;
      case Value::Type::Bool: return v.as_bool();
      case Value::Type::Int: return v.as_int() != 0;
      case Value::Type::Float: return v.as_double() != 0;
      case Value::Type::String: return !v.str().empty();
      case Value::Type::Seq: return v.size() > 0;
      case Value::Type::Map: return v.size() > 0;
    }
    return false;
  }

  static std::string fmt_float(double d) {
    if (d == std::floor(d) && std::fabs(d) < 1e21) {
      if (std::fabs(d) >= 1e21) return strfmt("%g", d);
      return strfmt("%.0f", d);
    }
    for (int p = 1; p <= 17; ++p) {
      std::string s = strfmt("%.*g", p, d);
      if (std::strtod(s.c_str(), nullptr) == d) return s;
    }
    return strfmt("%g", d);
  }

  static std::string print_value(const Value& v) {
    switch (v.type()) {
      case Value::Type::Null: return "";
      case Value::Type::Float: return fmt_float(v.as_double());
      case Value::Type::Seq: {
        std::vector<std::string> parts;
        for (auto& it : v.items()) parts.push_back(it.is_null() ? "<nil>" : print_value(it));
        return "[" + join(parts, " ") + "]";
      }
      case Value::Type::Map: {
        auto keys = v.keys();
        std::sort(keys.begin(), keys.end());
        std::vector<std::string> parts;
        for (auto& k : keys) parts.push_back(k + ":" + print_value(v.get(k)));
        return "map[" + join(parts, " ") + "]";
      }
      default: return v.as_string();
    }
  }

  static Value field_chain(Value cur, const std::string& chain) {
    for (auto& part : split(chain, ".")) {
      if (part.empty()) continue;
      if (cur.is_map()) {
        const Value* n = cur.find(part);
        if (!n && cur.has(kObjTag)) {  // niladic method: (.Files.Glob "x").AsConfig
          bool found = false;
          Value r = call_method(cur, part, {}, &found);
          if (found) {
            cur = r;
            continue;
          }
        }
        cur = n ? *n : Value();
      } else {
        return Value();  // missingkey=zero semantics (Helm)
      }
    }
    return cur;
  }

  // `.Files.Get "x"` / `$.Capabilities.APIVersions.Has "v"`: the command's first word is a
  // field chain ending in a method of a Helm object. Returns false if it is not a method call.
  bool try_method_call(Scope& sc, const Arg& first, std::vector<Value>& args, Value* out) {
    std::string chain;
    Value base;
    if (first.kind == Arg::Field) {
      chain = first.name;
      base = sc.dot;
    } else if (first.kind == Arg::Var) {
      size_t d = first.name.find('.');
      if (d == std::string::npos) return false;
      base = lookup_var(sc, first.name.substr(0, d));
      chain = first.name.substr(d);
    } else if (first.kind == Arg::Sub && !first.chain.empty()) {
      base = eval_pipeline(sc, *first.sub, false);
      chain = first.chain;
    } else {
      return false;
    }
    size_t last = chain.rfind('.');
    Value recv = field_chain(base, chain.substr(0, last));
    if (!recv.has(kObjTag)) return false;
    bool found = false;
    *out = call_method(recv, chain.substr(last + 1), args, &found);
    return found;
  }

  Value lookup_var(const Scope& sc, const std::string& ref) {
    std::string name = ref;
    std::string chain;
    size_t dot = ref.find('.');
    if (dot != std::string::npos) {
      name = ref.substr(0, dot);
      chain = ref.substr(dot);
    }
    for (auto it = sc.vars.rbegin(); it != sc.vars.rend(); ++it)
      if (it->first == name) return field_chain(it->second, chain);
    throw TemplateError("undefined variable: " + name);
  }

  Value eval_arg(Scope& sc, const Arg& a) {
    switch (a.kind) {
      case Arg::Field: return field_chain(sc.dot, a.name);
      case Arg::Var: return lookup_var(sc, a.name);
      case Arg::Lit: return a.lit;
      case Arg::Dot: return sc.dot;
      case Arg::Sub: return field_chain(eval_pipeline(sc, *a.sub, false), a.chain);
      case Arg::Ident: return call(sc, a.name, {}, nullptr);
    }
    return Value();
  }

  Value eval_pipeline(Scope& sc, const Pipeline& p, bool declare_in_scope) {
    Value last;
    bool have_last = false;
    for (auto& c : p.cmds) {
      const Arg& first = c.args[0];
      if (first.kind == Arg::Ident && (first.name == "and" || first.name == "or") && c.args.size() > 1) {
        // Go 1.18+: and/or evaluate their arguments lazily and stop at the first deciding one,
        // so `and (hasKey . "x") (gt .x 1)` never compares a missing value
        bool is_and = first.name == "and";
        Value v;
        bool decided = false;
        for (size_t i = 1; i < c.args.size(); ++i) {
          v = eval_arg(sc, c.args[i]);
          if (truth(v) != is_and) {
            decided = true;
            break;
          }
        }
        if (!decided && have_last) v = last;  // a piped value is the final argument
        last = v;
        have_last = true;
        continue;
      }
      if (first.kind == Arg::Ident) {
        std::vector<Value> args;
        for (size_t i = 1; i < c.args.size(); ++i) args.push_back(eval_arg(sc, c.args[i]));
        last = call(sc, first.name, std::move(args), have_last ? &last : nullptr);
      } else if (c.args.size() > 1 || have_last) {
        std::vector<Value> args;
        for (size_t i = 1; i < c.args.size(); ++i) args.push_back(eval_arg(sc, c.args[i]));
        if (have_last) args.push_back(last);
        if (!try_method_call(sc, first, args, &last)) {
          if (c.args.size() > 1) throw TemplateError("can't give argument to non-function");
          throw TemplateError("can't pipe into non-function");
        }
      } else {
        last = eval_arg(sc, first);
      }
      have_last = true;
    }
    if (!p.decl.empty() && declare_in_scope) {
      if (p.assign) {
        for (auto it = sc.vars.rbegin(); it != sc.vars.rend(); ++it)
          if (it->first == p.decl[0]) {
            it->second = last;
            return last;
          }
        throw TemplateError("undefined variable: " + p.decl[0]);
      }
      sc.vars.emplace_back(p.decl[0], last);
    }
    return last;
  }

  // ---------------------------------------------------------- functions

  static bool cmp_eq(const Value& a, const Value& b) {
    if (a.is_number() && b.is_number()) return a.as_double() == b.as_double();
    if (a.is_null() || b.is_null()) return a.is_null() && b.is_null();
    if (a.is_scalar() && b.is_scalar()) {
      if (a.type() != b.type()) return false;
      return a.as_string() == b.as_string();
    }
    return a == b;
  }

  static int cmp_order(const Value& a, const Value& b) {
    if (a.is_number() && b.is_number()) {
      double x = a.as_double(), y = b.as_double();
      return x < y ? -1 : x > y ? 1 : 0;
    }
    if (a.is_string() && b.is_string()) return a.str() < b.str() ? -1 : a.str() > b.str() ? 1 : 0;
    if (a.is_null() || b.is_null()) throw TemplateError("incompatible types for comparison");
    std::string x = a.as_string(), y = b.as_string();
    return x < y ? -1 : x > y ? 1 : 0;
  }

  static std::string go_quote(const std::string& s) {
    std::string out = "\"";
    for (unsigned char c : s) {
      switch (c) {
        case '"': out += "\\\""; break;
        case '\\': out += "\\\\"; break;
        case '\n': out += "\\n"; break;
        case '\t': out += "\\t"; break;
        case '\r': out += "\\r"; break;
        default:
          if (c < 0x20)
            out += strfmt("\\x%02x", c);
          else
            out.push_back((char)c);
      }
    }
    return out + "\"";
  }

  static std::string strval(const Value& v) { return v.is_null() ? "" : print_value(v); }
  // Generated sizes (until/untilStep/seq elements, repeat output) are bounded: a chart typo
  // such as `until 1000000000` must fail the render, not take the host's memory.
  static constexpr int64_t kMaxGenerated = 10000000;
  // |b - a| / |step| without overflow (a span beyond int64 is over any limit anyway)
  static int64_t span_count(int64_t a, int64_t b, int64_t st, const char* fn) {
    int64_t d;
    if (__builtin_sub_overflow(b, a, &d) || (st == -1 && d == INT64_MIN))
      throw TemplateError(std::string(fn) + ": the range exceeds the limit of " + std::to_string(kMaxGenerated));
    return d / st;
  }
  static void check_generated(int64_t n, const char* fn) {
    if (n > kMaxGenerated)
      throw TemplateError(std::string(fn) + ": " + std::to_string(n) + " elements exceed the limit of " +
                          std::to_string(kMaxGenerated));
  }
  // Go marshals map[string]interface{} with sorted keys (yaml and json alike): values that
  // went through toYaml/toJson render byte-identical to Helm's output (and to its checksums).
  static Value sorted_maps(const Value& v) {
    if (v.is_map()) {
      Value out = Value::map();
      std::vector<const std::pair<std::string, Value>*> es;
      for (auto& e : v.entries()) es.push_back(&e);
      std::sort(es.begin(), es.end(), [](auto* a, auto* b) { return a->first < b->first; });
      for (auto* e : es) out.entries().emplace_back(e->first, sorted_maps(e->second));
      return out;
    }
    if (v.is_seq()) {
      Value out = Value::seq();
      for (auto& it : v.items()) out.push(sorted_maps(it));
      return out;
    }
    return v;
  }
  // json.Marshal's HTML escaping of <, > and & (sprig toJson; toRawJson keeps them)
  static std::string html_escape_json(const std::string& j) {
    std::string o;
    o.reserve(j.size());
    for (char c : j) {
      if (c == '<') o += "\\u003c";
      else if (c == '>') o += "\\u003e";
      else if (c == '&') o += "\\u0026";
      else o.push_back(c);
    }
    return o;
  }
  // "2006-01-02T15:04:05Z07:00" (fractional seconds ignored) -> unix seconds; 0 if unparsable
  static int64_t parse_rfc3339(const std::string& t) {
    struct tm tm{};
    int off_h = 0, off_m = 0;
    char sign = 0;
    if (std::sscanf(t.c_str(), "%d-%d-%dT%d:%d:%d", &tm.tm_year, &tm.tm_mon, &tm.tm_mday, &tm.tm_hour, &tm.tm_min,
                    &tm.tm_sec) != 6)
      return 0;
    tm.tm_year -= 1900;
    tm.tm_mon -= 1;
    size_t z = t.find_first_of("+-Z", 19);
    if (z != std::string::npos && t[z] != 'Z' && std::sscanf(t.c_str() + z, "%c%d:%d", &sign, &off_h, &off_m) == 3) {
      int64_t off = off_h * 3600 + off_m * 60;
      return (int64_t)timegm(&tm) - (sign == '-' ? -off : off);
    }
    return (int64_t)timegm(&tm);
  }

  static std::string indent_str(int n, const std::string& s) {
    std::string pad(n, ' ');
    std::string out = pad;
    for (char c : s) {
      out.push_back(c);
      if (c == '\n') out += pad;
    }
    return out;
  }

  static std::string go_printf(const std::string& f, const std::vector<Value>& args) {
    std::string out;
    size_t ai = 0;
    for (size_t i = 0; i < f.size(); ++i) {
      if (f[i] != '%') {
        out.push_back(f[i]);
        continue;
      }
      if (i + 1 >= f.size()) break;
      size_t j = i + 1;
      std::string flags;
      while (j < f.size() && std::strchr("+-# 0123456789.", f[j])) flags.push_back(f[j++]);
      char verb = f[j];
      i = j;
      if (verb == '%') {
        out.push_back('%');
        continue;
      }
      Value a = ai < args.size() ? args[ai++] : Value();
      switch (verb) {
        case 'd': out += strfmt(("%" + flags + "lld").c_str(), (long long)a.as_int()); break;
        case 'f': case 'e': case 'g':
          out += strfmt(("%" + flags + std::string(1, verb)).c_str(), a.as_double());
          break;
        case 'x': out += a.is_number() ? strfmt("%llx", (long long)a.as_int()) : hex_encode(strval(a)); break;
        case 'q': out += go_quote(strval(a)); break;
        case 't': out += a.as_bool() ? "true" : "false"; break;
        default: {
          std::string s = strval(a);
          if (!flags.empty() && std::isdigit((unsigned char)flags.back()))
            out += strfmt(("%" + flags + "s").c_str(), s.c_str());
          else
            out += s;
        }
      }
    }
    return out;
  }

  std::string render_nodes(Scope& sc, const std::vector<NodeP>& nodes) {
    std::string out;
    for (auto& n : nodes) exec_node(sc, *n, out);
    return out;
  }

  int depth = 0;  // nested template/include calls

  std::string include(const std::string& name, const Value& dot) {
    auto it = templates.find(name);
    if (it == templates.end()) throw TemplateError("template: no template \"" + name + "\" associated");
    // Go's text/template stops runaway recursion with an error (maxExecDepth); here the
    // native stack is the limit, so stop well before it (100 levels fit an 8 MB stack even in
    // the ASan build, whose frames are several times larger; real charts nest ~10 deep)
    struct DepthGuard {
      int& d;
      explicit DepthGuard(int& x) : d(x) {
        if (++d > 100) {
          --d;
          throw TemplateError("template: exceeded maximum template depth (100)");
        }
      }
      ~DepthGuard() { --d; }
    } guard(depth);
    Scope sc;
    sc.dot = dot;
    sc.vars.emplace_back("$", dot);
    try {
      return render_nodes(sc, it->second);
    } catch (const LoopBreak&) {
      throw TemplateError("{{break}} outside {{range}}");
    } catch (const LoopContinue&) {
      throw TemplateError("{{continue}} outside {{range}}");
    }
  }

  Value call(Scope& sc, const std::string& fn, std::vector<Value> args, const Value* piped) {
    if (piped) args.push_back(*piped);
    auto need = [&](size_t n) {
      if (args.size() < n) throw TemplateError("wrong number of args for " + fn);
    };
    auto S = [](std::string s) {
      Value v(std::move(s));
      return v;
    };
    if (fn == "eq") {
      need(2);
      for (size_t i = 1; i < args.size(); ++i)
        if (cmp_eq(args[0], args[i])) return Value(true);
      return Value(false);
    }
    if (fn == "ne") { need(2); return Value(!cmp_eq(args[0], args[1])); }
    if (fn == "lt") { need(2); return Value(cmp_order(args[0], args[1]) < 0); }
    if (fn == "le") { need(2); return Value(cmp_order(args[0], args[1]) <= 0); }
    if (fn == "gt") { need(2); return Value(cmp_order(args[0], args[1]) > 0); }
    if (fn == "ge") { need(2); return Value(cmp_order(args[0], args[1]) >= 0); }
    if (fn == "and") {
      for (auto& a : args)
        if (!truth(a)) return a;
      return args.empty() ? Value() : args.back();
    }
    if (fn == "or") {
      for (auto& a : args)
        if (truth(a)) return a;
      return args.empty() ? Value() : args.back();
    }
    if (fn == "not") { need(1); return Value(!truth(args[0])); }
    if (fn == "len") {
      need(1);
      const Value& v = is_obj(args[0], "files") ? args[0].get(kObjData) : args[0];
      return Value((int64_t)(v.is_string() ? v.str().size() : v.size()));
    }
    if (fn == "index") {
      need(1);
      Value cur = args[0];
      for (size_t i = 1; i < args.size(); ++i) {
        if (cur.is_map())
          cur = cur.get(args[i].as_string());
        else if (cur.is_seq()) {
          int64_t k = args[i].as_int();
          if (k < 0 || k >= (int64_t)cur.size()) throw TemplateError("index out of range");
          cur = cur[(size_t)k];
        } else
          return Value();
      }
      return cur;
    }
    if (fn == "print" || fn == "println") {
      std::string s;
      for (size_t i = 0; i < args.size(); ++i) {
        if (i && fn == "println") s += " ";
        if (i && fn == "print" && !args[i].is_string() && !args[i - 1].is_string()) s += " ";
        s += strval(args[i]);
      }
      if (fn == "println") s += "\n";
      return S(s);
    }
    if (fn == "printf") {
      need(1);
      std::vector<Value> rest(args.begin() + 1, args.end());
      return S(go_printf(args[0].as_string(), rest));
    }
    if (fn == "default") {
      need(1);
      if (args.size() == 1) return args[0];
      return truth(args[1]) ? args[1] : args[0];
    }
    if (fn == "empty") { need(1); return Value(!truth(args[0])); }
    if (fn == "coalesce") {
      for (auto& a : args)
        if (truth(a)) return a;
      return Value();
    }
    if (fn == "ternary") { need(3); return truth(args[2]) ? args[0] : args[1]; }
    if (fn == "required") {
      need(2);
      if (args[1].is_null() || (args[1].is_string() && args[1].str().empty())) throw TemplateError(args[0].as_string());
      return args[1];
    }
    if (fn == "fail") { need(1); throw TemplateError(args[0].as_string()); }
    if (fn == "quote" || fn == "squote") {
      std::vector<std::string> parts;
      for (auto& a : args) {
        if (a.is_null()) continue;
        parts.push_back(fn == "quote" ? go_quote(strval(a)) : "'" + strval(a) + "'");
      }
      return S(join(parts, " "));
    }
    if (fn == "toYaml") {
      need(1);
      if (args[0].is_null()) return S("null");
      std::string y = yaml_dump(sorted_maps(args[0]));
      if (ends_with(y, "\n")) y.pop_back();
      return S(y);
    }
    if (fn == "toJson" || fn == "mustToJson") { need(1); return S(html_escape_json(json_dump(sorted_maps(args[0])))); }
    if (fn == "toRawJson") { need(1); return S(json_dump(sorted_maps(args[0]))); }
    if (fn == "toPrettyJson") { need(1); return S(html_escape_json(json_dump(sorted_maps(args[0]), 2))); }
    if (fn == "fromYaml") { need(1); return yaml_parse(args[0].as_string()); }
    if (fn == "fromJson") { need(1); return json_parse(args[0].as_string()); }
    if (fn == "indent") { need(2); return S(indent_str((int)args[0].as_int(), strval(args[1]))); }
    if (fn == "nindent") { need(2); return S("\n" + indent_str((int)args[0].as_int(), strval(args[1]))); }
    if (fn == "trim") { need(1); return S(trim(strval(args[0]), " \t\r\n")); }
    if (fn == "trimAll") { need(2); return S(trim(strval(args[1]), args[0].as_string())); }
    if (fn == "trimPrefix") {
      need(2);
      std::string s = strval(args[1]);
      return S(starts_with(s, args[0].as_string()) ? s.substr(args[0].as_string().size()) : s);
    }
    if (fn == "trimSuffix") {
      need(2);
      std::string s = strval(args[1]);
      return S(ends_with(s, args[0].as_string()) ? s.substr(0, s.size() - args[0].as_string().size()) : s);
    }
    if (fn == "upper") { need(1); return S(to_upper(strval(args[0]))); }
    if (fn == "lower") { need(1); return S(to_lower(strval(args[0]))); }
    if (fn == "title") {
      need(1);
      std::string s = strval(args[0]);
      bool up = true;
      for (auto& c : s) {
        if (up && std::isalpha((unsigned char)c)) c = (char)std::toupper((unsigned char)c);
        up = std::isspace((unsigned char)c);
      }
      return S(s);
    }
    if (fn == "replace") { need(3); return S(replace_all(strval(args[2]), args[0].as_string(), args[1].as_string())); }
    if (fn == "contains") { need(2); return Value(contains(strval(args[1]), args[0].as_string())); }
    if (fn == "hasPrefix") { need(2); return Value(starts_with(strval(args[1]), args[0].as_string())); }
    if (fn == "hasSuffix") { need(2); return Value(ends_with(strval(args[1]), args[0].as_string())); }
    if (fn == "trunc") {
      need(2);
      std::string s = strval(args[1]);
      int64_t n = args[0].as_int();
      if (n >= 0) return S(s.substr(0, std::min<size_t>((size_t)n, s.size())));
      size_t k = (size_t)(-n);
      return S(k >= s.size() ? s : s.substr(s.size() - k));
    }
    if (fn == "repeat") {
      need(2);
      std::string o, unit = strval(args[1]);
      int64_t n = args[0].as_int();
      // n * size can overflow int64: compare by division instead
      if (n > 0 && (n > kMaxGenerated || (int64_t)unit.size() > kMaxGenerated / n))
        throw TemplateError("repeat: " + std::to_string(n) + " x " + std::to_string(unit.size()) +
                            " bytes exceeds the limit of " + std::to_string(kMaxGenerated));
      for (int64_t i = 0; i < n; ++i) o += unit;
      return S(o);
    }
    if (fn == "join") {
      need(2);
      std::vector<std::string> parts;
      for (auto& it : args[1].items()) parts.push_back(strval(it));
      return S(join(parts, args[0].as_string()));
    }
    if (fn == "split" || fn == "splitList") {
      need(2);
      auto parts = split(strval(args[1]), args[0].as_string());
      if (fn == "splitList") return Value::strings(parts);
      Value m = Value::map();
      for (size_t i = 0; i < parts.size(); ++i) m["_" + std::to_string(i)] = parts[i];
      return m;
    }
    if (fn == "list" || fn == "tuple") {
      Value l = Value::seq();
      for (auto& a : args) l.push(a);
      return l;
    }
    if (fn == "dict") {
      Value m = Value::map();
      for (size_t i = 0; i + 1 < args.size(); i += 2) m[args[i].as_string()] = args[i + 1];
      return m;
    }
    if (fn == "get") { need(2); return args[0].get(args[1].as_string()); }
    if (fn == "hasKey") { need(2); return Value(args[0].has(args[1].as_string())); }
    if (fn == "set") { need(3); Value m = args[0]; m[args[1].as_string()] = args[2]; return m; }
    if (fn == "unset") { need(2); Value m = args[0]; m.erase(args[1].as_string()); return m; }
    if (fn == "keys") {
      Value l = Value::seq();
      for (auto& a : args)
        for (auto& k : a.keys()) l.push(Value(k));
      return l;
    }
    if (fn == "values") {
      need(1);
      Value l = Value::seq();
      for (auto& e : args[0].entries()) l.push(e.second);
      return l;
    }
    if (fn == "merge" || fn == "mergeOverwrite") {
      need(1);
      Value out = Value::map();
      if (fn == "merge") {
        for (auto it = args.rbegin(); it != args.rend(); ++it) merge_into(out, *it);
      } else {
        for (auto& a : args) merge_into(out, a);
      }
      return out;
    }
    if (fn == "first") { need(1); return args[0].size() ? args[0][(size_t)0] : Value(); }
    if (fn == "last") { need(1); return args[0].size() ? args[0][args[0].size() - 1] : Value(); }
    if (fn == "has") {
      need(2);
      for (auto& it : args[1].items())
        if (cmp_eq(it, args[0])) return Value(true);
      return Value(false);
    }
    if (fn == "int" || fn == "int64" || fn == "atoi") { need(1); return Value(args[0].as_int()); }
    if (fn == "float64") { need(1); return Value(args[0].as_double()); }
    if (fn == "toString") { need(1); return S(strval(args[0])); }
    if (fn == "toStrings") {
      Value l = Value::seq();
      for (auto& it : args[0].items()) l.push(Value(strval(it)));
      return l;
    }
    auto arith = [&](auto op) -> Value {
      need(1);
      bool f = false;
      for (auto& a : args) f |= a.is_float();
      if (f) {
        double r = args[0].as_double();
        for (size_t i = 1; i < args.size(); ++i) r = op(r, args[i].as_double());
        return Value(r);
      }
      int64_t r = args[0].as_int();
      for (size_t i = 1; i < args.size(); ++i) r = (int64_t)op((double)r, (double)args[i].as_int());
      return Value(r);
    };
    if (fn == "add") return arith([](double a, double b) { return a + b; });
    if (fn == "sub") return arith([](double a, double b) { return a - b; });
    if (fn == "mul") return arith([](double a, double b) { return a * b; });
    if (fn == "div") {
      need(2);
      if (args[1].as_double() == 0) throw TemplateError("division by zero");
      if (args[0].is_int() && args[1].is_int()) return Value(args[0].as_int() / args[1].as_int());
      return Value(args[0].as_double() / args[1].as_double());
    }
    if (fn == "mod") { need(2); return Value(args[1].as_int() ? args[0].as_int() % args[1].as_int() : 0); }
    if (fn == "max" || fn == "min") {
      need(1);
      Value best = args[0];
      for (auto& a : args)
        if ((fn == "max") ? cmp_order(a, best) > 0 : cmp_order(a, best) < 0) best = a;
      return best;
    }
    if (fn == "until") {
      need(1);
      Value l = Value::seq();
      check_generated(args[0].as_int(), "until");
      for (int64_t i = 0; i < args[0].as_int(); ++i) l.push(Value(i));
      return l;
    }
    if (fn == "b64enc") { need(1); return S(base64_encode(strval(args[0]))); }
    if (fn == "b64dec") { need(1); return S(base64_decode(strval(args[0]))); }
    if (fn == "sha256sum") { need(1); return S(sha256_hex(strval(args[0]))); }
    if (fn == "kindIs") {
      need(2);
      std::string k = args[0].as_string();
      const Value& v = args[1];
      std::string kind = v.is_map() ? "map" : v.is_seq() ? "slice" : v.is_string() ? "string" : v.is_int() ? "int64"
                         : v.is_float() ? "float64" : v.is_bool() ? "bool" : "invalid";
      return Value(kind == k || (k == "int" && kind == "int64"));
    }
    if (fn == "typeOf") {
      need(1);
      const Value& v = args[0];
      return S(v.is_map() ? "map[string]interface {}" : v.is_seq() ? "[]interface {}" : v.is_string() ? "string"
               : v.is_int() ? "int64" : v.is_float() ? "float64" : v.is_bool() ? "bool" : "<nil>");
    }
    if (fn == "regexMatch") { need(2); return Value(safe_regex_search(strval(args[1]), std::regex(args[0].as_string()))); }
    if (fn == "regexReplaceAll") {
      need(3);
      return S(safe_regex_replace(strval(args[1]), std::regex(args[0].as_string()), args[2].as_string()));
    }
    if (fn == "semverCompare" || fn == "mustSemverCompare") {
      need(2);
      return Value(semver_satisfies(args[0].as_string(), args[1].as_string()));
    }
    if (fn == "semver") {
      need(1);
      Semver v = parse_semver(args[0].as_string());
      if (!v.ok) throw TemplateError("invalid semantic version: " + args[0].as_string());
      Value m = Value::map();
      m["Major"] = v.major;
      m["Minor"] = v.minor;
      m["Patch"] = v.patch;
      m["Prerelease"] = v.pre;
      m["Original"] = args[0].as_string();
      return m;
    }
    if (fn == "include") { need(2); return S(include(args[0].as_string(), args[1])); }
    if (fn == "tpl") {
      need(2);
      std::string nm = "tpl-" + sha256_hex(args[0].as_string()).substr(0, 12);
      if (!templates.count(nm)) templates[nm] = parse(nm, args[0].as_string());
      return S(include(nm, args[1]));
    }
    if (fn == "lookup") {
      need(4);
      if (owner->lookup) return owner->lookup(args[0].as_string(), args[1].as_string(), args[2].as_string(), args[3].as_string());
      return Value::map();
    }
    if (fn == "now") return S(std::to_string((long long)std::time(nullptr)));
    if (fn == "date") {
      need(1);
      std::time_t t = std::time(nullptr);
      char buf[64];
      std::strftime(buf, sizeof(buf), "%Y-%m-%d", std::gmtime(&t));
      return S(buf);
    }
    if (fn == "uuidv4") {
      std::string h = hex_encode(random_string(16));
      return S(h.substr(0, 8) + "-" + h.substr(8, 4) + "-4" + h.substr(13, 3) + "-a" + h.substr(17, 3) + "-" + h.substr(20, 12));
    }
    if (fn == "randAlphaNum" || fn == "randAlpha") { need(1); return S(random_string((size_t)args[0].as_int())); }
    // ---- certificates and encryption (sprig crypto.go)
    auto strings_of = [](const Value& l) {
      std::vector<std::string> out;
      for (auto& it : l.items()) out.push_back(strval(it));
      return out;
    };
    if (fn == "genPrivateKey") { need(1); return S(sprig::gen_private_key(args[0].as_string())); }
    if (fn == "genCA") { need(2); return sprig::gen_ca(strval(args[0]), (int)args[1].as_int()); }
    if (fn == "genSelfSignedCert") {
      need(4);
      return sprig::gen_self_signed_cert(strval(args[0]), strings_of(args[1]), strings_of(args[2]), (int)args[3].as_int());
    }
    if (fn == "genSignedCert") {
      need(5);
      return sprig::gen_signed_cert(strval(args[0]), strings_of(args[1]), strings_of(args[2]), (int)args[3].as_int(),
                                    args[4]);
    }
    if (fn == "encryptAES") { need(2); return S(sprig::encrypt_aes(strval(args[0]), strval(args[1]))); }
    if (fn == "decryptAES") { need(2); return S(sprig::decrypt_aes(strval(args[0]), strval(args[1]))); }
    if (fn == "htpasswd") { need(2); return S(sprig::htpasswd(strval(args[0]), strval(args[1]))); }
    // ---- durations (sprig date.go): Go's time.Duration.String() of whole seconds
    auto go_duration = [](int64_t sec) {
      if (sec == 0) return std::string("0s");
      std::string sign = sec < 0 ? "-" : "";
      uint64_t a = (uint64_t)(sec < 0 ? -sec : sec);
      uint64_t h = a / 3600, m = a % 3600 / 60, x = a % 60;
      if (h) return sign + std::to_string(h) + "h" + std::to_string(m) + "m" + std::to_string(x) + "s";
      if (m) return sign + std::to_string(m) + "m" + std::to_string(x) + "s";
      return sign + std::to_string(x) + "s";
    };
    if (fn == "duration") {
      need(1);
      int64_t sec = 0;
      parse_int64(strval(args[0]), &sec);
      return S(go_duration(sec));
    }
    if (fn == "ago") {
      need(1);
      int64_t t = 0;
      if (!parse_int64(strval(args[0]), &t)) t = parse_rfc3339(strval(args[0]));
      return S(go_duration((int64_t)std::time(nullptr) - t));
    }
    // ---- wider Sprig set (strings)
    if (fn == "sha1sum") { need(1); return S(digest_hex(EVP_sha1(), strval(args[0]))); }
    if (fn == "adler32sum") {
      need(1);
      std::string d = strval(args[0]);
      return S(std::to_string(::adler32(::adler32(0L, Z_NULL, 0), (const Bytef*)d.data(), (uInt)d.size())));
    }
    if (fn == "b32enc") { need(1); return S(b32_encode(strval(args[0]))); }
    if (fn == "b32dec") { need(1); return S(b32_decode(strval(args[0]))); }
    if (fn == "abbrev") {
      need(2);
      std::string str = strval(args[1]);
      int64_t w = args[0].as_int();
      if (w < 4 || (int64_t)str.size() <= w) return S(str);
      return S(str.substr(0, (size_t)w - 3) + "...");
    }
    if (fn == "abbrevboth") {
      need(3);
      std::string str = strval(args[2]);
      int64_t l = args[0].as_int(), w = args[1].as_int();
      if ((int64_t)str.size() <= w) return S(str);
      if (l > 4) str = "..." + str.substr((size_t)std::min<int64_t>(l, (int64_t)str.size()));
      if ((int64_t)str.size() > w) str = str.substr(0, (size_t)std::max<int64_t>(0, w - 3)) + "...";
      return S(str);
    }
    if (fn == "camelcase") {
      need(1);
      std::string o;
      for (auto& w : words_of(strval(args[0]))) {
        std::string x = to_lower(w);
        x[0] = (char)std::toupper((unsigned char)x[0]);
        o += x;
      }
      return S(o);
    }
    if (fn == "snakecase" || fn == "kebabcase") {
      need(1);
      std::vector<std::string> ws;
      for (auto& w : words_of(strval(args[0]))) ws.push_back(to_lower(w));
      return S(join(ws, fn == "snakecase" ? "_" : "-"));
    }
    if (fn == "swapcase") {
      need(1);
      std::string o = strval(args[0]);
      for (auto& c : o)
        c = std::isupper((unsigned char)c) ? (char)std::tolower((unsigned char)c) : (char)std::toupper((unsigned char)c);
      return S(o);
    }
    if (fn == "untitle") {
      need(1);
      std::string o = strval(args[0]);
      bool start = true;
      for (auto& c : o) {
        if (start && std::isalpha((unsigned char)c)) c = (char)std::tolower((unsigned char)c);
        start = std::isspace((unsigned char)c);
      }
      return S(o);
    }
    if (fn == "initials") {
      need(1);
      std::string o;
      for (auto& w : split(strval(args[0]), " "))
        if (!w.empty()) o.push_back(w[0]);
      return S(o);
    }
    if (fn == "nospace") {
      need(1);
      std::string o;
      for (char c : strval(args[0]))
        if (!std::isspace((unsigned char)c)) o.push_back(c);
      return S(o);
    }
    if (fn == "substr") {
      need(3);
      std::string str = strval(args[2]);
      int64_t a = args[0].as_int(), b = args[1].as_int();
      if (a < 0) return S(str.substr(0, (size_t)std::min<int64_t>(b, (int64_t)str.size())));
      if (b < 0 || b > (int64_t)str.size()) return S(a < (int64_t)str.size() ? str.substr((size_t)a) : "");
      return S(a < b ? str.substr((size_t)a, (size_t)(b - a)) : "");
    }
    if (fn == "wrap" || fn == "wrapWith") {
      need(fn == "wrap" ? 2 : 3);
      size_t width = (size_t)args[0].as_int();
      std::string nl = fn == "wrap" ? "\n" : args[1].as_string();
      std::string out, line;
      for (auto& w : split(strval(args.back()), " ")) {
        if (w.empty()) continue;
        if (!line.empty() && line.size() + 1 + w.size() > width) {
          out += line + nl;
          line.clear();
        }
        line += (line.empty() ? "" : " ") + w;
      }
      return S(out + line);
    }
    if (fn == "cat") {
      std::vector<std::string> parts;
      for (auto& a : args)
        if (!a.is_null()) parts.push_back(strval(a));
      return S(join(parts, " "));
    }
    if (fn == "plural") { need(3); return S(args[2].as_int() == 1 ? args[0].as_string() : args[1].as_string()); }
    if (fn == "randNumeric" || fn == "randAscii") {
      need(1);
      std::string r = random_string((size_t)args[0].as_int());
      if (fn == "randNumeric")
        for (auto& c : r) c = (char)('0' + ((unsigned char)c % 10));
      return S(r);
    }
    if (fn == "trimall") { need(2); return S(trim(strval(args[1]), args[0].as_string())); }
    // ---- lists
    if (fn == "append" || fn == "push") { need(2); Value l = args[0].is_null() ? Value::seq() : args[0]; l.push(args[1]); return l; }
    if (fn == "prepend") {
      need(2);
      Value l = Value::seq();
      l.push(args[1]);
      for (auto& it : args[0].items()) l.push(it);
      return l;
    }
    if (fn == "concat") {
      Value l = Value::seq();
      for (auto& a : args)
        for (auto& it : a.items()) l.push(it);
      return l;
    }
    if (fn == "uniq") {
      need(1);
      Value l = Value::seq();
      for (auto& it : args[0].items()) {
        bool dup = false;
        for (auto& x : l.items()) dup |= cmp_eq(x, it);
        if (!dup) l.push(it);
      }
      return l;
    }
    if (fn == "compact") {
      need(1);
      Value l = Value::seq();
      for (auto& it : args[0].items())
        if (truth(it)) l.push(it);
      return l;
    }
    if (fn == "without") {
      need(1);
      Value l = Value::seq();
      for (auto& it : args[0].items()) {
        bool drop = false;
        for (size_t i = 1; i < args.size(); ++i) drop |= cmp_eq(args[i], it);
        if (!drop) l.push(it);
      }
      return l;
    }
    if (fn == "rest" || fn == "initial" || fn == "reverse") {
      need(1);
      Value l = Value::seq();
      const auto& its = args[0].items();
      if (fn == "rest")
        for (size_t i = 1; i < its.size(); ++i) l.push(its[i]);
      else if (fn == "initial")
        for (size_t i = 0; i + 1 < its.size(); ++i) l.push(its[i]);
      else
        for (auto it = its.rbegin(); it != its.rend(); ++it) l.push(*it);
      return l;
    }
    if (fn == "sortAlpha") {
      need(1);
      std::vector<std::string> v;
      for (auto& it : args[0].items()) v.push_back(strval(it));
      std::sort(v.begin(), v.end());
      return Value::strings(v);
    }
    if (fn == "slice") {
      need(1);
      if (args[0].is_string()) {
        const std::string& str = args[0].str();
        size_t a = args.size() > 1 ? (size_t)args[1].as_int() : 0, b = args.size() > 2 ? (size_t)args[2].as_int() : str.size();
        if (a > b || b > str.size()) throw TemplateError("slice: index out of range");
        return S(str.substr(a, b - a));
      }
      const auto& its = args[0].items();
      size_t a = args.size() > 1 ? (size_t)args[1].as_int() : 0, b = args.size() > 2 ? (size_t)args[2].as_int() : its.size();
      if (a > b || b > its.size()) throw TemplateError("slice: index out of range");
      Value l = Value::seq();
      for (size_t i = a; i < b; ++i) l.push(its[i]);
      return l;
    }
    if (fn == "untilStep") {
      need(3);
      Value l = Value::seq();
      int64_t a = args[0].as_int(), b = args[1].as_int(), st = args[2].as_int();
      if (st == 0) return l;
      check_generated(span_count(a, b, st, "untilStep"), "untilStep");
      for (int64_t i = a; st > 0 ? i < b : i > b;) {
        l.push(Value(i));
        if (__builtin_add_overflow(i, st, &i)) break;  // the next value is past int64: done
      }
      return l;
    }
    if (fn == "seq") {
      need(1);
      int64_t a = 1, b = args.back().as_int(), st = 1;
      if (args.size() == 2) a = args[0].as_int(), b = args[1].as_int();
      if (args.size() >= 3) a = args[0].as_int(), st = args[1].as_int(), b = args[2].as_int();
      if (args.size() >= 2 && args.size() < 3 && a > b) st = -1;
      std::vector<std::string> o;
      if (st != 0) check_generated(span_count(a, b, st, "seq"), "seq");
      if (st != 0)
        for (int64_t i = a; st > 0 ? i <= b : i >= b;) {
          o.push_back(std::to_string(i));
          if (__builtin_add_overflow(i, st, &i)) break;
        }
      return S(join(o, " "));
    }
    if (fn == "all") {
      for (auto& a : args)
        if (!truth(a)) return Value(false);
      return Value(true);
    }
    if (fn == "any") {
      for (auto& a : args)
        if (truth(a)) return Value(true);
      return Value(false);
    }
    // ---- dicts
    if (fn == "pick" || fn == "omit") {
      need(1);
      Value m = Value::map();
      for (auto& e : args[0].entries()) {
        bool listed = false;
        for (size_t i = 1; i < args.size(); ++i) listed |= args[i].as_string() == e.first;
        if (listed == (fn == "pick")) m[e.first] = e.second;
      }
      return m;
    }
    if (fn == "pluck") {
      need(1);
      Value l = Value::seq();
      for (size_t i = 1; i < args.size(); ++i)
        if (args[i].has(args[0].as_string())) l.push(args[i].get(args[0].as_string()));
      return l;
    }
    if (fn == "dig") {
      need(3);
      Value cur = args.back();
      for (size_t i = 0; i + 2 < args.size(); ++i) {
        const Value* n = cur.is_map() ? cur.find(args[i].as_string()) : nullptr;
        if (!n) return args[args.size() - 2];
        cur = *n;
      }
      return cur;
    }
    if (fn == "deepCopy") { need(1); return args[0]; }
    if (fn == "deepEqual") { need(2); return Value(args[0] == args[1]); }
    if (fn == "kindOf") {
      need(1);
      const Value& v = args[0];
      return S(v.is_map() ? "map" : v.is_seq() ? "slice" : v.is_string() ? "string" : v.is_int() ? "int64"
               : v.is_float() ? "float64" : v.is_bool() ? "bool" : "invalid");
    }
    if (fn == "typeIs" || fn == "typeIsLike") {
      need(2);
      const Value& v = args[1];
      std::string t = v.is_map() ? "map[string]interface {}" : v.is_seq() ? "[]interface {}" : v.is_string() ? "string"
                      : v.is_int() ? "int64" : v.is_float() ? "float64" : v.is_bool() ? "bool" : "<nil>";
      std::string want = args[0].as_string();
      if (fn == "typeIsLike" && starts_with(want, "*")) want = want.substr(1);
      return Value(t == want || (want == "int" && t == "int64"));
    }
    // ---- regex / paths / math / encodings
    if (fn == "regexFind") {
      need(2);
      std::smatch m;
      std::string str = strval(args[1]);
      return S(safe_regex_search(str, &m, std::regex(args[0].as_string())) ? m.str(0) : "");
    }
    if (fn == "regexFindAll" || fn == "regexSplit") {
      need(3);
      std::string str = strval(args[1]);
      std::regex re(args[0].as_string());
      int64_t n = args[2].as_int();
      std::vector<std::string> out;
      safe_regex_run(str.size(), [&] {
      if (fn == "regexFindAll") {
        for (auto it = std::sregex_iterator(str.begin(), str.end(), re); it != std::sregex_iterator(); ++it) {
          if (n >= 0 && (int64_t)out.size() >= n) break;
          out.push_back(it->str(0));
        }
      } else {
        size_t pos = 0;
        for (auto it = std::sregex_iterator(str.begin(), str.end(), re); it != std::sregex_iterator(); ++it) {
          if (n > 0 && (int64_t)out.size() >= n - 1) break;
          out.push_back(str.substr(pos, (size_t)it->position(0) - pos));
          pos = (size_t)(it->position(0) + it->length(0));
        }
        out.push_back(str.substr(pos));
      }
      });
      return Value::strings(out);
    }
    if (fn == "regexReplaceAllLiteral") {
      need(3);
      std::string str = strval(args[1]), out;
      std::regex re(args[0].as_string());
      safe_regex_run(str.size(), [&] { out = std::regex_replace(str, re, args[2].as_string(), std::regex_constants::format_sed); });
      return S(out);
    }
    if (fn == "regexQuoteMeta") {
      need(1);
      std::string o;
      for (char c : strval(args[0])) {
        if (std::strchr("\\.+*?()|[]{}^$", c)) o.push_back('\\');
        o.push_back(c);
      }
      return S(o);
    }
    if (fn == "base") { need(1); std::string p = path_clean(strval(args[0])); return S(p == "/" ? "/" : base_name(p)); }
    if (fn == "dir") {
      need(1);
      std::string p = path_clean(strval(args[0]));
      size_t k = p.rfind('/');
      return S(k == std::string::npos ? "." : k == 0 ? "/" : p.substr(0, k));
    }
    if (fn == "ext") {
      need(1);
      std::string b = base_name(strval(args[0]));
      size_t k = b.rfind('.');
      return S(k == std::string::npos ? "" : b.substr(k));
    }
    if (fn == "clean") { need(1); return S(path_clean(strval(args[0]))); }
    if (fn == "isAbs") { need(1); return Value(!strval(args[0]).empty() && strval(args[0])[0] == '/'); }
    if (fn == "floor") { need(1); return Value(std::floor(args[0].as_double())); }
    if (fn == "ceil") { need(1); return Value(std::ceil(args[0].as_double())); }
    if (fn == "round") {
      need(2);
      double p = std::pow(10.0, (double)args[1].as_int());
      return Value(std::round(args[0].as_double() * p) / p);
    }
    if (fn == "add1") { need(1); return Value(args[0].as_int() + 1); }
    if (fn == "addf" || fn == "subf" || fn == "mulf" || fn == "divf" || fn == "maxf" || fn == "minf") {
      need(1);
      double r = args[0].as_double();
      for (size_t i = 1; i < args.size(); ++i) {
        double x = args[i].as_double();
        if (fn == "addf") r += x;
        else if (fn == "subf") r -= x;
        else if (fn == "mulf") r *= x;
        else if (fn == "divf") r /= x;
        else if (fn == "maxf") r = std::max(r, x);
        else r = std::min(r, x);
      }
      return Value(r);
    }
    if (fn == "toDecimal") { need(1); return Value((int64_t)std::strtoll(strval(args[0]).c_str(), nullptr, 8)); }
    if (fn == "toToml") {
      need(1);
      std::string o;
      if (args[0].is_map()) toml_table(sorted_maps(args[0]), "", o);
      return S(o);
    }
    if (fn == "fromYamlArray" || fn == "fromJsonArray") {
      need(1);
      Value v = fn == "fromYamlArray" ? yaml_parse(args[0].as_string()) : json_parse(args[0].as_string());
      return v.is_seq() ? v : Value::seq();
    }
    if (fn == "urlquery") {
      std::string o;
      for (auto& a : args) o += strval(a);
      std::string r;
      for (unsigned char c : o) {
        if (std::isalnum(c) || c == '-' || c == '_' || c == '.' || c == '~') r.push_back((char)c);
        else if (c == ' ') r.push_back('+');
        else r += strfmt("%%%02X", c);
      }
      return S(r);
    }
    if (fn == "html" || fn == "js") {
      std::string o;
      for (auto& a : args) o += strval(a);
      std::string r;
      for (char c : o) {
        if (fn == "html") {
          if (c == '<') r += "&lt;"; else if (c == '>') r += "&gt;"; else if (c == '&') r += "&amp;";
          else if (c == '"') r += "&#34;"; else if (c == '\'') r += "&#39;"; else r.push_back(c);
        } else {
          if (c == '\\' || c == '\'' || c == '"') r += std::string("\\") + c;
          else if (c == '<') r += "\\u003C"; else if (c == '>') r += "\\u003E"; else if (c == '&') r += "\\u0026";
          else if (c == '=') r += "\\u003D"; else if (c == '\n') r += "\\n"; else r.push_back(c);
        }
      }
      return S(r);
    }
    if (fn == "unixEpoch") return S(std::to_string((long long)std::time(nullptr)));
    if (fn == "dateInZone" || fn == "htmlDate") {
      std::time_t t = std::time(nullptr);
      char buf[64];
      std::strftime(buf, sizeof(buf), "%Y-%m-%d", std::gmtime(&t));
      return S(buf);
    }
    // ---- remaining Sprig functions: os* aliases, biggest, sha512sum, shuffle, chunk, URLs, DNS
    static const std::map<std::string, std::string> kAliases = {
        {"osBase", "base"}, {"osDir", "dir"}, {"osClean", "clean"}, {"osExt", "ext"}, {"osIsAbs", "isAbs"},
        {"biggest", "max"}};
    auto al = kAliases.find(fn);
    if (al != kAliases.end()) return call(sc, al->second, std::move(args), nullptr);
    if (fn == "sha512sum") { need(1); return S(digest_hex(EVP_sha512(), strval(args[0]))); }
    if (fn == "shuffle") {
      need(1);
      std::string t = strval(args[0]);
      std::string r = random_string(t.size() * 4 + 4);
      for (size_t i = t.size(); i > 1; --i) std::swap(t[i - 1], t[(unsigned char)r[i] * 131u % i]);
      return S(t);
    }
    if (fn == "chunk") {
      need(2);
      int64_t n = args[0].as_int();
      if (n <= 0) throw TemplateError("chunk: size must be positive");
      Value out = Value::seq(), cur = Value::seq();
      for (auto& it : args[1].items()) {
        cur.push(it);
        if ((int64_t)cur.size() == n) {
          out.push(cur);
          cur = Value::seq();
        }
      }
      if (cur.size()) out.push(cur);
      return out;
    }
    if (fn == "urlParse") {
      need(1);
      std::string u = strval(args[0]);
      Value m = Value::map();
      std::string rest = u, frag, query;
      size_t h = rest.find('#');
      if (h != std::string::npos) frag = rest.substr(h + 1), rest = rest.substr(0, h);
      size_t q = rest.find('?');
      if (q != std::string::npos) query = rest.substr(q + 1), rest = rest.substr(0, q);
      std::string scheme, host, userinfo, path = rest, opaque;
      size_t c = rest.find(':');
      if (c != std::string::npos && c > 0 && rest.find('/') > c) {
        scheme = rest.substr(0, c);
        rest = rest.substr(c + 1);
        if (starts_with(rest, "//")) {
          rest = rest.substr(2);
          size_t sl = rest.find('/');
          std::string auth = rest.substr(0, sl);
          path = sl == std::string::npos ? "" : rest.substr(sl);
          size_t at = auth.rfind('@');
          if (at != std::string::npos) userinfo = auth.substr(0, at), auth = auth.substr(at + 1);
          host = auth;
        } else {
          opaque = rest;
          path = "";
        }
      }
      std::string hostname = host;
      if (!hostname.empty() && hostname[0] == '[') hostname = hostname.substr(1, hostname.find(']') - 1);
      else if (hostname.find(':') != std::string::npos) hostname = hostname.substr(0, hostname.find(':'));
      m["scheme"] = scheme;
      m["host"] = host;
      m["hostname"] = hostname;
      m["path"] = path;
      m["query"] = query;
      m["opaque"] = opaque;
      m["fragment"] = frag;
      m["userinfo"] = userinfo;
      return m;
    }
    if (fn == "urlJoin") {
      need(1);
      const Value& m = args[0];
      std::string out;
      if (!m.get("scheme").as_string().empty()) out += m.get("scheme").as_string() + ":";
      if (!m.get("opaque").as_string().empty()) {
        out += m.get("opaque").as_string();
      } else {
        if (!m.get("host").as_string().empty() || !m.get("userinfo").as_string().empty()) {
          out += "//";
          if (!m.get("userinfo").as_string().empty()) out += m.get("userinfo").as_string() + "@";
          out += m.get("host").as_string();
        }
        out += m.get("path").as_string();
      }
      if (!m.get("query").as_string().empty()) out += "?" + m.get("query").as_string();
      if (!m.get("fragment").as_string().empty()) out += "#" + m.get("fragment").as_string();
      return S(out);
    }
    if (fn == "getHostByName") {
      need(1);
      auto addrs = net::resolve(strval(args[0]), 0);
      return S(addrs.empty() ? "" : addrs[0].text);
    }
    // mustX is X that returns its error instead of panicking; errors already throw here
    if (starts_with(fn, "must") && fn.size() > 4 && std::isupper((unsigned char)fn[4])) {
      std::string base(1, (char)std::tolower((unsigned char)fn[4]));
      base += fn.substr(5);
      return call(sc, base, std::move(args), nullptr);
    }
    throw TemplateError("function \"" + fn + "\" not defined");
  }

  void exec_node(Scope& sc, const Node& n, std::string& out) {
    switch (n.kind) {
      case Node::Text: out += n.text; return;
      case Node::Action: {
        Value v = eval_pipeline(sc, *n.pipe, true);
        if (n.pipe->decl.empty()) out += print_value(v);
        return;
      }
      case Node::If: {
        size_t mark = sc.vars.size();
        Value v = eval_pipeline(sc, *n.pipe, true);
        struct Restore {  // loop control may unwind through this scope
          Scope& sc;
          size_t mark;
          ~Restore() { sc.vars.resize(mark); }
        } restore{sc, mark};
        for (auto& child : (truth(v) ? n.body : n.else_body)) exec_node(sc, *child, out);
        return;
      }
      case Node::With: {
        size_t mark = sc.vars.size();
        Value v = eval_pipeline(sc, *n.pipe, true);
        struct Restore {  // loop control may unwind through this scope
          Scope& sc;
          size_t mark;
          Value dot;
          ~Restore() {
            sc.vars.resize(mark);
            sc.dot = dot;
          }
        } restore{sc, mark, sc.dot};
        if (truth(v)) {
          sc.dot = v;
          for (auto& child : n.body) exec_node(sc, *child, out);
        } else {
          for (auto& child : n.else_body) exec_node(sc, *child, out);
        }
        return;
      }
      case Node::Range: {
        Pipeline p = *n.pipe;
        std::vector<std::string> decl = p.decl;
        p.decl.clear();
        Value v = eval_pipeline(sc, p, false);
        if (is_obj(v, "files")) v = v.get(kObjData);  // range over .Files: path -> bytes
        std::vector<std::pair<Value, Value>> items;
        if (v.is_seq()) {
          for (size_t i = 0; i < v.size(); ++i) items.emplace_back(Value((int64_t)i), v[i]);
        } else if (v.is_map()) {
          auto keys = v.keys();
          std::sort(keys.begin(), keys.end());
          for (auto& k : keys) items.emplace_back(Value(k), v.get(k));
        } else if (v.is_int()) {
          for (int64_t i = 0; i < v.as_int(); ++i) items.emplace_back(Value(i), Value(i));
        }
        if (items.empty()) {
          out += render_nodes(sc, n.else_body);
          return;
        }
        Value saved = sc.dot;
        for (auto& kv : items) {
          size_t mark = sc.vars.size();
          if (decl.size() == 1) sc.vars.emplace_back(decl[0], kv.second);
          if (decl.size() >= 2) {
            sc.vars.emplace_back(decl[0], kv.first);
            sc.vars.emplace_back(decl[1], kv.second);
          }
          sc.dot = kv.second;
          bool brk = false;
          try {
            for (auto& child : n.body) exec_node(sc, *child, out);
          } catch (const LoopContinue&) {
          } catch (const LoopBreak&) {
            brk = true;
          }
          // assignments with "=" to outer vars must survive: only drop the loop's own vars
          sc.vars.resize(mark);
          if (brk) break;
        }
        sc.dot = saved;
        return;
      }
      case Node::Template: {
        Value dot = n.pipe ? eval_pipeline(sc, *n.pipe, false) : Value();
        out += include(n.name, dot);
        return;
      }
      case Node::List: out += render_nodes(sc, n.body); return;
      case Node::Break: throw LoopBreak{};
      case Node::Continue: throw LoopContinue{};
    }
  }
};

Engine::Engine() : impl_(std::make_unique<Impl>()) { impl_->owner = this; }
Engine::~Engine() = default;

void Engine::add(const std::string& name, const std::string& text) {
  try {
    impl_->templates[name] = impl_->parse(name, text);
  } catch (const TemplateError& e) {
    throw TemplateError("parse error in " + name + ": " + e.what());
  }
}

bool Engine::has(const std::string& name) const { return impl_->templates.count(name) > 0; }

std::string Engine::execute(const std::string& name, const Value& dot) {
  try {
    return impl_->include(name, dot);
  } catch (const TemplateError& e) {
    throw TemplateError("render error in " + name + ": " + e.what());
  }
}

}  // namespace tmpl
}  // namespace ds

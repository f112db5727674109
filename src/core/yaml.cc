// YAML 1.2-subset reader/writer (block + flow collections, quoted/plain/block scalars,
// anchors/aliases/merge keys, multi-document streams). The reference uses gopkg.in/yaml.v2;
// the writer follows that library's layout (sequences inside maps are not indented) so files
// round-trip with minimal diff (config/configutil/save.go:15).
#include <cctype>
#include <fstream>
#include <map>
#include <sstream>

#include "core/strutil.h"
#include "core/value.h"

namespace ds {

namespace {

struct Line {
  int indent;
  std::string content;  // text after indentation (raw, comments not yet stripped)
  int lineno;
  bool blank;  // empty or comment only
};

bool is_blank_content(const std::string& c) { return c.empty() || c[0] == '#'; }

Value resolve_plain(const std::string& s) {
  if (s.empty() || s == "~" || s == "null" || s == "Null" || s == "NULL") return Value();
  if (s == "true" || s == "True" || s == "TRUE") return Value(true);
  if (s == "false" || s == "False" || s == "FALSE") return Value(false);
  int64_t iv;
  if (parse_int64(s, &iv)) {
    // leading zeros like "0755" are octal in YAML 1.1; keep as string unless simple
    if (s.size() > 1 && s[0] == '0') {
      int64_t o = 0;
      bool ok = true;
      for (size_t i = 1; i < s.size(); ++i) {
        if (s[i] < '0' || s[i] > '7') ok = false;
        o = o * 8 + (s[i] - '0');
      }
      if (ok) return Value(o);
      return Value(s);
    }
    return Value(iv);
  }
  if (s.size() > 2 && s[0] == '0' && (s[1] == 'x' || s[1] == 'X')) {
    char* end = nullptr;
    long long v = strtoll(s.c_str() + 2, &end, 16);
    if (end && *end == 0) return Value((int64_t)v);
  }
  if (s == ".inf" || s == ".Inf" || s == "+.inf") return Value(1.0 / 0.0);
  if (s == "-.inf" || s == "-.Inf") return Value(-1.0 / 0.0);
  if (s == ".nan" || s == ".NaN") return Value(0.0 / 0.0);
  // floats: require a digit and only float chars
  bool floaty = false, digit = false;
  for (char c : s) {
    if (std::isdigit((unsigned char)c))
      digit = true;
    else if (c == '.' || c == 'e' || c == 'E' || c == '-' || c == '+')
      floaty = true;
    else
      return Value(s);
  }
  if (digit && floaty) {
    double d;
    if (parse_double(s, &d)) return Value(d);
  }
  return Value(s);
}

class Parser {
 public:
  explicit Parser(const std::string& text) {
    std::string cur;
    int lineno = 0;
    std::istringstream is(text);
    std::string raw;
    while (std::getline(is, raw)) {
      ++lineno;
      if (!raw.empty() && raw.back() == '\r') raw.pop_back();
      int ind = 0;
      while (ind < (int)raw.size() && raw[ind] == ' ') ++ind;
      std::string content = raw.substr(ind);
      // tabs as leading indentation are not valid YAML; treat them as blank-ish content
      Line l{ind, content, lineno, is_blank_content(trim(content))};
      if (!l.blank && trim_right(content).empty()) l.blank = true;
      lines_.push_back(l);
      raw_.push_back(raw);
    }
  }

  std::vector<Value> parse_all() {
    std::vector<Value> docs;
    pos_ = 0;
    while (true) {
      skip_blank();
      if (pos_ >= lines_.size()) break;
      // document markers
      if (is_doc_start(lines_[pos_])) {
        std::string rest = trim(lines_[pos_].content.substr(3));
        ++pos_;
        if (!rest.empty() && rest[0] != '#') {
          // "--- value" inline
          docs.push_back(parse_inline(rest, 0));
          continue;
        }
        skip_blank();
        if (pos_ >= lines_.size() || is_doc_start(lines_[pos_]) || is_doc_end(lines_[pos_])) {
          docs.push_back(Value());
          continue;
        }
      }
      if (is_doc_end(lines_[pos_])) {
        ++pos_;
        continue;
      }
      anchors_.clear();
      Value v = parse_block(lines_[pos_].indent);
      docs.push_back(v);
      skip_blank();
      if (pos_ < lines_.size() && !is_doc_start(lines_[pos_]) && !is_doc_end(lines_[pos_])) {
        fail("unexpected content (bad indentation?)");
      }
    }
    return docs;
  }

 private:
  std::vector<Line> lines_;
  std::vector<std::string> raw_;
  size_t pos_ = 0;
  std::map<std::string, Value> anchors_;

  [[noreturn]] void fail(const std::string& msg) const {
    int ln = pos_ < lines_.size() ? lines_[pos_].lineno : (int)lines_.size();
    throw ParseError("yaml: line " + std::to_string(ln) + ": " + msg);
  }

  static bool is_doc_start(const Line& l) {
    return l.indent == 0 && starts_with(l.content, "---") &&
           (l.content.size() == 3 || l.content[3] == ' ' || l.content[3] == '\t');
  }
  static bool is_doc_end(const Line& l) {
    return l.indent == 0 && starts_with(l.content, "...") && trim(l.content) == "...";
  }

  void skip_blank() {
    while (pos_ < lines_.size() && lines_[pos_].blank) ++pos_;
  }

  static bool is_seq_item(const std::string& c) {
    return !c.empty() && c[0] == '-' && (c.size() == 1 || c[1] == ' ' || c[1] == '\t');
  }

  // Returns position of the ':' separating key and value, or npos.
  static size_t find_map_colon(const std::string& c) {
    if (c.empty()) return std::string::npos;
    if (c[0] == '[' || c[0] == '{' || c[0] == '#' || c[0] == '|' || c[0] == '>') return std::string::npos;
    if (c[0] == '"' || c[0] == '\'') {
      char q = c[0];
      size_t i = 1;
      while (i < c.size()) {
        if (q == '"' && c[i] == '\\') {
          i += 2;
          continue;
        }
        if (c[i] == q) {
          if (q == '\'' && i + 1 < c.size() && c[i + 1] == '\'') {
            i += 2;
            continue;
          }
          break;
        }
        ++i;
      }
      if (i >= c.size()) return std::string::npos;
      size_t j = i + 1;
      while (j < c.size() && c[j] == ' ') ++j;
      if (j < c.size() && c[j] == ':' && (j + 1 == c.size() || c[j + 1] == ' ' || c[j + 1] == '\t'))
        return j;
      return std::string::npos;
    }
    for (size_t i = 0; i < c.size(); ++i) {
      if (c[i] == '#' && i > 0 && (c[i - 1] == ' ' || c[i - 1] == '\t')) return std::string::npos;
      if (c[i] == ':' && (i + 1 == c.size() || c[i + 1] == ' ' || c[i + 1] == '\t')) return i;
    }
    return std::string::npos;
  }

  static std::string strip_comment(const std::string& s) {
    // plain text: comment starts at " #"
    bool in_s = false, in_d = false;
    for (size_t i = 0; i < s.size(); ++i) {
      char c = s[i];
      if (in_d) {
        if (c == '\\') {
          ++i;
          continue;
        }
        if (c == '"') in_d = false;
        continue;
      }
      if (in_s) {
        if (c == '\'') in_s = false;
        continue;
      }
      if (c == '"' && (i == 0 || s[i - 1] == ' ' || s[i - 1] == '[' || s[i - 1] == '{' || s[i - 1] == ',' ||
                       s[i - 1] == ':'))
        in_d = true;
      else if (c == '\'' && (i == 0 || s[i - 1] == ' ' || s[i - 1] == '[' || s[i - 1] == '{' ||
                             s[i - 1] == ',' || s[i - 1] == ':'))
        in_s = true;
      else if (c == '#' && (i == 0 || s[i - 1] == ' ' || s[i - 1] == '\t'))
        return trim_right(s.substr(0, i));
    }
    return trim_right(s);
  }

  std::string parse_key(const std::string& raw) {
    std::string k = trim(raw);
    if (!k.empty() && (k[0] == '"' || k[0] == '\'')) {
      size_t p = 0;
      Value v = parse_quoted(k, &p);
      return v.as_string();
    }
    return k;
  }

  Value parse_block(int indent) {
    Nest nest(nest_);
    skip_blank();
    if (pos_ >= lines_.size()) return Value();
    Line& l = lines_[pos_];
    if (l.indent < indent || is_doc_start(l) || is_doc_end(l)) return Value();
    if (is_seq_item(l.content)) return parse_seq(l.indent);
    if (find_map_colon(l.content) != std::string::npos) return parse_map(l.indent);
    // scalar / flow at block position (possibly multi-line)
    int ind = l.indent;
    std::string text = l.content;
    ++pos_;
    return parse_inline_multiline(text, ind - 1);
  }

  // Parses an inline value that may continue on more-indented following lines.
  Value parse_inline_multiline(std::string text, int parent_indent) {
    std::string t = trim(text);
    if (t.empty()) return Value();
    char c0 = t[0];
    if (c0 == '[' || c0 == '{') {
      // join lines until balanced
      std::string acc = t;
      while (!flow_balanced(acc) && pos_ < lines_.size()) {
        acc += " " + trim(lines_[pos_].content);
        ++pos_;
      }
      return parse_inline(acc, parent_indent);
    }
    if (c0 == '"' || c0 == '\'') {
      std::string acc = t;
      while (!quote_closed(acc) && pos_ < lines_.size()) {
        std::string nxt = trim(lines_[pos_].content);
        size_t bs = 0;
        while (bs < acc.size() && acc[acc.size() - 1 - bs] == '\\') ++bs;
        if (c0 == '"' && bs % 2 == 1) {
          // an escaped line break (PyYAML writes long strings this way): the break and the next
          // line's leading white space vanish, nothing takes their place
          acc.pop_back();
          acc += nxt;
        } else {
          acc += nxt.empty() ? "\n" : (ends_with(acc, "\n") ? nxt : " " + nxt);
        }
        ++pos_;
      }
      return parse_inline(acc, parent_indent);
    }
    Value v = parse_inline(t, parent_indent);
    if (v.is_string() && !v.quoted() && c0 != '|' && c0 != '>' && c0 != '&' && c0 != '*' && c0 != '!') {
      // "key: a: b" — a plain scalar cannot hold ": " (or end in ':'); go-yaml reports it
      // rather than reading a typo as a string
      std::string body = strip_comment(t);
      if (body.find(": ") != std::string::npos || body.find(":\t") != std::string::npos ||
          (!body.empty() && body.back() == ':')) {
        int ln = pos_ > 0 && pos_ - 1 < lines_.size() ? lines_[pos_ - 1].lineno : (int)lines_.size();
        throw ParseError("yaml: line " + std::to_string(ln) + ": mapping values are not allowed in this context");
      }
    }
    if (v.is_string() && !v.quoted() && c0 != '|' && c0 != '>') {
      // plain multi-line continuation
      std::string acc = v.str();
      bool cont = false;
      while (pos_ < lines_.size() && !lines_[pos_].blank && lines_[pos_].indent > parent_indent &&
             find_map_colon(lines_[pos_].content) == std::string::npos && !is_seq_item(lines_[pos_].content)) {
        acc += " " + strip_comment(trim(lines_[pos_].content));
        ++pos_;
        cont = true;
      }
      if (cont) return Value(acc);
    }
    return v;
  }

  static bool quote_closed(const std::string& s) {
    char q = s[0];
    for (size_t i = 1; i < s.size(); ++i) {
      if (q == '"' && s[i] == '\\') {
        ++i;
        continue;
      }
      if (s[i] == q) {
        if (q == '\'' && i + 1 < s.size() && s[i + 1] == '\'') {
          ++i;
          continue;
        }
        return true;
      }
    }
    return false;
  }

  static bool flow_balanced(const std::string& s) {
    int depth = 0;
    bool in_s = false, in_d = false;
    for (size_t i = 0; i < s.size(); ++i) {
      char c = s[i];
      if (in_d) {
        if (c == '\\')
          ++i;
        else if (c == '"')
          in_d = false;
        continue;
      }
      if (in_s) {
        if (c == '\'') in_s = false;
        continue;
      }
      if (c == '"')
        in_d = true;
      else if (c == '\'')
        in_s = true;
      else if (c == '[' || c == '{')
        ++depth;
      else if (c == ']' || c == '}')
        --depth;
    }
    return depth <= 0;
  }

  Value parse_seq(int indent) {
    Value out = Value::seq();
    while (true) {
      skip_blank();
      if (pos_ >= lines_.size()) break;
      Line& l = lines_[pos_];
      if (is_doc_start(l) || is_doc_end(l)) break;
      if (l.indent != indent || !is_seq_item(l.content)) break;
      std::string rest = l.content.substr(1);
      size_t sp = 0;
      while (sp < rest.size() && (rest[sp] == ' ' || rest[sp] == '\t')) ++sp;
      rest = rest.substr(sp);
      if (rest.empty() || rest[0] == '#') {
        ++pos_;
        skip_blank();
        if (pos_ < lines_.size() && lines_[pos_].indent > indent)
          out.push(parse_block(lines_[pos_].indent));
        else
          out.push(Value());
        continue;
      }
      int new_indent = indent + 1 + (int)sp;
      // Re-interpret the remainder as a line at the deeper indent.
      l.indent = new_indent;
      l.content = rest;
      if (is_seq_item(rest)) {
        out.push(parse_seq(new_indent));
      } else if (find_map_colon(rest) != std::string::npos && rest[0] != '&' && rest[0] != '*') {
        out.push(parse_map(new_indent));
      } else if (rest[0] == '&' && find_map_colon(rest) != std::string::npos) {
        // "- &anchor key: value" is unusual; treat anchor on the map
        size_t spc = rest.find(' ');
        std::string anchor = rest.substr(1, spc - 1);
        l.content = trim(rest.substr(spc));
        l.indent = new_indent + (int)spc + 1;
        Value m = parse_map(l.indent);
        anchors_[anchor] = m;
        out.push(m);
      } else {
        ++pos_;
        out.push(parse_value_after_indicator(rest, indent));
      }
    }
    return out;
  }

  // A value found inline after "key:" or "- ". `owner_indent` is the indentation of the owning
  // key / dash, used for block scalars and nested blocks.
  Value parse_value_after_indicator(const std::string& rest_raw, int owner_indent) {
    std::string rest = trim(rest_raw);
    std::string anchor;
    if (!rest.empty() && rest[0] == '&') {
      size_t spc = rest.find_first_of(" \t");
      anchor = rest.substr(1, spc == std::string::npos ? std::string::npos : spc - 1);
      rest = spc == std::string::npos ? "" : trim(rest.substr(spc));
    }
    // skip tags like !!map / !!str
    bool force_str = false;
    if (!rest.empty() && rest[0] == '!') {
      size_t spc = rest.find_first_of(" \t");
      std::string tag = rest.substr(0, spc);
      force_str = tag == "!!str";
      rest = spc == std::string::npos ? "" : trim(rest.substr(spc));
    }
    Value v;
    if (rest.empty() || rest[0] == '#') {
      skip_blank();
      if (pos_ < lines_.size()) {
        Line& n = lines_[pos_];
        if (n.indent > owner_indent)
          v = parse_block(n.indent);
        else if (n.indent == owner_indent && is_seq_item(n.content))
          v = parse_seq(owner_indent);
      }
    } else if (rest[0] == '|' || rest[0] == '>') {
      v = parse_block_scalar(rest, owner_indent);
    } else {
      v = parse_inline_multiline(rest, owner_indent);
      if (force_str && !v.is_string()) {
        Value s(v.as_string());
        s.set_quoted(true);
        v = s;
      }
    }
    if (!anchor.empty()) anchors_[anchor] = v;
    return v;
  }

  Value parse_map(int indent) {
    Value out = Value::map();
    while (true) {
      skip_blank();
      if (pos_ >= lines_.size()) break;
      Line& l = lines_[pos_];
      if (is_doc_start(l) || is_doc_end(l)) break;
      if (l.indent != indent) {
        if (l.indent > indent) fail("bad indentation of a mapping entry");
        break;
      }
      if (is_seq_item(l.content)) break;
      size_t colon = find_map_colon(l.content);
      if (colon == std::string::npos) fail("could not find expected ':'");
      std::string key = parse_key(l.content.substr(0, colon));
      std::string rest = l.content.substr(colon + 1);
      ++pos_;
      Value v = parse_value_after_indicator(rest, indent);
      if (key == "<<") {
        // merge key: copy entries not already present
        auto apply = [&](const Value& src) {
          if (!src.is_map()) return;
          for (auto& e : src.entries())
            if (!out.has(e.first)) out[e.first] = e.second;
        };
        if (v.is_seq())
          for (auto& it : v.items()) apply(it);
        else
          apply(v);
        continue;
      }
      if (out.has(key)) fail("mapping key \"" + key + "\" already defined");
      out.entries().emplace_back(key, std::move(v));
    }
    return out;
  }

  Value parse_block_scalar(const std::string& header, int owner_indent) {
    bool literal = header[0] == '|';
    char chomp = 'c';  // clip
    int explicit_indent = 0;
    for (size_t i = 1; i < header.size(); ++i) {
      char c = header[i];
      if (c == '-')
        chomp = 's';
      else if (c == '+')
        chomp = 'k';
      else if (std::isdigit((unsigned char)c))
        explicit_indent = c - '0';
      else if (c == ' ' || c == '#')
        break;
    }
    // determine content indent
    int content_indent = -1;
    if (explicit_indent > 0) content_indent = owner_indent + explicit_indent;
    std::vector<std::string> body;
    while (pos_ < lines_.size()) {
      const std::string& raw = raw_[pos_];
      bool blank = trim(raw).empty();
      if (blank) {
        body.push_back("");
        ++pos_;
        continue;
      }
      int ind = lines_[pos_].indent;
      if (content_indent < 0) {
        if (ind <= owner_indent) break;
        content_indent = ind;
      }
      if (ind < content_indent) break;
      body.push_back(raw.substr(content_indent));
      ++pos_;
    }
    // trailing blank lines belong to chomping
    int trailing = 0;
    while (!body.empty() && body.back().empty()) {
      body.pop_back();
      ++trailing;
    }
    std::string out;
    if (literal) {
      for (size_t i = 0; i < body.size(); ++i) {
        out += body[i];
        if (i + 1 < body.size()) out += "\n";
      }
    } else {
      // folded: single newlines become spaces, blank lines become newlines
      bool prev_blank = false;
      for (size_t i = 0; i < body.size(); ++i) {
        const std::string& b = body[i];
        if (b.empty()) {
          out += "\n";
          prev_blank = true;
          continue;
        }
        if (i > 0 && !prev_blank && !(b[0] == ' ')) out += " ";
        if (i > 0 && (b[0] == ' ') && !prev_blank) out += "\n";
        out += b;
        prev_blank = false;
      }
    }
    if (!body.empty()) {
      if (chomp == 'c')
        out += "\n";
      else if (chomp == 'k')
        out += std::string(1 + trailing, '\n');
    }
    Value v(out);
    v.set_quoted(true);
    return v;
  }

  Value parse_quoted(const std::string& s, size_t* p) {
    char q = s[*p];
    std::string out;
    size_t i = *p + 1;
    for (; i < s.size(); ++i) {
      char c = s[i];
      if (q == '\'') {
        if (c == '\'') {
          if (i + 1 < s.size() && s[i + 1] == '\'') {
            out.push_back('\'');
            ++i;
            continue;
          }
          break;
        }
        out.push_back(c);
        continue;
      }
      if (c == '"') break;
      if (c == '\\' && i + 1 < s.size()) {
        char e = s[++i];
        switch (e) {
          case 'n': out.push_back('\n'); break;
          case 't': out.push_back('\t'); break;
          case 'r': out.push_back('\r'); break;
          case '0': out.push_back('\0'); break;
          case '"': out.push_back('"'); break;
          case '\\': out.push_back('\\'); break;
          case '/': out.push_back('/'); break;
          case ' ': out.push_back(' '); break;
          case 'e': out.push_back('\x1b'); break;
          case 'x':
          case 'u':
          case 'U': {
            int n = e == 'x' ? 2 : e == 'u' ? 4 : 8;
            unsigned cp = (unsigned)strtoul(s.substr(i + 1, n).c_str(), nullptr, 16);
            i += n;
            if (cp < 0x80) {
              out.push_back((char)cp);
            } else if (cp < 0x800) {
              out.push_back((char)(0xC0 | (cp >> 6)));
              out.push_back((char)(0x80 | (cp & 0x3F)));
            } else if (cp < 0x10000) {
              out.push_back((char)(0xE0 | (cp >> 12)));
              out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
              out.push_back((char)(0x80 | (cp & 0x3F)));
            } else {
              out.push_back((char)(0xF0 | (cp >> 18)));
              out.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
              out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
              out.push_back((char)(0x80 | (cp & 0x3F)));
            }
            break;
          }
          default: out.push_back(e);
        }
        continue;
      }
      out.push_back(c);
    }
    if (i >= s.size()) throw ParseError("yaml: unterminated quoted string: " + s);
    *p = i + 1;
    Value v(out);
    v.set_quoted(true);
    return v;
  }

  // Flow / scalar parser working on one logical line.
  Value parse_inline(const std::string& text, int parent_indent) {
    (void)parent_indent;
    std::string t = trim(text);
    if (t.empty()) return Value();
    if (t[0] == '|' || t[0] == '>') return parse_block_scalar(t, parent_indent);
    size_t p = 0;
    Value v = parse_flow_value(t, &p, false);
    // rest must be comment/empty
    while (p < t.size() && (t[p] == ' ' || t[p] == '\t')) ++p;
    if (p < t.size() && t[p] != '#') {
      throw ParseError("yaml: unexpected trailing content: " + t.substr(p));
    }
    return v;
  }

  void skip_ws(const std::string& s, size_t* p) {
    while (*p < s.size() && (s[*p] == ' ' || s[*p] == '\t' || s[*p] == '\n')) ++*p;
  }

  struct Nest {
    int& d;
    explicit Nest(int& x) : d(x) {
      if (++d > 1000) {
        --d;
        throw ParseError("yaml: exceeded max depth (1000)");
      }
    }
    ~Nest() { --d; }
  };
  int nest_ = 0;  // collection nesting (flow and block): untrusted documents cannot exhaust the stack

  Value parse_flow_value(const std::string& s, size_t* p, bool in_flow) {
    Nest nest(nest_);
    skip_ws(s, p);
    if (*p >= s.size()) return Value();
    char c = s[*p];
    if (c == '&') {
      size_t e = *p + 1;
      while (e < s.size() && s[e] != ' ' && s[e] != ',' && s[e] != ']' && s[e] != '}') ++e;
      std::string name = s.substr(*p + 1, e - *p - 1);
      *p = e;
      Value v = parse_flow_value(s, p, in_flow);
      anchors_[name] = v;
      return v;
    }
    if (c == '*') {
      size_t e = *p + 1;
      while (e < s.size() && s[e] != ' ' && s[e] != ',' && s[e] != ']' && s[e] != '}') ++e;
      std::string name = s.substr(*p + 1, e - *p - 1);
      *p = e;
      auto it = anchors_.find(name);
      if (it == anchors_.end()) throw ParseError("yaml: unknown anchor '" + name + "' referenced");
      return it->second;
    }
    if (c == '!') {
      size_t e = *p;
      while (e < s.size() && s[e] != ' ') ++e;
      bool force_str = s.substr(*p, e - *p) == "!!str";
      *p = e;
      Value v = parse_flow_value(s, p, in_flow);
      if (force_str && !v.is_string()) {
        Value sv(v.as_string());
        sv.set_quoted(true);
        return sv;
      }
      return v;
    }
    if (c == '"' || c == '\'') return parse_quoted(s, p);
    if (c == '[') {
      ++*p;
      Value out = Value::seq();
      while (true) {
        skip_ws(s, p);
        if (*p >= s.size()) throw ParseError("yaml: unterminated flow sequence");
        if (s[*p] == ']') {
          ++*p;
          break;
        }
        Value item = parse_flow_value(s, p, true);
        skip_ws(s, p);
        // single-pair map inside a flow seq: [a: b]
        if (*p < s.size() && s[*p] == ':') {
          ++*p;
          Value m = Value::map();
          m[item.as_string()] = parse_flow_value(s, p, true);
          item = m;
          skip_ws(s, p);
        }
        out.push(item);
        if (*p < s.size() && s[*p] == ',') {
          ++*p;
          continue;
        }
        skip_ws(s, p);
        if (*p < s.size() && s[*p] == ']') {
          ++*p;
          break;
        }
        throw ParseError("yaml: expected ',' or ']' in flow sequence");
      }
      return out;
    }
    if (c == '{') {
      ++*p;
      Value out = Value::map();
      while (true) {
        skip_ws(s, p);
        if (*p >= s.size()) throw ParseError("yaml: unterminated flow mapping");
        if (s[*p] == '}') {
          ++*p;
          break;
        }
        Value k = parse_flow_value(s, p, true);
        skip_ws(s, p);
        Value v;
        if (*p < s.size() && s[*p] == ':') {
          ++*p;
          skip_ws(s, p);
          if (*p < s.size() && (s[*p] == ',' || s[*p] == '}'))
            v = Value();
          else
            v = parse_flow_value(s, p, true);
        }
        out[k.as_string()] = v;
        skip_ws(s, p);
        if (*p < s.size() && s[*p] == ',') {
          ++*p;
          continue;
        }
        if (*p < s.size() && s[*p] == '}') {
          ++*p;
          break;
        }
        throw ParseError("yaml: expected ',' or '}' in flow mapping");
      }
      return out;
    }
    // plain scalar
    size_t start = *p;
    size_t e = *p;
    while (e < s.size()) {
      char ch = s[e];
      if (in_flow && (ch == ',' || ch == ']' || ch == '}')) break;
      if (in_flow && ch == ':' && (e + 1 == s.size() || s[e + 1] == ' ' || s[e + 1] == ',')) break;
      if (ch == '#' && e > start && (s[e - 1] == ' ' || s[e - 1] == '\t')) break;
      ++e;
    }
    *p = e;
    return resolve_plain(trim(s.substr(start, e - start)));
  }
};

bool needs_quotes(const std::string& s) {
  if (s.empty()) return true;
  Value r = resolve_plain(s);
  if (!r.is_string()) return true;
  std::string l = to_lower(s);
  if (l == "yes" || l == "no" || l == "on" || l == "off" || l == "y" || l == "n") return true;
  char c0 = s[0];
  if (std::string("-?:,[]{}#&*!|>'\"%@` \t").find(c0) != std::string::npos) {
    // "-foo" is fine as plain but "- foo" / "-" are not; keep it simple and quote.
    if (!(c0 == '-' && s.size() > 1 && s[1] != ' ')) return true;
  }
  if (s.back() == ' ' || s.back() == ':' || s.back() == '\t') return true;
  if (s.find(": ") != std::string::npos || s.find(" #") != std::string::npos) return true;
  for (char c : s) {
    if ((unsigned char)c < 0x20) return true;
  }
  return false;
}

std::string dq(const std::string& s) {
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
  out += "\"";
  return out;
}

std::string scalar_text(const Value& v) {
  switch (v.type()) {
    case Value::Type::Null: return "null";
    case Value::Type::String: return needs_quotes(v.str()) ? dq(v.str()) : v.str();
    default: return v.as_string();
  }
}

std::string key_text(const std::string& k) { return needs_quotes(k) ? dq(k) : k; }

bool use_block_literal(const Value& v) {
  if (!v.is_string()) return false;
  const std::string& s = v.str();
  if (s.find('\n') == std::string::npos) return false;
  for (unsigned char c : s)
    if (c < 0x20 && c != '\n') return false;
  // trailing spaces on lines break literal blocks
  for (auto& line : split(s, "\n"))
    if (!line.empty() && (line.back() == ' ' || line[0] == ' ')) return false;
  return true;
}

void emit_block_literal(const std::string& s, int indent, std::string& out) {
  std::string body = s;
  std::string hdr = "|";
  if (!ends_with(body, "\n"))
    hdr = "|-";
  else if (ends_with(body, "\n\n"))
    hdr = "|+";
  out += hdr + "\n";
  std::string content = body;
  if (ends_with(content, "\n")) content.pop_back();
  for (auto& line : split(content, "\n")) {
    if (line.empty())
      out += "\n";
    else
      out += std::string(indent, ' ') + line + "\n";
  }
}

void emit(const Value& v, int indent, std::string& out);

void emit_seq(const Value& v, int indent, std::string& out) {
  for (auto& it : v.items()) {
    out += std::string(indent, ' ') + "-";
    if (it.is_map() && it.size() > 0) {
      // first key inline after "- "
      std::string sub;
      emit(it, indent + 2, sub);
      out += " " + sub.substr(indent + 2);
    } else if (it.is_seq() && it.size() > 0) {
      std::string sub;
      emit_seq(it, indent + 2, sub);
      out += " " + sub.substr(indent + 2);
    } else if (it.is_map()) {
      out += " {}\n";
    } else if (it.is_seq()) {
      out += " []\n";
    } else if (use_block_literal(it)) {
      out += " ";
      emit_block_literal(it.str(), indent + 2, out);
    } else {
      out += " " + scalar_text(it) + "\n";
    }
  }
}

void emit(const Value& v, int indent, std::string& out) {
  if (v.is_map()) {
    for (auto& e : v.entries()) {
      out += std::string(indent, ' ') + key_text(e.first) + ":";
      const Value& c = e.second;
      if (c.is_map()) {
        if (c.size() == 0) {
          out += " {}\n";
        } else {
          out += "\n";
          emit(c, indent + 2, out);
        }
      } else if (c.is_seq()) {
        if (c.size() == 0) {
          out += " []\n";
        } else {
          out += "\n";
          emit_seq(c, indent, out);
        }
      } else if (use_block_literal(c)) {
        out += " ";
        emit_block_literal(c.str(), indent + 2, out);
      } else {
        out += " " + scalar_text(c) + "\n";
      }
    }
  } else if (v.is_seq()) {
    emit_seq(v, indent, out);
  } else {
    out += std::string(indent, ' ') + scalar_text(v) + "\n";
  }
}

}  // namespace

std::vector<Value> yaml_parse_all(const std::string& text) {
  // a UTF-8 byte order mark (Windows editors) is not content, as in go-yaml's reader
  static const std::string kBom = "\xEF\xBB\xBF";
  Parser p(text.compare(0, kBom.size(), kBom) == 0 ? text.substr(kBom.size()) : text);
  return p.parse_all();
}

Value yaml_parse(const std::string& text) {
  auto docs = yaml_parse_all(text);
  if (docs.empty()) return Value();
  return docs[0];
}

std::string yaml_dump(const Value& v) {
  std::string out;
  if (v.is_map() && v.size() == 0) return "{}\n";
  if (v.is_seq() && v.size() == 0) return "[]\n";
  emit(v, 0, out);
  return out;
}

Value yaml_load_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("open " + path + ": no such file or directory");
  std::stringstream ss;
  ss << f.rdbuf();
  try {
    return yaml_parse(ss.str());
  } catch (const ParseError& e) {
    throw ParseError(path + ": " + e.what());
  }
}

}  // namespace ds

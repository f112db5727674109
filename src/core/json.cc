// JSON reader/writer over the shared Value tree (Kubernetes REST bodies, docker API streams,
// JSON log lines; the reference uses encoding/json + logrus.JSONFormatter).
#include <cmath>

#include "core/strutil.h"
#include "core/value.h"

namespace ds {

namespace {

struct JParser {
  const std::string& s;
  size_t p = 0;
  int depth = 0;  // nesting of objects/arrays: bounded like Go's encoding/json (10000) but
                  // sized for the native stack (API responses are untrusted input)

  [[noreturn]] void fail(const std::string& m) {
    throw ParseError("json: " + m + " at offset " + std::to_string(p));
  }
  void ws() {
    while (p < s.size() && (s[p] == ' ' || s[p] == '\n' || s[p] == '\t' || s[p] == '\r')) ++p;
  }
  static void put_utf8(std::string& out, unsigned cp) {
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
  }
  std::string str() {
    if (s[p] != '"') fail("expected string");
    ++p;
    std::string out;
    while (p < s.size()) {
      char c = s[p++];
      if (c == '"') return out;
      if (c == '\\') {
        if (p >= s.size()) fail("bad escape");
        char e = s[p++];
        switch (e) {
          case 'n': out.push_back('\n'); break;
          case 't': out.push_back('\t'); break;
          case 'r': out.push_back('\r'); break;
          case 'b': out.push_back('\b'); break;
          case 'f': out.push_back('\f'); break;
          case '/': out.push_back('/'); break;
          case '\\': out.push_back('\\'); break;
          case '"': out.push_back('"'); break;
          case 'u': {
            if (p + 4 > s.size()) fail("bad unicode escape");
            unsigned cp = (unsigned)strtoul(s.substr(p, 4).c_str(), nullptr, 16);
            p += 4;
            if (cp >= 0xD800 && cp <= 0xDBFF && p + 6 <= s.size() && s[p] == '\\' && s[p + 1] == 'u') {
              unsigned lo = (unsigned)strtoul(s.substr(p + 2, 4).c_str(), nullptr, 16);
              if (lo >= 0xDC00 && lo <= 0xDFFF) {
                cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                p += 6;
              }
            }
            put_utf8(out, cp);
            break;
          }
          default: fail("bad escape");
        }
      } else {
        out.push_back(c);
      }
    }
    fail("unterminated string");
  }
  Value val() {
    ws();
    if (p >= s.size()) fail("unexpected end");
    struct Nest {
      JParser& j;
      explicit Nest(JParser& x) : j(x) {
        if (++j.depth > 1000) j.fail("exceeded max depth (1000)");
      }
      ~Nest() { --j.depth; }
    } nest(*this);
    char c = s[p];
    if (c == '{') {
      ++p;
      Value m = Value::map();
      ws();
      if (p < s.size() && s[p] == '}') {
        ++p;
        return m;
      }
      while (true) {
        ws();
        std::string k = str();
        ws();
        if (p >= s.size() || s[p] != ':') fail("expected ':'");
        ++p;
        Value v = val();
        m.entries().emplace_back(std::move(k), std::move(v));
        ws();
        if (p < s.size() && s[p] == ',') {
          ++p;
          continue;
        }
        if (p < s.size() && s[p] == '}') {
          ++p;
          return m;
        }
        fail("expected ',' or '}'");
      }
    }
    if (c == '[') {
      ++p;
      Value a = Value::seq();
      ws();
      if (p < s.size() && s[p] == ']') {
        ++p;
        return a;
      }
      while (true) {
        a.push(val());
        ws();
        if (p < s.size() && s[p] == ',') {
          ++p;
          continue;
        }
        if (p < s.size() && s[p] == ']') {
          ++p;
          return a;
        }
        fail("expected ',' or ']'");
      }
    }
    if (c == '"') {
      Value v(str());
      v.set_quoted(true);
      return v;
    }
    if (s.compare(p, 4, "true") == 0) {
      p += 4;
      return Value(true);
    }
    if (s.compare(p, 5, "false") == 0) {
      p += 5;
      return Value(false);
    }
    if (s.compare(p, 4, "null") == 0) {
      p += 4;
      return Value();
    }
    size_t st = p;
    bool isf = false;
    while (p < s.size() && (std::isdigit((unsigned char)s[p]) || s[p] == '-' || s[p] == '+' || s[p] == '.' ||
                            s[p] == 'e' || s[p] == 'E')) {
      if (s[p] == '.' || s[p] == 'e' || s[p] == 'E') isf = true;
      ++p;
    }
    if (st == p) fail("unexpected character");
    std::string num = s.substr(st, p - st);
    if (!isf) {
      int64_t iv;
      if (parse_int64(num, &iv)) return Value(iv);
    }
    double d;
    if (!parse_double(num, &d)) fail("bad number");
    return Value(d);
  }
};

void dump(const Value& v, int indent, int level, std::string& out) {
  auto nl = [&](int lvl) {
    if (indent >= 0) {
      out.push_back('\n');
      out.append((size_t)(indent * lvl), ' ');
    }
  };
  switch (v.type()) {
    case Value::Type::Null: out += "null"; break;
    case Value::Type::Bool: out += v.as_bool() ? "true" : "false"; break;
    case Value::Type::Int: out += std::to_string(v.as_int()); break;
    case Value::Type::Float: {
      double d = v.as_double();
      if (std::isfinite(d)) {
        if (d == std::floor(d) && std::fabs(d) < 1e15)
          out += strfmt("%.1f", d);
        else
          out += strfmt("%.17g", d);
      } else {
        out += "null";
      }
      break;
    }
    case Value::Type::String: out += "\"" + json_escape(v.str()) + "\""; break;
    case Value::Type::Seq: {
      out.push_back('[');
      bool first = true;
      for (auto& it : v.items()) {
        if (!first) out.push_back(',');
        first = false;
        nl(level + 1);
        dump(it, indent, level + 1, out);
      }
      if (!v.items().empty()) nl(level);
      out.push_back(']');
      break;
    }
    case Value::Type::Map: {
      out.push_back('{');
      bool first = true;
      for (auto& e : v.entries()) {
        if (!first) out.push_back(',');
        first = false;
        nl(level + 1);
        out += "\"" + json_escape(e.first) + "\":";
        if (indent >= 0) out.push_back(' ');
        dump(e.second, indent, level + 1, out);
      }
      if (!v.entries().empty()) nl(level);
      out.push_back('}');
      break;
    }
  }
}

}  // namespace

std::string json_escape(const std::string& s) {
  std::string out;
  out.reserve(s.size() + 8);
  for (unsigned char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      case '\b': out += "\\b"; break;
      case '\f': out += "\\f"; break;
      default:
        if (c < 0x20)
          out += strfmt("\\u%04x", c);
        else
          out.push_back((char)c);
    }
  }
  return out;
}

Value json_parse(const std::string& text) {
  JParser jp{text};
  Value v = jp.val();
  jp.ws();
  if (jp.p != text.size()) jp.fail("trailing content");
  return v;
}

std::string json_dump(const Value& v, int indent) {
  std::string out;
  dump(v, indent, 0, out);
  return out;
}

}  // namespace ds

// String helpers shared by every module (the reference leans on Go's strings package).
#pragma once

#include <algorithm>
#include <cctype>
#include <cstdint>
#include <sstream>
#include <string>
#include <vector>

namespace ds {

inline std::vector<std::string> split(const std::string& s, const std::string& sep) {
  std::vector<std::string> out;
  if (sep.empty()) {
    out.push_back(s);
    return out;
  }
  size_t start = 0;
  while (true) {
    size_t pos = s.find(sep, start);
    if (pos == std::string::npos) {
      out.push_back(s.substr(start));
      break;
    }
    out.push_back(s.substr(start, pos - start));
    start = pos + sep.size();
  }
  return out;
}

inline std::vector<std::string> split_nonempty(const std::string& s, char sep) {
  std::vector<std::string> out;
  std::string cur;
  for (char c : s) {
    if (c == sep) {
      if (!cur.empty()) out.push_back(cur);
      cur.clear();
    } else {
      cur.push_back(c);
    }
  }
  if (!cur.empty()) out.push_back(cur);
  return out;
}

inline std::string join(const std::vector<std::string>& v, const std::string& sep) {
  std::string out;
  for (size_t i = 0; i < v.size(); ++i) {
    if (i) out += sep;
    out += v[i];
  }
  return out;
}

inline bool starts_with(const std::string& s, const std::string& p) {
  return s.size() >= p.size() && s.compare(0, p.size(), p) == 0;
}

inline bool ends_with(const std::string& s, const std::string& p) {
  return s.size() >= p.size() && s.compare(s.size() - p.size(), p.size(), p) == 0;
}

inline bool contains(const std::string& s, const std::string& p) { return s.find(p) != std::string::npos; }

inline std::string trim(const std::string& s, const std::string& chars = " \t\r\n") {
  size_t b = s.find_first_not_of(chars);
  if (b == std::string::npos) return "";
  size_t e = s.find_last_not_of(chars);
  return s.substr(b, e - b + 1);
}

inline std::string trim_left(const std::string& s, const std::string& chars = " \t\r\n") {
  size_t b = s.find_first_not_of(chars);
  return b == std::string::npos ? "" : s.substr(b);
}

inline std::string trim_right(const std::string& s, const std::string& chars = " \t\r\n") {
  size_t e = s.find_last_not_of(chars);
  return e == std::string::npos ? "" : s.substr(0, e + 1);
}

inline std::string replace_all(std::string s, const std::string& from, const std::string& to) {
  if (from.empty()) return s;
  size_t pos = 0;
  while ((pos = s.find(from, pos)) != std::string::npos) {
    s.replace(pos, from.size(), to);
    pos += to.size();
  }
  return s;
}

inline std::string to_lower(std::string s) {
  for (auto& c : s) c = (char)std::tolower((unsigned char)c);
  return s;
}

inline std::string to_upper(std::string s) {
  for (auto& c : s) c = (char)std::toupper((unsigned char)c);
  return s;
}

inline bool parse_int64(const std::string& s, int64_t* out) {
  if (s.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (s[0] == '-' || s[0] == '+') {
    neg = s[0] == '-';
    i = 1;
  }
  if (i >= s.size()) return false;
  int64_t v = 0;
  for (; i < s.size(); ++i) {
    if (!std::isdigit((unsigned char)s[i])) return false;
    v = v * 10 + (s[i] - '0');
  }
  *out = neg ? -v : v;
  return true;
}

inline bool parse_double(const std::string& s, double* out) {
  if (s.empty()) return false;
  char* end = nullptr;
  double v = std::strtod(s.c_str(), &end);
  if (end != s.c_str() + s.size()) return false;
  *out = v;
  return true;
}

inline std::string shell_quote(const std::string& s) {
  // single-quote for POSIX sh: ' -> '\''
  std::string out = "'";
  for (char c : s) {
    if (c == '\'')
      out += "'\\''";
    else
      out.push_back(c);
  }
  out += "'";
  return out;
}

// %XX decoding (userinfo of proxy URLs, query values).
inline std::string url_decode(const std::string& s) {
  std::string out;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '%' && i + 2 < s.size() && std::isxdigit((unsigned char)s[i + 1]) &&
        std::isxdigit((unsigned char)s[i + 2])) {
      out.push_back((char)std::stoi(s.substr(i + 1, 2), nullptr, 16));
      i += 2;
    } else {
      out.push_back(s[i]);
    }
  }
  return out;
}

template <typename... Args>
std::string cat(Args&&... args) {
  std::ostringstream os;
  (os << ... << args);
  return os.str();
}

// printf-style formatting into std::string.
std::string strfmt(const char* fmt, ...) __attribute__((format(printf, 1, 2)));

}  // namespace ds

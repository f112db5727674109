#include "core/match.h"

#include <algorithm>
#include <cstdint>
#include <functional>
#include <vector>

#include "core/fs.h"
#include "core/strutil.h"

namespace ds {

namespace {
// Failure memo for the backtracking matchers below: their result depends only on (pattern
// position, subject position), so a state that failed once fails again. This bounds every
// match to O(pattern x subject) states; without it patterns such as "**/**/**/**/x" or
// "*a*a*a*a*a*c" take exponential time (a `.dockerignore` line could hang a build).
struct FailMemo {
  std::vector<uint8_t> bits;
  size_t width = 0;
  void reset(size_t p, size_t s) {
    width = s + 1;
    bits.assign((p + 1) * width, 0);
  }
  bool failed(size_t pi, size_t si) const { return bits[pi * width + si] != 0; }
  bool fail(size_t pi, size_t si) {
    bits[pi * width + si] = 1;
    return false;
  }
};
thread_local FailMemo g_gi_memo, g_pm_memo, g_dk_memo, g_ds_memo;
}  // namespace

// ---------------------------------------------------------------- gitignore

void GitIgnore::add_lines(const std::vector<std::string>& lines) {
  for (auto& l : lines) add_line(l);
}

void GitIgnore::add_line(const std::string& raw) {
  std::string line = trim_right(raw, "\r");
  if (starts_with(line, "#")) return;
  line = trim(line, " ");
  if (line.empty()) return;
  Pat p;
  if (line[0] == '!') {
    p.negate = true;
    line = line.substr(1);
  }
  if (!line.empty() && (line[0] == '#' || line[0] == '!')) line = line.substr(1);
  if (line.empty()) return;
  // "foo/*.blah" inside a folder is anchored: a '/' after some non-'/' char followed by "*."
  {
    size_t slash = line.find('/');
    if (line[0] != '/' && slash != std::string::npos && slash > 0) {
      size_t star = line.find("*.", slash);
      if (star != std::string::npos) line = "/" + line;
    }
  }
  if (starts_with(line, "/**/")) line = line.substr(1);
  bool anchored = line[0] == '/';
  bool dir_suffix = ends_with(line, "/");
  if (anchored) {
    p.toks.push_back({Tok::OptSlash, 0});
    line = line.substr(1);
  } else {
    p.toks.push_back({Tok::OptAnySlash, 0});
  }
  for (size_t i = 0; i < line.size(); ++i) {
    char c = line[i];
    if (line.compare(i, 4, "/**/") == 0) {
      p.toks.push_back({Tok::SlashOrMid, 0});
      i += 3;
      continue;
    }
    if (line.compare(i, 3, "**/") == 0) {
      p.toks.push_back({Tok::OptAnySlash, 0});
      i += 2;
      continue;
    }
    if (line.compare(i, 3, "/**") == 0) {
      p.toks.push_back({Tok::OptSlashAny, 0});
      i += 2;
      continue;
    }
    if (c == '\\' && i + 1 < line.size() && line[i + 1] == '*') {
      p.toks.push_back({Tok::Any, 0});  // go-gitignore turns "\*" into ".*" via its magic star
      ++i;
      continue;
    }
    if (c == '*') {
      p.toks.push_back({Tok::Star, 0});
      continue;
    }
    p.toks.push_back({Tok::Lit, c});
  }
  // dir_suffix: "(|.*)$" else "(|/.*)$"
  p.toks.push_back({dir_suffix ? Tok::Any : Tok::OptSlashAny, 0});
  pats_.push_back(std::move(p));
}

static bool gi_match_(const std::vector<GitIgnore::Tok>& t, size_t ti, const std::string& s, size_t si);
static bool gi_match(const std::vector<GitIgnore::Tok>& t, size_t ti, const std::string& s, size_t si) {
  if (g_gi_memo.failed(ti, si)) return false;
  return gi_match_(t, ti, s, si) || g_gi_memo.fail(ti, si);
}

static bool gi_match_(const std::vector<GitIgnore::Tok>& t, size_t ti, const std::string& s, size_t si) {
  using Tok = GitIgnore::Tok;
  if (ti == t.size()) return si == s.size();
  const Tok& k = t[ti];
  switch (k.kind) {
    case Tok::Lit:
      return si < s.size() && s[si] == k.c && gi_match(t, ti + 1, s, si + 1);
    case Tok::Star: {
      for (size_t j = si;; ++j) {
        if (gi_match(t, ti + 1, s, j)) return true;
        if (j >= s.size() || s[j] == '/') return false;
      }
    }
    case Tok::Any: {
      for (size_t j = si; j <= s.size(); ++j)
        if (gi_match(t, ti + 1, s, j)) return true;
      return false;
    }
    case Tok::OptSlash:
      if (gi_match(t, ti + 1, s, si)) return true;
      return si < s.size() && s[si] == '/' && gi_match(t, ti + 1, s, si + 1);
    case Tok::OptAnySlash: {
      // (|.*/)
      if (gi_match(t, ti + 1, s, si)) return true;
      for (size_t j = si; j < s.size(); ++j)
        if (s[j] == '/' && gi_match(t, ti + 1, s, j + 1)) return true;
      return false;
    }
    case Tok::OptSlashAny: {
      // (|/.*)
      if (gi_match(t, ti + 1, s, si)) return true;
      if (si < s.size() && s[si] == '/') {
        for (size_t j = si + 1; j <= s.size(); ++j)
          if (gi_match(t, ti + 1, s, j)) return true;
      }
      return false;
    }
    case Tok::SlashOrMid: {
      // (/|/.+/)
      if (si >= s.size() || s[si] != '/') return false;
      if (gi_match(t, ti + 1, s, si + 1)) return true;
      for (size_t j = si + 2; j < s.size(); ++j)
        if (s[j] == '/' && gi_match(t, ti + 1, s, j + 1)) return true;
      return false;
    }
  }
  return false;
}

bool GitIgnore::matches(const std::string& path) const {
  bool m = false;
  for (auto& p : pats_) {
    g_gi_memo.reset(p.toks.size(), path.size());
    if (gi_match(p.toks, 0, path, 0)) {
      if (!p.negate)
        m = true;
      else if (m)
        m = false;
    }
  }
  return m;
}

// ---------------------------------------------------------------- filepath.Match

static bool match_class(const std::string& pat, size_t* pi, char c, bool* ok) {
  // pat[*pi] == '['
  size_t i = *pi + 1;
  bool neg = false;
  if (i < pat.size() && (pat[i] == '^' || pat[i] == '!')) {
    neg = true;
    ++i;
  }
  bool matched = false;
  bool first = true;
  while (i < pat.size() && (pat[i] != ']' || first)) {
    first = false;
    char lo = pat[i];
    if (lo == '\\' && i + 1 < pat.size()) lo = pat[++i];
    char hi = lo;
    if (i + 2 < pat.size() && pat[i + 1] == '-' && pat[i + 2] != ']') {
      hi = pat[i + 2];
      if (hi == '\\' && i + 3 < pat.size()) {
        hi = pat[i + 3];
        ++i;
      }
      i += 2;
    }
    if (lo <= c && c <= hi) matched = true;
    ++i;
  }
  if (i >= pat.size()) {
    *ok = false;
    return false;
  }
  *pi = i + 1;
  *ok = true;
  return matched != neg;
}

static bool pm_rec_(const std::string& p, size_t pi, const std::string& s, size_t si);
static bool pm_rec(const std::string& p, size_t pi, const std::string& s, size_t si) {
  if (g_pm_memo.failed(pi, si)) return false;
  return pm_rec_(p, pi, s, si) || g_pm_memo.fail(pi, si);
}

static bool pm_rec_(const std::string& p, size_t pi, const std::string& s, size_t si) {
  while (pi < p.size()) {
    char c = p[pi];
    if (c == '*') {
      while (pi < p.size() && p[pi] == '*') ++pi;
      for (size_t j = si;; ++j) {
        if (pm_rec(p, pi, s, j)) return true;
        if (j >= s.size() || s[j] == '/') return false;
      }
    }
    if (si >= s.size()) return false;
    if (c == '?') {
      if (s[si] == '/') return false;
      ++pi;
      ++si;
      continue;
    }
    if (c == '[') {
      bool ok;
      size_t np = pi;
      bool m = match_class(p, &np, s[si], &ok);
      if (!ok || !m || s[si] == '/') return false;
      pi = np;
      ++si;
      continue;
    }
    if (c == '\\' && pi + 1 < p.size()) {
      ++pi;
      c = p[pi];
    }
    if (s[si] != c) return false;
    ++pi;
    ++si;
  }
  return si == s.size();
}

bool path_match(const std::string& pattern, const std::string& name) {
  g_pm_memo.reset(pattern.size(), name.size());
  return pm_rec(pattern, 0, name, 0);
}

// ---------------------------------------------------------------- docker ignore

// Docker's pattern regex: "**" matches across separators, "*" doesn't, "?" single non-sep.
static bool docker_rec_(const std::string& p, size_t pi, const std::string& s, size_t si);
static bool docker_rec(const std::string& p, size_t pi, const std::string& s, size_t si) {
  if (g_dk_memo.failed(pi, si)) return false;
  return docker_rec_(p, pi, s, si) || g_dk_memo.fail(pi, si);
}

static bool docker_match(const std::string& p, const std::string& s) {
  g_dk_memo.reset(p.size(), s.size());
  return docker_rec(p, 0, s, 0);
}

static bool docker_rec_(const std::string& p, size_t pi, const std::string& s, size_t si) {
  while (pi < p.size()) {
    char c = p[pi];
    if (c == '*') {
      if (pi + 1 < p.size() && p[pi + 1] == '*') {
        pi += 2;
        // "**/" may match zero dirs
        if (pi < p.size() && p[pi] == '/') {
          if (docker_rec(p, pi + 1, s, si)) return true;
        }
        for (size_t j = si; j <= s.size(); ++j)
          if (docker_rec(p, pi, s, j)) return true;
        return false;
      }
      ++pi;
      for (size_t j = si;; ++j) {
        if (docker_rec(p, pi, s, j)) return true;
        if (j >= s.size() || s[j] == '/') return false;
      }
    }
    if (si >= s.size()) return false;
    if (c == '?') {
      if (s[si] == '/') return false;
      ++pi;
      ++si;
      continue;
    }
    if (c == '[') {
      bool ok;
      size_t np = pi;
      bool m = match_class(p, &np, s[si], &ok);
      if (!ok || !m) return false;
      pi = np;
      ++si;
      continue;
    }
    if (c == '\\' && pi + 1 < p.size()) {
      ++pi;
      c = p[pi];
    }
    if (s[si] != c) return false;
    ++pi;
    ++si;
  }
  return si == s.size();
}

DockerIgnore::DockerIgnore(const std::vector<std::string>& patterns) {
  for (auto raw : patterns) {
    std::string pat = trim(raw);
    if (pat.empty()) continue;
    P p;
    if (pat[0] == '!') {
      p.exclusion = true;
      pat = pat.substr(1);
      exclusions_ = true;
    }
    pat = fs::clean(pat);
    if (starts_with(pat, "/")) pat = pat.substr(1);
    if (pat.empty() || pat == ".") continue;
    p.pat = pat;
    p.dirs = split(pat, "/");
    pats_.push_back(p);
  }
}

bool DockerIgnore::matches(const std::string& rel_in) const {
  std::string rel = rel_in;
  if (starts_with(rel, "./")) rel = rel.substr(2);
  if (starts_with(rel, "/")) rel = rel.substr(1);
  std::vector<std::string> parent_dirs = split(fs::dirname(rel), "/");
  bool parent_is_root = fs::dirname(rel) == ".";
  bool matched = false;
  for (auto& p : pats_) {
    if (p.exclusion != matched) continue;  // only patterns that can flip the state matter
    bool m = docker_match(p.pat, rel);
    if (!m && !parent_is_root) {
      if (p.dirs.size() <= parent_dirs.size()) {
        std::vector<std::string> sub(parent_dirs.begin(), parent_dirs.begin() + p.dirs.size());
        m = docker_match(p.pat, join(sub, "/"));
      }
    }
    if (m) matched = !p.exclusion;
  }
  return matched;
}

bool DockerIgnore::dir_may_contain_exception(const std::string& rel_dir) const {
  if (!exclusions_) return false;
  std::string d = rel_dir;
  if (starts_with(d, "./")) d = d.substr(2);
  std::string dir_slash = d + "/";
  for (auto& p : pats_) {
    if (!p.exclusion) continue;
    if (starts_with(p.pat + "/", dir_slash)) return true;
    // wildcard exceptions may match anything below
    if (p.pat.find('*') != std::string::npos || p.pat.find('?') != std::string::npos) return true;
  }
  return false;
}

std::vector<std::string> read_dockerignore(const std::string& path) {
  std::vector<std::string> out;
  std::string data;
  if (!fs::read_file(path, &data)) return out;
  for (auto& line : split(data, "\n")) {
    std::string l = trim(line);
    if (l.empty() || l[0] == '#') continue;
    out.push_back(l);
  }
  return out;
}

// ---------------------------------------------------------------- doublestar

static bool brace_expand_match(const std::string& pattern, const std::string& path);

static bool seg_match(const std::string& pat, const std::string& seg) { return path_match(pat, seg); }

static bool ds_rec_(const std::vector<std::string>& p, size_t pi, const std::vector<std::string>& s, size_t si);
static bool ds_rec(const std::vector<std::string>& p, size_t pi, const std::vector<std::string>& s, size_t si) {
  if (g_ds_memo.failed(pi, si)) return false;
  return ds_rec_(p, pi, s, si) || g_ds_memo.fail(pi, si);
}

static bool ds_rec_(const std::vector<std::string>& p, size_t pi, const std::vector<std::string>& s, size_t si) {
  if (pi == p.size()) return si == s.size();
  if (p[pi] == "**") {
    for (size_t j = si; j <= s.size(); ++j)
      if (ds_rec(p, pi + 1, s, j)) return true;
    return false;
  }
  if (si >= s.size()) return false;
  if (!seg_match(p[pi], s[si])) return false;
  return ds_rec(p, pi + 1, s, si + 1);
}

static std::vector<std::string> expand_braces(const std::string& pat) {
  size_t open = pat.find('{');
  if (open == std::string::npos) return {pat};
  int depth = 0;
  size_t close = std::string::npos;
  std::vector<size_t> commas;
  for (size_t i = open; i < pat.size(); ++i) {
    if (pat[i] == '{')
      ++depth;
    else if (pat[i] == '}') {
      if (--depth == 0) {
        close = i;
        break;
      }
    } else if (pat[i] == ',' && depth == 1)
      commas.push_back(i);
  }
  if (close == std::string::npos) return {pat};
  std::vector<std::string> alts;
  size_t start = open + 1;
  for (size_t c : commas) {
    alts.push_back(pat.substr(start, c - start));
    start = c + 1;
  }
  alts.push_back(pat.substr(start, close - start));
  std::vector<std::string> out;
  for (auto& a : alts)
    for (auto& e : expand_braces(pat.substr(0, open) + a + pat.substr(close + 1))) out.push_back(e);
  return out;
}

static bool brace_expand_match(const std::string& pattern, const std::string& path) {
  for (auto& pat : expand_braces(pattern)) {
    bool abs = starts_with(pat, "/");
    if (abs != starts_with(path, "/")) continue;
    auto ps = split_nonempty(pat, '/');
    auto ss = split_nonempty(path, '/');
    g_ds_memo.reset(ps.size(), ss.size());
    if (ds_rec(ps, 0, ss, 0)) return true;
  }
  return false;
}

bool glob_match(const std::string& pattern, const std::string& path) { return brace_expand_match(pattern, path); }

std::vector<std::string> glob_expand(const std::string& pattern_in) {
  std::vector<std::string> out;
  for (auto& pattern : expand_braces(pattern_in)) {
    bool abs = fs::is_abs(pattern);
    std::string pat = pattern;
    if (starts_with(pat, "./")) pat = pat.substr(2);
    auto segs = split_nonempty(pat, '/');
    // find first segment with magic
    size_t first_magic = segs.size();
    for (size_t i = 0; i < segs.size(); ++i) {
      if (segs[i].find_first_of("*?[") != std::string::npos) {
        first_magic = i;
        break;
      }
    }
    std::string base = abs ? "/" : "";
    for (size_t i = 0; i < first_magic; ++i) base = fs::join(base, segs[i]);
    if (first_magic == segs.size()) {
      std::string p = base.empty() ? "." : base;
      if (fs::exists(p)) out.push_back(starts_with(pattern, "./") ? "./" + fs::relative(".", p) : p);
      continue;
    }
    std::string root = base.empty() ? "." : base;
    if (!fs::is_dir(root)) continue;
    fs::walk(root, [&](const std::string& p, const fs::StatInfo&) {
      std::string candidate = p;
      if (!abs) {
        candidate = p == "." ? "" : (starts_with(p, "./") ? p.substr(2) : p);
      }
      if (!candidate.empty() && brace_expand_match(abs ? pattern : pat, candidate)) {
        out.push_back(starts_with(pattern, "./") ? "./" + candidate : candidate);
      }
      return true;
    });
  }
  std::sort(out.begin(), out.end());
  out.erase(std::unique(out.begin(), out.end()), out.end());
  return out;
}

std::vector<std::string> collect_dockerignore_rules(const std::string& root) {
  std::vector<std::string> rules;
  std::vector<std::string> files;
  fs::walk(root, [&](const std::string& p, const fs::StatInfo& st) {
    if (!st.is_dir && fs::basename(p) == ".dockerignore") files.push_back(p);
    return true;
  });
  std::sort(files.begin(), files.end());
  for (auto& f : files) {
    std::string prefix = fs::relative(root, fs::dirname(f));
    if (!prefix.empty()) prefix = "/" + prefix;
    std::string data;
    if (!fs::read_file(f, &data)) continue;
    for (auto& line : split(data, "\n")) {
      std::string rule = trim(trim(line, "\r"), " ");
      if (rule.empty() || rule[0] == '#') continue;
      std::string out;
      if (!prefix.empty()) {
        size_t off = 0;
        if (rule[0] == '!') {
          out = "!";
          off = 1;
        }
        if (rule[off] == '/')
          out += rule.substr(off);
        else
          out += prefix + "/**/" + rule.substr(off);
      } else {
        out = rule;
      }
      if (out != "Dockerfile" && out != "/Dockerfile") rules.push_back(out);
    }
  }
  return rules;
}

}  // namespace ds

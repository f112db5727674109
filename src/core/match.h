// Path pattern matchers used across the tool:
//  * GitIgnore  — sync exclude / downloadExclude / uploadExclude lists. Semantics follow the
//                 gitignore line compiler the reference uses (sync/util.go:291 compilePaths,
//                 github.com/sabhiram/go-gitignore): "/x" anchors to the sync root, "x/" matches
//                 a directory subtree, "*" stays inside one segment, "**" spans segments, "!"
//                 re-includes.
//  * DockerIgnore — .dockerignore semantics (util/hash/hash.go:43, builder/docker/docker.go:94):
//                 filepath.Match per pattern, parent-directory matching, "!" exceptions.
//  * glob_match / glob_expand — doublestar globs (watch/watch.go:104, deploy/kubectl/manifests.go:35).
#pragma once

#include <string>
#include <vector>

namespace ds {

class GitIgnore {
 public:
  GitIgnore() = default;
  explicit GitIgnore(const std::vector<std::string>& lines) { add_lines(lines); }
  void add_lines(const std::vector<std::string>& lines);
  void add_line(const std::string& line);
  bool empty() const { return pats_.empty(); }
  // `path` is slash-separated, typically relative with a leading "/" ("/src/a.js").
  bool matches(const std::string& path) const;

  struct Tok {
    enum Kind { Lit, Star, OptAnySlash, OptSlashAny, Any, SlashOrMid, OptSlash } kind;
    char c;
  };
  struct Pat {
    std::vector<Tok> toks;
    bool negate = false;
  };

 private:
  std::vector<Pat> pats_;
};

// filepath.Match (Go) semantics: '*' no '/', '?', character classes, '\\' escapes.
bool path_match(const std::string& pattern, const std::string& name);

class DockerIgnore {
 public:
  DockerIgnore() = default;
  explicit DockerIgnore(const std::vector<std::string>& patterns);
  // `rel` is a slash-separated path relative to the context root, without leading "./" or "/".
  bool matches(const std::string& rel) const;
  bool has_exclusions() const { return exclusions_; }
  // True if a directory that matched may still contain re-included ("!") entries.
  bool dir_may_contain_exception(const std::string& rel_dir) const;
  bool empty() const { return pats_.empty(); }

  struct P {
    std::string pat;
    std::vector<std::string> dirs;
    bool exclusion = false;
  };

 private:
  std::vector<P> pats_;
  bool exclusions_ = false;
};

// Reads a .dockerignore file into cleaned patterns (comments/blank lines dropped).
std::vector<std::string> read_dockerignore(const std::string& path);

// Doublestar glob: "**" matches any number of path segments (including zero).
bool glob_match(const std::string& pattern, const std::string& path);
// Expands a glob against the filesystem (relative patterns are resolved against cwd and
// returned relative). Results are sorted.
std::vector<std::string> glob_expand(const std::string& pattern);

// util/ignoreutil/ignorefile.go:12 — gather all nested .dockerignore rules under root.
std::vector<std::string> collect_dockerignore_rules(const std::string& root);

}  // namespace ds

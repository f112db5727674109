// Go text/template interpreter (with the Sprig/Helm function subset charts use) so Helm charts
// render natively — no Tiller (helm/tiller.go) and no helm binary needed.
//
// Supported: text + {{ }} actions with {{- -}} trimming, comments, pipelines, variables
// ($x := / $x =, $ root), field chains, if/else if/else, range (with $i, $v := ; else),
// with/else, define/template/include/block, parenthesized pipelines, and functions:
// eq ne lt le gt ge and or not len index print printf println default empty coalesce ternary
// required fail quote squote toYaml toJson fromYaml indent nindent trim trimAll trimPrefix
// trimSuffix upper lower title replace contains hasPrefix hasSuffix trunc repeat join split
// splitList list dict get set unset hasKey keys values merge int int64 float64 toString atoi
// add sub mul div mod max min until b64enc b64dec sha256sum kindIs typeOf regexMatch
// regexReplaceAll semverCompare tpl lookup (nil) now date uuidv4 randAlphaNum, plus the wider
// Sprig set stable charts use (string case/abbrev/wrap/substr, list append/prepend/concat/uniq/
// without/rest/initial/reverse/sortAlpha/compact/slice, dict pick/omit/pluck/dig/deepCopy,
// regexFind(All)/regexSplit, path base/dir/ext/clean, math floor/ceil/round, sha1/adler32,
// b32enc/dec, semver, toToml, fromYamlArray/fromJsonArray, urlquery, and the must* variants),
// and method calls on Helm's Files / APIVersions objects (see below).
#pragma once

#include <functional>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "core/value.h"

namespace ds {
namespace tmpl {

struct TemplateError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

class Engine {
 public:
  Engine();
  ~Engine();
  // Parse a named template (its {{define}} blocks are registered too).
  void add(const std::string& name, const std::string& text);
  // Execute a template with `dot` as data; returns the rendered text.
  std::string execute(const std::string& name, const Value& dot);
  bool has(const std::string& name) const;
  // Optional hook for `lookup` (api server queries); default returns an empty map.
  std::function<Value(const std::string& api_version, const std::string& kind, const std::string& ns,
                      const std::string& name)>
      lookup;

  struct Impl;

 private:
  std::unique_ptr<Impl> impl_;
};

// Helm's built-in objects with methods. Go templates call methods on values
// (`.Files.Get "x"`, `(.Files.Glob "conf/*").AsConfig`, `.Capabilities.APIVersions.Has "apps/v1"`);
// these are maps tagged with a reserved key that the engine dispatches method calls on.
//   Files:       Get GetBytes Glob Lines AsConfig AsSecrets   (helm pkg/engine/files.go)
//   APIVersions: Has
Value make_files_object(const std::vector<std::pair<std::string, std::string>>& files);
Value make_api_versions_object(const std::vector<std::string>& versions);

// Masterminds/semver constraint check (semverCompare, requirements version ranges):
// "^1.2", "~1.2.3", ">=1.19-0", "1.x", "1.2 - 1.4", "a || b", "a, b". Throws on a bad version.
bool semver_match(const std::string& constraint, const std::string& version);

}  // namespace tmpl
}  // namespace ds

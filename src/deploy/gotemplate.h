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
// regexReplaceAll semverCompare tpl lookup (nil) now date uuidv4 randAlphaNum.
#pragma once

#include <functional>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>

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

}  // namespace tmpl
}  // namespace ds

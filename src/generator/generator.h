// Project scaffolding for `devspace init` (generator/generator.go): language detection and
// chart + Dockerfile creation. Unlike the reference, which git-clones a template repository at
// init time (generator.go:129), the templates are compiled into the binary (templates/ in the
// source tree) so init works offline; a local template directory (--templateRepoPath) with the
// same layout (`_base/` + one directory per language) takes precedence when given.
#pragma once

#include <map>
#include <string>
#include <vector>

namespace ds {
namespace generator {

class ChartGenerator {
 public:
  // template_dir: optional on-disk template repository; empty = embedded templates.
  explicit ChartGenerator(std::string project_dir, std::string template_dir = "");
  std::vector<std::string> supported_languages() const;
  bool is_supported(const std::string& lang) const;
  // Bytes-by-language over the project tree (vendor/dot/doc/config paths skipped, 10 s cap);
  // returns the supported language with the most bytes, or "" (generator.go:160).
  std::string detect_language() const;
  // Copies _base/ then <language>/ into the project without overwriting existing files
  // unless `overwrite` (generator.go:88 CreateChart).
  void create_chart(const std::string& language, bool overwrite) const;
  // Files of a template (relative path -> content), for tests.
  std::map<std::string, std::string> files(const std::string& dir) const;

 private:
  std::string project_, template_dir_;
};

// Language for a file name (extension / well-known file name), "" if unknown.
std::string language_of(const std::string& path);
// All embedded template files (relative path -> bytes).
const std::map<std::string, std::string>& embedded_templates();

}  // namespace generator
}  // namespace ds

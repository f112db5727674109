#include "generator/generator.h"

#include <chrono>
#include <set>

#include "core/fs.h"
#include "core/strutil.h"

namespace ds {
namespace generator {

const std::map<std::string, std::string>& embedded_templates() {
  static const std::map<std::string, std::string> m = {
#include "embedded_templates.inc"
  };
  return m;
}

ChartGenerator::ChartGenerator(std::string project_dir, std::string template_dir)
    : project_(std::move(project_dir)), template_dir_(std::move(template_dir)) {}

std::map<std::string, std::string> ChartGenerator::files(const std::string& dir) const {
  std::map<std::string, std::string> out;
  if (!template_dir_.empty()) {
    std::string root = fs::join(template_dir_, dir);
    if (!fs::is_dir(root)) return out;
    fs::walk(root, [&](const std::string& p, const fs::StatInfo& st) {
      if (st.is_dir) return fs::basename(p) != ".git";
      out[fs::relative(root, p)] = fs::read_file(p);
      return true;
    });
    return out;
  }
  std::string prefix = dir + "/";
  for (auto& kv : embedded_templates())
    if (starts_with(kv.first, prefix)) out[kv.first.substr(prefix.size())] = kv.second;
  return out;
}

std::vector<std::string> ChartGenerator::supported_languages() const {
  std::set<std::string> langs;
  if (!template_dir_.empty()) {
    for (auto& e : fs::list_dir(template_dir_))
      if (e.is_dir && e.name[0] != '_' && e.name[0] != '.') langs.insert(e.name);
  } else {
    for (auto& kv : embedded_templates()) {
      size_t s = kv.first.find('/');
      if (s == std::string::npos) continue;
      std::string d = kv.first.substr(0, s);
      if (d[0] != '_' && d[0] != '.') langs.insert(d);
    }
  }
  return {langs.begin(), langs.end()};
}

bool ChartGenerator::is_supported(const std::string& lang) const {
  for (auto& l : supported_languages())
    if (l == lang) return true;
  return false;
}

std::string language_of(const std::string& path) {
  static const std::map<std::string, std::string> ext = {
      {".js", "javascript"}, {".mjs", "javascript"}, {".jsx", "javascript"}, {".ts", "javascript"},
      {".tsx", "javascript"}, {".py", "python"},     {".go", "go"},          {".java", "java"},
      {".kt", "java"},       {".scala", "java"},     {".php", "php"},        {".rb", "ruby"},
      {".hip", "rocm-pytorch"}, {".cu", "rocm-pytorch"}};
  static const std::map<std::string, std::string> names = {
      {"package.json", "javascript"}, {"requirements.txt", "python"}, {"setup.py", "python"},
      {"go.mod", "go"},               {"pom.xml", "java"},            {"build.gradle", "java"},
      {"composer.json", "php"},       {"Gemfile", "ruby"},            {"Rakefile", "ruby"}};
  std::string base = fs::basename(path);
  auto n = names.find(base);
  if (n != names.end()) return n->second;
  auto e = ext.find(to_lower(fs::extension(path)));
  return e == ext.end() ? "" : e->second;
}

static bool skipped_path(const std::string& rel, bool is_dir) {
  std::string base = fs::basename(rel);
  if (!base.empty() && base[0] == '.') return true;  // dot files / dirs
  static const std::set<std::string> vendor = {"node_modules", "vendor", "bower_components", "__pycache__",
                                               "site-packages", "venv", "env", "third_party", "dist", "build",
                                               "target", "docs", "doc", "Documentation", "chart", "charts"};
  if (is_dir) return vendor.count(base) > 0;
  static const std::set<std::string> doc_ext = {".md", ".rst", ".txt", ".yaml", ".yml", ".json", ".toml",
                                                ".ini", ".cfg", ".lock", ".xml"};
  std::string e = to_lower(fs::extension(rel));
  if (doc_ext.count(e) && language_of(rel).empty()) return true;
  return false;
}

std::string ChartGenerator::detect_language() const {
  std::map<std::string, int64_t> bytes;
  auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(10);
  bool torch = false;
  fs::walk(project_, [&](const std::string& p, const fs::StatInfo& st) {
    if (std::chrono::steady_clock::now() > deadline) return false;
    std::string rel = fs::relative(project_, p);
    if (rel == "." || rel.empty()) return true;
    if (skipped_path(rel, st.is_dir)) return false;
    if (st.is_dir) return true;
    std::string lang = language_of(p);
    if (lang.empty()) return true;
    bytes[lang] += st.size ? st.size : 1;
    // GPU training code: python importing torch is served by the ROCm PyTorch template.
    if (lang == "python" && !torch && st.size < (4 << 20)) {
      std::string src;
      if (fs::read_file(p, &src) &&
          (contains(src, "import torch") || contains(src, "from torch") || contains(src, "torch.distributed")))
        torch = true;
    }
    return true;
  });
  if (torch) {
    bytes["rocm-pytorch"] += bytes["python"] + 1;
    bytes.erase("python");
  }
  std::string best;
  int64_t most = 0;
  for (auto& kv : bytes)
    if (is_supported(kv.first) && kv.second > most) {
      best = kv.first;
      most = kv.second;
    }
  return best;
}

// The python/ruby templates start `main.<ext>`; a project whose entry file has another
// conventional name (app.py, server.py, ...) or that has a single top-level source file gets
// that file in the generated Dockerfile's CMD instead of a CMD that crashes on start.
static std::string entry_file(const std::string& project, const std::string& ext) {
  if (fs::exists(fs::join(project, "main" + ext))) return "main" + ext;
  for (const char* base : {"app", "server", "run", "wsgi", "__main__"})
    if (fs::exists(fs::join(project, base + ext))) return base + ext;
  std::vector<std::string> top;
  for (auto& e : fs::list_dir(project))
    if (!e.is_dir && ends_with(e.name, ext)) top.push_back(e.name);
  return top.size() == 1 ? top[0] : "main" + ext;
}

void ChartGenerator::create_chart(const std::string& language, bool overwrite) const {
  if (!is_supported(language)) throw std::runtime_error("Language Template not found");
  for (const std::string& dir : {std::string("_base"), language}) {
    for (auto& kv : files(dir)) {
      std::string dst = fs::join(project_, kv.first);
      if (!overwrite && fs::exists(dst)) continue;
      std::string content = kv.second;
      if (kv.first == "Dockerfile") {
        for (const char* ext : {".py", ".rb"}) {
          std::string tmpl = std::string("\"main") + ext + "\"";
          size_t at = content.find(tmpl);
          if (at != std::string::npos) content.replace(at, tmpl.size(), "\"" + entry_file(project_, ext) + "\"");
        }
      }
      fs::write_file(dst, content, ends_with(kv.first, ".sh") ? 0755 : 0644);
    }
  }
}

}  // namespace generator
}  // namespace ds

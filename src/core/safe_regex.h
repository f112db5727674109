// std::regex (libstdc++) matches recursively, one stack frame chain per input character: a
// 100 kB line overflows an 8 MB stack and kills the process. These wrappers run matches on
// long inputs on a thread whose stack is sized for the input (reserved lazily by mmap, so an
// unused reserve costs nothing), with the same results as the std:: calls. Inputs over 1 MiB
// throw instead.
#pragma once

#include <functional>
#include <regex>
#include <string>

namespace ds {

bool safe_regex_search(const std::string& s, std::smatch* m, const std::regex& re);
bool safe_regex_search(const std::string& s, const std::regex& re);
bool safe_regex_match(const std::string& s, std::smatch* m, const std::regex& re);
bool safe_regex_match(const std::string& s, const std::regex& re);
std::string safe_regex_replace(const std::string& s, const std::regex& re, const std::string& fmt);
// Runs `fn` (regex work over an input of `input_bytes`) with a stack sized for it.
void safe_regex_run(size_t input_bytes, const std::function<void()>& fn);

}  // namespace ds

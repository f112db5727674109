// Counterparts of the reference's small utility tests, so every `*_test.go` of
// /root/reference has one here (the sync and config ones are in test_sync.cc / test_config.cc /
// test_core.cc):
//   pkg/util/randutil/rand_test.go        TestGenerateRandomString
//   pkg/util/paramutil/param_test.go      TestSetDefaults (prompt parameters' defaults)
//   pkg/util/processutil/pipe_test.go     TestPipe, TestPipeWithWaitGroup
//   pkg/util/fsutil/filesystem_test.go    (commented out upstream) write/read/overwrite, copy, home
//   pkg/util/log/logger_test.go           (commented out upstream) JSON file logger levels
// pkg/util/jujuerr_test.go only logs a juju error trace; errors here are exceptions with their
// message, covered wherever an error is asserted.
#include <unistd.h>

#include <cstdlib>
#include <regex>
#include <set>
#include <thread>

#include "core/codec.h"
#include "core/fs.h"
#include "core/strutil.h"
#include "core/value.h"
#include "core/log.h"
#include "core/proc.h"
#include "core/prompt.h"
#include "testing.h"

using namespace ds;

TEST(ref_rand_generates_alphanumeric_strings) {
  // rand_test.go:8 — 10000 one-character strings, letters and digits only
  std::regex forbidden("[^a-zA-Z0-9]");
  std::set<char> seen;
  for (int i = 0; i < 10000; ++i) {
    std::string s = random_string(1);
    EXPECT_EQ(s.size(), (size_t)1);
    EXPECT_TRUE(!std::regex_search(s, forbidden));
    seen.insert(s[0]);
  }
  EXPECT_EQ(seen.size(), (size_t)62);  // and every one of them turns up
  for (int i = 0; i < 1000; ++i) {
    std::string s = random_lower_alnum(8);
    EXPECT_EQ(s.size(), (size_t)8);
    EXPECT_TRUE(!std::regex_search(s, std::regex("[^a-z0-9]")));
  }
}

TEST(ref_prompt_parameters_default_when_empty) {
  // param_test.go:15 — an empty validation pattern means "anything" (the reference fills in
  // ".*"); a given one is kept and enforced
  prompt::Params any;
  any.question = "Anything?";
  any.key = "ref-any";
  prompt::set_answer("ref-any", "x y z");
  EXPECT_EQ(prompt::ask(any), std::string("x y z"));
  prompt::Params digits;
  digits.question = "A number?";
  digits.validation_regex = "[0-9]+";
  digits.key = "ref-digits";
  prompt::set_answer("ref-digits", "42");
  EXPECT_EQ(prompt::ask(digits), std::string("42"));
  prompt::set_answer("ref-digits", "4x2");
  bool threw = false;
  try {
    prompt::ask(digits);
  } catch (const std::exception&) {
    threw = true;
  }
  EXPECT_TRUE(threw);  // a preset answer is checked like a typed one
  EXPECT_EQ(digits.validation_regex, std::string("[0-9]+"));  // the caller's params are untouched
}

TEST(ref_pipe_copies_in_order_and_stops_at_eof) {
  // pipe_test.go:12,31 — a reader's bytes reach the writer in order, in buffer-sized pieces,
  // and the copy ends at EOF (or an error) without reading on
  int in[2], out[2];
  EXPECT_EQ(::pipe(in), 0);
  EXPECT_EQ(::pipe(out), 0);
  const std::string message = "Hello World";  // longer than the buffer
  std::thread copier([&] {
    char buf[10];
    size_t reads = 0;
    while (true) {
      ssize_t n = read_some(in[0], buf, sizeof(buf), 2000);
      ++reads;
      if (n <= 0) break;
      if (!write_all(out[1], buf, (size_t)n)) break;
    }
    ::close(out[1]);
    EXPECT_TRUE(reads >= 3);  // two pieces and the end
  });
  EXPECT_TRUE(write_all(in[1], message));
  ::close(in[1]);
  std::string got = read_all(out[0]);
  copier.join();
  ::close(in[0]);
  ::close(out[0]);
  EXPECT_EQ(got, message);
}

TEST(ref_fs_write_read_overwrite_copy_home) {
  // filesystem_test.go (commented out upstream, Windows paths): write a new file under missing
  // directories, read it back, overwrite it, copy it; the home directory is $HOME's
  std::string root = fs::make_temp_dir("ref-fs-");
  std::string name = random_string(10);
  std::string p = root + "/" + name + "/" + name;
  fs::write_file(p, "Content " + name);
  EXPECT_EQ(fs::read_file(p), "Content " + name);
  fs::write_file(p, "New Content " + name);
  EXPECT_EQ(fs::read_file(p), "New Content " + name);
  std::string q = root + "/" + random_string(10) + "/copy";
  fs::copy(p, q);
  EXPECT_EQ(fs::read_file(q), "New Content " + name);
  fs::write_file(p, "");
  fs::copy(p, q);  // no overwrite by default
  EXPECT_EQ(fs::read_file(q), "New Content " + name);
  fs::copy(p, q, true);
  EXPECT_EQ(fs::read_file(q), std::string());
  const char* home = std::getenv("HOME");
  if (home && *home) EXPECT_EQ(fs::home_dir(), std::string(home));
  fs::remove_all(root);
}

TEST(ref_file_logger_writes_levels_and_messages) {
  // logger_test.go (commented out upstream): a named file logger writes one JSON object per
  // line with the level and the message
  std::string dir = fs::make_temp_dir("ref-log-");
  std::string saved = log::logdir();
  log::logdir() = dir;
  auto l = log::file_logger("TestLogger");
  l->info("Some Test Log");
  l->warn("More Logs");
  log::logdir() = saved;
  std::vector<std::string> lines;
  for (auto& s : split(fs::read_file(l->path()), "\n"))
    if (!s.empty()) lines.push_back(s);
  EXPECT_EQ(lines.size(), (size_t)2);
  Value a = json_parse(lines[0]), b = json_parse(lines[1]);
  EXPECT_EQ(a.get("level").as_string(), std::string("info"));
  EXPECT_EQ(a.get("msg").as_string(), std::string("Some Test Log"));
  EXPECT_EQ(b.get("level").as_string(), std::string("warning"));
  EXPECT_EQ(b.get("msg").as_string(), std::string("More Logs"));
  fs::remove_all(dir);
}

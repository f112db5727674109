// Build-context hashing (util/hash/hash.go DirectoryExcludes semantics + incremental CRC cache),
// Dockerfile entrypoint override, image name helpers.
#include <unistd.h>

#include "build/docker.h"
#include "core/fs.h"
#include "core/strutil.h"
#include "testing.h"

using namespace ds;

TEST(context_hash_incremental_cache_matches_full_hash) {
  std::string d = fs::make_temp_dir("ctx-");
  fs::write_file(fs::join(d, "a.txt"), "alpha");
  fs::write_file(fs::join(d, "sub/b.bin"), std::string(1 << 20, 'b'));
  fs::write_file(fs::join(d, "node_modules/x.js"), "ignored");
  std::string cache = fs::join(d, "../" + fs::basename(d) + "-crc.json");
  std::vector<std::string> ex = {"node_modules"};
  std::string full = build::hash_directory_excludes(d, ex);
  std::string first = build::hash_directory_excludes(d, ex, cache);
  EXPECT_EQ(first, full);
  EXPECT_TRUE(fs::exists(cache));
  EXPECT_TRUE(contains(fs::read_file(cache), "b.bin"));
  EXPECT_TRUE(!contains(fs::read_file(cache), "x.js"));
  std::string second = build::hash_directory_excludes(d, ex, cache);  // served from the cache
  EXPECT_EQ(second, full);
  // excluded files do not affect the hash
  fs::write_file(fs::join(d, "node_modules/x.js"), "changed");
  EXPECT_EQ(build::hash_directory_excludes(d, ex, cache), full);
  // a content change with a new mtime is detected
  usleep(10000);
  fs::write_file(fs::join(d, "a.txt"), "ALPHA");
  std::string third = build::hash_directory_excludes(d, ex, cache);
  EXPECT_TRUE(third != full);
  EXPECT_EQ(third, build::hash_directory_excludes(d, ex));
  // a stale/corrupt cache is ignored
  fs::write_file(cache, "{not json");
  EXPECT_EQ(build::hash_directory_excludes(d, ex, cache), third);
  fs::remove_all(d);
  fs::remove(cache);
}

TEST(image_name_helpers) {
  EXPECT_EQ(build::registry_from_image("nginx"), std::string(""));
  EXPECT_EQ(build::registry_from_image("user/app:1"), std::string(""));
  EXPECT_EQ(build::registry_from_image("gcr.io/proj/app:1"), std::string("gcr.io"));
  EXPECT_EQ(build::registry_from_image("localhost:5000/app"), std::string("localhost:5000"));
  EXPECT_EQ(build::split_image_tag("reg:5000/a/b:tag").second, std::string("tag"));
  EXPECT_EQ(build::split_image_tag("reg:5000/a/b").second, std::string(""));
  EXPECT_EQ(build::pull_secret_name("my.Reg:5000"), std::string("devspace-auth-my-reg-5000"));
}

// util/dockerfile/get.go:14 GetPorts
TEST(dockerfile_ports_like_get_ports) {
  EXPECT_TRUE(build::dockerfile_ports("FROM node\nRUN x\n").empty());
  auto p = build::dockerfile_ports("FROM node\r\nEXPOSE 3000 8080/tcp\rEXPOSE 3000\nEXPOSE  9229/udp\n  EXPOSE 1\nexpose 2\n");
  EXPECT_EQ(p.size(), (size_t)3);
  EXPECT_EQ(p[0], 3000);
  EXPECT_EQ(p[1], 8080);
  EXPECT_EQ(p[2], 9229);
  EXPECT_THROWS(build::dockerfile_ports("EXPOSE $PORT\n"));
}

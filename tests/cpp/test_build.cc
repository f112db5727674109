// Build-context hashing (util/hash/hash.go DirectoryExcludes semantics + incremental CRC cache),
// Dockerfile entrypoint override, image name helpers.
#include <unistd.h>

#include <map>

#include "build/docker.h"
#include "core/codec.h"
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

// The build context as the daemon receives it (archive.TarWithOptions in the reference,
// pkg/devspace/builder/docker/docker.go:96-140): .dockerignore rules with a "!" exception, a
// symlink kept as a symlink (never followed), ownership reset to 0:0, and the Dockerfile
// replaced by the override (the entrypoint rewrite of `devspace dev`) when one is given.
TEST(build_context_archive_keeps_symlinks_and_applies_dockerignore) {
  std::string d = fs::make_temp_dir("ctx-");
  fs::write_file(fs::join(d, "app.js"), "console.log(1)\n");
  fs::write_file(fs::join(d, "lib/util.js"), "module.exports = 2\n");
  fs::write_file(fs::join(d, "debug.log"), "noise");
  fs::write_file(fs::join(d, "logs/keep.log"), "kept by the exception");
  fs::write_file(fs::join(d, "Dockerfile"), "FROM node\nCMD [\"node\", \"app.js\"]\n");
  fs::write_file(fs::join(d, ".dockerignore"), "*.log\n**/*.log\n!logs/keep.log\n");
  EXPECT_EQ(::symlink("app.js", fs::join(d, "current.js").c_str()), 0);
  std::vector<std::string> ex = {"*.log", "**/*.log", "!logs/keep.log"};
  std::string override_df = "FROM node\nENTRYPOINT [\"sleep\", \"999\"]\n";
  std::string tar = build::context_tar(d, ex, "Dockerfile", override_df);
  TarReader tr(string_source(&tar));
  std::map<std::string, TarEntry> got;
  std::map<std::string, std::string> data;
  TarEntry e;
  while (tr.next(&e)) {
    got[e.name] = e;
    data[e.name] = tr.read_all();
  }
  EXPECT_TRUE(got.count("app.js") && got.count("lib/util.js") && got.count(".dockerignore"));
  EXPECT_TRUE(!got.count("debug.log"));
  EXPECT_TRUE(got.count("logs/keep.log"));
  EXPECT_EQ(data["logs/keep.log"], std::string("kept by the exception"));
  EXPECT_TRUE(got.count("current.js"));
  EXPECT_EQ(got["current.js"].type, '2');
  EXPECT_EQ(got["current.js"].linkname, std::string("app.js"));
  EXPECT_EQ(got["current.js"].size, (int64_t)0);
  EXPECT_EQ(data["Dockerfile"], override_df);
  EXPECT_EQ((int)got["Dockerfile"].mode, 0600);
  for (auto& kv : got) EXPECT_TRUE(kv.second.uid == 0 && kv.second.gid == 0);
  // no override: the Dockerfile goes in as it is on disk
  std::string plain = build::context_tar(d, ex, "Dockerfile", std::nullopt);
  TarReader tr2(string_source(&plain));
  std::string df;
  while (tr2.next(&e)) {
    std::string body = tr2.read_all();
    if (e.name == "Dockerfile") df = body;
  }
  EXPECT_EQ(df, fs::read_file(fs::join(d, "Dockerfile")));
  fs::remove_all(d);
}

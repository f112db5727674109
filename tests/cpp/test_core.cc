// Core library tests: YAML/JSON, matchers, tar/gzip, hashing, CLI parser.
#include <unistd.h>

#include <chrono>

#include "core/cli.h"
#include "core/codec.h"
#include "core/fs.h"
#include "core/match.h"
#include "core/proc.h"
#include "core/strutil.h"
#include "core/value.h"
#include "testing.h"

using namespace ds;

TEST(yaml_basic_map_and_seq) {
  Value v = yaml_parse(
      "version: v1alpha2\n"
      "cluster:\n"
      "  namespace: test   # comment\n"
      "dev:\n"
      "  sync:\n"
      "  - containerPath: /app\n"
      "    localSubPath: ./\n"
      "    uploadExcludePaths:\n"
      "    - Dockerfile\n"
      "    - node_modules/\n"
      "  ports:\n"
      "    - portMappings:\n"
      "        - localPort: 3000\n"
      "          remotePort: 3000\n");
  EXPECT_EQ(v.get("version").as_string(), std::string("v1alpha2"));
  EXPECT_EQ(v.at_path("cluster.namespace").as_string(), std::string("test"));
  const Value& sync = v.at_path("dev.sync");
  EXPECT_TRUE(sync.is_seq());
  EXPECT_EQ(sync.size(), (size_t)1);
  EXPECT_EQ(sync[0].get("containerPath").as_string(), std::string("/app"));
  EXPECT_EQ(sync[0].get("uploadExcludePaths").size(), (size_t)2);
  const Value& pm = v.at_path("dev.ports")[0].get("portMappings")[0];
  EXPECT_EQ(pm.get("localPort").as_int(), (int64_t)3000);
  EXPECT_TRUE(pm.get("localPort").is_int());
}

TEST(yaml_bom_and_crlf) {
  Value v = yaml_parse("\xEF\xBB\xBFversion: v1alpha2\r\nimages:\r\n  default:\r\n    image: x\r\n");
  EXPECT_EQ(v.get("version").as_string(), std::string("v1alpha2"));
  EXPECT_EQ(v.at_path("images.default.image").as_string(), std::string("x"));
}

TEST(yaml_colon_space_in_plain_value_is_an_error) {
  for (const char* bad : {"a: b: c\n", "a: b:\n", "- a: b\n- c: d: e\n"}) {
    bool threw = false;
    try {
      yaml_parse(bad);
    } catch (const std::exception& e) {
      threw = contains(e.what(), "mapping values are not allowed");
    }
    EXPECT_TRUE(threw);
  }
  EXPECT_EQ(yaml_parse("a: http://x:80/y\n").get("a").as_string(), std::string("http://x:80/y"));
  EXPECT_EQ(yaml_parse("a: b # c: d\n").get("a").as_string(), std::string("b"));
  EXPECT_EQ(yaml_parse("a: \"b: c\"\n").get("a").as_string(), std::string("b: c"));
  EXPECT_EQ(yaml_parse("a: b:c\n").get("a").as_string(), std::string("b:c"));
}

TEST(yaml_scalars_and_quotes) {
  Value v = yaml_parse(
      "a: \"123\"\n"
      "b: 123\n"
      "c: 'it''s'\n"
      "d: true\n"
      "e: ~\n"
      "f: \"line\\nbreak\"\n"
      "g: 1.5\n"
      "h: [a, 'b', {x: 1}]\n"
      "i: {k: v, n: 2}\n"
      "j: \"999999999999\"\n"
      "k: http://example.com:8080/x\n");
  EXPECT_TRUE(v.get("a").is_string());
  EXPECT_TRUE(v.get("b").is_int());
  EXPECT_EQ(v.get("c").as_string(), std::string("it's"));
  EXPECT_TRUE(v.get("d").as_bool());
  EXPECT_TRUE(v.get("e").is_null());
  EXPECT_EQ(v.get("f").as_string(), std::string("line\nbreak"));
  EXPECT_TRUE(v.get("g").is_float());
  EXPECT_EQ(v.get("h").size(), (size_t)3);
  EXPECT_EQ(v.get("h")[2].get("x").as_int(), (int64_t)1);
  EXPECT_EQ(v.get("i").get("n").as_int(), (int64_t)2);
  EXPECT_EQ(v.get("k").as_string(), std::string("http://example.com:8080/x"));
}

TEST(yaml_block_scalars_and_anchors) {
  Value v = yaml_parse(
      "lit: |\n"
      "  line1\n"
      "  line2\n"
      "fold: >-\n"
      "  a\n"
      "  b\n"
      "base: &b\n"
      "  x: 1\n"
      "derived:\n"
      "  <<: *b\n"
      "  y: 2\n");
  EXPECT_EQ(v.get("lit").as_string(), std::string("line1\nline2\n"));
  EXPECT_EQ(v.get("fold").as_string(), std::string("a b"));
  EXPECT_EQ(v.get("derived").get("x").as_int(), (int64_t)1);
  EXPECT_EQ(v.get("derived").get("y").as_int(), (int64_t)2);
}

TEST(yaml_multi_document) {
  auto docs = yaml_parse_all("a: 1\n---\nb: 2\n---\n# only comment\n---\nc: 3\n");
  EXPECT_EQ(docs.size(), (size_t)4);
  EXPECT_EQ(docs[1].get("b").as_int(), (int64_t)2);
  EXPECT_TRUE(docs[2].is_null());
}

TEST(yaml_roundtrip) {
  std::string src =
      "version: v1alpha2\n"
      "images:\n"
      "  default:\n"
      "    image: dscr.io/user/devspace\n"
      "    createPullSecret: true\n"
      "deployments:\n"
      "- name: devspace-app\n"
      "  helm:\n"
      "    chartPath: ./chart\n"
      "dev:\n"
      "  overrideImages:\n"
      "  - name: default\n"
      "    entrypoint:\n"
      "    - sleep\n"
      "    - \"999999999999\"\n";
  Value v = yaml_parse(src);
  std::string out = yaml_dump(v);
  EXPECT_EQ(out, src);
  Value v2 = yaml_parse(out);
  EXPECT_TRUE(v == v2);
  Value ml = Value::map();
  ml["s"] = "a\nb\n";
  ml["e"] = "";
  ml["n"] = "true";
  Value back = yaml_parse(yaml_dump(ml));
  EXPECT_EQ(back.get("s").as_string(), std::string("a\nb\n"));
  EXPECT_TRUE(back.get("e").is_string());
  EXPECT_TRUE(back.get("n").is_string());
}

TEST(json_roundtrip) {
  Value v = json_parse("{\"a\": [1, 2.5, \"x\\u00e9\", true, null], \"b\": {\"c\": \"d\"}}");
  EXPECT_EQ(v.get("a")[2].as_string(), std::string("x\xc3\xa9"));
  std::string d = json_dump(v);
  EXPECT_TRUE(json_parse(d) == v);
  EXPECT_EQ(json_dump(json_parse("{}")), std::string("{}"));
}

TEST(merge_semantics) {
  // config/configutil/merge_test.go:10 TestSimpleMerge — maps merge, slices replace.
  Value base = yaml_parse("a: 1\nm:\n  x: 1\n  y: [1, 2]\n");
  Value over = yaml_parse("b: 2\nm:\n  y: [3]\n  z: 4\n");
  merge_into(base, over);
  EXPECT_EQ(base.get("a").as_int(), (int64_t)1);
  EXPECT_EQ(base.get("b").as_int(), (int64_t)2);
  EXPECT_EQ(base.at_path("m.x").as_int(), (int64_t)1);
  EXPECT_EQ(base.at_path("m.y").size(), (size_t)1);
  EXPECT_EQ(base.at_path("m.z").as_int(), (int64_t)4);
}

TEST(gitignore_matcher) {
  GitIgnore gi({"/.devspace/logs", "node_modules/", "*.pyc", "ignoreFileLocal", "testFolder/deep", "!keep.pyc"});
  EXPECT_TRUE(gi.matches("/.devspace/logs"));
  EXPECT_TRUE(gi.matches("/.devspace/logs/sync.log"));
  EXPECT_TRUE(!gi.matches("/x/.devspace/logs"));
  EXPECT_TRUE(gi.matches("/node_modules/"));
  EXPECT_TRUE(gi.matches("/node_modules/a/b.js"));
  EXPECT_TRUE(gi.matches("/a/b/c.pyc"));
  EXPECT_TRUE(!gi.matches("/a/keep.pyc"));
  EXPECT_TRUE(gi.matches("/ignoreFileLocal"));
  EXPECT_TRUE(gi.matches("/testFolder/ignoreFileLocal"));
  EXPECT_TRUE(!gi.matches("/ignoreFileLocalX"));
  EXPECT_TRUE(gi.matches("/testFolder/deep/x"));
  GitIgnore g2({"Dockerfile", ".devspace/", "chart/"});
  EXPECT_TRUE(g2.matches("/Dockerfile"));
  EXPECT_TRUE(g2.matches("/chart/templates/a.yaml"));
  EXPECT_TRUE(g2.matches("/.devspace/config.yaml"));
  EXPECT_TRUE(!g2.matches("/index.js"));
  GitIgnore g3({"**/tmp", "logs/**"});
  EXPECT_TRUE(g3.matches("/a/b/tmp"));
  EXPECT_TRUE(g3.matches("/logs/x/y"));
}

TEST(docker_ignore_and_glob) {
  DockerIgnore di({"node_modules", "*.log", "!important.log", "build/**/*.o"});
  EXPECT_TRUE(di.matches("node_modules"));
  EXPECT_TRUE(di.matches("node_modules/x/y.js"));
  EXPECT_TRUE(di.matches("a.log"));
  EXPECT_TRUE(!di.matches("important.log"));
  EXPECT_TRUE(di.matches("build/a/b/c.o"));
  EXPECT_TRUE(!di.matches("src/a.js"));
  EXPECT_TRUE(glob_match("chart/**", "chart/templates/a.yaml"));
  EXPECT_TRUE(glob_match("kube/*.yaml", "kube/dep.yaml"));
  EXPECT_TRUE(!glob_match("kube/*.yaml", "kube/x/dep.yaml"));
  EXPECT_TRUE(glob_match("**/*.{yaml,yml}", "a/b/c.yml"));
  EXPECT_TRUE(path_match("[a-c]?.txt", "bx.txt"));
}

TEST(tar_gzip_roundtrip) {
  std::string out;
  {
    GzipWriter gz(string_sink(&out), 1);
    TarWriter tw([&](const char* d, size_t n) { return gz.write(d, n); });
    TarEntry f;
    f.name = "dir/file.txt";
    f.mode = 0640;
    f.mtime = 1500000000;
    tw.add_file(f, "hello world");
    TarEntry d;
    d.name = "emptydir";
    d.mtime = 1500000001;
    d.mode = 0755;
    tw.add_dir(d);
    TarEntry lf;
    lf.name = std::string(150, 'x') + "/long.txt";
    tw.add_file(lf, std::string(1000, 'z'));
    tw.finish();
    gz.finish();
  }
  GzipReader gr(string_source(&out));
  TarReader tr([&](char* b, size_t n) { return gr.read(b, n); });
  TarEntry e;
  EXPECT_TRUE(tr.next(&e));
  EXPECT_EQ(e.name, std::string("dir/file.txt"));
  EXPECT_EQ(e.mode, (uint32_t)0640);
  EXPECT_EQ(e.mtime, (int64_t)1500000000);
  EXPECT_EQ(tr.read_all(), std::string("hello world"));
  EXPECT_TRUE(tr.next(&e));
  EXPECT_EQ(e.type, '5');
  EXPECT_TRUE(tr.next(&e));
  EXPECT_EQ(e.name.size(), (size_t)159);
  EXPECT_EQ(tr.read_all().size(), (size_t)1000);
  EXPECT_TRUE(!tr.next(&e));
}

TEST(tar_interop_with_gnu_tar) {
  if (which("tar").empty()) return;
  std::string dir = fs::make_temp_dir();
  fs::write_file(fs::join(dir, "src/a.txt"), "A");
  fs::write_file(fs::join(dir, "src/sub/b.txt"), "BB");
  RunResult r = run({"tar", "-czf", fs::join(dir, "x.tgz"), "-C", fs::join(dir, "src"), "."});
  EXPECT_EQ(r.code, 0);
  std::string data = fs::read_file(fs::join(dir, "x.tgz"));
  GzipReader gr(string_source(&data));
  TarReader tr([&](char* b, size_t n) { return gr.read(b, n); });
  TarEntry e;
  int files = 0;
  while (tr.next(&e))
    if (e.type == '0') ++files;
  EXPECT_EQ(files, 2);
  // and the other direction: our archive extracts with GNU tar
  std::string ours;
  {
    GzipWriter gz(string_sink(&ours));
    TarWriter tw([&](const char* d, size_t n) { return gz.write(d, n); });
    TarEntry f;
    f.name = "deep/dir/" + std::string(120, 'q') + ".txt";
    f.mode = 0644;
    tw.add_file(f, "payload");
    tw.finish();
    gz.finish();
  }
  fs::write_file(fs::join(dir, "ours.tgz"), ours);
  fs::mkdirs(fs::join(dir, "out"));
  r = run({"tar", "-xzf", fs::join(dir, "ours.tgz"), "-C", fs::join(dir, "out")});
  EXPECT_EQ(r.code, 0);
  EXPECT_EQ(fs::read_file(fs::join(dir, "out/deep/dir/" + std::string(120, 'q') + ".txt")), std::string("payload"));
  fs::remove_all(dir);
}

TEST(hash_and_encodings) {
  EXPECT_EQ(sha256_hex("abc"), std::string("ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"));
  EXPECT_EQ(base64_encode("hello"), std::string("aGVsbG8="));
  EXPECT_EQ(base64_decode("aGVsbG8="), std::string("hello"));
  EXPECT_EQ(base64_decode(base64_encode(std::string("\xff\xfe\x01", 3), true)), std::string("\xff\xfe\x01", 3));
  std::string r = random_string(7);
  EXPECT_EQ(r.size(), (size_t)7);
  for (char c : r) EXPECT_TRUE(std::isalnum((unsigned char)c));
}

TEST(cli_flags) {
  cli::Command root("devspace", "root");
  root.persistent_bool("debug", "", false, "debug");
  auto dev = std::make_unique<cli::Command>("dev", "start dev");
  std::string seen;
  dev->boolean("force-build", "b", false, "force build")
      .boolean("sync", "", true, "sync")
      .str("namespace", "n", "", "ns")
      .slice("exclude", "", "excludes")
      .integer("lines", "", 200, "lines");
  dev->run = [&](cli::Command& c, const std::vector<std::string>& args) {
    seen = std::to_string(c.get_bool("force-build")) + std::to_string(c.get_bool("sync")) + c.get_str("namespace") +
           std::to_string(c.get_slice("exclude").size()) + std::to_string(c.get_int("lines")) +
           std::to_string(args.size()) + std::to_string(c.get_bool("debug"));
    return 0;
  };
  dev->aliases = {"up"};
  root.add(std::move(dev));
  EXPECT_EQ(root.execute({"up", "-b", "--sync=false", "-n", "ns1", "--exclude", "a,b", "--lines=5", "x", "--debug"}), 0);
  EXPECT_EQ(seen, std::string("10ns12511"));
}

TEST(fs_paths) {
  EXPECT_EQ(fs::clean("/a/b/../c/./d/"), std::string("/a/c/d"));
  EXPECT_EQ(fs::dirname("/a/b/c"), std::string("/a/b"));
  EXPECT_EQ(fs::basename("/a/b/c/"), std::string("c"));
  EXPECT_EQ(fs::relative("/a/b", "/a/b/c/d"), std::string("c/d"));
  EXPECT_EQ(fs::join("a/", "/b"), std::string("a/b"));
}

// Mutation fuzz of the YAML reader/writer: every mutated document parses or throws a
// std::exception, and what parses dumps to YAML that reads back to the same value.
TEST(yaml_mutation_fuzz_roundtrip) {
  const std::vector<std::string> seeds = {
      "version: v1alpha2\nimages:\n  default:\n    image: reg/app\n    build:\n      kaniko:\n        cache: true\n"
      "dev:\n  sync:\n  - containerPath: /app\n    excludePaths: [node_modules/, '*.pyc']\n  ports:\n"
      "  - portMappings:\n    - {localPort: 3000, remotePort: 3000}\n",
      "a: |\n  line one\n  line two\nb: >-\n  folded\n  text\nc: &anc {x: 1, y: [1, 2]}\nd: *anc\ne: \"q\\\"s\"\n"
      "f: 'it''s'\ng: ~\nh: 0x1F\ni: -1.5e3\n---\n- x\n- - nested\n  - seq\n- k: v\n  k2: v2\n"};
  const std::string alphabet = " \n\t:-[]{},#&*!|>'\"%@?ab01.";
  uint64_t rng = 0xD1B54A32D192ED03ull;
  auto next = [&rng] {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return rng;
  };
  int ok = 0;
  for (int it = 0; it < 20000; ++it) {
    std::string t = seeds[next() % seeds.size()];
    int nmut = 1 + (int)(next() % 4);
    for (int m = 0; m < nmut && !t.empty(); ++m) {
      size_t i = next() % t.size();
      switch (next() % 3) {
        case 0: t[i] = alphabet[next() % alphabet.size()]; break;
        case 1: t.erase(i, 1 + next() % 6); break;
        default: t.insert(i, 1, alphabet[next() % alphabet.size()]);
      }
    }
    std::vector<Value> docs;
    try {
      docs = yaml_parse_all(t);
    } catch (const std::exception&) {
      continue;
    }
    ++ok;
    for (auto& d : docs) {
      std::string out = yaml_dump(d);
      Value back = yaml_parse(out);
      if (!(back == d)) {
        std::fprintf(stderr, "roundtrip mismatch for:\n%s\n--- dumped:\n%s\n", t.c_str(), out.c_str());
        EXPECT_TRUE(false);
        return;
      }
    }
  }
  EXPECT_TRUE(ok > 1000);
}

// Archives and JSON arrive from containers and API servers: corrupted tar, gzip and JSON input
// is rejected with an exception or read partially, never a crash or an unbounded allocation.
TEST(untrusted_tar_gzip_json_mutation_fuzz) {
  std::string tar;
  {
    TarWriter tw(string_sink(&tar));
    TarEntry e;
    e.name = "dir/file.txt";
    tw.add_file(e, std::string(3000, 'x'));
    e.name = std::string(150, 'n') + "/long-name-needs-pax.txt";
    tw.add_file(e, "hello");
    TarEntry d;
    d.name = "dir/sub";
    d.type = '5';
    tw.add_dir(d);
    tw.finish();
  }
  std::string gz = gzip_compress(tar);
  std::string js = "{\"kind\":\"Pod\",\"metadata\":{\"name\":\"p\",\"labels\":{\"a\":\"b\"}},"
                   "\"items\":[1,2.5,-3e2,true,null,\"\\u00e9\\n\"],\"s\":\"x\"}";
  uint64_t rng = 0x2545F4914F6CDD1Dull;
  auto next = [&rng] {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return rng;
  };
  auto mutate = [&](std::string t) {
    int n = 1 + (int)(next() % 4);
    for (int m = 0; m < n && !t.empty(); ++m) {
      size_t i = next() % t.size();
      switch (next() % 3) {
        case 0: t[i] = (char)(next() & 0xff); break;
        case 1: t.erase(i, 1 + next() % 8); break;
        default: t.insert(i, 1, (char)(next() & 0xff));
      }
    }
    return t;
  };
  for (int it = 0; it < 3000; ++it) {
    std::string t = mutate(tar);
    try {
      TarReader r(string_source(&t));
      TarEntry e;
      int entries = 0;
      while (r.next(&e) && entries++ < 100) {
        std::string body = r.read_all();
        EXPECT_TRUE((int64_t)body.size() <= (int64_t)t.size());
      }
    } catch (const std::exception&) {
    }
    std::string g = mutate(gz);
    try {
      std::string out = gzip_decompress(g);
      EXPECT_TRUE(out.size() <= (size_t)64 << 20);
    } catch (const std::exception&) {
    }
    std::string j = mutate(js);
    try {
      json_parse(j);
    } catch (const std::exception&) {
    }
  }
}

TEST(parsers_bound_nesting_depth) {
  auto nested = [](size_t n) { return std::string(n, '[') + std::string(n, ']'); };
  EXPECT_TRUE(json_parse(nested(500)).is_seq());
  EXPECT_TRUE(yaml_parse(nested(500)).is_seq());
  for (auto* parse : {+[](const std::string& t) { json_parse(t); }, +[](const std::string& t) { yaml_parse(t); }}) {
    bool threw = false;
    try {
      parse(nested(200000));  // would overflow the stack without the bound
    } catch (const std::exception& e) {
      threw = contains(e.what(), "max depth");
    }
    EXPECT_TRUE(threw);
  }
}

// Patterns that make a plain backtracking matcher exponential finish at once (failure memo).
TEST(matchers_pathological_patterns_are_fast) {
  std::string deep;
  for (int i = 0; i < 40; ++i) deep += "a/";
  deep += "b";
  std::string stars;
  for (int i = 0; i < 25; ++i) stars += "*a";
  stars += "c";
  std::string dstars;
  for (int i = 0; i < 10; ++i) dstars += "**/";
  dstars += "c";
  auto t0 = std::chrono::steady_clock::now();
  EXPECT_TRUE(!glob_match(dstars, deep));
  EXPECT_TRUE(!path_match(stars, std::string(60, 'a')));
  GitIgnore gi;
  gi.add_line(dstars);
  gi.add_line(stars);
  EXPECT_TRUE(!gi.matches(deep) && !gi.matches(std::string(60, 'a')));
  DockerIgnore di({dstars, stars});
  EXPECT_TRUE(!di.matches(deep) && !di.matches(std::string(60, 'a')));
  // and they still match what they should
  EXPECT_TRUE(glob_match(dstars, deep.substr(0, deep.size() - 1) + "c"));
  EXPECT_TRUE(path_match(stars, std::string(59, 'a') + "c"));
  auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
  EXPECT_TRUE(ms < 500);
}


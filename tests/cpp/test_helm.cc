// Helm chart semantics on in-repo fixtures (tests/fixtures/charts): .Files, .Capabilities,
// NOTES.txt, .helmignore, dependencies (condition / tags / alias / import-values / library
// charts, Chart.yaml v2 and requirements.yaml v1), hooks, Helm 3 release records, and the
// wider Sprig function set. Golden renders live in tests/fixtures/golden/ (regenerate with
// DS_UPDATE_GOLDEN=1 bin/devspace_tests helm_golden).
#include <algorithm>

#include "core/codec.h"
#include "core/fs.h"
#include "core/strutil.h"
#include "deploy/gotemplate.h"
#include "deploy/helm.h"
#include "testing.h"

using namespace ds;

static const std::string kCharts = std::string(DEVSPACE_SOURCE_DIR) + "/tests/fixtures/charts/";
static const std::string kGolden = std::string(DEVSPACE_SOURCE_DIR) + "/tests/fixtures/golden/";

static helm::RenderOptions opts(const std::string& caps_yaml = "") {
  helm::RenderOptions o;
  o.release_name = "rel";
  o.namespace_ = "ns1";
  if (!caps_yaml.empty()) o.capabilities = yaml_parse(caps_yaml);
  return o;
}

static std::string render_chart(const std::string& name, const Value& user = Value::map(),
                                const std::string& caps_yaml = "") {
  helm::Chart c = helm::load_chart(kCharts + name);
  helm::process_dependencies(c, user);
  return helm::render_to_string(c, helm::coalesce_values(c, user), opts(caps_yaml));
}

static const Value* find_named(const std::vector<Value>& docs, const std::string& name) {
  for (auto& d : docs)
    if (d.at_path("metadata.name").as_string() == name) return &d;
  return nullptr;
}

static std::vector<Value> docs_of(const std::string& text) {
  std::vector<Value> out;
  for (auto& d : yaml_parse_all(text))
    if (d.is_map() && !d.get("kind").is_null()) out.push_back(d);
  return out;
}

static void check_golden(const std::string& name, const std::string& got) {
  std::string path = kGolden + name + ".yaml";
  const char* upd = getenv("DS_UPDATE_GOLDEN");
  if (upd && std::string(upd) == "1") fs::write_file(path, got);
  EXPECT_TRUE(fs::exists(path));
  EXPECT_EQ(got, fs::read_file(path));
}

TEST(helm_files_object) {
  std::string out = render_chart("files-chart");
  auto docs = docs_of(out);
  const Value* cm = find_named(docs, "rel-conf");
  EXPECT_TRUE(cm != nullptr);
  const Value& d = cm->get("data");
  // (.Files.Glob "conf/*").AsConfig: one key per base name
  EXPECT_EQ(d.get("a.conf").as_string(), std::string("listen 80\nworkers 4\n"));
  EXPECT_EQ(d.get("b.conf").as_string(), std::string("level: debug\n"));
  EXPECT_EQ(d.get("readme").as_string(), std::string("readme text"));
  EXPECT_EQ(d.get("missing").as_string(), std::string(""));
  // .helmignore drops *.tmp and scratch/; templates/, Chart.yaml, values.yaml are not files
  EXPECT_EQ(d.get("ignored").as_string(), std::string(""));
  EXPECT_EQ(d.get("file-count").as_string(), std::string("5"));  // README, 2 conf, 2 data
  EXPECT_EQ(d.get("lines").as_string(), std::string("alpha;beta;gamma;"));
  EXPECT_EQ(d.get("first-line").as_string(), std::string("alpha"));
  EXPECT_EQ(d.get("bytes-b64").as_string(), base64_encode("s3cr3t"));
  EXPECT_EQ(cm->at_path("metadata.labels.chart").as_string(), std::string("files-chart-0.3.1"));
  EXPECT_EQ(cm->at_path("metadata.labels.app-version").as_string(), std::string("1.4"));
  EXPECT_EQ(cm->at_path("metadata.labels.chart-api").as_string(), std::string("v2"));
  const Value* sec = find_named(docs, "rel-token");
  EXPECT_TRUE(sec != nullptr);
  EXPECT_EQ(sec->at_path("data").get("token.txt").as_string(), base64_encode("s3cr3t"));
  // hidden files under templates/ are not templates
  EXPECT_TRUE(!contains(out, "hidden"));
  check_golden("files-chart", out);
}

TEST(helm_capabilities_and_notes) {
  std::string caps = "KubeVersion: {Major: '1', Minor: '20', GitVersion: v1.20.15-gke.100}\n"
                     "APIVersions: [v1, apps/v1, batch/v1beta1]\n";
  auto docs = docs_of(render_chart("files-chart", Value::map(), caps));
  const Value& d = find_named(docs, "rel-caps")->get("data");
  EXPECT_EQ(d.get("kube").as_string(), std::string("v1.20.15-gke.100"));
  EXPECT_EQ(d.get("minor").as_string(), std::string("20"));
  EXPECT_EQ(d.get("has-apps").as_string(), std::string("true"));
  EXPECT_EQ(d.get("has-bogus").as_string(), std::string("false"));
  EXPECT_EQ(d.get("cronjob-api").as_string(), std::string("batch/v1beta1"));  // 1.20 < 1.21-0
  auto docs2 = docs_of(render_chart("files-chart", Value::map(),
                                    "KubeVersion: {Major: '1', Minor: '29', GitVersion: v1.29.2}\nAPIVersions: [v1]\n"));
  const Value& d2 = find_named(docs2, "rel-caps")->get("data");
  EXPECT_EQ(d2.get("cronjob-api").as_string(), std::string("batch/v1"));
  EXPECT_EQ(d2.get("has-apps").as_string(), std::string("false"));
  EXPECT_TRUE(starts_with(d2.get("helm").as_string(), "v3."));
  // NOTES.txt renders (top chart only) but is not part of the manifest
  helm::Chart c = helm::load_chart(kCharts + "files-chart");
  bool notes = false;
  for (auto& f : helm::render_files(c, helm::coalesce_values(c, Value::map()), opts()))
    if (f.first == "files-chart/templates/NOTES.txt") {
      notes = true;
      EXPECT_EQ(f.second, std::string("hello from rel in ns1.\n"));
    }
  EXPECT_TRUE(notes);
  EXPECT_TRUE(!contains(helm::render_to_string(c, c.values, opts()), "hello from"));
}

TEST(helm_dependencies_v2) {
  std::string out = render_chart("deps-chart");
  auto docs = docs_of(out);
  // condition db.enabled=true (parent values) beats the subchart's own enabled: false
  EXPECT_TRUE(find_named(docs, "rel-db") != nullptr);
  EXPECT_EQ(find_named(docs, "rel-db")->at_path("data.env").as_string(), std::string("staging"));  // globals
  EXPECT_EQ(find_named(docs, "rel-db")->at_path("data.image").as_string(), std::string("postgres:16"));
  // tags: backend=true keeps cache
  EXPECT_TRUE(find_named(docs, "rel-cache") != nullptr);
  // aliases: two copies of worker; worker-b disabled by its condition
  EXPECT_TRUE(find_named(docs, "rel-worker-a") != nullptr);
  EXPECT_EQ(find_named(docs, "rel-worker-a")->at_path("data.queue").as_string(), std::string("fast"));
  EXPECT_TRUE(find_named(docs, "rel-worker-b") == nullptr);
  // library chart: defines are usable, its templates never render
  EXPECT_TRUE(find_named(docs, "must-not-render") == nullptr);
  const Value* app = find_named(docs, "rel-deps-chart");
  EXPECT_TRUE(app != nullptr);
  EXPECT_EQ(app->at_path("metadata.labels").get("app.kubernetes.io/managed-by").as_string(), std::string("Helm"));
  // import-values: exports form (db.exports.data -> parent top level) ...
  EXPECT_EQ(app->at_path("data").get("db-exported-user").as_string(), std::string("admin"));
  EXPECT_EQ(app->at_path("data").get("db-exported-pool").as_string(), std::string("5"));
  // ... and child/parent form, where the parent's own value wins
  EXPECT_EQ(app->at_path("data").get("cache-port").as_string(), std::string("7000"));
  EXPECT_EQ(app->at_path("data").get("cache-proto").as_string(), std::string("resp"));
  check_golden("deps-chart", out);

  // user values flip conditions and tags
  Value user = yaml_parse("db: {enabled: false}\ntags: {backend: false}\nworkerB: {enabled: true}\n");
  auto d2 = docs_of(render_chart("deps-chart", user));
  EXPECT_TRUE(find_named(d2, "rel-db") == nullptr);
  EXPECT_TRUE(find_named(d2, "rel-cache") == nullptr);
  EXPECT_TRUE(find_named(d2, "rel-worker-b") != nullptr);
  EXPECT_EQ(find_named(d2, "rel-worker-b")->at_path("data.queue").as_string(), std::string("default"));
  // disabled charts export nothing
  EXPECT_EQ(find_named(d2, "rel-deps-chart")->at_path("data").get("db-exported-user").as_string(), std::string("none"));
  // a null user value deletes a default (Helm coalesce), imported values included
  Value del = yaml_parse("cacheService: null\n");
  auto d3 = docs_of(render_chart("deps-chart", del));
  EXPECT_EQ(find_named(d3, "rel-deps-chart")->at_path("data").get("cache-port").as_string(), std::string(""));
}

TEST(helm_requirements_v1) {
  auto docs = docs_of(render_chart("reqs-chart"));
  EXPECT_TRUE(find_named(docs, "rel-svc") != nullptr);
  EXPECT_TRUE(find_named(docs, "rel-redis") == nullptr);  // condition redis.enabled=false
  EXPECT_TRUE(find_named(docs, "rel-mysql") == nullptr);  // tag database=false
  auto on = docs_of(render_chart("reqs-chart", yaml_parse("redis: {enabled: true}\ntags: {database: true}\n")));
  EXPECT_TRUE(find_named(on, "rel-redis") != nullptr);
  EXPECT_TRUE(find_named(on, "rel-mysql") != nullptr);
}

TEST(helm_release_record_layout) {
  helm::Release r;
  r.name = "app";
  r.namespace_ = "ns";
  r.version = 3;
  r.status = "deployed";
  r.first_deployed = "2026-01-01T00:00:00Z";
  r.last_deployed = "2026-01-02T00:00:00Z";
  r.description = "Upgrade complete";
  r.notes = "hi";
  r.manifest = "---\n# Source: c/templates/a.yaml\nkind: ConfigMap\n";
  r.config = yaml_parse("a: 1\n");
  helm::Chart c = helm::load_chart(kCharts + "files-chart");
  helm::Hook h;
  h.name = "mig";
  h.kind = "Job";
  h.path = "c/templates/j.yaml";
  h.manifest = "kind: Job\n";
  h.events = {"pre-install"};
  h.weight = -5;
  r.hooks.push_back(h);
  Value v = helm::release_to_json(r);
  // pkg/release/release.go field names
  for (auto k : {"name", "info", "chart", "config", "manifest", "hooks", "version", "namespace"})
    EXPECT_TRUE(v.has(k));
  for (auto k : {"first_deployed", "last_deployed", "deleted", "description", "status", "notes"})
    EXPECT_TRUE(v.get("info").has(k));
  for (auto k : {"name", "kind", "path", "manifest", "events", "last_run", "weight"})
    EXPECT_TRUE(v.get("hooks")[0].has(k));
  helm::Release back = helm::release_from_json(json_parse(json_dump(v)));
  EXPECT_EQ(back.version, 3);
  EXPECT_EQ(back.description, std::string("Upgrade complete"));
  EXPECT_EQ(back.hooks.size(), (size_t)1);
  EXPECT_EQ(back.hooks[0].weight, -5);
  EXPECT_EQ(back.config.get("a").as_int(), (int64_t)1);
}

TEST(sprig_extended_functions) {
  auto R = [](const std::string& src, const std::string& data = "{}") {
    tmpl::Engine e;
    e.add("t", src);
    return e.execute("t", yaml_parse(data));
  };
  EXPECT_EQ(R("{{ camelcase \"http_server-name\" }}"), std::string("HttpServerName"));
  EXPECT_EQ(R("{{ snakecase \"HTTPServerName\" }}"), std::string("http_server_name"));
  EXPECT_EQ(R("{{ kebabcase \"fooBar\" }}"), std::string("foo-bar"));
  EXPECT_EQ(R("{{ abbrev 5 \"hello world\" }}"), std::string("he..."));
  EXPECT_EQ(R("{{ substr 0 5 \"hello world\" }}"), std::string("hello"));
  EXPECT_EQ(R("{{ nospace \"a b  c\" }}"), std::string("abc"));
  EXPECT_EQ(R("{{ append (list 1 2) 3 | toJson }}"), std::string("[1,2,3]"));
  EXPECT_EQ(R("{{ prepend (list 2 3) 1 | toJson }}"), std::string("[1,2,3]"));
  EXPECT_EQ(R("{{ concat (list 1) (list 2 3) | toJson }}"), std::string("[1,2,3]"));
  EXPECT_EQ(R("{{ list 1 1 2 | uniq | toJson }}"), std::string("[1,2]"));
  EXPECT_EQ(R("{{ without (list 1 2 3) 2 | toJson }}"), std::string("[1,3]"));
  EXPECT_EQ(R("{{ list \"b\" \"a\" | sortAlpha | toJson }}"), std::string("[\"a\",\"b\"]"));
  EXPECT_EQ(R("{{ list 1 2 3 | rest | toJson }}{{ list 1 2 3 | initial | toJson }}"), std::string("[2,3][1,2]"));
  EXPECT_EQ(R("{{ compact (list \"\" \"a\") | toJson }}"), std::string("[\"a\"]"));
  EXPECT_EQ(R("{{ pick .m \"a\" | toJson }}", "m: {a: 1, b: 2}"), std::string("{\"a\":1}"));
  EXPECT_EQ(R("{{ omit .m \"a\" | toJson }}", "m: {a: 1, b: 2}"), std::string("{\"b\":2}"));
  EXPECT_EQ(R("{{ dig \"a\" \"b\" \"dflt\" .m }}", "m: {a: {b: deep}}"), std::string("deep"));
  EXPECT_EQ(R("{{ dig \"a\" \"x\" \"dflt\" .m }}", "m: {a: {b: deep}}"), std::string("dflt"));
  EXPECT_EQ(R("{{ regexFind \"[0-9]+\" \"ab123cd45\" }}"), std::string("123"));
  EXPECT_EQ(R("{{ regexFindAll \"[0-9]+\" \"ab123cd45\" -1 | toJson }}"), std::string("[\"123\",\"45\"]"));
  EXPECT_EQ(R("{{ regexSplit \",\" \"a,b,c\" -1 | toJson }}"), std::string("[\"a\",\"b\",\"c\"]"));
  EXPECT_EQ(R("{{ base \"/a/b/c.txt\" }} {{ dir \"/a/b/c.txt\" }} {{ ext \"c.tar.gz\" }} {{ clean \"a/../b/./c\" }}"),
            std::string("c.txt /a/b .gz b/c"));
  EXPECT_EQ(R("{{ sha1sum \"abc\" }}"), std::string("a9993e364706816aba3e25717850c26c9cd0d89d"));
  EXPECT_EQ(R("{{ adler32sum \"abc\" }}"), std::string("38600999"));
  EXPECT_EQ(R("{{ b32enc \"hi\" }} {{ b32dec \"NBUQ====\" }}"), std::string("NBUQ==== hi"));
  EXPECT_EQ(R("{{ floor 1.7 }} {{ ceil 1.2 }} {{ round 1.256 2 }}"), std::string("1 2 1.26"));
  EXPECT_EQ(R("{{ toToml .m }}", "m: {a: 1, s: x, t: {b: true}}"), std::string("a = 1\ns = \"x\"\n\n[t]\nb = true\n"));
  EXPECT_EQ(R("{{ (semver \"1.2.3-rc.1\").Minor }}"), std::string("2"));
  EXPECT_EQ(R("{{ mustToJson (list 1) }} {{ mustRegexMatch \"^a\" \"abc\" }}"), std::string("[1] true"));
  EXPECT_EQ(R("{{ urlquery \"a b&c\" }}"), std::string("a+b%26c"));
  EXPECT_EQ(R("{{ slice (list 1 2 3) 1 | toJson }} {{ slice \"hello\" 1 3 }}"), std::string("[2,3] el"));
  EXPECT_EQ(R("{{ seq 3 }}"), std::string("1 2 3"));
  EXPECT_EQ(R("{{ wrap 5 \"aa bb cc\" }}"), std::string("aa bb\ncc"));
}

TEST(semver_constraints) {
  EXPECT_TRUE(tmpl::semver_match(">=1.21-0", "v1.29.2"));
  EXPECT_TRUE(tmpl::semver_match(">=1.21-0", "v1.21.3-gke.100"));
  EXPECT_TRUE(!tmpl::semver_match(">=1.21-0", "v1.20.15"));
  EXPECT_TRUE(!tmpl::semver_match(">=1.21", "v1.22.0-rc.1"));  // prerelease needs a prerelease constraint
  EXPECT_TRUE(tmpl::semver_match("~2.1.0", "2.1.4"));
  EXPECT_TRUE(!tmpl::semver_match("~2.1.0", "2.2.0"));
  EXPECT_TRUE(tmpl::semver_match("^1.2", "1.9.0"));
  EXPECT_TRUE(!tmpl::semver_match("^1.2", "2.0.0"));
  EXPECT_TRUE(tmpl::semver_match("^0.2.3", "0.2.9"));
  EXPECT_TRUE(!tmpl::semver_match("^0.2.3", "0.3.0"));
  EXPECT_TRUE(tmpl::semver_match("1.x", "1.7.0"));
  EXPECT_TRUE(tmpl::semver_match("3.x", "3.2.1"));
  EXPECT_TRUE(tmpl::semver_match("1.2 - 1.4.5", "1.4.5"));
  EXPECT_TRUE(!tmpl::semver_match("1.2 - 1.4.5", "1.4.6"));
  EXPECT_TRUE(tmpl::semver_match("<1.0 || >=2.1", "2.3.0"));
  EXPECT_TRUE(tmpl::semver_match(">=1.2, <2", "1.5.0"));
  EXPECT_TRUE(!tmpl::semver_match(">=1.2, <2", "2.0.0"));
  EXPECT_TRUE(tmpl::semver_match("0.10.2", "0.10.2"));
  EXPECT_THROWS(tmpl::semver_match(">=1", "not-a-version"));
}

TEST(gotemplate_go118_control_flow) {
  auto R = [](const std::string& src, const std::string& data = "{}") {
    tmpl::Engine e;
    e.add("t", src);
    return e.execute("t", yaml_parse(data));
  };
  // {{break}} / {{continue}} inside range (also from inside if/with bodies)
  EXPECT_EQ(R("{{ range $i, $v := .l }}{{ if eq $v 3 }}{{ break }}{{ end }}{{ $v }},{{ end }}", "l: [1, 2, 3, 4]"),
            std::string("1,2,"));
  EXPECT_EQ(R("{{ range .l }}{{ with . }}{{ if eq . 2 }}{{ continue }}{{ end }}{{ . }}{{ end }};{{ end }}",
              "l: [1, 2, 3]"),
            std::string("1;3;"));
  EXPECT_THROWS(R("{{ break }}"));
  // and/or stop at the first deciding argument: the comparison with a missing value never runs
  EXPECT_EQ(R("{{ if and (hasKey . \"x\") (gt .x 1) }}big{{ else }}none{{ end }}"), std::string("none"));
  EXPECT_EQ(R("{{ if or (not (hasKey . \"x\")) (gt .x 1) }}ok{{ end }}"), std::string("ok"));
  EXPECT_EQ(R("{{ and 1 0 2 }}|{{ or 0 \"\" 3 }}|{{ 5 | and 1 }}|{{ 0 | or \"\" }}"), std::string("0|3|5|0"));
}

TEST(helm_values_schema_validation) {
  helm::Chart c = helm::load_chart(kCharts + "schema-chart");
  EXPECT_TRUE(!c.schema.empty());
  helm::validate_values(c, helm::coalesce_values(c, Value::map()));  // defaults are valid
  Value bad = yaml_parse(
      "replicas: 40\ngpus: 3\nimage: {repository: 'Bad Repo', pullPolicy: Sometimes, extra: 1}\nsub: {mode: turbo}\n");
  std::string msg;
  try {
    helm::validate_values(c, helm::coalesce_values(c, bad));
  } catch (const std::exception& e) {
    msg = e.what();
  }
  EXPECT_TRUE(starts_with(msg, "values don't meet the specifications of the schema(s) in the following chart(s):"));
  EXPECT_TRUE(contains(msg, "schema-chart:\n"));
  EXPECT_TRUE(contains(msg, "- replicas: Must be less than or equal to 16"));
  EXPECT_TRUE(contains(msg, "- gpus: must be one of the following: [0,1,2,4,8]"));
  EXPECT_TRUE(contains(msg, "- image.repository: Does not match pattern"));
  EXPECT_TRUE(contains(msg, "- image.pullPolicy: must be one of the following"));  // via $ref
  EXPECT_TRUE(contains(msg, "- image: Additional property extra is not allowed"));
  EXPECT_TRUE(contains(msg, "sub:\n- mode: must be one of the following"));  // subchart schema
  Value wrong_type = yaml_parse("replicas: 'two'\n");
  msg.clear();
  try {
    helm::validate_values(c, helm::coalesce_values(c, wrong_type));
  } catch (const std::exception& e) {
    msg = e.what();
  }
  EXPECT_TRUE(contains(msg, "- replicas: Invalid type. Expected: integer, given: string"));
  Value missing = yaml_parse("image: null\n");  // a null user value deletes the default
  msg.clear();
  try {
    helm::validate_values(c, helm::coalesce_values(c, missing));
  } catch (const std::exception& e) {
    msg = e.what();
  }
  EXPECT_TRUE(contains(msg, "- (root): image is required"));
}

// Go-template engine, Helm chart rendering (the embedded component chart), generator language
// detection and config mutations (configure/*).
#include <algorithm>
#include <cstring>

#include <crypt.h>
#include <openssl/pem.h>
#include <openssl/x509.h>
#include <openssl/x509v3.h>

#include "analyze/analyze.h"
#include "config/config.h"
#include "configure/configure.h"
#include "core/fs.h"
#include "core/strutil.h"
#include "deploy/gotemplate.h"
#include "deploy/helm.h"
#include "deploy/helmrepo.h"
#include "build/docker.h"
#include "generator/generator.h"
#include "gpu/sizing.h"
#include <regex>

#include "testing.h"

using namespace ds;

static std::string render_tmpl(const std::string& src, const Value& data) {
  tmpl::Engine e;
  e.add("t", src);
  return e.execute("t", data);
}

TEST(gotemplate_basics) {
  Value d = yaml_parse("name: app\nitems: [a, b]\nm: {x: 1, z: 2}\nflag: false\nn: 3\n");
  EXPECT_EQ(render_tmpl("{{ .name | upper }}", d), std::string("APP"));
  EXPECT_EQ(render_tmpl("{{ range $i, $v := .items }}{{ $i }}={{ $v }};{{ end }}", d), std::string("0=a;1=b;"));
  EXPECT_EQ(render_tmpl("{{ range $k, $v := .m }}{{ $k }}{{ $v }}{{ end }}", d), std::string("x1z2"));
  EXPECT_EQ(render_tmpl("{{ if .flag }}yes{{ else }}no{{ end }}", d), std::string("no"));
  EXPECT_EQ(render_tmpl("{{ default \"z\" .missing }}", d), std::string("z"));
  EXPECT_EQ(render_tmpl("{{- $x := 1 }}{{ $x = add $x .n }}{{ $x }}", d), std::string("4"));
  EXPECT_EQ(render_tmpl("{{ toYaml .m | nindent 2 }}", d), std::string("\n  x: 1\n  z: 2"));
  EXPECT_EQ(render_tmpl("{{ printf \"%s-%d\" .name .n }}", d), std::string("app-3"));
  EXPECT_EQ(render_tmpl("{{ if and .m .m.x }}ok{{ end }}", d), std::string("ok"));
  EXPECT_EQ(render_tmpl("{{ if and .nothing .nothing.deep }}bad{{ else }}ok{{ end }}", d), std::string("ok"));
  EXPECT_EQ(render_tmpl("{{ list 1 2 3 | len }}", d), std::string("3"));
  EXPECT_EQ(render_tmpl("{{ define \"p\" }}[{{ . }}]{{ end }}{{ include \"p\" .name }}", d), std::string("[app]"));
}

static Value component_values(int gpus, bool with_volume, int max_replicas) {
  std::string y =
      "components:\n"
      "- name: default\n"
      "  replicas: 1\n"
      "  containers:\n"
      "  - image: reg/app:tag\n"
      "    resources:\n"
      "      limits:\n"
      "        cpu: \"2\"\n"
      "        ephemeralStorage: 1Gi\n"
      "        gpu: " + std::to_string(gpus) + "\n"
      "      requests:\n"
      "        memory: 1Gi\n"
      "    env:\n"
      "    - name: A\n"
      "      value: b\n";
  if (with_volume)
    y += "    volumeMounts:\n    - containerPath: /data\n      volume:\n        name: data\n        subPath: /d\n";
  if (max_replicas) y += "  autoScaling:\n    horizontal:\n      maxReplicas: " + std::to_string(max_replicas) +
                         "\n      averageCPU: 80\n";
  y += "  service:\n    name: external\n    ports:\n    - externalPort: 80\n      containerPort: 3000\n";
  y += with_volume ? "volumes:\n- name: data\n  size: 2Gi\n" : "volumes: []\n";
  y += "pullSecrets: [devspace-auth-reg]\n";
  return yaml_parse(y);
}

static const Value* find_kind(const std::vector<Value>& objs, const std::string& kind) {
  for (auto& o : objs)
    if (o.get("kind").as_string() == kind) return &o;
  return nullptr;
}

TEST(component_chart_cpu_deployment) {
  helm::Chart c = helm::load_chart(std::string(DEVSPACE_SOURCE_DIR) + "/templates/_base/chart");
  helm::RenderOptions o;
  o.release_name = "devspace-app";
  o.namespace_ = "ns";
  auto objs = helm::render(c, component_values(0, false, 0), o);
  const Value* d = find_kind(objs, "Deployment");
  EXPECT_TRUE(d != nullptr);
  EXPECT_TRUE(find_kind(objs, "StatefulSet") == nullptr);
  EXPECT_TRUE(find_kind(objs, "HorizontalPodAutoscaler") == nullptr);
  const Value& ct = d->at_path("spec.template.spec.containers")[0];
  EXPECT_EQ(ct.get("image").as_string(), std::string("reg/app:tag"));
  EXPECT_TRUE(ct.at_path("resources.limits").find("amd.com/gpu") == nullptr);
  EXPECT_EQ(ct.at_path("resources.limits.ephemeral-storage").as_string(), std::string("1Gi"));
  EXPECT_EQ(ct.at_path("resources.requests.memory").as_string(), std::string("1Gi"));
  EXPECT_EQ(d->at_path("spec.template.metadata.labels.app.kubernetes.io/name").as_string(""), std::string(""));
  const Value& labels = d->at_path("spec.template.metadata.labels");
  EXPECT_EQ(labels.get("app.kubernetes.io/name").as_string(), std::string("devspace-app"));
  EXPECT_EQ(labels.get("app.kubernetes.io/component").as_string(), std::string("default"));
  EXPECT_EQ(d->at_path("spec.template.spec.imagePullSecrets")[0].get("name").as_string(),
            std::string("devspace-auth-reg"));
  const Value* svc = find_kind(objs, "Service");
  EXPECT_TRUE(svc != nullptr);
  EXPECT_EQ(svc->at_path("spec.ports")[0].get("targetPort").as_int(), (int64_t)3000);
  // install order: Service before Deployment
  auto si = std::find_if(objs.begin(), objs.end(), [](const Value& v) { return v.get("kind").as_string() == "Service"; });
  auto di = std::find_if(objs.begin(), objs.end(), [](const Value& v) { return v.get("kind").as_string() == "Deployment"; });
  EXPECT_TRUE(si < di);
}

TEST(component_chart_gpu_statefulset_hpa) {
  helm::Chart c = helm::load_chart(std::string(DEVSPACE_SOURCE_DIR) + "/templates/_base/chart");
  helm::RenderOptions o;
  o.release_name = "train";
  auto objs = helm::render(c, component_values(8, true, 4), o);
  const Value* s = find_kind(objs, "StatefulSet");
  EXPECT_TRUE(s != nullptr);
  EXPECT_TRUE(find_kind(objs, "Deployment") == nullptr);
  EXPECT_EQ(s->at_path("spec.serviceName").as_string(), std::string("external"));
  const Value& ct = s->at_path("spec.template.spec.containers")[0];
  EXPECT_EQ(ct.at_path("resources.limits").get("amd.com/gpu").as_int(), (int64_t)8);
  bool nproc = false, shm = false;
  for (auto& e : ct.get("env").items())
    if (e.get("name").as_string() == "DEVSPACE_NPROC") nproc = e.get("value").as_string() == "8";
  for (auto& m : ct.get("volumeMounts").items())
    if (m.get("mountPath").as_string() == "/dev/shm") shm = true;
  EXPECT_TRUE(nproc);
  EXPECT_TRUE(shm);
  std::string shm_size;
  for (auto& v : s->at_path("spec.template.spec.volumes").items())
    if (v.get("name").as_string() == "dshm") shm_size = v.at_path("emptyDir.sizeLimit").as_string();
  EXPECT_EQ(shm_size, std::string("128Gi"));
  const Value* pvc = find_kind(objs, "PersistentVolumeClaim");
  EXPECT_TRUE(pvc != nullptr);
  EXPECT_EQ(pvc->at_path("spec.resources.requests.storage").as_string(), std::string("2Gi"));
  const Value* hpa = find_kind(objs, "HorizontalPodAutoscaler");
  EXPECT_TRUE(hpa != nullptr);
  EXPECT_EQ(hpa->at_path("spec.maxReplicas").as_int(), (int64_t)4);
}

TEST(generator_detects_languages) {
  std::string d = fs::make_temp_dir("gen-");
  generator::ChartGenerator g(d);
  auto langs = g.supported_languages();
  EXPECT_TRUE(std::find(langs.begin(), langs.end(), "rocm-pytorch") != langs.end());
  EXPECT_TRUE(std::find(langs.begin(), langs.end(), "javascript") != langs.end());
  EXPECT_EQ(g.detect_language(), std::string(""));
  fs::write_file(fs::join(d, "index.js"), std::string(300, 'x'));
  fs::write_file(fs::join(d, "node_modules/dep/big.py"), std::string(5000, 'x'));  // vendored: ignored
  EXPECT_EQ(g.detect_language(), std::string("javascript"));
  fs::write_file(fs::join(d, "tool.py"), "print(1)\n" + std::string(500, '#'));
  EXPECT_EQ(g.detect_language(), std::string("python"));
  fs::write_file(fs::join(d, "train.py"), "import torch\n");
  EXPECT_EQ(g.detect_language(), std::string("rocm-pytorch"));
  g.create_chart("rocm-pytorch", false);
  EXPECT_TRUE(fs::exists(fs::join(d, "chart/Chart.yaml")));
  EXPECT_TRUE(fs::exists(fs::join(d, "chart/templates/deployments.yaml")));
  EXPECT_TRUE(contains(fs::read_file(fs::join(d, "Dockerfile")), "rocm/pytorch"));
  EXPECT_TRUE(contains(fs::read_file(fs::join(d, "devspace_amd/runner.py")), "Hot-reload runner"));
  EXPECT_TRUE(contains(fs::read_file(fs::join(d, "devspace_amd/ops/fused_ops.hip")), "gfx950"));
  EXPECT_TRUE(fs::exists(fs::join(d, "devspace_amd/ops/build.py")));
  // no overwrite of user files
  EXPECT_TRUE(contains(fs::read_file(fs::join(d, "train.py")), "import torch"));
  fs::remove_all(d);
}

TEST(generator_dockerfile_cmd_uses_the_entry_file) {
  auto cmd_of = [](const std::vector<std::string>& files) {
    std::string d = fs::make_temp_dir("gen-");
    for (auto& f : files) fs::write_file(fs::join(d, f), "print(1)\n");
    generator::ChartGenerator(d).create_chart("python", false);
    std::string df = fs::read_file(fs::join(d, "Dockerfile"));
    fs::remove_all(d);
    return df.substr(df.find("CMD"));
  };
  EXPECT_EQ(cmd_of({"main.py", "app.py"}), std::string("CMD [\"python\", \"main.py\"]\n"));
  EXPECT_EQ(cmd_of({"util.py", "app.py"}), std::string("CMD [\"python\", \"app.py\"]\n"));
  EXPECT_EQ(cmd_of({"hello.py"}), std::string("CMD [\"python\", \"hello.py\"]\n"));
  EXPECT_EQ(cmd_of({"a.py", "b.py"}), std::string("CMD [\"python\", \"main.py\"]\n"));
}

TEST(configure_mutations) {
  std::string d = fs::make_temp_dir("cfg-");
  std::string old = fs::cwd();
  fs::chdir(d);
  fs::write_file(".devspace/config.yaml",
                 "version: v1alpha2\ndeployments:\n- name: app\n  helm:\n    chartPath: ./chart\n"
                 "dev:\n  selectors:\n  - name: default\n    labelSelector:\n      app: web\n");
  {
    config::Context ctx;
    configure::add_port(ctx, "", "", "", "8080,9000:90");
  }
  {
    config::Context ctx;
    const Value& p = ctx.base().at_path("dev.ports");
    EXPECT_EQ(p.size(), (size_t)1);
    EXPECT_EQ(p[0].get("labelSelector").get("app").as_string(), std::string("web"));
    EXPECT_EQ(p[0].get("portMappings")[1].get("remotePort").as_int(), (int64_t)90);
    configure::add_port(ctx, "", "app=web", "", "7000");  // same selector: appended
  }
  {
    config::Context ctx;
    EXPECT_EQ(ctx.base().at_path("dev.ports")[0].get("portMappings").size(), (size_t)3);
    configure::remove_port(ctx, false, "", "8080,90");
  }
  {
    config::Context ctx;
    auto& pm = ctx.base().at_path("dev.ports")[0].get("portMappings");
    EXPECT_EQ(pm.size(), (size_t)1);
    EXPECT_EQ(pm[0].get("localPort").as_int(), (int64_t)7000);
    EXPECT_THROWS(configure::add_sync(ctx, "./", "relative", "", "", "", ""));
    configure::add_sync(ctx, "./src", "/app/src", "", "", "a/, b", "");
    configure::add_deployment(ctx, "k", "", "kube/*.yaml, more.yaml", "");
    EXPECT_THROWS(configure::add_deployment(ctx, "k", "", "x.yaml", ""));
    EXPECT_THROWS(configure::add_deployment(ctx, "z", "", "x.yaml", "./c"));
  }
  {
    config::Context ctx;
    const Value& s = ctx.base().at_path("dev.sync")[0];
    EXPECT_EQ(s.get("excludePaths")[1].as_string(), std::string("b"));
    EXPECT_EQ(s.get("labelSelector").get("app").as_string(), std::string("web"));
    EXPECT_EQ(ctx.base().get("deployments")[1].at_path("kubectl.manifests")[1].as_string(), std::string("more.yaml"));
    configure::remove_deployment(ctx, false, "k");
    configure::remove_sync(ctx, false, "", "/app/src", "");
  }
  {
    config::Context ctx;
    EXPECT_EQ(ctx.base().get("deployments").size(), (size_t)1);
    EXPECT_EQ(ctx.base().at_path("dev.sync").size(), (size_t)0);
  }
  EXPECT_THROWS(configure::parse_selectors("a=b,c"));
  EXPECT_THROWS(configure::parse_port_mappings("1:2:3"));
  fs::chdir(old);
  fs::remove_all(d);
}

TEST(helmrepo_versions_and_search) {
  EXPECT_EQ(helmrepo::compare_versions("1.10.0", "1.9.3"), 1);
  EXPECT_EQ(helmrepo::compare_versions("v2.0", "2.0.0"), 0);
  EXPECT_EQ(helmrepo::compare_versions("0.1.0", "0.1.1"), -1);
  std::string home = fs::make_temp_dir("helmhome-");
  setenv("DEVSPACE_HELM_HOME", home.c_str(), 1);
  std::string repo = fs::make_temp_dir("repo-");
  fs::write_file(fs::join(repo, "index.yaml"),
                 "apiVersion: v1\nentries:\n  mysql:\n  - name: mysql\n    version: 0.9.0\n    appVersion: 5.7.1\n"
                 "    urls: [mysql-0.9.0.tgz]\n  - name: mysql\n    version: 0.10.2\n    appVersion: 5.7.14\n"
                 "    urls: [mysql-0.10.2.tgz]\n");
  helmrepo::add_repo({"local", "file://" + repo});
  helmrepo::update();
  auto v = helmrepo::search("mysql");
  EXPECT_EQ(v.version, std::string("0.10.2"));
  EXPECT_EQ(helmrepo::search("mysql", "", "5.7.1").version, std::string("0.9.0"));
  EXPECT_THROWS(helmrepo::search("nope"));
  unsetenv("DEVSPACE_HELM_HOME");
  fs::remove_all(home);
  fs::remove_all(repo);
}

// Mutation fuzz of the template engine over the embedded component chart: every mutated
// template either renders or throws a std::exception (parse/exec error) — no crash, hang or
// other exception type. Under scripts/sanitize.sh this also checks memory safety.
TEST(gotemplate_mutation_fuzz_never_crashes) {
  const auto& emb = generator::embedded_templates();
  std::string helpers = emb.at("_base/chart/templates/_helpers.tpl");
  Value values = yaml_parse(emb.at("_base/chart/values.yaml"));
  Value data = Value::map();
  data["Values"] = values;
  data["Release"]["Name"] = "rel";
  data["Release"]["Namespace"] = "ns";
  data["Chart"]["Name"] = "chart";
  std::vector<std::string> seeds;
  for (auto& kv : emb)
    if (starts_with(kv.first, "_base/chart/templates/") && ends_with(kv.first, ".yaml")) seeds.push_back(kv.second);
  EXPECT_TRUE(seeds.size() >= 3);
  const std::string alphabet = "{}|$.()\"- :=,_abeinrtV0123\n";
  uint64_t rng = 0x9E3779B97F4A7C15ull;
  auto next = [&rng] {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return rng;
  };
  int rendered = 0, errors = 0;
  for (int it = 0; it < 4000; ++it) {
    std::string t = seeds[next() % seeds.size()];
    int nmut = 1 + (int)(next() % 3);
    for (int m = 0; m < nmut && !t.empty(); ++m) {
      size_t i = next() % t.size();
      switch (next() % 3) {
        case 0: t[i] = alphabet[next() % alphabet.size()]; break;
        case 1: t.erase(i, 1 + next() % 4); break;
        default: t.insert(i, 1, alphabet[next() % alphabet.size()]);
      }
    }
    try {
      tmpl::Engine e;
      e.add("_helpers.tpl", helpers);
      e.add("t", t);
      e.execute("t", data);
      ++rendered;
    } catch (const std::exception&) {
      ++errors;
    }
  }
  EXPECT_TRUE(rendered > 100 && errors > 100);
}

TEST(sprig_certificates_encryption_durations) {
  Value d = Value::map();
  std::string out = render_tmpl(
      "{{ $ca := genCA \"my-ca\" 365 }}{{ $c := genSignedCert \"svc\" (list \"10.0.0.1\") (list \"svc.ns.svc\") 30 $ca }}"
      "{{ $ca.Cert }}|{{ $c.Cert }}|{{ $c.Key }}|{{ (genSelfSignedCert \"self\" nil (list \"a.b\") 1).Cert }}",
      d);
  auto parts = split(out, "|");
  EXPECT_EQ(parts.size(), (size_t)4);
  auto read_cert = [](const std::string& pem) {
    BIO* b = BIO_new_mem_buf(pem.data(), (int)pem.size());
    X509* x = PEM_read_bio_X509(b, nullptr, nullptr, nullptr);
    BIO_free(b);
    return x;
  };
  X509* ca = read_cert(parts[0]);
  X509* leaf = read_cert(parts[1]);
  X509* self = read_cert(parts[3]);
  EXPECT_TRUE(ca && leaf && self);
  EXPECT_EQ(X509_check_ca(ca), 1);
  EVP_PKEY* ca_pub = X509_get_pubkey(ca);
  EXPECT_EQ(X509_verify(leaf, ca_pub), 1);  // signed by the CA
  EXPECT_EQ(X509_check_host(leaf, "svc.ns.svc", 0, 0, nullptr), 1);
  EXPECT_EQ(X509_check_ip_asc(leaf, "10.0.0.1", 0), 1);
  EXPECT_EQ(X509_check_host(self, "a.b", 0, 0, nullptr), 1);
  EXPECT_TRUE(contains(parts[2], "BEGIN RSA PRIVATE KEY"));
  EVP_PKEY_free(ca_pub);
  X509_free(ca);
  X509_free(leaf);
  X509_free(self);
  for (const char* t : {"rsa", "ecdsa", "ed25519"})
    EXPECT_TRUE(contains(render_tmpl(std::string("{{ genPrivateKey \"") + t + "\" }}", d), "PRIVATE KEY-----"));
  EXPECT_EQ(render_tmpl("{{ encryptAES \"secretkey\" \"plaintext\" | decryptAES \"secretkey\" }}", d),
            std::string("plaintext"));
  EXPECT_EQ(render_tmpl("{{ duration 3725 }} {{ duration \"95\" }} {{ duration 0 }}", d), std::string("1h2m5s 1m35s 0s"));
  std::string line = render_tmpl("{{ htpasswd \"admin\" \"s3cret\" }}", d);
  EXPECT_TRUE(starts_with(line, "admin:$2a$10$") && line.size() == 6 + 60);
  struct crypt_data cd;
  std::memset(&cd, 0, sizeof(cd));
  std::string hash = line.substr(6);
  EXPECT_EQ(std::string(crypt_r("s3cret", hash.c_str(), &cd)), hash);  // verifies as bcrypt
}

TEST(sprig_remaining_functions) {
  Value d = Value::map();
  EXPECT_EQ(render_tmpl("{{ osBase \"/a/b.txt\" }} {{ osExt \"x.tar.gz\" }} {{ biggest 1 7 3 }}", d), std::string("b.txt .gz 7"));
  EXPECT_EQ(render_tmpl("{{ sha512sum \"abc\" | trunc 16 }}", d), std::string("ddaf35a193617aba"));
  EXPECT_EQ(render_tmpl("{{ chunk 2 (list 1 2 3 4 5) | toJson }}", d), std::string("[[1,2],[3,4],[5]]"));
  std::string sh = render_tmpl("{{ shuffle \"abcdef\" }}", d);
  std::string sorted = sh;
  std::sort(sorted.begin(), sorted.end());
  EXPECT_EQ(sorted, std::string("abcdef"));
  EXPECT_EQ(render_tmpl("{{ $u := urlParse \"https://me:pw@example.com:8443/p/q?x=1#frag\" }}"
                        "{{ $u.scheme }}|{{ $u.host }}|{{ $u.hostname }}|{{ $u.path }}|{{ $u.query }}|{{ $u.fragment }}|{{ $u.userinfo }}",
                        d),
            std::string("https|example.com:8443|example.com|/p/q|x=1|frag|me:pw"));
  EXPECT_EQ(render_tmpl("{{ urlJoin (dict \"scheme\" \"http\" \"host\" \"h:80\" \"path\" \"/x\" \"query\" \"a=b\") }}", d),
            std::string("http://h:80/x?a=b"));
  EXPECT_EQ(render_tmpl("{{ getHostByName \"localhost\" | empty | not }}", d), std::string("true"));
  EXPECT_EQ(render_tmpl("{{ mustMerge (dict \"a\" 1) (dict \"a\" 2 \"b\" 3) | toJson }}", d), std::string("{\"a\":1,\"b\":3}"));
}

// Behaviours of Go's text/template + Sprig that charts rely on (checked against Go semantics).
TEST(gotemplate_go_semantics_corner_cases) {
  Value d = yaml_parse("list: [1, 2]\nm: {b: 1, a: 2}\nzero: 0\nf: 1.5\nbig: 1000000\ntwo: 2.0\nhuge: 1.0e+21\nsmall: 1.0e-7\n");
  struct Case {
    const char* tmpl;
    const char* want;
  } cases[] = {
      {"{{ and 1 0 2 }}", "0"},
      {"{{ or 0 \"\" \"x\" }}", "x"},
      {"{{ range $k, $v := .m }}{{ $k }}{{ end }}", "ab"},
      {"{{ with .missing }}x{{ else }}y{{ end }}", "y"},
      {"{{ \"a\" | printf \"%s-%s\" \"b\" }}", "b-a"},
      {"{{ 3 | add 1 }}", "4"},
      {"{{ printf \"%v\" .list }}", "[1 2]"},
      {"{{ .f }} {{ 1e3 }}", "1.5 1000"},
      {"{{ default 5 .zero }}", "5"},
      {"{{ empty (list) }}", "true"},
      {"{{ ternary \"a\" \"b\" true }}", "a"},
      {"[{{ quote .missing }}]", "[]"},
      {"{{ quote 1 \"x\" }}", "\"1\" \"x\""},
      {"{{ eq 1 2 1 }}", "true"},
      {"{{ len .m }}", "2"},
      {"{{ index .list 1 }}", "2"},
      {"{{- \"x\" -}}  {{- \"y\" }}", "xy"},
      {"{{ toYaml .m | trim }}", "a: 2\nb: 1"},
      {"{{ $x := 1 }}{{ if true }}{{ $x = 2 }}{{ end }}{{ $x }}", "2"},
      {"{{ range $i, $e := until 3 }}{{ $i }}{{ end }}", "012"},
      {"{{ int \"12\" | add 1 }} {{ atoi \"7\" }}", "13 7"},
      {"{{ not 0 }} {{ not 1 }}", "true false"},
      {"{{ lt 1 2 }} {{ ge 2 2 }}", "true true"},
      {"{{ print 1 2 \"a\" \"b\" 3 }}", "1 2ab3"},  // fmt.Sprint: spaces only between two non-strings
      {"{{ .big }} {{ .two }} {{ .huge }} {{ .small }}", "1000000 2 1e+21 1e-07"},
      {"a{{/* c */}}b{{- /* c2 */ -}} c", "abc"},
      {"{{ define \"tt\" }}<{{ . }}>{{ end }}{{ template \"tt\" 5 }}", "<5>"},
      {"{{ define \"rec\" }}{{ include \"rec\" . }}{{ end }}{{ include \"rec\" 1 }}",
       "ERROR: render error in t: template: exceeded maximum template depth (100)"},
      {"{{ block \"blk\" . }}dflt{{ end }}", "dflt"},
      {"{{ range .list }}{{ $.f }}{{ end }}", "1.51.5"},
      {"{{ .missing | default \"a\" | upper }}", "A"},
      {"{{ if eq .missing nil }}nil{{ end }}", "nil"},
      {"{{ (index .m \"a\") }} {{ .m.b }}", "2 1"},
      {"{{ printf \"%d %s %q %5.2f\" 3 \"x\" \"y\" 3.14159 }}", "3 x \"y\"  3.14"},
      {"{{ until 1000000000 | len }}",
       "ERROR: render error in t: until: 1000000000 elements exceed the limit of 10000000"},
      {"{{ repeat 3 \"ab\" }} {{ seq 3 }} {{ untilStep 0 6 2 | len }}", "ababab 1 2 3 3"},
      // n * size wraps int64 for these: the guard must not be fooled
      {"{{ repeat 4611686018427387904 \"ab\" }}",
       "ERROR: render error in t: repeat: 4611686018427387904 x 2 bytes exceeds the limit of 10000000"},
      {"{{ repeat 6000000 \"ab\" | len }}",
       "ERROR: render error in t: repeat: 6000000 x 2 bytes exceeds the limit of 10000000"},
      {"{{ untilStep -9223372036854775807 9223372036854775807 1 | len }}",
       "ERROR: render error in t: untilStep: the range exceeds the limit of 10000000"},
      {"{{ untilStep 9223372036854775806 9223372036854775807 5 | len }}", "1"},
      {"{{ seq 9223372036854775806 5 9223372036854775807 }}", "9223372036854775806"},
      {"{{ seq -9223372036854775807 2 9223372036854775807 | len }}",
       "ERROR: render error in t: seq: the range exceeds the limit of 10000000"},
  };
  for (auto& c : cases) {
    std::string got;
    try {
      got = render_tmpl(c.tmpl, d);
    } catch (const std::exception& e) {
      got = std::string("ERROR: ") + e.what();
    }
    if (got != c.want) std::fprintf(stderr, "  %s -> [%s], want [%s]\n", c.tmpl, got.c_str(), c.want);
    EXPECT_EQ(got, std::string(c.want));
  }
}

// std::regex recurses per input character; long inputs used to overflow the stack (a 100 kB
// container log line crashed `devspace analyze`).
TEST(regex_on_long_inputs_does_not_crash) {
#if defined(__SANITIZE_THREAD__)
#define DS_TSAN 1
#elif defined(__has_feature)
#if __has_feature(thread_sanitizer)
#define DS_TSAN 1
#endif
#endif
#ifdef DS_TSAN
  // ThreadSanitizer's runtime does not cope with std::regex's deep recursion on a large
  // custom thread stack (it faults inside the runtime); this test is about stack depth, which
  // the release and ASan builds cover, not about races.
  return;
#endif
  std::string m;
  // 60 kB: twice what overflows an 8 MB stack in a plain std::regex call
  EXPECT_TRUE(analyze::log_has_gpu_runtime_error(std::string(60000, 'y') + "\nNCCL error: boom\n", &m));
  EXPECT_EQ(m, std::string("NCCL error"));
  EXPECT_TRUE(!analyze::log_has_gpu_runtime_error(std::string(60000, 'z'), &m));
  Value d = Value::map();
  d["s"] = std::string(60000, 'a') + "b";
  EXPECT_EQ(render_tmpl("{{ regexFind \"a*b\" .s | len }}", d), std::string("60001"));
  EXPECT_EQ(render_tmpl("{{ regexMatch \"^a+b$\" .s }}", d), std::string("true"));
  EXPECT_EQ(render_tmpl("{{ regexReplaceAll \"a+\" .s \"x\" }}", d), std::string("xb"));
  EXPECT_EQ(render_tmpl("{{ regexFindAll \"a+b\" .s -1 | len }}", d), std::string("1"));
}


// ---------------------------------------------------------------- MI355X pod sizing

static Value init_values(int gpus, const std::vector<gpu::GpuNode>& nodes = {}) {
  // what `devspace init` writes into the base chart's values.yaml for a rocm-pytorch project
  std::string v = fs::read_file(std::string(DEVSPACE_SOURCE_DIR) + "/templates/_base/chart/values.yaml");
  gpu::PodSizing s = gpu::size_pod(gpus, nodes);
  v = replace_all(v, "#image#", "reg/train:tag");
  v = replace_all(v, "#port#", "29500");
  v = replace_all(v, "#resources#", gpu::resources_yaml(s));
  std::string settings = gpu::gpu_settings_yaml(s);
  v = replace_all(v, settings.empty() ? "#gpu-settings#\n" : "#gpu-settings#", settings);
  return yaml_parse(v);
}

static void check_gpu_pod_invariants(const Value& spec, int gpus, const std::string& resource = "amd.com/gpu") {
  const Value& ct = spec.get("containers")[0];
  const Value& lim = ct.at_path("resources.limits");
  const Value& req = ct.at_path("resources.requests");
  EXPECT_EQ(lim.get(resource).as_int(), (int64_t)gpus);
  double cpu = gpu::parse_cpu(lim.get("cpu").as_string());
  int64_t mem = gpu::parse_memory_bytes(lim.get("memory").as_string());
  EXPECT_TRUE(cpu >= gpus);  // at least one core per rank
  EXPECT_EQ(req.get("cpu").as_string(), lim.get("cpu").as_string());
  EXPECT_EQ(req.get("memory").as_string(), lim.get("memory").as_string());
  int64_t shm = -1;
  for (auto& v : spec.get("volumes").items())
    if (v.get("name").as_string() == "dshm") shm = gpu::parse_memory_bytes(v.at_path("emptyDir.sizeLimit").as_string());
  EXPECT_TRUE(shm > 0);
  // tmpfs pages are charged to the container: memory covers shm plus a host budget per rank
  EXPECT_TRUE(mem >= shm + (int64_t)gpus * (8ll << 30));
  bool tol = false;
  for (auto& t : spec.get("tolerations").items())
    if (t.get("key").as_string() == "amd.com/gpu" && t.get("effect").as_string() == "NoSchedule") tol = true;
  EXPECT_TRUE(tol);
  EXPECT_TRUE(gpu::pod_sizing_problems(spec).empty());
}

TEST(component_chart_gpu_sizing_1_2_4_8) {
  helm::Chart c = helm::load_chart(std::string(DEVSPACE_SOURCE_DIR) + "/templates/_base/chart");
  helm::RenderOptions o;
  o.release_name = "train";
  for (int g : {1, 2, 4, 8}) {
    auto objs = helm::render(c, init_values(g), o);
    const Value* d = find_kind(objs, "Deployment");
    EXPECT_TRUE(d != nullptr);
    const Value& spec = d->at_path("spec.template.spec");
    check_gpu_pod_invariants(spec, g);
    // defaults: 12 CPUs and 80 Gi (16 Gi shm + 64 Gi) per GPU
    const Value& lim = spec.get("containers")[0].at_path("resources.limits");
    EXPECT_EQ(lim.get("cpu").as_string(), std::to_string(12 * g));
    EXPECT_EQ(lim.get("memory").as_string(), std::to_string(80 * g) + "Gi");
    EXPECT_TRUE(spec.find("nodeSelector") == nullptr);
  }
}

TEST(component_chart_gpu_sizing_from_node_allocatable) {
  // an 8x MI355X node with 256 CPUs and 3 TiB allocatable, labelled by the GPU operator
  Value nodes = yaml_parse(
      "items:\n"
      "- metadata: {name: mi355x-0, labels: {amd.com/gpu.product-name: AMD_Instinct_MI355X}}\n"
      "  status: {allocatable: {cpu: '256', memory: 3221225472Ki, amd.com/gpu: '8'}}\n"
      "- metadata: {name: cpu-0}\n"
      "  status: {allocatable: {cpu: '64', memory: 256Gi}}\n");
  auto gn = gpu::gpu_nodes(nodes);
  EXPECT_EQ(gn.size(), (size_t)1);
  EXPECT_EQ(gn[0].memory, (int64_t)3221225472ll * 1024);
  gpu::PodSizing s = gpu::size_pod(4, gn);
  EXPECT_EQ(s.cpu_per_gpu, 28);  // floor(256 * 0.9 / 8)
  EXPECT_EQ(s.shm_per_gpu_gi + s.host_per_gpu_gi, 345);  // floor(3072 GiB * 0.9 / 8)
  EXPECT_EQ(s.product, std::string("AMD_Instinct_MI355X"));
  helm::Chart c = helm::load_chart(std::string(DEVSPACE_SOURCE_DIR) + "/templates/_base/chart");
  helm::RenderOptions o;
  o.release_name = "train";
  auto objs = helm::render(c, init_values(4, gn), o);
  const Value& spec = find_kind(objs, "Deployment")->at_path("spec.template.spec");
  check_gpu_pod_invariants(spec, 4);
  EXPECT_EQ(spec.at_path("nodeSelector").get("amd.com/gpu.product-name").as_string(),
            std::string("AMD_Instinct_MI355X"));
  EXPECT_EQ(spec.get("containers")[0].at_path("resources.limits.cpu").as_string(), std::string("112"));
}

// MI355X nodes in SPX mode advertise 8 devices of 288 GB; in CPX mode (one
// partition per XCD) 64 devices of an even 36 GB share. The node labeller says which.
static Value mi355x_node(const std::string& name, const std::string& mode, const std::string& nps,
                         const std::string& resource, int64_t capacity, int64_t allocatable) {
  return yaml_parse(
      "items:\n"
      "- metadata:\n"
      "    name: " + name + "\n"
      "    labels: {amd.com/gpu.product-name: AMD_Instinct_MI355X, amd.com/gpu.vram: 288G,\n"
      "             amd.com/gpu.compute-partitioning-mode: " + mode + ", amd.com/gpu.memory-partitioning-mode: " + nps + "}\n"
      "  status:\n"
      "    capacity: {cpu: '256', memory: 3221225472Ki, " + resource + ": '" + std::to_string(capacity) + "'}\n"
      "    allocatable: {cpu: '256', memory: 3221225472Ki, " + resource + ": '" + std::to_string(allocatable) + "'}\n");
}

TEST(gpu_sizing_spx_x8_node) {
  auto gn = gpu::gpu_nodes(mi355x_node("mi355x-spx", "spx", "nps1", "amd.com/gpu", 8, 8));
  EXPECT_EQ(gn.size(), (size_t)1);
  EXPECT_EQ(gn[0].parts(), 1);
  EXPECT_EQ(gn[0].hbm_per_device(), (int64_t)288000000000LL);
  EXPECT_EQ(gn[0].unhealthy(), (int64_t)0);
  EXPECT_TRUE(contains(gn[0].describe(), "8 x AMD_Instinct_MI355X, SPX/NPS1: 8 schedulable amd.com/gpu of 288 GB"));
  gpu::PodSizing s = gpu::size_pod(8, gn);
  EXPECT_EQ(s.cpu_per_gpu, 28);
  EXPECT_EQ(s.hbm_per_device, (int64_t)288000000000LL);
  EXPECT_TRUE(contains(gpu::resources_yaml(s), "288 GB HBM each"));
  helm::Chart c = helm::load_chart(std::string(DEVSPACE_SOURCE_DIR) + "/templates/_base/chart");
  helm::RenderOptions o;
  o.release_name = "train";
  auto objs = helm::render(c, init_values(8, gn), o);
  check_gpu_pod_invariants(find_kind(objs, "Deployment")->at_path("spec.template.spec"), 8);
}

// a node with fewer CPUs than devices. The pod never asks for the whole node
// (requests = limits: a DaemonSet's CPU request would leave it Unschedulable); init warns.
TEST(gpu_sizing_leaves_headroom_on_a_node_with_a_cpu_per_gpu) {
  Value nodes = yaml_parse(
      "items:\n"
      "- metadata: {name: small}\n"
      "  status: {allocatable: {cpu: '8', memory: 64Gi, amd.com/gpu: '8'}}\n");
  auto gn = gpu::gpu_nodes(nodes);
  gpu::PodSizing s = gpu::size_pod(8, gn);
  EXPECT_TRUE(s.cpu_milli() <= 7000);
  EXPECT_EQ(s.cpu_quantity(), std::string("7"));
  EXPECT_TRUE(contains(s.warning, "fewer than one CPU each"));
  std::string res = gpu::resources_yaml(s);
  EXPECT_TRUE(contains(res, "cpu: \"7\""));
  gpu::PodSizing one = gpu::size_pod(1, gn);
  EXPECT_EQ(one.cpu_quantity(), std::string("900m"));
  // a node with CPUs to spare: whole CPUs per device, no warning
  gpu::PodSizing big = gpu::size_pod(8, gpu::gpu_nodes(mi355x_node("n", "spx", "nps1", "amd.com/gpu", 8, 8)));
  EXPECT_TRUE(big.warning.empty());
  EXPECT_EQ(big.cpu_quantity(), std::string("224"));
}

TEST(gpu_sizing_cpx_x64_node) {
  auto gn = gpu::gpu_nodes(mi355x_node("mi355x-cpx", "CPX", "NPS2", "amd.com/gpu", 64, 64));
  EXPECT_EQ(gn.size(), (size_t)1);
  EXPECT_EQ(gn[0].parts(), 8);
  EXPECT_EQ(gn[0].hbm_per_device(), (int64_t)36000000000LL);  // 288 GB / 8 partitions
  EXPECT_TRUE(contains(gn[0].describe(), "8 x AMD_Instinct_MI355X, CPX/NPS2: 64 schedulable amd.com/gpu of 36 GB"));
  gpu::PodSizing s = gpu::size_pod(8, gn);
  // a 64th of the node per device, not an 8th
  EXPECT_EQ(s.cpu_per_gpu, 3);                             // floor(256 * 0.9 / 64)
  EXPECT_EQ(s.shm_per_gpu_gi + s.host_per_gpu_gi, 43);     // floor(3072 GiB * 0.9 / 64)
  EXPECT_EQ(s.shm_per_gpu_gi, 10);
  EXPECT_EQ(s.partition, std::string("CPX/NPS2"));
  std::string res = gpu::resources_yaml(s);
  EXPECT_TRUE(contains(res, "CPX/NPS2 partition") && contains(res, "36 GB") && contains(res, "288 GB for the 8"));
  EXPECT_TRUE(!contains(res, "288 GB per GPU"));
  helm::Chart c = helm::load_chart(std::string(DEVSPACE_SOURCE_DIR) + "/templates/_base/chart");
  helm::RenderOptions o;
  o.release_name = "train";
  auto objs = helm::render(c, init_values(8, gn), o);
  check_gpu_pod_invariants(find_kind(objs, "Deployment")->at_path("spec.template.spec"), 8);
  // the init prompt's bound is the largest node's allocatable
  EXPECT_EQ(gpu::largest(gn)->gpus, (int64_t)64);
  std::regex r("^" + gpu::range_regex(64) + "$");
  EXPECT_TRUE(std::regex_match("64", r) && std::regex_match("1", r) && std::regex_match("9", r));
  EXPECT_TRUE(!std::regex_match("65", r) && !std::regex_match("0", r) && !std::regex_match("640", r));
}

TEST(gpu_sizing_mixed_strategy_resource_names) {
  EXPECT_TRUE(gpu::is_gpu_resource("amd.com/gpu") && gpu::is_gpu_resource("amd.com/cpx_nps2") &&
              gpu::is_gpu_resource("amd.com/spx"));
  EXPECT_TRUE(!gpu::is_gpu_resource("amd.com/gpu.product-name") && !gpu::is_gpu_resource("amd.com/cpx_npsx") &&
              !gpu::is_gpu_resource("nvidia.com/gpu"));
  auto gn = gpu::gpu_nodes(mi355x_node("mixed", "", "", "amd.com/cpx_nps2", 64, 62));
  EXPECT_EQ(gn.size(), (size_t)1);
  EXPECT_EQ(gn[0].resource, std::string("amd.com/cpx_nps2"));
  EXPECT_EQ(gn[0].compute_mode, std::string("cpx"));
  EXPECT_EQ(gn[0].memory_mode, std::string("nps2"));
  EXPECT_EQ(gn[0].unhealthy(), (int64_t)2);
  gpu::PodSizing s = gpu::size_pod(4, gn);
  EXPECT_EQ(s.resource, std::string("amd.com/cpx_nps2"));
  EXPECT_TRUE(contains(gpu::gpu_settings_yaml(s), "gpuResource: \"amd.com/cpx_nps2\""));
  helm::Chart c = helm::load_chart(std::string(DEVSPACE_SOURCE_DIR) + "/templates/_base/chart");
  helm::RenderOptions o;
  o.release_name = "train";
  auto objs = helm::render(c, init_values(4, gn), o);
  const Value& spec = find_kind(objs, "Deployment")->at_path("spec.template.spec");
  check_gpu_pod_invariants(spec, 4, "amd.com/cpx_nps2");
  EXPECT_TRUE(spec.get("containers")[0].at_path("resources.limits").find("amd.com/gpu") == nullptr);
  EXPECT_EQ(gpu::container_gpu_request(spec.get("containers")[0]), (int64_t)4);
}

TEST(component_chart_cpu_only_has_no_gpu_scheduling) {
  helm::Chart c = helm::load_chart(std::string(DEVSPACE_SOURCE_DIR) + "/templates/_base/chart");
  helm::RenderOptions o;
  o.release_name = "web";
  auto objs = helm::render(c, init_values(0), o);
  const Value& spec = find_kind(objs, "Deployment")->at_path("spec.template.spec");
  EXPECT_TRUE(spec.find("tolerations") == nullptr);
  const Value& ct = spec.get("containers")[0];
  EXPECT_EQ(ct.at_path("resources.limits.cpu").as_string(), std::string("2"));
  EXPECT_TRUE(ct.at_path("resources").find("requests") == nullptr);
  EXPECT_TRUE(ct.at_path("resources.limits").find("amd.com/gpu") == nullptr);
}

TEST(gpu_sizing_problems_flag_undersized_pods) {
  // the round-2 chart for 8 GPUs: 2 CPUs, 4 Gi memory, 128 Gi memory-backed shm
  Value spec = yaml_parse(
      "containers:\n"
      "- name: train\n"
      "  resources: {limits: {cpu: '2', memory: 4Gi, amd.com/gpu: 8}}\n"
      "  volumeMounts: [{name: dshm, mountPath: /dev/shm}]\n"
      "volumes: [{name: dshm, emptyDir: {medium: Memory, sizeLimit: 128Gi}}]\n");
  auto probs = gpu::pod_sizing_problems(spec);
  EXPECT_EQ(probs.size(), (size_t)2);
  EXPECT_TRUE(contains(probs[0], "/dev/shm") && contains(probs[0], "OOM"));
  EXPECT_TRUE(contains(probs[1], "2 CPU(s) for 8 GPU rank(s)"));
  Value nolimit = yaml_parse("containers:\n- name: t\n  resources: {limits: {amd.com/gpu: 1}}\n");
  EXPECT_EQ(gpu::pod_sizing_problems(nolimit).size(), (size_t)1);
  EXPECT_EQ(gpu::parse_memory_bytes("1.5Gi"), (int64_t)1610612736);
  EXPECT_EQ(gpu::parse_memory_bytes("500M"), (int64_t)500000000);
  EXPECT_EQ(gpu::parse_memory_bytes("1e3"), (int64_t)1000);
  EXPECT_EQ(gpu::parse_memory_bytes("12Qi"), (int64_t)-1);
  EXPECT_TRUE(gpu::parse_cpu("500m") == 0.5);
}

TEST(image_reference_validation) {
  for (const char* ok : {"devspace", "user/devspace", "local.registry/init-node", "localhost:5000/a/b:v1",
                         "rocm/pytorch:rocm7.0_ubuntu24.04_py3.12_pytorch_release_2.8.0", "gcr.io/p/img@sha256:"
                         "0123456789abcdef0123456789abcdef0123456789abcdef0123456789abcdef",
                         "my-reg.example.com:443/team/app__x.y-z:1.0"})
    EXPECT_EQ(build::image_reference_problem(ok), std::string(""));
  for (const char* bad : {"", "/devspace", "user//app", "user/", "User/App", "reg.io/", "app:", "app:-bad",
                          "a b", "user/app@sha256:xyz"})
    EXPECT_TRUE(!build::image_reference_problem(bad).empty());
}

// Config layer tests: ports of config/versions/v1alpha1/upgrade_test.go (TestEmpty, TestSimple)
// plus load/override/vars/save behaviour from config/configutil.
#include <cstdlib>

#include "config/config.h"
#include "core/fs.h"
#include "core/prompt.h"
#include "testing.h"

using namespace ds;

namespace {
struct TempProject {
  std::string old, dir;
  TempProject() {
    old = fs::cwd();
    dir = fs::make_temp_dir("cfgtest-");
    fs::chdir(dir);
  }
  ~TempProject() {
    fs::chdir(old);
    fs::remove_all(dir);
  }
};
}  // namespace

TEST(upgrade_v1alpha1_empty) {
  Value v = config::upgrade_v1alpha1(Value::map());
  EXPECT_EQ(v.get("version").as_string(), std::string("v1alpha2"));
  config::validate_strict(v, config::schema_latest());
}

TEST(upgrade_v1alpha1_simple) {
  Value old = yaml_parse(
      "version: v1alpha1\n"
      "devSpace:\n"
      "  deployments:\n"
      "  - name: test\n"
      "    helm:\n"
      "      devOverwrite: overwrite\n"
      "  services:\n"
      "  - name: test\n"
      "    namespace: testnamespace\n"
      "  ports:\n"
      "  - service: test\n"
      "  sync:\n"
      "  - namespace: test\n"
      "images:\n"
      "  test:\n"
      "    name: test\n"
      "    registry: test\n"
      "registries:\n"
      "  test:\n"
      "    url: test.io\n"
      "tiller:\n"
      "  namespace: tillernamespace\n");
  Value n = config::parse_versioned(old);
  EXPECT_EQ(n.at_path("deployments")[0].at_path("helm.overrides")[0].as_string(), std::string("overwrite"));
  EXPECT_EQ(n.at_path("deployments")[0].at_path("helm.tillerNamespace").as_string(), std::string("tillernamespace"));
  EXPECT_EQ(n.at_path("dev.selectors").size(), (size_t)1);
  EXPECT_EQ(n.at_path("dev.ports").size(), (size_t)1);
  EXPECT_EQ(n.at_path("dev.selectors")[0].get("name").as_string(), std::string("test"));
  EXPECT_EQ(n.at_path("dev.ports")[0].get("selector").as_string(), std::string("test"));
  EXPECT_EQ(n.at_path("images.test.image").as_string(), std::string("test.io/test"));
  EXPECT_EQ(n.at_path("dev.autoReload.images")[0].as_string(), std::string("test"));
}

TEST(strict_unknown_field) {
  EXPECT_THROWS(config::parse_versioned(yaml_parse("version: v1alpha2\ndev:\n  bogus: 1\n")));
  EXPECT_THROWS(config::parse_versioned(yaml_parse("version: v9\n")));
  // missing version => latest (overrides)
  Value v = config::parse_versioned(yaml_parse("cluster:\n  namespace: x\n"));
  EXPECT_EQ(v.get("version").as_string(), std::string("v1alpha2"));
}

TEST(load_with_configs_yaml_overrides_and_vars) {
  TempProject p;
  setenv("DEVSPACE_VAR_IMAGE", "myrepo/app", 1);
  fs::write_file(".devspace/base.yaml",
                 "version: v1alpha2\n"
                 "images:\n"
                 "  default:\n"
                 "    image: ${IMAGE}\n"
                 "dev:\n"
                 "  ports:\n"
                 "  - labelSelector:\n"
                 "      app: x\n"
                 "    portMappings:\n"
                 "    - localPort: ${PORT}\n"
                 "      remotePort: 3000\n");
  fs::write_file(".devspace/configs.yaml",
                 "default:\n"
                 "  config:\n"
                 "    path: .devspace/base.yaml\n"
                 "  vars:\n"
                 "    data:\n"
                 "    - name: PORT\n"
                 "      default: \"8080\"\n"
                 "  overrides:\n"
                 "  - data:\n"
                 "      cluster:\n"
                 "        namespace: overridden\n");
  prompt::set_scripted_answers({""});  // accept default for PORT
  config::Context ctx;
  const Value& c = ctx.get(true);
  EXPECT_EQ(c.at_path("images.default.image").as_string(), std::string("myrepo/app"));
  EXPECT_EQ(c.at_path("cluster.namespace").as_string(), std::string("overridden"));
  EXPECT_EQ(c.at_path("dev.ports")[0].get("portMappings")[0].get("localPort").as_int(), (int64_t)8080);
  // generated.yaml caches the answers
  config::Generated g = config::Generated::load();
  EXPECT_EQ(g.vars().get("PORT").as_int(), (int64_t)8080);
  EXPECT_EQ(g.vars().get("IMAGE").as_string(), std::string("myrepo/app"));
  unsetenv("DEVSPACE_VAR_IMAGE");
}

TEST(validation_messages) {
  config::Context ctx;
  try {
    ctx.validate(yaml_parse("deployments:\n- name: a\n"));
    EXPECT_TRUE(false);
  } catch (const config::ConfigError& e) {
    EXPECT_EQ(std::string(e.what()),
              std::string("Please specify either helm or kubectl as deployment type in deployment a"));
  }
  try {
    ctx.validate(yaml_parse("dev:\n  sync:\n  - selector: x\n"));
    EXPECT_TRUE(false);
  } catch (const config::ConfigError& e) {
    EXPECT_EQ(std::string(e.what()),
              std::string("Error in config: containerPath or localSubPath are nil in sync config at index 0"));
  }
}

TEST(save_base_strips_empty) {
  TempProject p;
  fs::write_file(".devspace/config.yaml", "version: v1alpha2\ndev:\n  sync: []\ncluster: {}\n");
  config::Context ctx;
  Value& b = ctx.base();
  Value img = Value::map();
  img["image"] = "repo/x";
  b["images"]["default"] = img;
  ctx.save_base();
  std::string out = fs::read_file(".devspace/config.yaml");
  EXPECT_EQ(out, std::string("version: v1alpha2\nimages:\n  default:\n    image: repo/x\n"));
}

TEST(resolve_selector_defaults) {
  Value cfg = yaml_parse(
      "cluster:\n  namespace: ns1\n"
      "deployments:\n- name: app\n  helm:\n    chartPath: ./chart\n"
      "dev:\n  selectors:\n  - name: default\n    containerName: c1\n    labelSelector:\n      a: b\n");
  auto r = config::resolve_selector(cfg, yaml_parse("selector: default\n"));
  EXPECT_EQ(r.labels.to_query(), std::string("a=b"));
  EXPECT_EQ(r.container, std::string("c1"));
  EXPECT_EQ(r.namespace_, std::string("ns1"));
  auto r2 = config::resolve_selector(cfg, yaml_parse("namespace: other\n"));
  EXPECT_EQ(r2.labels.to_query(), std::string("app.kubernetes.io/name=app"));
  EXPECT_EQ(r2.namespace_, std::string("other"));
}

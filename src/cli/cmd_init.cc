// `devspace init` (cmd/init.go:98 Run): fresh config with the default helm deployment,
// auto-reload + entrypoint override, language detection + chart/Dockerfile generation,
// cluster (kube context + namespace, or cloud provider), selector/port/sync defaults, image
// name + registry. MI355X additions: a `rocm-pytorch` template (GPU training pod running the
// hot-reload runner) and a GPU-count question that fills amd.com/gpu limits in the chart.
#include <set>

#include "build/docker.h"
#include "cli/common.h"
#include "cloud/cloud.h"
#include "configure/configure.h"
#include "core/fs.h"
#include "core/log.h"
#include "core/proc.h"
#include "core/prompt.h"
#include "core/strutil.h"
#include "generator/generator.h"
#include "gpu/sizing.h"
#include "kube/client.h"
#include "kube/kubeconfig.h"

namespace ds {
namespace cmd {

namespace {

const char* const kConfigGitignore = "logs/\ngenerated.yaml\n";

bool yes_no(const std::string& q, const std::string& def) {
  prompt::Params p;
  p.question = q;
  p.default_value = def;
  p.options = {"yes", "no"};
  return prompt::ask(p) == "yes";
}

struct InitState {
  std::string port;
  std::string gpus = "0";
  std::string language;
  gpu::PodSizing sizing;
};

// Default base image of the rocm-pytorch template. A concrete, immutable tag: `latest` moves
// under the developer (and GPU nodes are often air-gapped, with images pre-pulled by tag).
const char* kDefaultRocmImage = "rocm/pytorch:rocm7.0_ubuntu24.04_py3.12_pytorch_release_2.8.0";

// The cluster's GPU nodes when they can be listed (3 s budget; init also works offline): what
// the device plugin advertises (whole GPUs or compute partitions) and the node labeller's labels.
std::vector<gpu::GpuNode> discover_gpu_nodes() {
  std::vector<gpu::GpuNode> nodes;
  if (getenv("DEVSPACE_INIT_NO_NODE_DISCOVERY")) return nodes;
  try {
    auto k = kube::Client::from_devspace_config(Value::map(), false);
    net::Response r = k->raw("GET", "/api/v1/nodes", "", "application/json", 3000);
    if (r.status == 200) nodes = gpu::gpu_nodes(json_parse(r.body));
  } catch (const std::exception&) {
    // no cluster configured / reachable, or nodes not listable for this user
  }
  return nodes;
}

// Per-device CPU/memory from the nodes, otherwise the per-GPU defaults.
gpu::PodSizing discover_sizing(int gpus, const std::vector<gpu::GpuNode>& nodes) {
  gpu::PodSizing s = gpu::size_pod(gpus, nodes);
  if (gpus > 0)
    log::infof("Sizing the pod for %d device(s) (%s): %s CPUs, %d Gi memory incl. %d Gi /dev/shm", gpus, s.basis.c_str(),
               s.cpu_quantity().c_str(), s.memory_gi(), s.shm_gi());
  if (gpus > 0 && !s.warning.empty()) log::warn(s.warning);
  if (gpus > 0 && s.hbm_per_device > 0)
    log::infof("HBM per device: %.0f GB%s (not a schedulable resource)", s.hbm_per_device / 1e9,
               s.partition.empty() ? "" : (" (" + s.partition + " partition)").c_str());
  return s;
}

void configure_cluster_local(Value& cfg) {
  std::string current;
  try {
    current = kube::KubeConfig::load().current_context();
  } catch (const std::exception& e) {
    log::fatal(std::string("Couldn't determine current kubernetes context: ") + e.what());
  }
  prompt::Params p;
  p.question = "Which namespace should the app run in?";
  p.default_value = "default";
  p.key = "namespace";
  p.env = "DEVSPACE_INIT_NAMESPACE";
  std::string ns = prompt::ask(p);
  cfg["cluster"]["kubeContext"] = current;
  cfg["cluster"]["namespace"] = ns;
}

void add_default_selector(Value& cfg) {
  Value s = Value::map();
  s["name"] = "default";
  s["labelSelector"]["app.kubernetes.io/name"] = config::kDefaultDeploymentName;
  s["labelSelector"]["app.kubernetes.io/component"] = "default";
  cfg["dev"]["selectors"] = Value::seq_of({s});
}

void add_default_ports(Value& cfg, InitState& st) {
  // an existing Dockerfile's first EXPOSEd port is the default (util/dockerfile.GetPorts)
  std::string def = "3000";
  try {
    std::string df;
    if (fs::read_file("Dockerfile", &df)) {
      auto ports = build::dockerfile_ports(df);
      if (!ports.empty()) def = std::to_string(ports[0]);
    }
  } catch (const std::exception&) {
  }
  prompt::Params p;
  p.question = "Which port is the app listening on? (Default: " + def + ")";
  p.default_value = "";
  p.optional = true;  // the default is applied below
  p.key = "port";
  p.env = "DEVSPACE_INIT_PORT";
  p.validation_regex = "[0-9]{0,5}";
  std::string port = prompt::ask(p);
  if (port.empty()) port = def;
  Value pms = Value::seq();
  int64_t n;
  if (parse_int64(port, &n)) {
    Value m = Value::map();
    m["localPort"] = n;
    m["remotePort"] = n;
    pms.push(m);
  }
  Value e = Value::map();
  e["selector"] = "default";
  e["portMappings"] = pms;
  cfg["dev"]["ports"] = Value::seq_of({e});
  st.port = port;
}

// Machine-learning projects: byte-code caches, notebook checkpoints, model checkpoints, run
// logs and datasets are per-side artefacts (multi-GB on MI355X nodes), never synced.
const char* kMlSyncExcludes[] = {"__pycache__/", "*.pyc", ".ipynb_checkpoints/", "checkpoints/", "*.pt",
                                 "*.pth", "*.safetensors", "wandb/", "data/"};

void add_default_sync(Value& cfg, const std::string& language) {
  Value& sync = cfg.ensure_path("dev.sync");
  if (!sync.is_seq()) sync = Value::seq();
  for (auto& s : sync.items())
    if (s.get("localSubPath").as_string() == "./" || s.get("containerPath").as_string() == "/app") return;
  Value ex = Value::seq();
  std::set<std::string> seen;
  auto add = [&](const std::string& r) {
    if (!r.empty() && seen.insert(r).second) ex.push(Value(r));
  };
  std::string di;
  if (fs::read_file(".dockerignore", &di))
    for (auto& r : split(di, "\n")) add(trim(r));
  if (language == "rocm-pytorch") {
    for (const char* r : kMlSyncExcludes) add(r);
  } else if (language == "python") {
    add("__pycache__/");
    add("*.pyc");
  }
  Value s = Value::map();
  s["selector"] = "default";
  s["containerPath"] = "/app";
  s["localSubPath"] = "./";
  s["excludePaths"] = ex;
  sync.push(s);
}

void configure_image(config::Context& ctx, bool use_cloud) {
  Value& cfg = ctx.base();
  std::string username;
  bool kaniko = false;
  std::unique_ptr<build::DockerClient> dc;
  try {
    dc = build::DockerClient::from_env(true, false);
  } catch (const std::exception& e) {
    log::fatal(std::string("Cannot create docker client: ") + e.what());
  }
  if (!dc->ping()) {
    if (!which("docker").empty() && use_cloud)
      log::fatal("Docker seems to be installed but is not running. Please start docker and restart `devspace init`");
    if (use_cloud) log::fatal("Please install docker in order to use `devspace init`");
    kaniko = true;
    log::info("No docker daemon reachable: images will be built in-cluster with kaniko");
    cfg["images"]["default"]["build"]["kaniko"]["cache"] = true;
    cfg["images"]["default"]["build"]["kaniko"]["namespace"] = "";
  }
  if (!kaniko) {
    log::start_wait("Checking Docker credentials");
    build::AuthConfig a = build::DockerConfigFile::load().get("https://index.docker.io/v1/");
    log::stop_wait();
    username = a.username;
    std::string kctx;
    try {
      kctx = kube::KubeConfig::load().current_context();
    } catch (...) {
    }
    if (!use_cloud && kctx == "minikube") {
      cfg["images"]["default"]["skipPush"] = true;
      return;
    }
  }
  try {
    configure::init_image(ctx, username, use_cloud);
  } catch (const std::exception& e) {
    log::fatal(e.what());
  }
}

void replace_placeholders(Value& cfg, InitState& st) {
  std::string image = "devspace";
  for (auto& e : cfg.get("images").entries()) {
    image = e.second.get("image").as_string(image);
    break;
  }
  if (st.port.empty()) {
    st.port = "3000";
    const Value& pm = cfg.at_path("dev.ports");
    if (pm.size() > 0 && pm[0].get("portMappings").size() > 0)
      st.port = std::to_string(pm[0].get("portMappings")[0].get("remotePort").as_int());
  }
  std::string data;
  if (!fs::read_file("chart/values.yaml", &data)) log::fatal("Couldn't find chart/values.yaml");
  data = replace_all(data, "#image#", image);
  data = replace_all(data, "#port#", st.port);
  data = replace_all(data, "#gpus#", st.gpus);
  data = replace_all(data, "#resources#", gpu::resources_yaml(st.sizing));
  std::string settings = gpu::gpu_settings_yaml(st.sizing);
  data = replace_all(data, settings.empty() ? "#gpu-settings#\n" : "#gpu-settings#", settings);
  fs::write_file("chart/values.yaml", data);
  // ROCm base image pin (GPU nodes are often air-gapped: a tag that is pre-pulled there)
  std::string df;
  if (fs::read_file("Dockerfile", &df) && contains(df, "#rocm-image#")) {
    const char* env = getenv("DEVSPACE_ROCM_IMAGE");
    std::string img = env && *env ? env : kDefaultRocmImage;
    std::string tag = build::split_image_tag(img).second;
    if (tag.empty() || tag == "latest")
      log::fatal("DEVSPACE_ROCM_IMAGE=" + img + " has no concrete tag: pin one, e.g. " + kDefaultRocmImage);
    fs::write_file("Dockerfile", replace_all(df, "#rocm-image#", img));
  }
}

int run_init(cli::Command& c, const std::vector<std::string>&) {
  config::Context ctx;
  bool exists = ctx.config_exists();
  bool reconfigure = c.get_bool("reconfigure");
  bool overwrite = c.get_bool("overwrite");
  bool use_cloud = c.get_bool("cloud");
  InitState st;
  if (exists && !reconfigure) {
    log::start_file_logging();
    try {
      ctx.base();
    } catch (const std::exception& e) {
      log::fatal(e.what());
    }
  } else {
    fs::remove_all(".devspace");
    log::start_file_logging();
    ctx.init_empty();
    Value& cfg = ctx.base();
    Value d = Value::map();
    d["name"] = config::kDefaultDeploymentName;
    d["helm"]["chartPath"] = "./chart";
    cfg["deployments"] = Value::seq_of({d});
    cfg["dev"]["autoReload"]["deployments"] = Value::strings({config::kDefaultDeploymentName});
  }
  Value& cfg = ctx.base();
  cfg["version"] = config::kLatestVersion;
  if (!cfg.get("images").has("default")) cfg["images"]["default"]["image"] = "devspace";

  log::get().write(log::color("\n     ____              ____\n    |  _ \\  _____   __/ ___| _ __   __ _  ___ ___\n"
                              "    | | | |/ _ \\ \\ / /\\___ \\| '_ \\ / _` |/ __/ _ \\\n"
                              "    | |_| |  __/\\ V /  ___) | |_) | (_| | (_|  __/\n"
                              "    |____/ \\___| \\_/  |____/| .__/ \\__,_|\\___\\___|   MI355X\n"
                              "                            |_|\n\n",
                              "cyan"));

  generator::ChartGenerator gen(fs::cwd(), c.get_str("templateRepoPath"));
  bool create_chart = overwrite;
  if (!overwrite) {
    if (fs::exists("chart"))
      create_chart = yes_no("Do you want to overwrite existing files in /chart?", "no");
    else
      create_chart = true;
  }
  if (create_chart) {
    log::start_wait("Detecting programming language");
    std::string detected = gen.detect_language();
    auto langs = gen.supported_languages();
    log::stop_wait();
    if (detected.empty()) detected = "none";
    if (langs.empty()) langs = {"none"};
    prompt::Params p;
    p.question = "Select programming language of project";
    p.default_value = detected;
    p.options = langs;
    p.key = "language";
    p.env = "DEVSPACE_INIT_LANGUAGE";
    st.language = prompt::ask(p);
    if (st.language == "rocm-pytorch") {
      prompt::Params g;
      // HBM is not a schedulable resource: the pod asks for devices, whole MI355X GPUs (SPX) or
      // compute partitions of them; the bound is what the largest node advertises (8 GPUs, or up
      // to 64 partitions in CPX mode), 8 when the nodes cannot be listed.
      auto nodes = discover_gpu_nodes();
      const gpu::GpuNode* big = gpu::largest(nodes);
      int max = big != nullptr ? (int)big->gpus : 8;
      std::string on = big != nullptr ? "; largest node " + big->name + ": " + big->describe() : "";
      g.question = strfmt("How many %s devices (1-%d%s) should the container request? (Default: 1)",
                          big != nullptr ? big->resource.c_str() : "amd.com/gpu (MI355X GPU)", max, on.c_str());
      g.default_value = "1";
      g.validation_regex = gpu::range_regex(max);
      g.key = "gpus";
      g.env = "DEVSPACE_INIT_GPUS";
      st.gpus = prompt::ask(g);
      st.sizing = discover_sizing(std::atoi(st.gpus.c_str()), nodes);
    }
  }
  // Dev-mode entrypoint override: keep the container idle for sync + terminal, except for
  // GPU training pods where the hot-reload runner (the image CMD) must keep running.
  if (!exists || reconfigure) {
    if (st.language != "rocm-pytorch") {
      Value o = Value::map();
      o["name"] = "default";
      o["entrypoint"] = Value::strings({"sleep", "999999999999"});
      cfg["dev"]["overrideImages"] = Value::seq_of({o});
    }
  }

  if (reconfigure || !exists) {
    if (fs::exists(fs::join(fs::home_dir(), ".kube/config")) && use_cloud)
      use_cloud = yes_no("Do you want to use DevSpace.cloud?", "yes");
    if (!use_cloud) {
      configure_cluster_local(cfg);
    } else {
      auto providers = cloud::load_providers();
      std::string provider = cloud::kDefaultProviderName;
      if (providers.size() > 1) {
        std::vector<std::string> names;
        for (auto& kv : providers) names.push_back(kv.first);
        provider = prompt::select("Select cloud provider", names);
      }
      cfg["cluster"]["cloudProvider"] = provider;
      try {
        cloud::ensure_logged_in(provider);
      } catch (const std::exception& e) {
        log::fatal(e.what());
      }
    }
    add_default_selector(cfg);
    add_default_ports(cfg, st);
    add_default_sync(cfg, st.language);
    configure_image(ctx, use_cloud);
    try {
      ctx.save_base();
    } catch (const std::exception& e) {
      log::fatal(std::string("Config error: ") + e.what());
    }
    std::string gi = fs::join(fs::dirname(ctx.config_path), ".gitignore");
    if (!fs::exists(gi)) fs::write_file(gi, kConfigGitignore);
  }

  if (create_chart) {
    try {
      gen.create_chart(st.language, create_chart && (overwrite || fs::exists("chart")));
    } catch (const std::exception& e) {
      log::fatal(std::string("Error while creating Helm chart and Dockerfile: ") + e.what());
    }
    replace_placeholders(cfg, st);
  }

  log::done("Project successfully initialized");
  if (use_cloud)
    log::info("\nPlease run: \n- `" + log::color("devspace create space [NAME]", "white+b") +
              "` to create a new space\n- `" + log::color("devspace use space [NAME]", "white+b") +
              "` to use an existing space");
  else
    log::info("Run:\n- `" + log::color("devspace dev", "white+b") + "` to develop application\n- `" +
              log::color("devspace deploy", "white+b") + "` to deploy application");
  return 0;
}

}  // namespace

void register_init(cli::Command& root) {
  auto c = std::make_unique<cli::Command>(
      "init", "Initializes your DevSpace",
      "\n#######################################################\n#################### devspace init "
      "####################\n#######################################################\nGets your project ready to "
      "start a DevSpaces.\nCreates the following files and "
      "directories:\n\nYOUR_PROJECT_PATH/\n|\n|-- Dockerfile\n|\n|-- chart/\n|   |-- Chart.yaml\n|   |-- "
      "values.yaml\n|   |-- templates/\n|\n|-- .devspace/\n|   |-- .gitignore\n|   |-- generated.yaml\n|   |-- "
      "config.yaml\n\nLanguages: none, javascript, python, go, java, php, ruby and rocm-pytorch\n(PyTorch on AMD "
      "Instinct MI355X with amd.com/gpu requests and a\nhot-reload training runner).\n"
      "#######################################################");
  c->max_args = 0;
  c->boolean("reconfigure", "r", false, "Change existing configuration")
      .boolean("overwrite", "o", false, "Overwrite existing chart files and Dockerfile")
      .str("templateRepoUrl", "", "", "Git repository for chart templates (embedded templates when empty)")
      .str("templateRepoPath", "", "", "Local path of a chart template repository (embedded templates when empty)")
      .boolean("cloud", "", false, "Use a DevSpace cloud provider for this project")
      // every question has an answer on the command line (CI, DEVSPACE_NONINTERACTIVE=1)
      .str("language", "", "", "Programming language of the project (skips the question)")
      .str("gpus", "", "", "GPU devices the container requests, rocm-pytorch only (skips the question)")
      .str("namespace", "", "", "Namespace the app runs in (skips the question)")
      .str("port", "", "", "Port the app listens on (skips the question)")
      .str("registry", "", "", "Registry to push to: hub.docker.com or a URL (skips the question)")
      .str("image", "", "", "Image name to push to; no Docker Hub account needed (skips the question)")
      .str("pullSecret", "", "", "Create a pull secret for the image: yes | no (skips the question)");
  c->run = [](cli::Command& cc, const std::vector<std::string>& a) {
    std::string url = cc.get_str("templateRepoUrl");
    if (!url.empty() && cc.get_str("templateRepoPath").empty()) {
      // Clone the repository into a temp dir (generator.go:129); requires git + network.
      std::string dir = fs::make_temp_dir("devspace-templates-");
      RunResult r = run({"git", "clone", "--depth", "1", url, dir}, "", {}, 120000);
      if (r.code != 0) log::fatal("Error cloning template repository " + url + ": " + r.err);
      cc.flag("templateRepoPath")->s = dir;
    }
    for (const char* k : {"language", "gpus", "namespace", "port", "registry", "image", "pullSecret"})
      if (cc.flag(k)->changed || !cc.get_str(k).empty()) prompt::set_answer(k, cc.get_str(k));
    return run_init(cc, a);
  };
  root.add(std::move(c));
}

}  // namespace cmd
}  // namespace ds

#include "build/image.h"

#include <poll.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <mutex>
#include <regex>
#include <set>
#include <thread>

#include "core/codec.h"
#include "core/fs.h"
#include "core/log.h"
#include "core/match.h"
#include "core/proc.h"
#include "core/safe_regex.h"
#include "core/strutil.h"
#include "core/trace.h"
#include "generator/generator.h"
#include "sync/sync.h"

namespace ds {
namespace build {

// the reference's executor (pkg/devspace/builder/kaniko/kaniko.go:120); images.*.build.kaniko.image
// or DEVSPACE_KANIKO_IMAGE choose another
static const char* const kKanikoImage = "gcr.io/kaniko-project/executor:debug-5ac29a97734170a0547fea33b348dc7c328e2f8a";
static const char* const kDefaultEmail = "noreply@devspace.cloud";

static void write_out(const std::string& s) { log::get().write(s); }

// ------------------------------------------------------------------------------ pull secrets

static std::mutex g_secrets_mu;
static std::vector<std::string> g_secret_names;

std::vector<std::string> pull_secret_names() {
  std::lock_guard<std::mutex> g(g_secrets_mu);
  return g_secret_names;
}

void create_pull_secret(kube::Client& k, const std::string& ns, const std::string& registry,
                        const std::string& username, const std::string& password_or_token, const std::string& email) {
  std::string name = pull_secret_name(registry);
  std::string url = registry.empty() || registry == "hub.docker.com" ? kDefaultIndexServer : registry;
  std::string token = username.empty() ? password_or_token : username + ":" + password_or_token;
  Value cfgjson = Value::map();
  Value& entry = cfgjson["auths"][url];
  entry["auth"] = base64_encode(token);
  entry["email"] = email;
  Value secret = Value::map();
  secret["apiVersion"] = "v1";
  secret["kind"] = "Secret";
  secret["metadata"]["name"] = name;
  secret["type"] = "kubernetes.io/dockerconfigjson";
  secret["data"][".dockerconfigjson"] = base64_encode(json_dump(cfgjson));
  std::string base = "/api/v1/namespaces/" + ns + "/secrets";
  if (!k.try_get(base + "/" + name)) {
    try {
      k.post(base, secret);
    } catch (const std::exception& e) {
      throw std::runtime_error(std::string("Unable to create image pull secret: ") + e.what());
    }
    log::donef("Created image pull secret %s/%s", ns.c_str(), name.c_str());
  } else {
    try {
      k.put(base + "/" + name, secret);
    } catch (const std::exception& e) {
      throw std::runtime_error(std::string("Unable to update image pull secret: ") + e.what());
    }
  }
  std::lock_guard<std::mutex> g(g_secrets_mu);
  if (std::find(g_secret_names.begin(), g_secret_names.end(), name) == g_secret_names.end())
    g_secret_names.push_back(name);
}

void init_registries(const Value& cfg, std::shared_ptr<kube::Client> kube, const std::string& default_ns) {
  for (auto& e : cfg.get("images").entries()) {
    const Value& ic = e.second;
    if (!ic.get("createPullSecret").as_bool(false)) continue;
    std::string registry = registry_from_image(ic.get("image").as_string());
    log::start_wait("Creating image pull secret for registry: " + registry);
    try {
      std::string user, pw;
      try {
        AuthConfig a = DockerClient::from_env(false, false)->auth_config(registry, true);
        user = a.username;
        pw = a.password;
      } catch (const std::exception&) {
      }
      if (cfg.get("deployments").size() > 0 && !user.empty() && !pw.empty()) {
        for (auto& d : cfg.get("deployments").items()) {
          std::string ns = d.get("namespace").as_string();
          create_pull_secret(*kube, ns.empty() ? default_ns : ns, registry, user, pw, kDefaultEmail);
        }
      }
    } catch (const std::exception& ex) {
      log::stop_wait();
      throw std::runtime_error(std::string("Failed to create pull secret for registry: ") + ex.what());
    }
    log::stop_wait();
  }
}

std::string image_with_tag(config::Generated& gen, const Value& image_conf, bool is_dev) {
  std::string image = image_conf.get("image").as_string();
  std::string tag = image_conf.get("tag").as_string();
  if (!tag.empty()) return image + ":" + tag;
  const Value& tags = gen.cache(is_dev).get("imageTags");
  if (!tags.has(image)) throw std::runtime_error("Couldn't find image tag in generated.yaml. Did the build succeed?");
  return image + ":" + tags.get(image).as_string();
}

// ------------------------------------------------------------------------------ kaniko output

std::pair<std::string, std::string> format_kaniko_line(const std::string& line) {
  static const std::regex logrus(R"re(^time="(.*)" level=(.*) msg="(.*)"$)re");
  static const std::regex klog(R"(^(INFO|WARN|ERRO|DEBU|FATA)\[\d+\] (.*)$)");
  static const std::vector<std::pair<std::regex, std::string>> formats = {
      {std::regex(R"re(^(?:Downloading base image|Retrieving image manifest) (.*)$)re"), " FROM $1"},
      {std::regex(R"re(^(Unpacking layer: \d+)$)re"), ">> $1"},
      {std::regex(R"re(^cmd: Add \[(.*)\]$)re"), " ADD $1"},
      {std::regex(R"re(^cmd: copy \[(.*)\]$)re"), " COPY $1"},
      {std::regex(R"re(^dest: (.*)$)re"), ">> destination: $1"},
      {std::regex(R"re(^args: \[-c (.*)\]$)re"), " RUN $1"},
      {std::regex(R"re(^Replacing CMD in config with \[(.*)\]$)re"), " CMD $1"},
      {std::regex(R"re(^Changed working directory to (.*)$)re"), " WORKDIR $1"},
      {std::regex(R"re(^Taking snapshot of full filesystem\.\.\.$)re"), " Packaging layers"},
      {std::regex(R"re(^Step \d+/\d+ : (.*)$)re"), " $1"},
      {std::regex(R"re(^(Pushed image to .*)$)re"), " $1"},
  };
  std::smatch m;
  std::string msg;
  bool is_log = false;
  if (safe_regex_match(line, &m, logrus)) {
    msg = m[3];
    is_log = true;
  } else if (safe_regex_match(line, &m, klog)) {
    msg = m[2];
    is_log = true;
  } else {
    msg = line;
  }
  for (auto& f : formats) {
    if (safe_regex_match(msg, f.first)) return {"done", safe_regex_replace(msg, f.first, f.second)};
  }
  if (!is_log) return {"info", ">> " + line};
  return {"", msg};
}

// ------------------------------------------------------------------------------ builders

namespace {

// A project whose Dockerfile runs the workload kit (`python -m devspace_amd.runner`, the
// rocm-pytorch template) but whose context lacks devspace_amd/ — a clean clone of
// examples/rocm-pytorch, where the checkout's build writes the kit (git-ignored), or a project
// whose kit copy was deleted — gets the kit this binary ships (the files `devspace init`
// vendors) added to its build context, with a notice. A copy in the project always wins.
std::vector<std::pair<std::string, std::string>> missing_workload_kit(const std::string& ctx,
                                                                      const std::string& dockerfile_text) {
  std::vector<std::pair<std::string, std::string>> out;
  if (dockerfile_text.find("devspace_amd") == std::string::npos) return out;
  if (fs::exists(fs::join(ctx, "devspace_amd/runner.py"))) return out;
  const std::string prefix = "rocm-pytorch/";
  for (auto& kv : generator::embedded_templates())
    if (starts_with(kv.first, prefix + "devspace_amd/")) out.emplace_back(kv.first.substr(prefix.size()), kv.second);
  if (!out.empty())
    log::info("[image] " + ctx + " has no devspace_amd/ (the workload kit its Dockerfile runs): adding the kit "
              "this devspace ships to the build context (`devspace init` vendors the same files)");
  return out;
}

class DockerBuilder : public Builder {
 public:
  DockerBuilder(std::unique_ptr<DockerClient> c, ImageBuildSettings s) : c_(std::move(c)), s_(std::move(s)) {}
  std::string engine() const override { return "docker"; }
  std::string url() const { return s_.image + ":" + s_.tag; }

  void authenticate() override {
    auth_ = c_->login(registry_from_image(url()), "", "", true, false, false);
    authed_ = true;
  }

  void build_image(const std::string& ctx, const std::string& dockerfile,
                   const std::vector<std::string>& entrypoint) override {
    std::string rel = fs::relative(ctx, dockerfile);
    bool outside = rel == dockerfile || starts_with(rel, "../") || rel.empty();
    std::vector<std::string> excludes = context_excludes(ctx, outside ? "" : rel);
    std::optional<std::string> override_df;
    if (!entrypoint.empty()) override_df = dockerfile_with_entrypoint(fs::read_file(dockerfile), entrypoint);
    auto kit = missing_workload_kit(ctx, fs::read_file(dockerfile));
    if (outside) {
      // build.AddDockerfileToBuildContext: ship it under a random name next to the context
      rel = ".dockerfile." + hex_encode(random_string(10)).substr(0, 20);
      if (!override_df) override_df = fs::read_file(dockerfile);
    }
    BuildRequest req;
    req.tag = url();
    req.dockerfile = rel;
    req.build_args = s_.build_args;
    req.target = s_.target;
    req.network_mode = s_.network;
    try {
      req.auth_configs = DockerConfigFile::load().all();
    } catch (const std::exception&) {
    }
    // the context tar streams to the daemon while the tree is walked (bounded memory)
    c_->build_stream([&](const Sink& sink) { return write_context_tar(sink, ctx, excludes, rel, override_df, kit); },
                     req, write_out);
  }

  void push_image() override {
    if (!authed_) authenticate();
    c_->push(url(), auth_, write_out);
  }

 private:
  std::unique_ptr<DockerClient> c_;
  ImageBuildSettings s_;
  AuthConfig auth_;
  bool authed_ = false;
};

// Reads an exec session's stdout + stderr line by line until both reach EOF.
void pump_lines(kube::ExecSession& s, const std::function<void(const std::string&)>& on_line) {
  int fds[2] = {s.out(), s.err()};
  std::string buf[2];
  bool open[2] = {fds[0] >= 0, fds[1] >= 0};
  char tmp[8192];
  while (open[0] || open[1]) {
    struct pollfd p[2];
    int n = 0, map[2];
    for (int i = 0; i < 2; ++i)
      if (open[i]) {
        p[n] = {fds[i], POLLIN, 0};
        map[n++] = i;
      }
    if (::poll(p, n, 500) < 0 && errno != EINTR) break;
    for (int j = 0; j < n; ++j) {
      if (!(p[j].revents & (POLLIN | POLLHUP | POLLERR))) continue;
      int i = map[j];
      ssize_t r = ::read(fds[i], tmp, sizeof(tmp));
      if (r <= 0) {
        open[i] = false;
        if (!buf[i].empty()) on_line(buf[i]);
        buf[i].clear();
        continue;
      }
      buf[i].append(tmp, (size_t)r);
      size_t nl;
      while ((nl = buf[i].find('\n')) != std::string::npos) {
        on_line(trim_right(buf[i].substr(0, nl), "\r"));
        buf[i].erase(0, nl + 1);
      }
    }
  }
}

class KanikoBuilder : public Builder {
 public:
  KanikoBuilder(std::shared_ptr<kube::Client> k, ImageBuildSettings s, BuildOptions o)
      : k_(std::move(k)), s_(std::move(s)), o_(std::move(o)) {}
  std::string engine() const override { return "kaniko"; }
  std::string url() const { return s_.image + ":" + s_.tag; }

  // builder/kaniko/kaniko.go:53 — the build pod gets the local docker credentials as a secret.
  void authenticate() override {
    if (!s_.kaniko_pull_secret.empty()) return;
    std::string registry = registry_from_image(url());
    AuthConfig a;
    try {
      a = DockerClient::from_env(false, false)->auth_config(registry, true);
    } catch (const std::exception&) {
    }
    std::string password = a.password.empty() ? a.identity_token : a.password;
    create_pull_secret(*k_, s_.kaniko_namespace, registry, a.username, password,
                       a.email.empty() ? kDefaultEmail : a.email);
  }

  void build_image(const std::string& ctx, const std::string& dockerfile_in,
                   const std::vector<std::string>& entrypoint) override {
    std::string dockerfile = dockerfile_in, tmpdir;
    if (!entrypoint.empty()) {
      tmpdir = fs::make_temp_dir("devspace-dockerfile-");
      dockerfile = fs::join(tmpdir, fs::basename(dockerfile_in));
      fs::write_file(dockerfile, dockerfile_with_entrypoint(fs::read_file(dockerfile_in), entrypoint));
    }
    struct TmpGuard {
      std::string d;
      ~TmpGuard() {
        if (!d.empty()) fs::remove_all(d);
      }
    } tmp_guard{tmpdir};

    std::string registry = registry_from_image(url());
    std::string secret = s_.kaniko_pull_secret.empty() ? pull_secret_name(registry) : s_.kaniko_pull_secret;
    std::string ns = s_.kaniko_namespace;
    Value pod = Value::map();
    pod["apiVersion"] = "v1";
    pod["kind"] = "Pod";
    pod["metadata"]["generateName"] = "devspace-build-";
    pod["metadata"]["labels"]["devspace-build-id"] = random_lower_alnum(12);
    Value c = Value::map();
    c["name"] = "kaniko";
    c["image"] = s_.kaniko_image.empty() ? std::string(kKanikoImage) : s_.kaniko_image;
    c["imagePullPolicy"] = "IfNotPresent";
    c["command"] = Value::strings({"/busybox/sleep"});
    c["args"] = Value::strings({"36000"});
    Value vm = Value::map();
    vm["name"] = secret;
    vm["mountPath"] = "/root/.docker";
    c["volumeMounts"].push(vm);
    pod["spec"]["containers"].push(c);
    Value vol = Value::map();
    vol["name"] = secret;
    vol["secret"]["secretName"] = secret;
    Value item = Value::map();
    item["key"] = ".dockerconfigjson";
    item["path"] = "config.json";
    vol["secret"]["items"].push(item);
    pod["spec"]["volumes"].push(vol);
    pod["spec"]["restartPolicy"] = "OnFailure";

    std::string base = "/api/v1/namespaces/" + ns + "/pods";
    Value created;
    try {
      created = k_->post(base, pod);
    } catch (const std::exception& e) {
      throw std::runtime_error(std::string("Unable to create build pod: ") + e.what());
    }
    std::string name = created.at_path("metadata.name").as_string();
    // deleteBuildPod runs on every exit path (the reference: interrupt handler + Close)
    struct PodGuard {
      kube::Client& k;
      std::string path;
      ~PodGuard() {
        try {
          Value opts = Value::map();
          opts["gracePeriodSeconds"] = 3;
          k.del(path, opts);
        } catch (const std::exception& e) {
          log::error(std::string("Failed to delete build pod: ") + e.what());
        }
      }
    } pod_guard{*k_, base + "/" + name};

    log::start_wait("Waiting for kaniko build pod to start");
    bool ready = false;
    auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(120);
    while (std::chrono::steady_clock::now() < deadline) {
      if (o_.interrupted && o_.interrupted()) {
        log::stop_wait();
        throw std::runtime_error("interrupted");
      }
      try {
        created = k_->get(base + "/" + name);
        const Value& cs = created.at_path("status.containerStatuses");
        if (cs.size() > 0 && cs[0].get("ready").as_bool()) {
          ready = true;
          break;
        }
        std::string st = kube::pod_status(created);
        if (kube::pod_status_is_fatal(st)) {
          log::stop_wait();
          throw std::runtime_error("Unable to start build pod: pod status " + st);
        }
      } catch (const kube::ApiError&) {
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(100));
    }
    log::stop_wait();
    if (!ready) throw std::runtime_error("Unable to start build pod");
    log::done("Kaniko build pod started (" + c["image"].as_string() + ")");

    std::vector<std::string> ignore = collect_dockerignore_rules(ctx);
    log::start_wait("Uploading files to build container");
    try {
      auto t = std::make_shared<kube::ExecTransport>(k_, created, "kaniko");
      sync::Session::copy_to_container(t, ctx, "/src", ignore);
      sync::Session::copy_to_container(t, dockerfile, "/src", ignore);
      auto kit = missing_workload_kit(ctx, fs::read_file(dockerfile));
      if (!kit.empty()) {
        std::string tmp = fs::make_temp_dir("devspace-kit-");
        for (auto& f : kit) {
          fs::mkdirs(fs::dirname(fs::join(tmp, f.first)));
          fs::write_file(fs::join(tmp, f.first), f.second);
        }
        try {
          sync::Session::copy_to_container(t, tmp, "/src", {});
        } catch (...) {
          fs::remove_all(tmp);
          throw;
        }
        fs::remove_all(tmp);
      }
    } catch (const std::exception& e) {
      log::stop_wait();
      throw std::runtime_error(std::string("Error uploading files to container: ") + e.what());
    }
    log::stop_wait();
    log::done("Uploaded files to container");

    log::start_wait("Building container image");
    std::vector<std::string> cmd = {"/kaniko/executor", "--dockerfile=/src/" + fs::basename(dockerfile),
                                    "--context=dir:///src", "--destination=" + url(), "--single-snapshot"};
    for (auto& kv : s_.build_args) {
      cmd.push_back("--build-arg");
      cmd.push_back(kv.first + "=" + kv.second);
    }
    if (!s_.target.empty()) cmd.push_back("--target=" + s_.target);
    if (!s_.no_cache) {
      // layer cache next to the image (the reference passes the previous tag, which kaniko
      // would read as a repository name)
      cmd.push_back("--cache=true");
      cmd.push_back("--cache-repo=" + s_.image + "-cache");
    }
    if (s_.insecure) {
      cmd.push_back("--insecure");
      cmd.push_back("--skip-tls-verify");
    }
    std::string last;
    int code = -1;
    {
      auto sess = k_->exec(ns, name, "kaniko", cmd, false, false);
      pump_lines(*sess, [&](const std::string& line) {
        if (trim(line).empty()) return;
        auto f = format_kaniko_line(line);
        if (f.first == "done")
          log::done("build >" + f.second);
        else if (f.first == "info")
          log::info("build >" + f.second);
        last = f.first.empty() ? f.second : line;
      });
      code = sess->wait(60000);
      if (code != 0 && !sess->error_message().empty() && last.empty()) last = sess->error_message();
    }
    log::stop_wait();
    if (code != 0)
      throw std::runtime_error("Error: command terminated with exit code " + std::to_string(code) +
                               ", Last Kaniko Output: " + last);
    log::done("Done building image");
  }

  void push_image() override {}  // kaniko pushes as part of the build

 private:
  std::shared_ptr<kube::Client> k_;
  ImageBuildSettings s_;
  BuildOptions o_;
};

}  // namespace

std::unique_ptr<Builder> create_builder(const Value& cfg, const Value& ic, const ImageBuildSettings& s_in,
                                        std::shared_ptr<kube::Client> kube, const BuildOptions& o) {
  ImageBuildSettings s = s_in;
  const Value& kan = ic.at_path("build.kaniko");
  if (kan.is_map()) {
    if (!kube) throw std::runtime_error("Error creating kaniko builder: no kubernetes client");
    s.kaniko_namespace = kan.get("namespace").as_string();
    if (s.kaniko_namespace.empty()) s.kaniko_namespace = config::default_namespace(cfg);
    s.kaniko_pull_secret = kan.get("pullSecret").as_string();
    s.kaniko_image = kan.get("image").as_string();
    if (const char* e = getenv("DEVSPACE_KANIKO_IMAGE"); e && *e && s.kaniko_image.empty()) s.kaniko_image = e;
    if (!s.kaniko_image.empty()) {
      std::string why = image_reference_problem(s.kaniko_image);
      if (!why.empty()) throw std::runtime_error("invalid kaniko image \"" + s.kaniko_image + "\": " + why);
      if (!contains(split_image_tag(s.kaniko_image).second, "debug"))
        log::warn("kaniko image " + s.kaniko_image +
                  " is not a debug build: devspace runs the build by exec and needs its /busybox shell");
    }
    s.no_cache = kan.has("cache") && !kan.get("cache").as_bool(true);
    return std::make_unique<KanikoBuilder>(kube, s, o);
  }
  bool prefer_minikube = ic.at_path("build.docker.preferMinikube").as_bool(true);
  std::unique_ptr<DockerClient> c;
  try {
    c = DockerClient::from_env(prefer_minikube, kube && kube->is_minikube());
  } catch (const std::exception& e) {
    throw std::runtime_error(std::string("Error creating docker client: ") + e.what());
  }
  return std::make_unique<DockerBuilder>(std::move(c), s);
}

// ------------------------------------------------------------------------------ orchestration

// Guards the shared generated.yaml cache when several images build at once.
static std::mutex& gen_mu() {
  static std::mutex m;
  return m;
}

static std::string context_cache_path(const std::string& abs_ctx) {
  return fs::join(".devspace", "cache", "context-" + sha256_hex(abs_ctx).substr(0, 16) + ".json");
}

bool should_rebuild(config::Generated& gen, const Value& ic, const std::string& context_path,
                    const std::string& dockerfile_path, bool force, bool is_dev) {
  fs::StatInfo st = fs::stat(dockerfile_path);
  if (!st.exists) throw std::runtime_error("Dockerfile " + dockerfile_path + " missing: no such file or directory");
  std::string abs_ctx = fs::abs_path(context_path);
  std::string rel = fs::relative(abs_ctx, fs::abs_path(dockerfile_path));
  if (starts_with(rel, "/")) rel.clear();
  std::vector<std::string> excludes = context_excludes(abs_ctx, rel);
  excludes.push_back(".devspace/");
  std::string hash;
  {
    trace::Span span("image.context_hash", {{"context", context_path}});
    hash = hash_directory_excludes(abs_ctx, excludes, context_cache_path(abs_ctx));
  }
  std::lock_guard<std::mutex> g(gen_mu());  // images build concurrently (build_all)
  Value& cache = gen.cache(is_dev);
  bool must = true;
  if (!force)
    must = cache.get("dockerfileTimestamps").get(dockerfile_path).as_int(-1) != st.mtime_sec ||
           cache.get("dockerContextPaths").get(context_path).as_string() != hash;
  cache["dockerfileTimestamps"][dockerfile_path] = Value((int64_t)st.mtime_sec);
  cache["dockerContextPaths"][context_path] = Value(hash);
  if (!cache.get("imageTags").has(ic.get("image").as_string())) return true;
  return must;
}

bool build_image(const Value& cfg, config::Generated& gen, const std::string& name, const Value& ic,
                 std::shared_ptr<kube::Client> kube, const BuildOptions& o) {
  std::string dockerfile = "./Dockerfile", context = "./";
  std::string image = ic.get("image").as_string();
  if (!ic.at_path("build.dockerfilePath").as_string().empty()) dockerfile = ic.at_path("build.dockerfilePath").as_string();
  if (!ic.at_path("build.contextPath").as_string().empty()) context = ic.at_path("build.contextPath").as_string();

  bool need;
  try {
    need = should_rebuild(gen, ic, context, dockerfile, o.force_rebuild, o.is_dev);
  } catch (const std::exception& e) {
    throw std::runtime_error(std::string("Error during shouldRebuild check: ") + e.what());
  }
  if (!need) {
    log::info("Skip building image '" + name + "'");
    return false;
  }
  std::string abs_df = fs::abs_path(dockerfile), abs_ctx = fs::abs_path(context);

  ImageBuildSettings s;
  s.image = image;
  s.tag = ic.get("tag").as_string().empty() ? random_string(7) : ic.get("tag").as_string();
  {
    std::lock_guard<std::mutex> g(gen_mu());
    s.last_tag = gen.cache(o.is_dev).get("imageTags").get(image).as_string();
  }
  for (auto& kv : ic.at_path("build.options.buildArgs").entries()) s.build_args[kv.first] = kv.second.as_string();
  s.target = ic.at_path("build.options.target").as_string();
  if (!o.docker_target.empty()) s.target = o.docker_target;
  s.network = ic.at_path("build.options.network").as_string();
  s.insecure = ic.get("insecure").as_bool(false);
  std::unique_ptr<Builder> b = create_builder(cfg, ic, s, kube, o);
  log::info("Building image '" + image + "' with engine '" + b->engine() + "'");

  std::string registry = registry_from_image(image);
  std::string display = registry.empty() ? "hub.docker.com" : registry;
  bool skip_push = ic.get("skipPush").as_bool(false);
  if (!skip_push) {
    log::start_wait("Authenticating (" + display + ")");
    try {
      b->authenticate();
    } catch (const std::exception& e) {
      log::stop_wait();
      throw std::runtime_error(std::string("Error during image registry authentication: ") + e.what());
    }
    log::stop_wait();
    log::done("Authentication successful (" + display + ")");
  }

  std::vector<std::string> entrypoint;
  if (o.is_dev) {
    for (auto& ov : cfg.at_path("dev.overrideImages").items()) {
      if (ov.get("name").as_string() == name) {
        for (auto& x : ov.get("entrypoint").items()) entrypoint.push_back(x.as_string());
        break;
      }
    }
  }
  {
    trace::Span span("image.build", {{"image", image}, {"engine", b->engine()}});
    try {
      b->build_image(abs_ctx, abs_df, entrypoint);
    } catch (const std::exception& e) {
      throw std::runtime_error(std::string("Error during image build: ") + e.what());
    }
  }
  if (!skip_push) {
    trace::Span span("image.push", {{"image", image}});
    try {
      b->push_image();
    } catch (const std::exception& e) {
      throw std::runtime_error(std::string("Error during image push: ") + e.what());
    }
    log::info("Image pushed to registry (" + display + ")");
  } else {
    log::info("Skip image push for " + image);
  }
  {
    std::lock_guard<std::mutex> g(gen_mu());
    gen.cache(o.is_dev)["imageTags"][image] = s.tag;
  }
  log::done("Done processing image '" + image + "'");
  return true;
}

bool build_all(const Value& cfg, config::Generated& gen, std::shared_ptr<kube::Client> kube, const BuildOptions& o) {
  std::vector<const std::pair<std::string, Value>*> todo;
  for (auto& e : cfg.get("images").entries()) {
    if (e.second.at_path("build.disabled").as_bool(false)) {
      log::info("Skipping building image " + e.first);
      continue;
    }
    todo.push_back(&e);
  }
  const char* par = getenv("DEVSPACE_BUILD_PARALLEL");
  if (todo.size() <= 1 || (par && std::string(par) == "0")) {
    bool rebuilt = false;
    for (auto* e : todo)
      if (build_image(cfg, gen, e->first, e->second, kube, o)) rebuilt = true;
    return rebuilt;
  }
  // The reference builds images one after another (image/build.go); independent images build
  // and push concurrently here, so a multi-service project waits for its slowest image, not the
  // sum. The first failure is reported after every build has finished.
  std::vector<std::thread> threads;
  std::vector<std::string> errors(todo.size());
  std::atomic<bool> rebuilt{false};
  for (size_t i = 0; i < todo.size(); ++i) {
    threads.emplace_back([&, i] {
      try {
        if (build_image(cfg, gen, todo[i]->first, todo[i]->second, kube, o)) rebuilt = true;
      } catch (const std::exception& e) {
        errors[i] = e.what();
      }
    });
  }
  for (auto& t : threads) t.join();
  for (auto& e : errors)
    if (!e.empty()) throw std::runtime_error(e);
  return rebuilt.load();
}

}  // namespace build
}  // namespace ds

#include "cloud/cloud.h"

#include <arpa/inet.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstring>

#include "build/docker.h"
#include "core/codec.h"
#include "core/fs.h"
#include "core/log.h"
#include "core/net.h"
#include "core/proc.h"
#include "core/prompt.h"
#include "core/strutil.h"
#include "kube/kubeconfig.h"
#include "platform/platform.h"

namespace ds {
namespace cloud {

const char* const kDefaultProviderName = "app.devspace.cloud";
const char* const kKubeContextPrefix = "devspace";

static std::string providers_path() { return fs::join(fs::home_dir(), ".devspace/clouds.yaml"); }

std::map<std::string, Provider> load_providers() {
  std::map<std::string, Provider> out;
  std::string data;
  if (fs::read_file(providers_path(), &data)) {
    Value v = yaml_parse(data);
    for (auto& e : v.entries()) {
      Provider p;
      p.name = e.first;
      p.host = e.second.get("host").as_string();
      p.token = e.second.get("token").as_string();
      out[e.first] = p;
    }
  }
  Provider& def = out[kDefaultProviderName];
  def.name = kDefaultProviderName;
  def.host = "https://app.devspace.cloud";
  return out;
}

void save_providers(const std::map<std::string, Provider>& ps) {
  Value v = Value::map();
  for (auto& kv : ps) {
    Value e = Value::map();
    if (kv.first != kDefaultProviderName) e["host"] = kv.second.host;
    if (!kv.second.token.empty()) e["token"] = kv.second.token;
    v[kv.first] = e;
  }
  fs::write_file(providers_path(), yaml_dump(v), 0600);
}

Value Space::to_generated() const {
  Value v = Value::map();
  v["spaceID"] = id;
  v["providerName"] = provider_name;
  v["name"] = name;
  v["namespace"] = namespace_;
  v["created"] = created;
  v["serviceAccountToken"] = service_account_token;
  v["caCert"] = ca_cert;
  v["server"] = server;
  v["domain"] = domain.empty() ? Value() : Value(domain);
  return v;
}

Space Space::from_generated(const Value& v) {
  Space s;
  s.id = v.get("spaceID").as_int();
  s.provider_name = v.get("providerName").as_string();
  s.name = v.get("name").as_string();
  s.namespace_ = v.get("namespace").as_string();
  s.created = v.get("created").as_string();
  s.service_account_token = v.get("serviceAccountToken").as_string();
  s.ca_cert = v.get("caCert").as_string();
  s.server = v.get("server").as_string();
  s.domain = v.get("domain").as_string();
  return s;
}

Value Client::graphql(const std::string& query, const Value& vars) {
  net::HttpClient http(p_.host);
  net::Request r;
  r.method = "POST";
  r.path = "/graphql";
  Value body = Value::map();
  body["query"] = query;
  body["variables"] = vars.is_null() ? Value::map() : vars;
  r.body = json_dump(body);
  r.headers = {{"Content-Type", "application/json"}, {"Authorization", "Bearer " + p_.token}};
  net::Response resp = http.request(r);
  if (resp.status != 200) throw std::runtime_error("graphql request failed: " + std::to_string(resp.status) + " " + resp.body);
  Value v = json_parse(resp.body);
  if (v.get("errors").size() > 0) throw std::runtime_error(v.get("errors")[0].get("message").as_string("graphql error"));
  return v.get("data");
}

static const char* kSpaceFields = R"(
      id
      name
      kubeContextBykubeContextId {
        namespace
        service_account_token
        clusterByclusterId { ca_cert server }
        kubeContextDomainsBykubeContextId(limit:1) { url }
      }
      created_at)";

static Space parse_space(const Value& s, const std::string& provider) {
  const Value& kc = s.get("kubeContextBykubeContextId");
  if (!kc.is_map()) throw std::runtime_error("KubeContext is nil for space " + s.get("name").as_string());
  const Value& cl = kc.get("clusterByclusterId");
  if (!cl.is_map()) throw std::runtime_error("Cluster is nil for space " + s.get("name").as_string());
  Space sp;
  sp.id = s.get("id").as_int();
  sp.name = s.get("name").as_string();
  sp.namespace_ = kc.get("namespace").as_string();
  sp.service_account_token = kc.get("service_account_token").as_string();
  sp.server = cl.get("server").as_string();
  sp.ca_cert = cl.get("ca_cert").as_string();
  sp.created = s.get("created_at").as_string();
  sp.provider_name = provider;
  const Value& d = kc.get("kubeContextDomainsBykubeContextId");
  if (d.size() > 0) sp.domain = d[0].get("url").as_string();
  return sp;
}

std::vector<Space> Client::spaces() {
  Value d = graphql(std::string("query { space {") + kSpaceFields + " } }");
  if (!d.get("space").is_seq()) throw std::runtime_error("Wrong answer from graphql server: Spaces is nil");
  std::vector<Space> out;
  for (auto& s : d.get("space").items()) out.push_back(parse_space(s, p_.name));
  return out;
}

Space Client::space(int64_t id) {
  Value vars = Value::map();
  vars["ID"] = id;
  Value d = graphql(std::string("query($ID:Int!) { space_by_pk(id:$ID) {") + kSpaceFields + " } }", vars);
  if (!d.get("space_by_pk").is_map()) throw std::runtime_error("Space " + std::to_string(id) + " not found");
  return parse_space(d.get("space_by_pk"), p_.name);
}

Space Client::space_by_name(const std::string& name) {
  Value vars = Value::map();
  vars["name"] = name;
  Value d = graphql(std::string("query($name:String!) { space(where:{name:{_eq:$name}}) {") + kSpaceFields + " } }", vars);
  if (d.get("space").size() == 0) throw std::runtime_error("Space " + name + " not found");
  return parse_space(d.get("space")[0], p_.name);
}

int64_t Client::create_space(const std::string& name, int64_t project_id, int64_t cluster_id) {
  Value vars = Value::map();
  vars["spaceName"] = name;
  vars["projectID"] = project_id;
  vars["clusterID"] = cluster_id ? Value(cluster_id) : Value();
  Value d = graphql(
      "mutation($spaceName: String!, $clusterID: Int, $projectID: Int!) { manager_createSpace(spaceName: $spaceName, "
      "clusterID: $clusterID, projectID: $projectID) { SpaceID } }",
      vars);
  return d.at_path("manager_createSpace.SpaceID").as_int();
}

int64_t Client::create_project(const std::string& name, int64_t cluster_id) {
  Value vars = Value::map();
  vars["projectName"] = name;
  vars["clusterID"] = cluster_id;
  Value d = graphql(
      "mutation($clusterID: Int!, $projectName: String!) { manager_createProject(clusterID: $clusterID, projectName: "
      "$projectName) { ProjectID } }",
      vars);
  return d.at_path("manager_createProject.ProjectID").as_int();
}

std::vector<std::pair<int64_t, std::string>> Client::projects() {
  Value d = graphql("query { project { id name } }");
  std::vector<std::pair<int64_t, std::string>> out;
  for (auto& p : d.get("project").items()) out.emplace_back(p.get("id").as_int(), p.get("name").as_string());
  return out;
}

std::vector<std::pair<int64_t, std::string>> Client::clusters() {
  Value d = graphql("query { cluster { id name } }");
  std::vector<std::pair<int64_t, std::string>> out;
  for (auto& c : d.get("cluster").items()) out.emplace_back(c.get("id").as_int(), c.get("name").as_string());
  return out;
}

void Client::delete_space(int64_t id) {
  Value vars = Value::map();
  vars["spaceID"] = id;
  graphql("mutation($spaceID: Int!) { manager_deleteSpace(spaceID: $spaceID) }", vars);
}

std::vector<std::string> Client::registries() {
  Value d = graphql("query { image_registry { url } }");
  std::vector<std::string> out;
  for (auto& r : d.get("image_registry").items()) out.push_back(r.get("url").as_string());
  return out;
}

std::string Client::login_via_browser(int timeout_s) {
  int fd = plat::socket_cloexec(AF_INET, SOCK_STREAM);
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  struct sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(25853);
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  if (::bind(fd, (struct sockaddr*)&a, sizeof(a)) != 0 || ::listen(fd, 4) != 0) {
    ::close(fd);
    throw std::runtime_error("cannot listen on :25853 for the login callback");
  }
  std::string url = p_.host + "/login?cli=true";
  for (const char* opener : {"xdg-open", "open"})
    if (!which(opener).empty()) {
      ProcOptions o;
      o.pipe_stdout = o.pipe_stderr = false;
      Process pr;
      pr.start({opener, url}, o);
      break;
    }
  log::info("Please open " + url + " in your browser to log in");
  auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(timeout_s);
  std::string token;
  while (token.empty() && std::chrono::steady_clock::now() < deadline) {
    struct pollfd pf{fd, POLLIN, 0};
    if (::poll(&pf, 1, 500) <= 0) continue;
    int c = ::accept(fd, nullptr, nullptr);
    if (c < 0) continue;
    char buf[8192];
    struct pollfd cp{c, POLLIN, 0};
    ssize_t n = ::poll(&cp, 1, 2000) > 0 ? ::recv(c, buf, sizeof(buf) - 1, 0) : 0;  // a silent client cannot stall login
    std::string req(buf, n > 0 ? (size_t)n : 0);
    size_t p = req.find("/token?token=");
    if (p != std::string::npos) {
      size_t e = req.find_first_of(" &\r\n", p + 13);
      token = req.substr(p + 13, e - p - 13);
      std::string resp = "HTTP/1.1 303 See Other\r\nLocation: " + p_.host + "/login-success\r\nContent-Length: 0\r\n\r\n";
      write_all(c, resp);
    } else {
      write_all(c, std::string("HTTP/1.1 400 Bad Request\r\nContent-Length: 0\r\n\r\n"));
    }
    ::close(c);
  }
  ::close(fd);
  if (token.empty()) throw std::runtime_error("login timed out");
  return token;
}

Provider ensure_logged_in(const std::string& name) {
  auto ps = load_providers();
  auto it = ps.find(name);
  if (it == ps.end())
    throw std::runtime_error("Cloud provider not found! Did you run `devspace add provider [url]`? Existing cloud providers: " +
                             [&] {
                               std::vector<std::string> n;
                               for (auto& kv : ps) n.push_back(kv.first);
                               return join(n, ", ");
                             }());
  if (it->second.token.empty()) return login(name, "");
  return it->second;
}

Provider login(const std::string& name, const std::string& token) {
  auto ps = load_providers();
  auto it = ps.find(name);
  if (it == ps.end()) throw std::runtime_error("Cloud provider " + name + " not found");
  if (token.empty() && !prompt::interactive())
    // the browser flow waits for a callback on localhost:25853: nothing will ever call it in
    // a CI job or a piped session (the reference waits forever there)
    throw std::runtime_error("Not logged in to " + name + " and this session is not interactive: run `devspace login --provider " +
                             name + " --token <token>` first");
  it->second.token = token.empty() ? Client(it->second).login_via_browser() : token;
  save_providers(ps);
  // cloud/registry.go:27 LoginIntoRegistries: docker credentials for every provider registry
  try {
    Client c(it->second);
    build::DockerConfigFile dcf = build::DockerConfigFile::load();
    for (auto& reg : c.registries()) {
      build::AuthConfig a;
      a.server_address = reg;
      a.username = token_account(it->second.token);
      a.password = it->second.token;
      a.auth = base64_encode(a.username + ":" + a.password);
      dcf.store(a);
    }
    dcf.save();
  } catch (const std::exception& e) {
    log::warn(std::string("Error logging into docker registries: ") + e.what());
  }
  return it->second;
}

std::string kube_context_for(const Space& s) { return std::string(kKubeContextPrefix) + "-" + to_lower(s.name); }

void update_kube_config(const std::string& context, const Space& s, bool set_active) {
  kube::KubeConfig kc = kube::KubeConfig::load();
  kc.set_cluster(context, s.server, s.ca_cert, false);
  kc.set_user_token(context, s.service_account_token);
  kc.set_context(context, context, context, s.namespace_);
  if (set_active) kc.set_current_context(context);
  kc.save();
}

void delete_kube_context(const Space& s) {
  kube::KubeConfig kc = kube::KubeConfig::load();
  kc.delete_context(kube_context_for(s));
  kc.save();
}

std::string token_account(const std::string& jwt) {
  auto parts = split(jwt, ".");
  if (parts.size() != 3) throw std::runtime_error("token is not a valid JWT");
  Value claims = json_parse(base64_decode(parts[1]));
  return claims.get("sub").as_string();
}

void configure(config::Context& ctx, const std::string& space_name) {
  Value& cfg = ctx.mutable_config();
  std::string provider = cfg.at_path("cluster.cloudProvider").as_string();
  if (provider.empty()) return;
  Provider p = ensure_logged_in(provider);
  Client c(p);
  Space s;
  config::Generated& gen = ctx.generated();
  if (!space_name.empty()) {
    s = c.space_by_name(space_name);
  } else {
    if (!gen.has_space())
      throw std::runtime_error(
          "No space configured\n\nPlease run: \n- `devspace create space [NAME]` to create a new space\n- `devspace use "
          "space [NAME]` to use an existing space");
    s = Space::from_generated(gen.space());
    try {
      s = c.space(s.id);
      gen.space() = s.to_generated();
    } catch (const std::exception& e) {
      log::warn("Couldn't get space " + s.name + ": " + e.what());
    }
    ctx.save_generated();
  }
  log::info("Using space " + s.name);
  bool use_kube_context = cfg.at_path("cluster.apiServer").is_null();
  Value cl = Value::map();
  cl["cloudProvider"] = provider;
  cl["namespace"] = s.namespace_;
  if (use_kube_context) {
    std::string kctx = kube_context_for(s);
    cl["kubeContext"] = kctx;
    update_kube_config(kctx, s, false);
  } else {
    cl["apiServer"] = s.server;
    cl["caCert"] = s.ca_cert;
    cl["user"]["token"] = s.service_account_token;
  }
  cfg["cluster"] = cl;
}

}  // namespace cloud
}  // namespace ds

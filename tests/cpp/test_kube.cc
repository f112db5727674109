// Kubernetes adapter units: pod status (kubectl printer port, kubectl/client.go:224), resource
// paths, kubeconfig resolution (inline data, tokens, namespaces), analyze's GPU log matcher.
#include <zlib.h>

#include "analyze/analyze.h"
#include "core/codec.h"
#include "core/fs.h"
#include "core/strutil.h"
#include "kube/client.h"
#include "kube/kubeconfig.h"
#include "testing.h"

using namespace ds;

static std::string status_of(const std::string& yaml) { return kube::pod_status(yaml_parse(yaml)); }

TEST(pod_status_printer) {
  EXPECT_EQ(status_of("status: {phase: Running, containerStatuses: [{ready: true, state: {running: {}}}]}"),
            std::string("Running"));
  EXPECT_EQ(status_of("status: {phase: Pending, containerStatuses: [{state: {waiting: {reason: ContainerCreating}}}]}"),
            std::string("ContainerCreating"));
  EXPECT_EQ(status_of("status: {phase: Running, containerStatuses: [{state: {waiting: {reason: CrashLoopBackOff}}}]}"),
            std::string("CrashLoopBackOff"));
  EXPECT_EQ(status_of("status: {phase: Failed, containerStatuses: [{state: {terminated: {exitCode: 3}}}]}"),
            std::string("ExitCode:3"));
  EXPECT_EQ(status_of("status: {phase: Failed, containerStatuses: [{state: {terminated: {exitCode: 0, signal: 9}}}]}"),
            std::string("Signal:9"));
  EXPECT_EQ(status_of("spec: {initContainers: [{name: a}, {name: b}]}\n"
                      "status: {phase: Pending, initContainerStatuses: [{state: {terminated: {exitCode: 0}}}, "
                      "{state: {running: {}}}]}"),
            std::string("Init:1/2"));
  EXPECT_EQ(status_of("spec: {initContainers: [{name: a}]}\n"
                      "status: {phase: Pending, initContainerStatuses: [{state: {terminated: {exitCode: 2}}}]}"),
            std::string("Init:ExitCode:2"));
  EXPECT_EQ(status_of("metadata: {deletionTimestamp: '2020-01-01T00:00:00Z'}\nstatus: {phase: Running}"),
            std::string("Terminating"));
  EXPECT_EQ(status_of("status: {phase: Failed, reason: Evicted}"), std::string("Evicted"));
  EXPECT_TRUE(kube::pod_status_is_fatal("ImagePullBackOff"));
  EXPECT_TRUE(kube::pod_status_is_fatal("CrashLoopBackOff"));
  EXPECT_TRUE(!kube::pod_status_is_fatal("ContainerCreating"));
}

TEST(resource_paths) {
  EXPECT_EQ(kube::resource_path("v1", "Service", "ns", "web"), std::string("/api/v1/namespaces/ns/services/web"));
  EXPECT_EQ(kube::resource_path("apps/v1", "Deployment", "ns", "d"),
            std::string("/apis/apps/v1/namespaces/ns/deployments/d"));
  EXPECT_EQ(kube::resource_path("rbac.authorization.k8s.io/v1", "ClusterRoleBinding", "ns", "x"),
            std::string("/apis/rbac.authorization.k8s.io/v1/clusterrolebindings/x"));
  EXPECT_EQ(kube::plural_of("Ingress"), std::string("ingresses"));
  EXPECT_EQ(kube::plural_of("NetworkPolicy"), std::string("networkpolicies"));
  EXPECT_TRUE(kube::is_cluster_scoped("Namespace"));
  EXPECT_TRUE(!kube::is_cluster_scoped("ConfigMap"));
}

TEST(kubeconfig_resolve_inline_credentials) {
  std::string d = fs::make_temp_dir("kc-");
  std::string path = fs::join(d, "config");
  fs::write_file(path,
                 "apiVersion: v1\nkind: Config\ncurrent-context: a\nclusters:\n"
                 "- name: ca\n  cluster:\n    server: https://10.0.0.1:6443\n    certificate-authority-data: " +
                     base64_encode("CA-PEM") +
                     "\n- name: cb\n  cluster:\n    server: http://127.0.0.1:8080\n    insecure-skip-tls-verify: true\n"
                     "contexts:\n- name: a\n  context: {cluster: ca, user: ua, namespace: team-a}\n"
                     "- name: b\n  context: {cluster: cb, user: ub}\n"
                     "users:\n- name: ua\n  user:\n    client-certificate-data: " +
                     base64_encode("CERT") + "\n    client-key-data: " + base64_encode("KEY") +
                     "\n- name: ub\n  user: {token: tok-b}\n");
  kube::KubeConfig kc = kube::KubeConfig::load(path);
  EXPECT_EQ(kc.current_context(), std::string("a"));
  kube::RestConfig a = kc.resolve();
  EXPECT_EQ(a.server, std::string("https://10.0.0.1:6443"));
  EXPECT_EQ(a.ca_pem, std::string("CA-PEM"));
  EXPECT_EQ(a.client_cert_pem, std::string("CERT"));
  EXPECT_EQ(a.client_key_pem, std::string("KEY"));
  EXPECT_EQ(a.namespace_, std::string("team-a"));
  kube::RestConfig b = kc.resolve("b");
  EXPECT_EQ(b.token, std::string("tok-b"));
  EXPECT_TRUE(b.insecure);
  EXPECT_EQ(b.namespace_, std::string(""));
  EXPECT_THROWS(kc.resolve("missing"));
  fs::remove_all(d);
}

// The other ways a kubeconfig names credentials (client-go's clientcmd): a token file and
// certificate files relative to the kubeconfig's directory, the cached token of a legacy
// auth-provider (oidc id-token, else gcp access-token), basic auth, and an exec plugin whose
// relative command is resolved against the kubeconfig's directory.
TEST(kubeconfig_resolve_files_auth_providers_and_exec) {
  std::string d = fs::make_temp_dir("kc-");
  std::string path = fs::join(d, "config");
  fs::write_file(fs::join(d, "sa/token"), "tok-from-file\n");
  fs::write_file(fs::join(d, "pki/ca.crt"), "CA-FILE");
  fs::write_file(fs::join(d, "pki/me.crt"), "CERT-FILE");
  fs::write_file(fs::join(d, "pki/me.key"), "KEY-FILE");
  fs::write_file(path,
                 "apiVersion: v1\nkind: Config\ncurrent-context: files\nclusters:\n"
                 "- name: c\n  cluster:\n    server: https://k8s.example:6443\n    certificate-authority: pki/ca.crt\n"
                 "    tls-server-name: api.internal\n    proxy-url: http://proxy:3128\n"
                 "contexts:\n- name: files\n  context: {cluster: c, user: files}\n"
                 "- name: oidc\n  context: {cluster: c, user: oidc}\n"
                 "- name: gcp\n  context: {cluster: c, user: gcp}\n"
                 "- name: basic\n  context: {cluster: c, user: basic}\n"
                 "- name: plugin\n  context: {cluster: c, user: plugin}\n"
                 "users:\n"
                 "- name: files\n  user:\n    tokenFile: sa/token\n    client-certificate: pki/me.crt\n"
                 "    client-key: pki/me.key\n"
                 "- name: oidc\n  user:\n    auth-provider:\n      name: oidc\n      config: {id-token: id-tok, "
                 "refresh-token: r}\n"
                 "- name: gcp\n  user:\n    auth-provider:\n      name: gcp\n      config: {access-token: acc-tok}\n"
                 "- name: basic\n  user: {username: admin, password: pw}\n"
                 "- name: plugin\n  user:\n    exec:\n      apiVersion: client.authentication.k8s.io/v1\n"
                 "      command: bin/get-token\n      args: [--cluster, c]\n      env: [{name: REGION, value: eu}]\n"
                 "      provideClusterInfo: true\n      installHint: install get-token\n");
  kube::KubeConfig kc = kube::KubeConfig::load(path);
  kube::RestConfig f = kc.resolve();
  EXPECT_EQ(f.token, std::string("tok-from-file"));
  EXPECT_EQ(f.token_file, fs::join(d, "sa/token"));
  EXPECT_EQ(f.ca_pem, std::string("CA-FILE"));
  EXPECT_EQ(f.client_cert_pem, std::string("CERT-FILE"));
  EXPECT_EQ(f.client_key_pem, std::string("KEY-FILE"));
  EXPECT_EQ(f.tls_server_name, std::string("api.internal"));
  EXPECT_EQ(f.proxy_url, std::string("http://proxy:3128"));
  EXPECT_EQ(kc.resolve("oidc").token, std::string("id-tok"));
  EXPECT_EQ(kc.resolve("gcp").token, std::string("acc-tok"));
  kube::RestConfig b = kc.resolve("basic");
  EXPECT_TRUE(b.username == "admin" && b.password == "pw" && b.token.empty());
  kube::RestConfig p = kc.resolve("plugin");
  EXPECT_EQ(p.exec_command.size(), (size_t)3);
  EXPECT_EQ(p.exec_command[0], fs::join(d, "bin/get-token"));
  EXPECT_EQ(p.exec_command[2], std::string("c"));
  EXPECT_EQ(p.exec_env.size(), (size_t)1);
  EXPECT_TRUE(p.exec_env[0].first == "REGION" && p.exec_env[0].second == "eu");
  EXPECT_EQ(p.exec_api_version, std::string("client.authentication.k8s.io/v1"));
  EXPECT_TRUE(p.exec_provide_cluster_info);
  EXPECT_EQ(p.exec_install_hint, std::string("install get-token"));
  fs::remove_all(d);
}

TEST(analyze_gpu_runtime_log_matcher) {
  std::string m;
  EXPECT_TRUE(analyze::log_has_gpu_runtime_error("RuntimeError: No HIP GPUs are available", &m));
  EXPECT_TRUE(analyze::log_has_gpu_runtime_error("NCCL WARN NET/Socket : no socket found\nncclSystemError", &m));
  EXPECT_TRUE(analyze::log_has_gpu_runtime_error("hipErrorNoDevice", &m));
  EXPECT_TRUE(!analyze::log_has_gpu_runtime_error("Example app listening on port 3000!", &m));
  EXPECT_TRUE(analyze::log_has_gpu_runtime_error("ERROR: Unexpected bus error encountered in worker. Bus error", &m));
  // multi-GPU pods need a memory-backed /dev/shm (RCCL); the devspace chart mounts one
  Value pod = yaml_parse(
      "spec:\n  containers:\n  - name: train\n    resources: {limits: {amd.com/gpu: 8}}\n    volumeMounts: []\n");
  EXPECT_TRUE(contains(analyze::shm_problem(pod, 8), "no memory-backed /dev/shm"));
  EXPECT_EQ(analyze::shm_problem(pod, 1), std::string(""));
  Value ok = yaml_parse(
      "spec:\n  volumes: [{name: shm, emptyDir: {medium: Memory, sizeLimit: 64Gi}}]\n  containers:\n  - name: train\n"
      "    resources: {limits: {amd.com/gpu: 8}}\n    volumeMounts: [{name: shm, mountPath: /dev/shm}]\n");
  EXPECT_EQ(analyze::shm_problem(ok, 8), std::string(""));
}

// The runner's state in a pod log (devspace_amd/runner.py output): a group down after a rank
// failed, a last edit that did not load, or training (no problem).
TEST(analyze_runner_state_from_pod_log) {
  std::string up = "[devspace-runner] started gen=1 marker=v0 digest=ab code=cd world=8\n"
                   "[devspace-runner] reloaded gen=2 marker=v1 digest=ef code=01 ranks=8 step=9\n";
  EXPECT_TRUE(analyze::runner_problems(up).empty());
  std::string down = up +
                     "[devspace-runner] rank=3 step failed gen=3 marker=bad: leaving the group (the supervisor restarts it)\n"
                     "Traceback (most recent call last):\n"
                     "  File \"/app/train.py\", line 40, in step\n"
                     "ValueError: shapes (4,8) and (9,8) not aligned\n"
                     "[devspace-runner] rank=3 exited with code 3: restarting the group of 8 (1/3 since the last edit)\n"
                     "[devspace-runner] rank=3 startup failed gen=1:\n"
                     "Traceback (most recent call last):\n"
                     "ValueError: shapes (4,8) and (9,8) not aligned\n"
                     "[devspace-runner] rank=3 exited with code 3 before every rank finished a first step: waiting for a "
                     "file change before starting the group again\n";
  auto p = analyze::runner_problems(down);
  EXPECT_EQ(p.size(), (size_t)1);
  EXPECT_TRUE(contains(p[0], "training group is down after rank=3 startup failed gen=1"));
  EXPECT_TRUE(contains(p[0], "ValueError: shapes (4,8) and (9,8) not aligned"));
  EXPECT_TRUE(analyze::runner_problems(down + "[devspace-runner] started gen=1 marker=fixed world=8\n").empty());
  // a multi-rank pod's log: each rank's lines carry "[rank N] " (devspace_amd/supervise.py LogRelay)
  std::string prefixed =
      "[rank 0] [devspace-runner] started gen=1 marker=v0 world=8\n"
      "[rank 3] [devspace-runner] rank=3 startup failed gen=1:\n"
      "[rank 3] Traceback (most recent call last):\n"
      "[rank 3]   File \"/app/train.py\", line 40, in step\n"
      "[rank 3] ValueError: shapes (4,8) and (9,8) not aligned\n"
      "[devspace-runner] rank=3 exited with code 3 before every rank finished a first step: waiting for a "
      "file change before starting the group again\n";
  p = analyze::runner_problems(prefixed);
  EXPECT_EQ(p.size(), (size_t)1);
  EXPECT_TRUE(contains(p[0], "ValueError: shapes (4,8) and (9,8) not aligned"));
  EXPECT_TRUE(!contains(p[0], "[rank 3]"));
  std::string bad_edit = up + "[devspace-runner] rank=1 load failed gen=3:\nTraceback (most recent call last):\n"
                              "ImportError: rank-local\n"
                              "[devspace-runner] reload failed gen=3 (failed on rank(s) [1]), keeping gen=2 on every rank\n";
  p = analyze::runner_problems(bad_edit);
  EXPECT_EQ(p.size(), (size_t)1);
  EXPECT_TRUE(contains(p[0], "the last edit did not load: reload failed gen=3"));
  EXPECT_TRUE(analyze::runner_problems(bad_edit + "[devspace-runner] reloaded gen=4 marker=ok ranks=8\n").empty());
  // the training state is no longer protected: said once, until fresh processes start
  std::string off = up + "[devspace-runner] rescue snapshots off (/dev/shm has 900 MiB free, a snapshot of every "
                         "rank needs 3072 MiB)\n";
  p = analyze::runner_problems(off);
  EXPECT_EQ(p.size(), (size_t)1);
  EXPECT_TRUE(contains(p[0], "stopped snapshotting the training state (/dev/shm has 900 MiB free"));
  EXPECT_TRUE(contains(p[0], "needs 3072 MiB): a restart"));
  EXPECT_TRUE(analyze::runner_problems(off + "[devspace-runner] started gen=1 marker=v0 world=8\n").empty());
  // a restart that could not load its snapshot started over: said until a restore succeeds
  std::string lost = up + "[devspace-runner] rescue: snapshot step=120 did not restore on rank 3 (ValueError: "
                          "state['model']: shape (8,) now, (4,) in the snapshot): starting from setup()\n"
                          "[devspace-runner] started gen=1 marker=v2 world=8\n";
  p = analyze::runner_problems(lost);
  EXPECT_EQ(p.size(), (size_t)1);
  EXPECT_TRUE(contains(p[0], "could not load its rescue snapshot (snapshot step=120 did not restore on rank 3"));
  EXPECT_TRUE(analyze::runner_problems(lost + "[devspace-runner] restored step=130 gen=1 from the rescue snapshot\n")
                  .empty());
}

// $KUBECONFIG with several files, merged like client-go's clientcmd loading rules.
TEST(kubeconfig_multi_file_merge_and_save) {
  std::string d = fs::make_temp_dir("kcmerge-");
  fs::mkdirs(fs::join(d, "one"));
  fs::mkdirs(fs::join(d, "two/certs"));
  std::string f1 = fs::join(d, "one/config"), f2 = fs::join(d, "two/config");
  fs::write_file(f1,
                 "apiVersion: v1\nkind: Config\ncurrent-context: a\n"
                 "clusters:\n- name: c1\n  cluster: {server: 'https://one:6443'}\n"
                 "contexts:\n- name: a\n  context: {cluster: c1, user: u1, namespace: ns-a}\n"
                 "users:\n- name: u1\n  user: {token: first}\n");
  fs::write_file(fs::join(d, "two/certs/ca.crt"), "CA-PEM");
  fs::write_file(f2,
                 "apiVersion: v1\nkind: Config\ncurrent-context: b\n"
                 "clusters:\n- name: c2\n  cluster: {server: 'https://two:6443', certificate-authority: certs/ca.crt}\n"
                 "contexts:\n- name: a\n  context: {cluster: c2, user: u2}\n"
                 "- name: b\n  context: {cluster: c2, user: u1}\n"
                 "users:\n- name: u1\n  user: {token: shadowed}\n- name: u2\n  user: {token: second}\n");
  setenv("KUBECONFIG", (f1 + ":" + f2 + ":" + f1).c_str(), 1);
  kube::KubeConfig kc = kube::KubeConfig::load();
  EXPECT_EQ(kc.files.size(), (size_t)2);
  EXPECT_EQ(kc.current_context(), std::string("a"));  // first file that sets it
  auto a = kc.resolve("a");
  EXPECT_EQ(a.server, std::string("https://one:6443"));  // first definition of "a" wins
  EXPECT_EQ(a.token, std::string("first"));
  auto b = kc.resolve("b");
  EXPECT_EQ(b.server, std::string("https://two:6443"));
  EXPECT_EQ(b.ca_pem, std::string("CA-PEM"));  // relative to the file that defines c2
  EXPECT_EQ(b.token, std::string("first"));    // u1 from the first file
  // edits go back where each entry lives; the current context to the file that set it
  kc.set_current_context("b");
  kc.set_context_namespace("b", "ns-b");
  kc.set_context("new", "c1", "u1", "");
  kc.save();
  Value v1 = yaml_load_file(f1), v2 = yaml_load_file(f2);
  EXPECT_EQ(v1.get("current-context").as_string(), std::string("b"));
  EXPECT_EQ(v2.get("current-context").as_string(), std::string("b"));  // untouched (was b)
  EXPECT_EQ(v1.get("contexts").size(), (size_t)2);                      // a + new
  bool b_ns = false, shadow_kept = false;
  for (auto& c : v2.get("contexts").items()) {
    if (c.get("name").as_string() == "b") b_ns = c.at_path("context.namespace").as_string() == "ns-b";
    if (c.get("name").as_string() == "a") shadow_kept = c.at_path("context.cluster").as_string() == "c2";
  }
  EXPECT_TRUE(b_ns);
  EXPECT_TRUE(shadow_kept);
  unsetenv("KUBECONFIG");
  fs::remove_all(d);
}

TEST(no_proxy_matching) {
  using net::no_proxy_matches;
  EXPECT_TRUE(no_proxy_matches("*", "api.example.com", 443));
  EXPECT_TRUE(no_proxy_matches("example.com", "api.example.com", 443));
  EXPECT_TRUE(no_proxy_matches(".example.com", "api.example.com", 443));
  EXPECT_TRUE(no_proxy_matches("example.com", "example.com", 443));
  EXPECT_TRUE(!no_proxy_matches("example.com", "badexample.com", 443));
  EXPECT_TRUE(no_proxy_matches("10.0.0.0/8, localhost", "10.96.0.1", 443));
  EXPECT_TRUE(!no_proxy_matches("10.0.0.0/8", "11.0.0.1", 443));
  EXPECT_TRUE(no_proxy_matches("kube.local:6443", "kube.local", 6443));
  EXPECT_TRUE(!no_proxy_matches("kube.local:6443", "kube.local", 443));
  EXPECT_TRUE(no_proxy_matches("127.0.0.1", "127.0.0.1", 8443));
  net::ProxyConfig p;
  p.https_proxy = "http://proxy:3128";
  p.no_proxy = "localhost";
  EXPECT_EQ(p.proxy_for("https", "api", 443), std::string("http://proxy:3128"));
  EXPECT_EQ(p.proxy_for("https", "localhost", 443), std::string(""));
  EXPECT_EQ(p.proxy_for("http", "api", 80), std::string(""));
}

TEST(websocket_accept_rfc6455_example) {
  // RFC 6455 §1.3 worked example
  EXPECT_EQ(net::websocket_accept("dGhlIHNhbXBsZSBub25jZQ=="), std::string("s3pPLMBiTxaQ9kYGzzhZRbK+xOo="));
}

// ---------------------------------------------------------------- SPDY/3.1 (the multiplexed port-forward tunnel)

TEST(spdy_dictionary_is_the_protocols) {
  const std::string& d = kube::spdy_dictionary();
  EXPECT_EQ(d.size(), (size_t)1423);
  // the zlib dictionary id a SPDY/3 peer checks (adler-32 of the dictionary)
  EXPECT_EQ((uint32_t)adler32(1L, (const Bytef*)d.data(), (uInt)d.size()), (uint32_t)0xe3c6a7c2u);
}

TEST(spdy_header_blocks_share_one_zlib_stream_per_direction) {
  kube::SpdyHeaderCodec a, b;
  kube::SpdyHeaders h1 = {{"streamtype", "error"}, {"port", "8080"}, {"requestid", "0"}};
  kube::SpdyHeaders h2 = {{"streamtype", "data"}, {"port", "8080"}, {"requestid", "0"}};
  std::string c1 = a.compress(h1), c2 = a.compress(h2);
  EXPECT_TRUE(c2.size() < c1.size());  // the second block refers back into the first
  kube::SpdyHeaders out;
  EXPECT_TRUE(b.decompress(c1, &out) && out == h1);
  EXPECT_TRUE(b.decompress(c2, &out) && out == h2);
  kube::SpdyHeaders empty;
  EXPECT_TRUE(b.decompress(a.compress(empty), &out) && out.empty());
}

TEST(spdy_frames_round_trip_and_split_anywhere) {
  std::string wire = kube::spdy::control_frame(kube::spdy::SynStream, 0, "0123456789") +
                     kube::spdy::data_frame(3, kube::spdy::kFlagFin, std::string(70000, 'x')) +
                     kube::spdy::control_frame(kube::spdy::Ping, 0, kube::spdy::u32(7));
  EXPECT_EQ((unsigned char)wire[0], 0x80);
  EXPECT_EQ((unsigned char)wire[1], 3);
  // the tunnel's WebSocket messages may cut frames anywhere: feed it in odd pieces
  std::string buf;
  std::vector<kube::spdy::Frame> got;
  for (size_t off = 0; off < wire.size(); off += 997) {
    buf += wire.substr(off, 997);
    kube::spdy::Frame f;
    while (kube::spdy::parse(&buf, &f)) got.push_back(f);
  }
  EXPECT_EQ(got.size(), (size_t)3);
  EXPECT_TRUE(got[0].control && got[0].type == kube::spdy::SynStream && got[0].body == "0123456789");
  EXPECT_TRUE(!got[1].control && got[1].stream_id == 3 && got[1].flags == kube::spdy::kFlagFin &&
              got[1].body.size() == 70000);
  EXPECT_TRUE(got[2].control && got[2].type == kube::spdy::Ping && kube::spdy::get_u32(got[2].body, 0) == 7);
}

// Without a spill budget a stream's mailbox holds at most `cap` unread bytes: the tunnel's reader
// waits for the consumer (as a spdystream frame loop), and a consumer that leaves unblocks it.
TEST(spdy_mailbox_bounds_unread_data) {
  kube::SpdyMailbox box;
  box.cap = 1000;
  box.spill_cap = 0;
  box.push({0, std::string(800, 'a')});
  std::atomic<bool> second_in{false};
  std::thread reader([&] {
    box.push({0, std::string(800, 'b')});  // 800 unread: still room
    box.push({0, std::string(800, 'c')});  // 1600 unread: waits for a pop
    second_in = true;
  });
  std::this_thread::sleep_for(std::chrono::milliseconds(50));
  EXPECT_TRUE(!second_in.load());
  kube::SpdyMailbox::Event e;
  EXPECT_TRUE(box.pop(&e, 1000) && e.data[0] == 'a');
  EXPECT_TRUE(box.pop(&e, 1000) && e.data[0] == 'b');
  reader.join();
  EXPECT_TRUE(second_in.load());
  // end events never wait for room; a closed mailbox drops data and ends pop()
  box.push({0, "", true});
  std::thread late([&] {
    box.push({0, std::string(800, 'd')});
    box.push({0, std::string(800, 'e')});  // over the cap: returns once the box is closed
  });
  std::this_thread::sleep_for(std::chrono::milliseconds(50));
  box.close();
  late.join();
  EXPECT_TRUE(!box.pop(&e, 10));
}

// Past `cap` in memory, events go to a nameless temp file in order (ends included) and push()
// does not wait: one slow local reader does not hold up the tunnel's other streams. Past
// `spill_cap` on disk it waits again. Drained, the box is back in memory.
TEST(spdy_mailbox_spills_past_its_memory_cap_in_order) {
  kube::SpdyMailbox box;
  box.cap = 1000;
  box.spill_cap = 3000;
  box.push({0, std::string(800, 'a')});
  box.push({0, std::string(800, 'b')});  // 800 in memory: still room
  box.push({0, std::string(900, 'c')});  // 1600 in memory: to disk
  box.push({1, "err"});
  box.push({0, "", true});               // the end comes after what is on disk
  EXPECT_EQ(box.bytes, (size_t)1600);
  {
    std::lock_guard<std::mutex> g(box.mu);
    EXPECT_TRUE(box.spilled() > 900);
  }
  std::atomic<bool> big_in{false};
  std::thread t([&] {
    box.push({0, std::string(2500, 'd')});  // over the disk budget: waits for the consumer
    big_in = true;
  });
  std::this_thread::sleep_for(std::chrono::milliseconds(50));
  EXPECT_TRUE(!big_in.load());
  kube::SpdyMailbox::Event e;
  EXPECT_TRUE(box.pop(&e, 1000) && e.data == std::string(800, 'a'));
  EXPECT_TRUE(box.pop(&e, 1000) && e.data == std::string(800, 'b'));
  EXPECT_TRUE(box.pop(&e, 1000) && e.channel == 0 && e.data == std::string(900, 'c') && !e.end);
  t.join();  // the disk budget had room again once 'c' was read
  EXPECT_TRUE(big_in.load());
  EXPECT_TRUE(box.pop(&e, 1000) && e.channel == 1 && e.data == "err");
  EXPECT_TRUE(box.pop(&e, 1000) && e.end && e.data.empty());
  EXPECT_TRUE(box.pop(&e, 1000) && e.data == std::string(2500, 'd'));
  {
    std::lock_guard<std::mutex> g(box.mu);
    EXPECT_EQ(box.spilled(), (uint64_t)0);
  }
  box.push({0, "mem"});  // drained: memory again
  EXPECT_EQ(box.bytes, (size_t)3);
  EXPECT_TRUE(box.pop(&e, 1000) && e.data == "mem");
  box.close();
  EXPECT_TRUE(!box.pop(&e, 10));
}

TEST(analyze_reports_a_long_step_holding_back_an_edit) {
  std::string up = "[devspace-runner] started gen=1 marker=v0\n";
  std::string held = up + "[devspace-runner] rank=0 in step for 75 s at train.py:42; edit pending: rank=0 is making "
                          "progress at train.py:42: not restarting\n";
  auto p = analyze::runner_problems(held);
  EXPECT_EQ(p.size(), (size_t)1);
  EXPECT_TRUE(contains(p[0], "the last edit is not loaded yet: training rank=0 in step for 75 s at train.py:42"));
  EXPECT_TRUE(contains(p[0], "making progress") && contains(p[0], "applies when that step ends"));
  // resolved: the edit loaded, or the group was restarted as stuck
  EXPECT_TRUE(analyze::runner_problems(held + "[devspace-runner] reloaded gen=2 marker=v1\n").empty());
  EXPECT_TRUE(analyze::runner_problems(held + "[devspace-runner] rank=0 made no progress for 90 s at train.py:42 and "
                                              "the code changed since (stuck in a step?): restarting\n").empty());
}

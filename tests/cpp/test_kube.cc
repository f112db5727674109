// Kubernetes adapter units: pod status (kubectl printer port, kubectl/client.go:224), resource
// paths, kubeconfig resolution (inline data, tokens, namespaces), analyze's GPU log matcher.
#include "analyze/analyze.h"
#include "core/codec.h"
#include "core/fs.h"
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

TEST(analyze_gpu_runtime_log_matcher) {
  std::string m;
  EXPECT_TRUE(analyze::log_has_gpu_runtime_error("RuntimeError: No HIP GPUs are available", &m));
  EXPECT_TRUE(analyze::log_has_gpu_runtime_error("NCCL WARN NET/Socket : no socket found\nncclSystemError", &m));
  EXPECT_TRUE(analyze::log_has_gpu_runtime_error("hipErrorNoDevice", &m));
  EXPECT_TRUE(!analyze::log_has_gpu_runtime_error("Example app listening on port 3000!", &m));
}

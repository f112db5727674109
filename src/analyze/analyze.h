// Namespace problem report (pkg/devspace/analyze): non-Normal events of live objects,
// pods with abnormal status, restarts, crash logs — plus MI355X checks: GPU scheduling
// (Insufficient amd.com/gpu, node allocatable), missing device plugin, ROCm/HIP/RCCL
// start-up errors in container logs, and (optionally) an in-pod GPU probe.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "kube/client.h"

namespace ds {
namespace analyze {

struct ReportItem {
  std::string name;
  std::vector<std::string> problems;
};

struct Options {
  bool wait = true;          // wait for pods leaving ContainerCreating/Pending/Terminating
  int wait_timeout_s = 120;  // analyze/pods.go:19
  int min_pod_age_s = 20;    // analyze/pods.go:16
  bool gpu_probe = false;    // exec the GPU probe inside GPU pods
};

std::vector<ReportItem> create_report(kube::Client& k, const std::string& ns, const Options& o);
std::string report_to_string(const std::vector<ReportItem>& report);
// Used by Helm deploy errors ("timed out waiting") to explain the failure.
std::string analyze(kube::Client& k, const std::string& ns, const Options& o);

// Helpers exposed for tests
std::vector<std::string> gpu_problems(kube::Client& k, const std::string& ns, const std::vector<Value>& pods,
                                      const Options& o);
bool log_has_gpu_runtime_error(const std::string& log, std::string* match);
// The hot-reload training runner's state from a container log ("[devspace-runner] ..." lines,
// devspace_amd/runner.py): a group that is down waiting for an edit after a rank failed, or a
// last edit that did not load (the ranks kept the previous code). Empty when it trains.
std::vector<std::string> runner_problems(const std::string& log);
// Multi-GPU pod without a memory-backed /dev/shm (RCCL): the problem text, or "".
std::string shm_problem(const Value& pod, int64_t gpus);
// Runs the shell-only GPU probe in a container; returns the problems it found (empty = fine).
// Works in images without devspace_amd (torch check) and without python3 (device nodes only,
// reported as "probe unavailable"). `summary` (optional) receives what was verified, e.g.
// "1 device(s) checked by the devspace probe: gpu0 gfx950 MFMA self-test err 0".
std::vector<std::string> probe_pod_gpus(kube::Client& k, const std::string& ns, const std::string& pod,
                                        const std::string& container, std::string* summary = nullptr);

}  // namespace analyze
}  // namespace ds

#include "analyze/analyze.h"
#include "gpu/sizing.h"

#include <time.h>

#include <chrono>
#include <map>
#include <regex>
#include <set>
#include <thread>

#include "core/log.h"
#include "core/safe_regex.h"
#include "core/strutil.h"

namespace ds {
namespace analyze {

static const int kHeaderWidth = 52;
static const std::string kPad = "  ";

static int64_t parse_time(const std::string& ts) {
  struct tm t{};
  if (ts.size() < 19 || !strptime(ts.c_str(), "%Y-%m-%dT%H:%M:%S", &t)) return 0;
  return (int64_t)timegm(&t);
}

static std::string human_age(int64_t secs) {
  if (secs < 0) secs = 0;
  if (secs < 60) return std::to_string(secs) + "s";
  if (secs < 3600) return std::to_string(secs / 60) + "m" + std::to_string(secs % 60) + "s";
  return std::to_string(secs / 3600) + "h" + std::to_string((secs % 3600) / 60) + "m";
}

static bool is_okay(const std::string& s) { return s == "Completed" || s == "Running"; }

std::vector<std::string> events_problems(kube::Client& k, const std::string& ns) {
  // events.go:20-55: every non-Normal event whose involved object still exists. One GET per
  // involved object (not per event), and events repeating the same message for the same
  // object are reported once with their counts summed (a correlator that did not aggregate
  // them would otherwise flood the report).
  Value evs = k.get("/api/v1/namespaces/" + ns + "/events");
  std::map<std::string, bool> exists;
  std::vector<std::pair<std::string, int64_t>> order;  // (header + message) -> count
  std::map<std::string, size_t> index;
  for (auto& e : evs.get("items").items()) {
    if (e.get("type").as_string() == "Normal") continue;
    const Value& io = e.get("involvedObject");
    std::string av = io.get("apiVersion").as_string("v1");
    std::string path = kube::resource_path(av, io.get("kind").as_string(), ns, io.get("name").as_string());
    auto it = exists.find(path);
    if (it == exists.end()) it = exists.emplace(path, (bool)k.try_get(path)).first;
    if (!it->second) continue;  // only objects that still exist
    std::string header = log::color(e.get("type").as_string() + " - " + io.get("kind").as_string() + " " +
                                        io.get("name").as_string() + ": ",
                                    "202+b");
    std::string key = header + "\n" + e.get("message").as_string();
    int64_t n = e.get("count").as_int(1);
    auto at = index.find(key);
    if (at != index.end()) {
      order[at->second].second += n;
      continue;
    }
    index[key] = order.size();
    order.push_back({key, n});
  }
  std::vector<std::string> out;
  for (auto& kv : order) {
    size_t nl = kv.first.find('\n');
    out.push_back(kPad + kv.first.substr(0, nl) + "\n" + kPad + std::to_string(kv.second) + "x " +
                  kv.first.substr(nl + 1) + " \n");
  }
  return out;
}

bool log_has_gpu_runtime_error(const std::string& text, std::string* match) {
  static const std::regex re(
      "(hipErrorNoDevice|hipErrorInvalidDevice|hipErrorOutOfMemory|HIP error|HSA_STATUS_ERROR[A-Z_]*|"
      "No HIP GPUs are available|RuntimeError: No CUDA GPUs are available|"
      "rccl.*(error|failed)|NCCL error|ncclSystemError|ncclInternalError|ncclUnhandledCudaError|"
      "amdgpu.ids: No such file|Unable to open /dev/kfd|/dev/kfd: (Permission denied|No such file)|"
      "torch.OutOfMemoryError|HIP out of memory|"
      "Bus error|unable to (write to|allocate) .*shared memory|shared memory segment|/dev/shm.*No space left)",
      std::regex::icase);
  // line by line (the patterns never span lines), each line capped: container logs can hold
  // megabyte-long lines (progress bars, JSON dumps) that std::regex cannot scan in one piece
  for (auto& full : split(text, "\n")) {
    std::string line = full.size() > 16384 ? full.substr(0, 16384) : full;
    std::smatch m;
    if (!safe_regex_search(line, &m, re)) continue;
    // amdgpu.ids is a benign warning on most images
    if (contains(m.str(0), "amdgpu.ids")) continue;
    if (match) *match = m.str(0);
    return true;
  }
  return false;
}

std::vector<std::string> runner_problems(const std::string& text) {
  const std::string tag = "[devspace-runner] ";
  std::string down, failed_reload, last_failure, last_exception, rescue_off, restore_failed, long_step;
  bool in_traceback = false;
  for (auto& raw : split(text, "\n")) {
    // a multi-rank pod's supervisor prefixes each rank's lines with "[rank N] "
    std::string line = raw;
    if (starts_with(line, "[rank ")) {
      size_t close = line.find("] ");
      if (close != std::string::npos && close < 12) line = line.substr(close + 2);
    }
    size_t at = line.find(tag);
    if (at == std::string::npos) {
      // the last line of a Python traceback printed after a failure: "<Error>: <message>"
      std::string t = trim(line);
      if (in_traceback && !t.empty() && t[0] != ' ' && t.find(": ") != std::string::npos &&
          !starts_with(t, "Traceback") && !starts_with(t, "File "))
        last_exception = t.size() > 300 ? t.substr(0, 300) + "..." : t;
      continue;
    }
    std::string msg = line.substr(at + tag.size());
    in_traceback = false;
    if (contains(msg, " step failed ") || contains(msg, " startup failed ") || contains(msg, " setup failed ") ||
        contains(msg, " load failed ") || contains(msg, "group failure")) {
      last_failure = msg.substr(0, msg.find(':') == std::string::npos ? msg.size() : msg.find(':'));
      last_exception.clear();
      in_traceback = true;
    } else if (contains(msg, "waiting for a file change before starting")) {  // a group, or one rank
      down = msg;
    } else if (starts_with(msg, "rank=") && contains(msg, " in step for ") && contains(msg, "; edit pending: ")) {
      // the supervisor's stuck-step rule saw a long step with an edit waiting and left it alone
      // (devspace_amd/supervise.py): the edit applies when the step ends
      long_step = msg;
    } else if (starts_with(msg, "started gen=")) {
      down.clear();
      failed_reload.clear();
      long_step.clear();
      rescue_off.clear();  // fresh processes take snapshots again
    } else if (starts_with(msg, "rescue: snapshot step=") && contains(msg, "did not restore")) {
      restore_failed = msg.substr(std::string("rescue: ").size());
    } else if (starts_with(msg, "restored step=")) {
      restore_failed.clear();
    } else if (starts_with(msg, "rescue snapshots off (")) {
      rescue_off = msg.substr(std::string("rescue snapshots off (").size());
      if (!rescue_off.empty() && rescue_off.back() == ')') rescue_off.pop_back();
    } else if (starts_with(msg, "reloaded gen=")) {
      failed_reload.clear();
      long_step.clear();
    } else if (contains(msg, " made no progress for ")) {
      long_step.clear();  // restarted as stuck
    } else if (starts_with(msg, "reload failed gen=")) {
      failed_reload = msg;
    }
  }
  std::vector<std::string> out;
  if (!down.empty()) {
    std::string why = last_failure.empty() ? "" : " after " + last_failure;
    if (!last_exception.empty()) why += " (" + last_exception + ")";
    out.push_back("training group is down" + why + "; the runner waits for an edit of the synced code to start it "
                  "again");
  } else if (!failed_reload.empty()) {
    std::string why = last_exception.empty() ? "" : " (" + last_exception + ")";
    out.push_back("the last edit did not load: " + failed_reload.substr(0, failed_reload.find('\n')) + why);
  }
  if (!long_step.empty()) {
    // "rank=0 in step for 75 s at train.py:42; edit pending: <why>"
    size_t semi = long_step.find("; edit pending: ");
    out.push_back("the last edit is not loaded yet: training " + long_step.substr(0, semi) + " (" +
                  long_step.substr(semi + std::string("; edit pending: ").size()) +
                  "); the edit applies when that step ends");
  }
  if (!restore_failed.empty())
    out.push_back("a restarted training group could not load its rescue snapshot (" + restore_failed +
                  "): training started over from setup()");
  if (!rescue_off.empty())
    out.push_back("the runner stopped snapshotting the training state (" + rescue_off +
                  "): a restart of the group or container would begin again from step 0 (a larger shmPerGPU, or "
                  "snapshot()/restore() in the module)");
  return out;
}

// RCCL between the GPUs of one pod (one process per GPU) and PyTorch's worker processes use
// /dev/shm; container runtimes give 64 MiB unless a memory-backed emptyDir is mounted there.
// Returns "" when a multi-GPU pod has one, else the problem.
std::string shm_problem(const Value& pod, int64_t gpus) {
  if (gpus < 2) return "";
  std::set<std::string> mem_volumes;
  for (auto& v : pod.at_path("spec.volumes").items())
    if (v.at_path("emptyDir.medium").as_string() == "Memory") mem_volumes.insert(v.get("name").as_string());
  for (auto& c : pod.at_path("spec.containers").items()) {
    if (gpu::container_gpu_request(c) == 0) continue;
    bool ok = false;
    for (auto& m : c.get("volumeMounts").items())
      if (m.get("mountPath").as_string() == "/dev/shm" && mem_volumes.count(m.get("name").as_string())) ok = true;
    if (!ok)
      return "container " + c.get("name").as_string() + " uses " + std::to_string(gpus) +
             " GPUs but has no memory-backed /dev/shm (RCCL intra-node transport; the runtime default is 64 MiB) — "
             "mount an emptyDir{medium: Memory} at /dev/shm";
  }
  return "";
}

static int64_t gpu_request(const Value& pod) {
  int64_t n = 0;
  for (auto& c : pod.at_path("spec.containers").items()) n += gpu::container_gpu_request(c);
  return n;
}

// Who holds a node's GPU devices: "ns/pod (4), ns2/pod2 (2)" from the pods bound to it (all
// namespaces; "" when that list is forbidden, with *why set).
static std::string gpu_holders(kube::Client& k, const std::string& node, std::string* why) {
  Value pods;
  try {
    pods = k.get("/api/v1/pods?fieldSelector=spec.nodeName%3D" + node);
  } catch (const std::exception& e) {
    if (why) *why = e.what();
    return "";
  }
  std::vector<std::string> out;
  for (auto& p : pods.get("items").items()) {
    std::string phase = p.at_path("status.phase").as_string();
    if (phase == "Succeeded" || phase == "Failed") continue;
    int64_t n = gpu_request(p);
    if (n > 0)
      out.push_back(p.at_path("metadata.namespace").as_string() + "/" + p.at_path("metadata.name").as_string() +
                    " (" + std::to_string(n) + ")");
  }
  return join(out, ", ");
}

// The scheduler's verdict on a Pending pod, when it is a lack of GPU devices.
static bool insufficient_gpus(const Value& pod) {
  for (auto& c : pod.at_path("status.conditions").items())
    if (c.get("reason").as_string() == "Unschedulable" && contains(c.get("message").as_string(), "Insufficient amd.com/"))
      return true;
  return false;
}

// In-pod GPU probe that depends on nothing but a POSIX shell: device nodes, ROCm tools, and —
// when python3 is there — the devspace gfx950 probe kernels (devspace_amd.gpucheck) or, in a
// stock rocm/pytorch image without devspace_amd, a torch/HIP check (device count, arch, a bf16
// matmul checked against fp32). Prints KEY=VALUE lines and at most one JSON report.
const char* const kGpuProbeScript = R"SH(
if [ -e /dev/kfd ]; then echo KFD=yes; else echo KFD=no; fi
n=0; for d in /dev/dri/renderD*; do [ -e "$d" ] && n=$((n+1)); done; echo RENDER=$n
echo "VISIBLE=${HIP_VISIBLE_DEVICES:-${ROCR_VISIBLE_DEVICES:-}}"
if command -v rocminfo >/dev/null 2>&1; then echo "ROCMINFO=$(rocminfo 2>/dev/null | grep -c 'Name: *gfx')"; else echo ROCMINFO=absent; fi
if command -v python3 >/dev/null 2>&1; then
  if python3 -c 'import devspace_amd.gpucheck' >/dev/null 2>&1; then
    echo PROBE=devspace; python3 -m devspace_amd.gpucheck --quick --json 2>/dev/null
  else
    echo PROBE=torch; python3 - <<'PY' 2>/dev/null || echo PROBE_FAILED=1
import json
rep = {"devices": [], "problems": []}
try:
    import torch
except Exception as e:
    rep["problems"].append("PyTorch is not importable (%s): only device nodes were checked" % e.__class__.__name__)
    print(json.dumps(rep)); raise SystemExit(0)
if not getattr(torch.version, "hip", None):
    rep["problems"].append("PyTorch build is not ROCm (torch.version.hip is empty)")
if not torch.cuda.is_available():
    rep["problems"].append("torch.cuda.is_available() is False: the HIP runtime sees no GPU")
else:
    for i in range(torch.cuda.device_count()):
        p = torch.cuda.get_device_properties(i)
        d = {"index": i, "name": p.name, "arch": getattr(p, "gcnArchName", ""), "hbm_gb": round(p.total_memory / 1e9, 1)}
        try:
            a = torch.randn(256, 256, device="cuda:%d" % i)
            b = torch.randn(256, 256, device="cuda:%d" % i)
            ref = (a.cpu() @ b.cpu())
            got = (a.bfloat16() @ b.bfloat16()).float().cpu()
            err = float((got - ref).abs().max() / ref.abs().max())
            d["matmul_rel_err"] = err
            if err > 5e-2:
                rep["problems"].append("GPU %d bf16 matmul mismatch (rel err %.3g)" % (i, err))
        except Exception as e:
            rep["problems"].append("GPU %d kernel launch failed: %s" % (i, e))
        rep["devices"].append(d)
print(json.dumps(rep))
PY
  fi
else
  echo PROBE=unavailable
fi
)SH";

std::vector<std::string> probe_pod_gpus(kube::Client& k, const std::string& ns, const std::string& pod,
                                        const std::string& container, std::string* summary) {
  auto s = k.exec(ns, pod, container, {"sh", "-c", kGpuProbeScript}, false, false);
  s->close_stdin_if_any();
  std::string outp = read_all(s->out());
  s->wait(60000);
  std::map<std::string, std::string> kv;
  std::string json_text;
  for (auto& line : split(outp, "\n")) {
    std::string t = trim(line);
    if (t.empty()) continue;
    if (t[0] == '{') {
      json_text = t;
      continue;
    }
    size_t eq = t.find('=');
    if (eq != std::string::npos && eq < 20) kv[t.substr(0, eq)] = t.substr(eq + 1);
  }
  std::vector<std::string> problems;
  if (kv["KFD"] == "no")
    problems.push_back("no /dev/kfd in the container (GPU not attached: amd.com/gpu request / device plugin?)");
  else if (kv["RENDER"] == "0")
    problems.push_back("/dev/kfd present but no /dev/dri/renderD* nodes (GPU not attached)");
  if (!json_text.empty()) {
    Value rep = json_parse(json_text);
    for (auto& pr : rep.get("problems").items()) problems.push_back(pr.as_string());
    // what the probe verified, so a clean report still says that the devices were exercised
    std::vector<std::string> devs;
    for (auto& d : rep.get("devices").items()) {
      std::string arch = d.get("arch").as_string();
      std::string dev = "gpu" + std::to_string(d.get("index").as_int()) + " " + (arch.empty() ? "?" : arch);
      if (!d.get("mfma_selftest_max_abs_err").is_null())
        dev += " MFMA self-test err " + json_dump(d.get("mfma_selftest_max_abs_err"));
      else if (!d.get("matmul_rel_err").is_null())
        dev += " bf16 matmul rel err " + json_dump(d.get("matmul_rel_err"));
      devs.push_back(dev);
    }
    if (summary)
      *summary = std::to_string(devs.size()) + " device(s) checked by the " + kv["PROBE"] + " probe" +
                 (devs.empty() ? "" : ": " + join(devs, ", "));
  } else if (kv["PROBE"] == "unavailable" || kv.count("PROBE_FAILED") || kv["PROBE"].empty()) {
    problems.push_back("GPU probe unavailable (no python3 in the image): only device nodes were checked");
  }
  return problems;
}

std::vector<std::string> gpu_problems(kube::Client& k, const std::string& ns, const std::vector<Value>& pods,
                                      const Options& o) {
  std::vector<std::string> out;
  // A crashed container whose log shows a ROCm/HIP/RCCL runtime error, in any pod: without an
  // amd.com/gpu request it is usually the missing request itself ("No HIP GPUs are available").
  auto crash_errors = [&](const Value& p, int64_t want) {
    std::string name = p.at_path("metadata.name").as_string();
    for (auto& c : p.at_path("status.containerStatuses").items()) {
      bool crashed = c.get("restartCount").as_int() > 0 || !c.at_path("state.terminated").is_null();
      if (!crashed) continue;
      std::string text;
      try {
        text = k.logs(ns, name, c.get("name").as_string(), 200, c.get("restartCount").as_int() > 0);
      } catch (...) {
        continue;
      }
      std::string m;
      if (log_has_gpu_runtime_error(text, &m))
        out.push_back(kPad + log::color("GPU: ", "202+b") + "container " + c.get("name").as_string() + " of pod " +
                      name + " failed with a ROCm/HIP/RCCL error: " + m +
                      (want == 0 ? " (the pod requests no amd.com/gpu: add resources.limits amd.com/gpu)" : "") +
                      "\n");
    }
  };
  int64_t requested = 0;
  for (auto& p : pods) requested += gpu_request(p);
  if (requested == 0) {
    for (auto& p : pods) crash_errors(p, 0);
    return out;
  }
  // what the AMD GPU device plugin advertises: whole GPUs or compute partitions, healthy or not
  std::vector<gpu::GpuNode> nodes;
  bool nodes_known = true;
  try {
    nodes = gpu::gpu_nodes(k.get("/api/v1/nodes"));
  } catch (const std::exception&) {
    nodes_known = false;  // listing nodes may be forbidden for namespace-scoped users
  }
  const gpu::GpuNode* big = gpu::largest(nodes);
  if (nodes_known && nodes.empty())
    out.push_back(kPad + log::color("GPU: ", "202+b") +
                  "no node advertises amd.com/gpu — is the AMD GPU device plugin DaemonSet running?\n");
  for (auto& n : nodes)
    if (n.unhealthy() > 0)
      out.push_back(kPad + log::color("GPU: ", "202+b") +
                    strfmt("node %s: %lld of %lld %s unhealthy (capacity %lld, allocatable %lld) — the device "
                           "plugin stopped offering them (a GPU fault, an ECC or XGMI error, a driver reset): "
                           "check the node's amdgpu kernel log or `amd-smi`",
                           n.name.c_str(), (long long)n.unhealthy(), (long long)n.capacity, n.resource.c_str(),
                           (long long)n.capacity, (long long)n.gpus) +
                    "\n");
  for (auto& p : pods) {
    int64_t want = gpu_request(p);
    if (want == 0) {
      crash_errors(p, 0);
      continue;
    }
    std::string name = p.at_path("metadata.name").as_string();
    if (big != nullptr && want > big->gpus)
      out.push_back(kPad + log::color("GPU: ", "202+b") + "pod " + name + " requests " + std::to_string(want) +
                    " GPU device(s) but the largest node has " + std::to_string(big->gpus) + " (" + big->name + ": " +
                    big->describe() + "; HBM is not a schedulable resource)\n");
    else if (insufficient_gpus(p) && nodes_known) {
      // it would fit on an empty node: say who holds the devices now
      for (auto& n : nodes) {
        if (n.gpus <= 0) continue;
        std::string why;
        std::string holders = gpu_holders(k, n.name, &why);
        if (!holders.empty())
          out.push_back(kPad + log::color("GPU: ", "202+b") + "pod " + name + " waits for " + std::to_string(want) +
                        " GPU device(s); node " + n.name + " (" + std::to_string(n.gpus) + " " + n.resource +
                        ") has them held by " + holders + "\n");
        else if (!why.empty())
          out.push_back(kPad + log::color("GPU: ", "202+b") + "pod " + name + " waits for " + std::to_string(want) +
                        " GPU device(s); the pods holding node " + n.name + "'s cannot be listed (" + why + ")\n");
      }
    }
    std::string shm = shm_problem(p, want);
    if (!shm.empty()) out.push_back(kPad + log::color("GPU: ", "202+b") + "pod " + name + ": " + shm + "\n");
    for (auto& prob : gpu::pod_sizing_problems(p.get("spec")))
      out.push_back(kPad + log::color("GPU: ", "202+b") + "pod " + name + ": " + prob + "\n");
    crash_errors(p, want);
    // a Running GPU pod can still be idle: its training group down after a rank failed, or the
    // last edit not loaded (the runner keeps the previous code)
    if (kube::pod_status(p) == "Running") {
      for (auto& c : p.at_path("spec.containers").items()) {
        std::string text;
        try {
          text = k.logs(ns, name, c.get("name").as_string(), 400);
        } catch (...) {
          continue;
        }
        for (auto& prob : runner_problems(text))
          out.push_back(kPad + log::color("GPU: ", "202+b") + "pod " + name + ": " + prob + "\n");
      }
    }
    if (o.gpu_probe && kube::pod_status(p) == "Running") {
      std::string c = p.at_path("spec.containers")[0].get("name").as_string();
      try {
        std::string summary;
        for (auto& line : probe_pod_gpus(k, ns, name, c, &summary))
          out.push_back(kPad + log::color("GPU: ", "202+b") + "pod " + name + ": " + line + "\n");
        if (!summary.empty()) log::infof("GPU probe of pod %s: %s", name.c_str(), summary.c_str());
      } catch (const std::exception& e) {
        out.push_back(kPad + log::color("GPU: ", "202+b") + "pod " + name + ": GPU probe unavailable (" + e.what() +
                      ")\n");
      }
    }
  }
  return out;
}

std::vector<std::string> pods_problems(kube::Client& k, const std::string& ns, const Options& o,
                                       std::vector<Value>* pods_out) {
  std::vector<std::string> out;
  // pods.go:50-117 waits (polling) while pods are starting or younger than min_pod_age_s; here
  // state changes arrive by watch and the age threshold is slept to exactly.
  auto t0 = std::chrono::steady_clock::now();
  auto deadline = t0 + std::chrono::seconds(o.wait_timeout_s);
  std::vector<Value> pods;
  auto state_waiting = [](const std::vector<Value>& ps) {
    for (auto& p : ps) {
      std::string st = kube::pod_status(p);
      if (st == "ContainerCreating" || st == "Pending" || st == "Terminating") {
        // Pending because of GPU scheduling will not resolve by waiting
        if (st == "Pending" && contains(json_dump(p.at_path("status.conditions")), "Unschedulable")) continue;
        return true;
      }
    }
    return false;
  };
  while (true) {
    pods = k.list_pods(ns, "");
    int64_t now = (int64_t)time(nullptr);
    int64_t age_wait_s = 0;
    for (auto& p : pods)
      age_wait_s = std::max(age_wait_s, o.min_pod_age_s - (now - parse_time(p.at_path("metadata.creationTimestamp").as_string())));
    bool waiting = state_waiting(pods);
    int64_t left_ms = std::chrono::duration_cast<std::chrono::milliseconds>(deadline - std::chrono::steady_clock::now()).count();
    if (!o.wait || (!waiting && age_wait_s <= 0) || left_ms <= 0) break;
    log::start_wait("Waiting for pods to become ready");
    if (!waiting) {
      std::this_thread::sleep_for(std::chrono::milliseconds(std::min<int64_t>(left_ms, age_wait_s * 1000)));
      continue;
    }
    int64_t budget = age_wait_s > 0 ? std::min<int64_t>(left_ms, age_wait_s * 1000) : left_ms;
    k.list_watch("/api/v1/namespaces/" + ns + "/pods", "", (int)budget,
                 [&](const std::vector<Value>& ps) { return !state_waiting(ps); });
  }
  log::stop_wait();
  int64_t now = (int64_t)time(nullptr);
  for (auto& p : pods) {
    std::string name = p.at_path("metadata.name").as_string();
    std::string st = kube::pod_status(p);
    std::vector<std::string> cps;
    int ready = 0, total = 0;
    bool problem = !is_okay(st) && !starts_with(st, "Init");
    for (auto& c : p.at_path("status.containerStatuses").items()) {
      ++total;
      if (c.get("ready").as_bool()) ++ready;
      std::vector<std::string> lines;
      bool cp = false;
      int64_t restarts = c.get("restartCount").as_int();
      const Value& last = c.at_path("lastState.terminated");
      if (restarts > 0 && last.is_map() &&
          (restarts > 4 || now - parse_time(last.get("finishedAt").as_string()) < 7200)) {
        cp = true;
        lines.push_back("        Restarts: " + log::color(std::to_string(restarts), "red+b"));
        lines.push_back("        Last Restart: " +
                        log::color(human_age(now - parse_time(last.get("finishedAt").as_string())), "white+b") + " ago");
        if (last.get("exitCode").as_int() != 0) {
          lines.push_back("        Last Exit: " + log::color(last.get("reason").as_string(), "red+b") + " (Code: " +
                          log::color(std::to_string(last.get("exitCode").as_int()), "red+b") + ")");
          try {
            std::string lg = k.logs(ns, name, c.get("name").as_string(), 50, true);
            if (!lg.empty()) lines.push_back("        Last Execution Log: \n" + lg);
          } catch (...) {
          }
        }
      }
      if (!c.get("ready").as_bool()) {
        cp = true;
        const Value& term = c.at_path("state.terminated");
        const Value& wait = c.at_path("state.waiting");
        if (term.is_map()) {
          lines.push_back("        Status: " + log::color("Terminated", "red+b") + " (reason: " +
                          log::color(term.get("reason").as_string(), "red+b") + ")");
        } else if (wait.is_map()) {
          lines.push_back("        Status: " + log::color("Waiting", "red+b") + " (reason: " +
                          log::color(wait.get("reason").as_string(), "red+b") + ")");
          if (!wait.get("message").as_string().empty())
            lines.push_back("        Message: " + log::color(wait.get("message").as_string(), "white+b"));
        }
      }
      if (cp) {
        problem = true;
        cps.push_back("      - Container: " + log::color(c.get("name").as_string(), "white+b"));
        for (auto& l : lines) cps.push_back(l);
      }
    }
    if (st == "Pending") {
      for (auto& cond : p.at_path("status.conditions").items())
        if (cond.get("reason").as_string() == "Unschedulable")
          cps.push_back("      - Scheduling: " + log::color(cond.get("message").as_string(), "red+b"));
    }
    if (!problem) continue;
    std::string color = is_okay(st) ? "green+b" : kube::pod_status_is_fatal(st) ? "red+b" : "yellow+b";
    std::string s = kPad + "Pod " + log::color(name, "white+b") + ":\n";
    s += kPad + "    Status: " + log::color(st, color) + "\n";
    s += kPad + "    Created: " + log::color(human_age(now - parse_time(p.at_path("metadata.creationTimestamp").as_string())), "white+b") + " ago\n";
    if (total > 0) {
      std::string r = std::to_string(ready);
      if (ready != total) r = log::color(r, "red+b");
      s += kPad + "    Container: " + r + "/" + std::to_string(total) + " running\n";
    }
    if (!cps.empty()) {
      s += kPad + "    Problems: \n";
      for (auto& l : cps) s += kPad + l + "\n";
    }
    out.push_back(s);
  }
  if (pods_out) *pods_out = pods;
  return out;
}

std::vector<ReportItem> create_report(kube::Client& k, const std::string& ns, const Options& o) {
  std::vector<ReportItem> report;
  log::start_wait("Analyzing events");
  std::vector<std::string> ev;
  try {
    ev = events_problems(k, ns);
  } catch (const std::exception& e) {
    log::stop_wait();
    throw std::runtime_error(std::string("Error during analyzing events: ") + e.what());
  }
  log::stop_wait();
  if (!ev.empty()) report.push_back({"Events", ev});
  std::vector<Value> pods;
  auto pp = pods_problems(k, ns, o, &pods);
  if (!pp.empty()) report.push_back({"Pods", pp});
  auto gp = gpu_problems(k, ns, pods, o);
  if (!gp.empty()) report.push_back({"GPUs", gp});
  return report;
}

std::string report_to_string(const std::vector<ReportItem>& report) {
  if (report.empty())
    return "\n" + kPad + "No problems found.\n" + kPad + "Run `" + log::color("devspace logs -p", "white+b") +
           "` if you want show pod logs\n\n";
  std::string out = "\n";
  for (auto& item : report) {
    std::string header = " " + item.name + " (" + std::to_string(item.problems.size()) + " potential issue(s)) ";
    if (header.size() % 2 == 1) header += " ";
    int padding = kHeaderWidth - (int)header.size();
    header = std::string(padding / 2, ' ') + header + std::string(padding / 2, ' ');
    out += log::color(kPad + std::string(kHeaderWidth, '=') + "\n" + kPad + header + "\n" + kPad +
                          std::string(kHeaderWidth, '=') + "\n",
                      "green+b");
    for (auto& p : item.problems) out += p + "\n";
  }
  return out;
}

std::string analyze(kube::Client& k, const std::string& ns, const Options& o) {
  return report_to_string(create_report(k, ns, o));
}

}  // namespace analyze
}  // namespace ds

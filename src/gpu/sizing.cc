#include "gpu/sizing.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <set>

#include "core/strutil.h"

namespace ds {
namespace gpu {

double parse_cpu(const std::string& q_in) {
  std::string q = trim(q_in);
  if (q.empty()) return 0;
  if (q.back() == 'm') return std::atof(q.substr(0, q.size() - 1).c_str()) / 1000.0;
  return std::atof(q.c_str());
}

int64_t parse_memory_bytes(const std::string& q_in) {
  std::string q = trim(q_in);
  if (q.empty()) return -1;
  size_t i = 0;
  while (i < q.size() && (isdigit((unsigned char)q[i]) || q[i] == '.' || q[i] == 'e' || q[i] == 'E' || q[i] == '+' ||
                          q[i] == '-'))
    ++i;
  // "1e3" is a number, "1E" / "1Ei" are suffixes: back off a trailing exponent letter
  if (i > 0 && (q[i - 1] == 'e' || q[i - 1] == 'E')) --i;
  if (i == 0) return -1;
  double v = std::atof(q.substr(0, i).c_str());
  std::string suf = q.substr(i);
  static const std::pair<const char*, double> kSuffixes[] = {
      {"", 1},           {"k", 1e3},           {"M", 1e6},           {"G", 1e9},           {"T", 1e12},
      {"P", 1e15},       {"E", 1e18},          {"Ki", 1024.0},       {"Mi", 1048576.0},    {"Gi", 1073741824.0},
      {"Ti", 1099511627776.0}, {"Pi", 1125899906842624.0}, {"Ei", 1152921504606846976.0}, {"m", 1e-3}};
  for (auto& s : kSuffixes)
    if (suf == s.first) return (int64_t)std::llround(v * s.second);
  return -1;
}

std::vector<GpuNode> gpu_nodes(const Value& node_list) {
  std::vector<GpuNode> out;
  for (auto& n : node_list.get("items").items()) {
    GpuNode g;
    g.gpus = n.at_path("status.allocatable").get("amd.com/gpu").as_int(0);
    if (g.gpus <= 0) continue;
    g.name = n.at_path("metadata.name").as_string();
    g.cpu = parse_cpu(n.at_path("status.allocatable").get("cpu").as_string());
    g.memory = parse_memory_bytes(n.at_path("status.allocatable").get("memory").as_string());
    g.product = n.at_path("metadata.labels").get("amd.com/gpu.product-name").as_string();
    out.push_back(g);
  }
  return out;
}

PodSizing size_pod(int gpus, const std::vector<GpuNode>& nodes) {
  PodSizing s;
  s.gpus = gpus;
  s.basis = "defaults";
  if (gpus <= 0 || nodes.empty()) return s;
  // the node type that can hold the most GPUs (a pod must fit on one node)
  const GpuNode* best = &nodes[0];
  for (auto& n : nodes)
    if (n.gpus > best->gpus) best = &n;
  if (best->cpu > 0) s.cpu_per_gpu = std::max(1, (int)std::floor(best->cpu * 0.9 / (double)best->gpus));
  if (best->memory > 0) {
    int per_gpu_gi = (int)(best->memory * 0.9 / (double)best->gpus / 1073741824.0);
    // keep shm at a quarter of the share when the node is small
    s.shm_per_gpu_gi = std::max(1, std::min(s.shm_per_gpu_gi, per_gpu_gi / 4));
    s.host_per_gpu_gi = std::max(1, per_gpu_gi - s.shm_per_gpu_gi);
  }
  s.product = best->product;
  s.basis = strfmt("node %s: %lld GPUs, %.0f CPUs, %lld GiB allocatable", best->name.c_str(), (long long)best->gpus,
                   best->cpu, (long long)(best->memory / 1073741824LL));
  return s;
}

std::string resources_yaml(const PodSizing& s) {
  if (s.gpus <= 0)
    return "      limits:\n"
           "        cpu: \"2\"\n"
           "        memory: \"4Gi\"\n"
           "        # AMD Instinct GPUs requested through the device plugin (amd.com/gpu)\n"
           "        gpu: 0";
  std::string cpu = std::to_string(s.cpu()), mem = std::to_string(s.memory_gi()) + "Gi";
  return strfmt(
      "      # MI355X sizing for %d GPU(s) (%s): %d CPUs and %d Gi host memory per GPU, i.e. a\n"
      "      # %d Gi memory-backed /dev/shm per rank (charged to this memory limit) + %d Gi per rank.\n"
      "      # HBM (288 GB per GPU) is not a schedulable resource: GPUs are requested whole.\n"
      "      limits:\n"
      "        gpu: %d\n"
      "        cpu: \"%s\"\n"
      "        memory: \"%s\"\n"
      "      requests:\n"
      "        cpu: \"%s\"\n"
      "        memory: \"%s\"",
      s.gpus, s.basis.c_str(), s.cpu_per_gpu, s.shm_per_gpu_gi + s.host_per_gpu_gi, s.shm_per_gpu_gi,
      s.host_per_gpu_gi, s.gpus, cpu.c_str(), mem.c_str(), cpu.c_str(), mem.c_str());
}

std::string gpu_settings_yaml(const PodSizing& s) {
  if (s.gpus <= 0) return "";
  std::string out = strfmt(
      "  # /dev/shm (emptyDir medium: Memory) per GPU, in Gi; host memory budget per rank, in Gi\n"
      "  shmPerGPU: %d\n"
      "  hostMemoryPerGPU: %d\n",
      s.shm_per_gpu_gi, s.host_per_gpu_gi);
  if (!s.product.empty())
    out += "  # schedule on nodes of this GPU model only (AMD GPU operator node label)\n  gpuProductName: \"" +
           s.product + "\"\n";
  else
    out += "  # gpuProductName: AMD_Instinct_MI355X   # pin to a GPU model (amd.com/gpu.product-name label)\n";
  return out.substr(0, out.size() - 1);  // the placeholder line supplies the newline
}

std::vector<std::string> pod_sizing_problems(const Value& spec) {
  std::vector<std::string> out;
  int64_t shm_bytes = 0;
  std::set<std::string> shm_vols;
  for (auto& v : spec.get("volumes").items()) {
    if (v.at_path("emptyDir.medium").as_string() != "Memory") continue;
    shm_vols.insert(v.get("name").as_string());
  }
  for (auto& c : spec.get("containers").items()) {
    const Value& lim = c.at_path("resources.limits");
    int64_t gpus = lim.get("amd.com/gpu").as_int(0);
    if (gpus <= 0) gpus = c.at_path("resources.requests").get("amd.com/gpu").as_int(0);
    if (gpus <= 0) continue;
    std::string name = c.get("name").as_string();
    shm_bytes = 0;
    for (auto& m : c.get("volumeMounts").items()) {
      if (m.get("mountPath").as_string() != "/dev/shm" || !shm_vols.count(m.get("name").as_string())) continue;
      for (auto& v : spec.get("volumes").items())
        if (v.get("name").as_string() == m.get("name").as_string()) {
          std::string sl = v.at_path("emptyDir.sizeLimit").as_string();
          shm_bytes = sl.empty() ? 0 : parse_memory_bytes(sl);
        }
    }
    std::string mem = lim.get("memory").as_string();
    int64_t mem_bytes = mem.empty() ? -1 : parse_memory_bytes(mem);
    if (mem_bytes < 0) {
      out.push_back("container " + name + " requests " + std::to_string(gpus) +
                    " GPU(s) but sets no memory limit: size it per GPU (shm + host budget per rank)");
    } else if (shm_bytes > 0 && shm_bytes >= mem_bytes) {
      out.push_back(strfmt("container %s: the memory-backed /dev/shm (sizeLimit %lld GiB) is at least its memory "
                           "limit (%s) — tmpfs pages are charged to the container, so the ranks will be OOM-killed "
                           "once shm fills; raise the memory limit to shm + a host budget per rank",
                           name.c_str(), (long long)(shm_bytes >> 30), mem.c_str()));
    }
    std::string cpu_s = lim.get("cpu").as_string();
    if (cpu_s.empty()) cpu_s = c.at_path("resources.requests").get("cpu").as_string();
    double cpu = cpu_s.empty() ? -1 : parse_cpu(cpu_s);
    if (cpu >= 0 && cpu < (double)gpus)
      out.push_back(strfmt("container %s: %s CPU(s) for %lld GPU rank(s) — one training process per GPU needs at "
                           "least one core each (plus dataloader workers)",
                           name.c_str(), cpu_s.c_str(), (long long)gpus));
  }
  return out;
}

}  // namespace gpu
}  // namespace ds

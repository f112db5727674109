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

bool is_gpu_resource(const std::string& name) {
  if (name == "amd.com/gpu") return true;
  static const char* kModes[] = {"spx", "dpx", "qpx", "cpx"};
  if (!starts_with(name, "amd.com/")) return false;
  std::string rest = name.substr(8);
  for (auto* m : kModes) {
    if (rest == m) return true;
    if (starts_with(rest, std::string(m) + "_nps") && rest.size() > 7) {  // "cpx_nps" + digits
      bool digits = true;
      for (size_t i = 7; i < rest.size(); ++i) digits = digits && isdigit((unsigned char)rest[i]);
      if (digits) return true;
    }
  }
  return false;
}

int partitions_per_gpu(const std::string& mode_in) {
  std::string mode = to_lower(trim(mode_in));
  if (mode == "spx") return 1;
  if (mode == "dpx") return 2;
  if (mode == "qpx") return 4;
  if (mode == "cpx") return 8;  // MI300X/MI325X/MI350X/MI355X: one partition per XCD, 8 XCDs
  return 0;
}

int64_t hbm_of_product(const std::string& product) {
  std::string p = to_lower(product);
  if (contains(p, "mi355") || contains(p, "mi350")) return 288LL * 1000 * 1000 * 1000;
  if (contains(p, "mi325")) return 256LL * 1000 * 1000 * 1000;
  if (contains(p, "mi300x")) return 192LL * 1000 * 1000 * 1000;
  return 0;
}

int GpuNode::parts() const {
  int p = partitions_per_gpu(compute_mode);
  return p > 0 ? p : 1;
}

int64_t GpuNode::hbm_per_device() const {
  int64_t v = vram_per_gpu > 0 ? vram_per_gpu : hbm_of_product(product);
  return v > 0 ? v / parts() : 0;
}

std::string GpuNode::describe() const {
  std::string out;
  int64_t physical = capacity > 0 ? capacity / parts() : gpus / parts();
  if (!product.empty()) out += std::to_string(physical) + " x " + product;
  if (!compute_mode.empty() || !memory_mode.empty()) {
    std::string mode = to_upper(compute_mode.empty() ? "spx" : compute_mode);
    if (!memory_mode.empty()) mode += "/" + to_upper(memory_mode);
    out += (out.empty() ? "" : ", ") + mode;
  }
  out += (out.empty() ? "" : ": ") + std::to_string(gpus) + " schedulable " + resource;
  if (hbm_per_device() > 0) out += strfmt(" of %.0f GB HBM each", hbm_per_device() / 1e9);
  return out;
}

// Node labeller labels, under amd.com/ or the older beta.amd.com/ prefix.
static std::string gpu_label(const Value& labels, const std::string& key) {
  std::string v = labels.get("amd.com/gpu." + key).as_string();
  if (v.empty()) v = labels.get("beta.amd.com/gpu." + key).as_string();
  return v;
}

std::vector<GpuNode> gpu_nodes(const Value& node_list) {
  std::vector<GpuNode> out;
  for (auto& n : node_list.get("items").items()) {
    const Value& alloc = n.at_path("status.allocatable");
    const Value& cap = n.at_path("status.capacity");
    const Value& labels = n.at_path("metadata.labels");
    std::set<std::string> resources;
    for (auto& k : alloc.keys())
      if (is_gpu_resource(k)) resources.insert(k);
    for (auto& k : cap.keys())
      if (is_gpu_resource(k)) resources.insert(k);
    int64_t node_devices = 0;
    for (auto& r : resources) node_devices += std::max<int64_t>(0, alloc.get(r).as_int(0));
    for (auto& r : resources) {
      GpuNode g;
      g.resource = r;
      g.gpus = alloc.get(r).as_int(0);
      g.capacity = cap.get(r).as_int(g.gpus);
      if (g.gpus <= 0 && g.capacity <= 0) continue;
      g.node_devices = node_devices;
      g.name = n.at_path("metadata.name").as_string();
      g.cpu = parse_cpu(alloc.get("cpu").as_string());
      g.memory = parse_memory_bytes(alloc.get("memory").as_string());
      g.product = gpu_label(labels, "product-name");
      g.compute_mode = to_lower(gpu_label(labels, "compute-partitioning-mode"));
      g.memory_mode = to_lower(gpu_label(labels, "memory-partitioning-mode"));
      if (r != "amd.com/gpu") {  // mixed strategy: the resource name is the partition type
        std::string rest = r.substr(8);
        size_t us = rest.find('_');
        g.compute_mode = rest.substr(0, us);
        if (us != std::string::npos) g.memory_mode = rest.substr(us + 1);
      }
      std::string vram = gpu_label(labels, "vram");
      if (!vram.empty()) {
        // the labeller writes e.g. "288G" (decimal) or "288Gi"
        g.vram_per_gpu = parse_memory_bytes(vram);
        if (g.vram_per_gpu < 0) g.vram_per_gpu = 0;
      }
      out.push_back(g);
    }
  }
  return out;
}

std::string PodSizing::cpu_quantity() const {
  int m = cpu_milli();
  return m % 1000 == 0 ? std::to_string(m / 1000) : std::to_string(m) + "m";
}

const GpuNode* largest(const std::vector<GpuNode>& nodes) {
  const GpuNode* best = nullptr;
  for (auto& n : nodes)
    if (n.gpus > 0 && (best == nullptr || n.gpus > best->gpus)) best = &n;
  return best;
}

PodSizing size_pod(int gpus, const std::vector<GpuNode>& nodes) {
  PodSizing s;
  s.gpus = gpus;
  s.basis = "defaults";
  const GpuNode* best = largest(nodes);
  if (gpus <= 0 || best == nullptr) return s;
  // CPU and memory are shared by every device the node can schedule (all GPU resources)
  double devices = (double)std::max<int64_t>(best->gpus, best->node_devices);
  if (best->cpu > 0) {
    // 90 % of the node's allocatable CPUs, shared by its devices. Less than one CPU each (an 8-CPU
    // node with 8 GPUs, a 64-core node in CPX x64): the pod gets its share, never the whole node.
    double share = best->cpu * 0.9 / devices;
    s.cpu_per_gpu = std::max(1, (int)std::floor(share));
    if (share < 1.0) {
      double total = share * gpus;
      s.cpu_total_milli = total >= 1.0 ? (int)std::floor(total) * 1000 : std::max(100, (int)std::floor(total * 10) * 100);
      s.warning = strfmt("node %s has %.0f allocatable CPUs for %.0f devices (%.2f per device after 10 %% headroom): "
                         "requesting %s CPU for %d device(s); the ranks share fewer than one CPU each",
                         best->name.c_str(), best->cpu, devices, share, s.cpu_quantity().c_str(), gpus);
    }
  }
  if (best->memory > 0) {
    int per_gpu_gi = (int)(best->memory * 0.9 / devices / 1073741824.0);
    // keep shm at a quarter of the share when the node is small
    s.shm_per_gpu_gi = std::max(1, std::min(s.shm_per_gpu_gi, per_gpu_gi / 4));
    s.host_per_gpu_gi = std::max(1, per_gpu_gi - s.shm_per_gpu_gi);
  }
  s.product = best->product;
  s.resource = best->resource;
  s.hbm_per_device = best->hbm_per_device();
  if (best->parts() > 1 || !best->memory_mode.empty())
    s.partition = to_upper(best->compute_mode.empty() ? "spx" : best->compute_mode) +
                  (best->memory_mode.empty() ? "" : "/" + to_upper(best->memory_mode));
  s.basis = strfmt("node %s: %s, %.0f CPUs, %lld GiB allocatable", best->name.c_str(), best->describe().c_str(),
                   best->cpu, (long long)(best->memory / 1073741824LL));
  return s;
}

int64_t container_gpu_request(const Value& c) {
  int64_t n = 0;
  for (auto* part : {"limits", "requests"}) {
    const Value& res = c.at_path("resources").get(part);
    for (auto& k : res.keys())
      if (is_gpu_resource(k)) n += res.get(k).as_int(0);
    if (n > 0) return n;
  }
  return n;
}

std::string range_regex(int max) {
  std::string out;
  for (int i = 1; i <= std::max(1, max); ++i) out += (i > 1 ? "|" : "") + std::to_string(i);
  return "(" + out + ")";
}

std::string resources_yaml(const PodSizing& s) {
  if (s.gpus <= 0)
    return "      limits:\n"
           "        cpu: \"2\"\n"
           "        memory: \"4Gi\"\n"
           "        # AMD Instinct GPUs requested through the device plugin (amd.com/gpu)\n"
           "        gpu: 0";
  std::string cpu = s.cpu_quantity(), mem = std::to_string(s.memory_gi()) + "Gi";
  std::string hbm;
  if (s.hbm_per_device > 0 && !s.partition.empty())
    hbm = strfmt("      # HBM is not a schedulable resource: each %s device is a %s partition with an even\n"
                 "      # share of its GPU's HBM, %.0f GB (%.0f GB for the %d devices).\n",
                 s.resource.c_str(), s.partition.c_str(), s.hbm_per_device / 1e9, s.hbm_per_device * s.gpus / 1e9,
                 s.gpus);
  else if (s.hbm_per_device > 0)
    hbm = strfmt("      # HBM is not a schedulable resource: devices are requested whole, %.0f GB HBM each.\n",
                 s.hbm_per_device / 1e9);
  else
    hbm = "      # HBM is not a schedulable resource: GPUs are requested whole (an MI355X has 288 GB; a\n"
          "      # compute partition of one, DPX/QPX/CPX, an even share of it).\n";
  return strfmt(
      "      # MI355X sizing for %d device(s) (%s): %s CPUs and %d Gi host memory per device, i.e. a\n"
      "      # %d Gi memory-backed /dev/shm per rank (charged to this memory limit) + %d Gi per rank.\n"
      "%s"
      "      limits:\n"
      "        gpu: %d\n"
      "        cpu: \"%s\"\n"
      "        memory: \"%s\"\n"
      "      requests:\n"
      "        cpu: \"%s\"\n"
      "        memory: \"%s\"",
      s.gpus, s.basis.c_str(),
      (s.cpu_total_milli >= 0 ? strfmt("%.2f", s.cpu_milli() / 1000.0 / std::max(1, s.gpus)) : std::to_string(s.cpu_per_gpu))
          .c_str(),
      s.shm_per_gpu_gi + s.host_per_gpu_gi, s.shm_per_gpu_gi,
      s.host_per_gpu_gi, hbm.c_str(), s.gpus, cpu.c_str(), mem.c_str(), cpu.c_str(), mem.c_str());
}

std::string gpu_settings_yaml(const PodSizing& s) {
  if (s.gpus <= 0) return "";
  std::string out = strfmt(
      "  # /dev/shm (emptyDir medium: Memory) per GPU, in Gi; host memory budget per rank, in Gi\n"
      "  shmPerGPU: %d\n"
      "  hostMemoryPerGPU: %d\n",
      s.shm_per_gpu_gi, s.host_per_gpu_gi);
  if (s.resource != "amd.com/gpu")
    out += "  # the device plugin's mixed strategy advertises partitions under their own resource name\n"
           "  gpuResource: \"" + s.resource + "\"\n";
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
    int64_t gpus = container_gpu_request(c);
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

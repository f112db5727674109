// MI355X pod sizing policy (SURVEY.md §7.5 "MI355X-node-aware features").
//
// HBM (288 GB per MI355X) is not a schedulable Kubernetes resource: a GPU pod asks for devices
// (amd.com/gpu via the AMD device plugin: whole GPUs, or compute partitions of them) plus host CPU
// and memory. Those must grow with
// the GPU count: one training process per GPU, RCCL's intra-node transport and PyTorch
// dataloaders in a memory-backed /dev/shm that is charged to the container's memory cgroup.
// The reference chart had a fixed resource block per container
// (/root/reference/examples/quickstart/chart/templates/deployments.yaml:63-82).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "core/value.h"

namespace ds {
namespace gpu {

// Kubernetes resource quantities ("500m", "16", "64Gi", "1.5G", "1e3").
double parse_cpu(const std::string& q);            // cores
int64_t parse_memory_bytes(const std::string& q);  // bytes; -1 when unparsable

// The AMD GPU device plugin advertises one schedulable device per GPU (SPX) or per compute
// partition: an MI355X in DPX/QPX/CPX mode is 2/4/8 devices (one per XCD group), so a node of 8
// MI355X in CPX mode advertises 64. With the "single" resource strategy every device is
// `amd.com/gpu`; with "mixed" each partition type is its own resource, `amd.com/<cpx>_<nps2>`.
// The node labeller labels the node with the product, the VRAM per GPU and the partition modes.
bool is_gpu_resource(const std::string& name);  // amd.com/gpu or amd.com/{spx,dpx,qpx,cpx}[_npsN]
int partitions_per_gpu(const std::string& compute_mode);  // spx 1, dpx 2, qpx 4, cpx 8; 0 unknown

struct GpuNode {
  std::string name;
  std::string resource = "amd.com/gpu";  // the resource name the devices are advertised under
  int64_t gpus = 0;          // status.allocatable[resource]: schedulable devices
  int64_t capacity = 0;      // status.capacity[resource]; > gpus when the plugin marked some unhealthy
  int64_t node_devices = 0;  // allocatable devices of every GPU resource on the node (CPU/memory share)
  double cpu = 0;            // allocatable cores
  int64_t memory = 0;        // allocatable bytes
  std::string product;       // amd.com/gpu.product-name (AMD GPU operator node labeller)
  std::string compute_mode;  // spx | dpx | qpx | cpx ("" unknown)
  std::string memory_mode;   // nps1 | nps2 | ... ("" unknown)
  int64_t vram_per_gpu = 0;  // bytes of HBM per physical GPU (amd.com/gpu.vram, else the product's)
  int64_t unhealthy() const { return capacity > gpus ? capacity - gpus : 0; }
  int parts() const;  // schedulable devices per physical GPU (1 unless a partition mode is known)
  int64_t hbm_per_device() const;  // even share of a GPU's HBM per device (0 unknown)
  std::string describe() const;  // "8 x AMD_Instinct_MI355X, CPX/NPS2: 64 devices of 36 GB HBM"
};
// GPU resources of the nodes, one entry per (node, GPU resource), from a NodeList's items.
std::vector<GpuNode> gpu_nodes(const Value& node_list);
// The entry with the most schedulable devices (a pod must fit on one node); nullptr when none.
const GpuNode* largest(const std::vector<GpuNode>& nodes);
int64_t hbm_of_product(const std::string& product);  // bytes per GPU, 0 unknown

struct PodSizing {
  int gpus = 0;               // schedulable devices requested (whole GPUs in SPX, partitions otherwise)
  int cpu_per_gpu = 12;       // default: 2 x 64-core EPYC hosts with 8 GPUs, leaving system headroom
  int shm_per_gpu_gi = 16;    // memory-backed /dev/shm per rank
  int host_per_gpu_gi = 64;   // host RSS budget per rank (interpreter, pinned buffers, dataloader)
  std::string product;        // node selector value when the nodes advertise one
  std::string resource = "amd.com/gpu";
  std::string partition;      // "CPX/NPS2" when the node runs partitioned GPUs
  int64_t hbm_per_device = 0; // bytes; 0 unknown (then: a whole MI355X, 288 GB)
  std::string basis;          // "defaults" | "node <name>: ..."
  // The pod's CPU request in millicores when the node has less than one CPU per device to give
  // (-1: gpus x cpu_per_gpu whole CPUs), and why, for `init` to say so.
  int cpu_total_milli = -1;
  std::string warning;
  int cpu_milli() const { return cpu_total_milli >= 0 ? cpu_total_milli : gpus * cpu_per_gpu * 1000; }
  // Kubernetes quantity of cpu_milli(): "112", "7", "900m"
  std::string cpu_quantity() const;
  int memory_gi() const { return gpus * (shm_per_gpu_gi + host_per_gpu_gi); }
  int shm_gi() const { return gpus * shm_per_gpu_gi; }
};

// Per-device defaults, or a per-device share (90 %) of the allocatable CPU and memory of the GPU
// node with the most schedulable devices when nodes are known (CPX: a 64th of an 8-GPU node).
PodSizing size_pod(int gpus, const std::vector<GpuNode>& nodes = {});

// values.yaml fragments for `devspace init` (#resources# / #gpu-settings# placeholders).
std::string resources_yaml(const PodSizing& s);  // indented for components[].containers[].resources
std::string gpu_settings_yaml(const PodSizing& s);  // indented for components[]

// Problems of a pod spec as scheduled on a GPU node: shm sizeLimit >= memory limit, fewer CPUs
// than ranks, no memory limit at all. Empty when fine.
std::vector<std::string> pod_sizing_problems(const Value& pod_spec);

// GPU devices a container requests: limits (else requests) of every GPU resource.
int64_t container_gpu_request(const Value& container);

// Anchored regex accepting the integers 1..max (the init prompt's bound).
std::string range_regex(int max);

}  // namespace gpu
}  // namespace ds

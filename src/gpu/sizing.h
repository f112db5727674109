// MI355X pod sizing policy (SURVEY.md §7.5 "MI355X-node-aware features").
//
// HBM (288 GB per MI355X) is not a schedulable Kubernetes resource: a GPU pod asks for whole
// GPUs (amd.com/gpu via the AMD device plugin) plus host CPU and memory. Those must grow with
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

struct GpuNode {
  std::string name;
  int64_t gpus = 0;        // status.allocatable["amd.com/gpu"]
  double cpu = 0;          // allocatable cores
  int64_t memory = 0;      // allocatable bytes
  std::string product;     // amd.com/gpu.product-name (AMD GPU operator node labeller)
};
// Nodes that advertise amd.com/gpu, from a NodeList's items.
std::vector<GpuNode> gpu_nodes(const Value& node_list);

struct PodSizing {
  int gpus = 0;
  int cpu_per_gpu = 12;       // default: 2 x 64-core EPYC hosts with 8 GPUs, leaving system headroom
  int shm_per_gpu_gi = 16;    // memory-backed /dev/shm per rank
  int host_per_gpu_gi = 64;   // host RSS budget per rank (interpreter, pinned buffers, dataloader)
  std::string product;        // node selector value when the nodes advertise one
  std::string basis;          // "defaults" | "node <name>: ..."
  int cpu() const { return gpus * cpu_per_gpu; }
  int memory_gi() const { return gpus * (shm_per_gpu_gi + host_per_gpu_gi); }
  int shm_gi() const { return gpus * shm_per_gpu_gi; }
};

// Per-GPU defaults, or a per-GPU share (90 %) of the allocatable CPU and memory of the GPU
// node type with the most GPUs when nodes are known.
PodSizing size_pod(int gpus, const std::vector<GpuNode>& nodes = {});

// values.yaml fragments for `devspace init` (#resources# / #gpu-settings# placeholders).
std::string resources_yaml(const PodSizing& s);  // indented for components[].containers[].resources
std::string gpu_settings_yaml(const PodSizing& s);  // indented for components[]

// Problems of a pod spec as scheduled on a GPU node: shm sizeLimit >= memory limit, fewer CPUs
// than ranks, no memory limit at all. Empty when fine.
std::vector<std::string> pod_sizing_problems(const Value& pod_spec);

}  // namespace gpu
}  // namespace ds

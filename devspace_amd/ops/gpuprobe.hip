// GPU health / sizing probe for MI355X dev pods (gfx950, CDNA4).
//
// `devspace analyze` (reference: pkg/devspace/analyze) reports why a pod is unhealthy; for
// GPU pods the question "did this pod get a working, full-speed MI355X?" needs a device-side
// answer: a scheduling success with a wedged/throttled GPU, a missing /dev/kfd or a wrong
// HIP_VISIBLE_DEVICES still looks "Running" to Kubernetes. This library measures, per device:
//   * MFMA correctness: one 32x32x16 bf16 tile against an exact host reference (identity A,
//     asymmetric B so a row/col swap cannot pass),
//   * HBM3E streaming bandwidth: float4 grid-stride copy, >>256 workgroups,
//   * dense bf16 MFMA throughput: register-resident v_mfma_f32_32x32x16_bf16 chains with
//     independent accumulators (one wave per SIMD class of measurement).
// Exposed through a C ABI and loaded with ctypes by devspace_amd/gpucheck.py.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::snprintf(g_err, sizeof(g_err), "%s failed: %s", #x, hipGetErrorString(e_)); \
      return -1;                                                                      \
    }                                                                                 \
  } while (0)

static char g_err[512];

// ------------------------------------------------------------------ kernels

// One wave: D(32x32) = A(32x16) * B(16x32) with the gfx950 bf16 fragment maps
// (lane l: r = l&31, h = l>>5 holds A[r][8h+j], B[8h+j][r]; D col = l&31,
// row = (reg&3) + 8*(reg>>2) + 4*h).
__global__ void __launch_bounds__(64) mfma_tile_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                       float* __restrict__ D) {
  const int l = threadIdx.x;
  const int r = l & 31, h = l >> 5;
  bf16x8 a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = (__bf16)A[r * 16 + 8 * h + j];
    b[j] = (__bf16)B[(8 * h + j) * 32 + r];
  }
  f32x16 acc = {};
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) {
    int row = (reg & 3) + 8 * (reg >> 2) + 4 * h;
    D[row * 32 + r] = acc[reg];
  }
}

// Streaming copy: 16-byte vectors (global_load/store_dwordx4), grid-stride, U independent
// vectors in flight per lane before the first store (keeps ~U*4 KiB of HBM reads outstanding
// per wave), nontemporal hints so the one-touch stream does not thrash L2/MALL.
template <int U, bool NT>
__global__ void __launch_bounds__(256) copy_kernel(const f32x4* __restrict__ src, f32x4* __restrict__ dst, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(&src[i + u * stride]) : src[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT)
        __builtin_nontemporal_store(v[u], &dst[i + u * stride]);
      else
        dst[i + u * stride] = v[u];
    }
  }
  for (; i < n; i += stride) dst[i] = src[i];
}

using copy_fn = void (*)(const f32x4*, f32x4*, size_t);
static copy_fn pick_copy(int unroll, int nt) {
  switch (unroll * 2 + (nt ? 1 : 0)) {
    case 2: return copy_kernel<1, false>;
    case 3: return copy_kernel<1, true>;
    case 4: return copy_kernel<2, false>;
    case 5: return copy_kernel<2, true>;
    case 8: return copy_kernel<4, false>;
    case 9: return copy_kernel<4, true>;
    case 16: return copy_kernel<8, false>;
    case 17: return copy_kernel<8, true>;
    default: return nullptr;
  }
}

// Register-resident MFMA chain: 4 independent accumulators per wave hide the MFMA latency.
__global__ void __launch_bounds__(256) mfma_rate_kernel(float* __restrict__ out, int iters, float seed) {
  bf16x8 a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = (__bf16)(seed + 0.001f * (threadIdx.x + j));
    b[j] = (__bf16)(seed - 0.002f * j);
  }
  f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  for (int it = 0; it < iters; ++it) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c3, 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
  if (s == 1234.5678f) out[blockIdx.x] = s;  // practically never true; keeps the chain live
}

// ------------------------------------------------------------------ C ABI

extern "C" {

const char* gp_last_error() { return g_err; }

int gp_device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// Writes a JSON object describing device `dev`.
int gp_device_info(int dev, char* buf, int cap) {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, dev));
  size_t free_b = 0, total_b = 0;
  CHECK(hipSetDevice(dev));
  CHECK(hipMemGetInfo(&free_b, &total_b));
  std::snprintf(buf, cap,
                "{\"index\": %d, \"name\": \"%s\", \"arch\": \"%s\", \"compute_units\": %d, "
                "\"clock_mhz\": %d, \"hbm_total_bytes\": %zu, \"hbm_free_bytes\": %zu, \"pci_bus\": %d, "
                "\"lds_per_cu_bytes\": %zu, \"warp_size\": %d}",
                dev, p.name, p.gcnArchName, p.multiProcessorCount, p.clockRate / 1000, total_b, free_b, p.pciBusID,
                (size_t)p.maxSharedMemoryPerMultiProcessor, p.warpSize);
  return 0;
}

// Returns max |D - A*B| for one MFMA tile (0.0 on a healthy device), or -1 on error.
double gp_mfma_selftest(int dev) {
  if (hipSetDevice(dev) != hipSuccess) return -1;
  std::vector<float> A(32 * 16, 0.f), B(16 * 32), D(32 * 32, -1.f);
  for (int i = 0; i < 16; ++i) A[i * 16 + i] = 1.f;  // identity on the first 16 rows
  for (int k = 0; k < 16; ++k)
    for (int j = 0; j < 32; ++j) B[k * 32 + j] = (float)((k * 7 + j * 3) % 64 - 17);  // asymmetric, bf16-exact
  float *dA, *dB, *dD;
  if (hipMalloc(&dA, A.size() * 4) || hipMalloc(&dB, B.size() * 4) || hipMalloc(&dD, D.size() * 4)) return -1;
  hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(mfma_tile_kernel, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
  hipFree(dA);
  hipFree(dB);
  hipFree(dD);
  double err = 0;
  for (int i = 0; i < 32; ++i)
    for (int j = 0; j < 32; ++j) {
      double want = i < 16 ? B[i * 32 + j] : 0.0;
      double d = D[i * 32 + j] - want;
      err = std::max(err, d < 0 ? -d : d);
    }
  return err;
}

// HBM copy bandwidth in GB/s for one kernel configuration (used by the tuning sweep).
double gp_hbm_copy_gbps_cfg(int dev, size_t bytes, int iters, int unroll, int nontemporal, int blocks_per_cu) {
  copy_fn fn = pick_copy(unroll, nontemporal);
  if (!fn || blocks_per_cu < 1 || hipSetDevice(dev) != hipSuccess) return -1;
  size_t n = bytes / sizeof(f32x4);
  f32x4 *src = nullptr, *dst = nullptr;
  if (hipMalloc(&src, n * sizeof(f32x4)) != hipSuccess) return -1;
  if (hipMalloc(&dst, n * sizeof(f32x4)) != hipSuccess) {
    hipFree(src);
    return -1;
  }
  hipMemset(src, 1, n * sizeof(f32x4));
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, dev);
  dim3 grid(p.multiProcessorCount * blocks_per_cu), block(256);
  hipLaunchKernelGGL(fn, grid, block, 0, 0, src, dst, n);  // warm-up
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(fn, grid, block, 0, 0, src, dst, n);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  hipFree(src);
  hipFree(dst);
  if (ms <= 0) return -1;
  return (2.0 * (double)n * sizeof(f32x4) * iters) / (ms * 1e-3) / 1e9;
}

// HBM copy bandwidth in GB/s (bytes read + written per second), default configuration.
// Tuned on MI355X (profiles/r1_hbm_copy_sweep.txt): 2 x dwordx4 in flight per lane,
// nontemporal, 2 workgroups of 256 per CU -> 6.0 TB/s (95% of the 6.3 TB/s achievable copy);
// more resident waves (8-16 WG/CU) thrash the HBM channels and drop to 4.3-5.2 TB/s.
double gp_hbm_copy_gbps(int dev, size_t bytes, int iters) {
  return gp_hbm_copy_gbps_cfg(dev, bytes, iters, 2, 1, 2);
}

// Dense bf16 MFMA rate in TFLOP/s.
double gp_mfma_bf16_tflops(int dev, int iters) {
  if (hipSetDevice(dev) != hipSuccess) return -1;
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, dev);
  float* out;
  if (hipMalloc(&out, 1 << 20) != hipSuccess) return -1;
  // 4 waves per block (one per SIMD), 2 blocks per CU
  dim3 grid(p.multiProcessorCount * 2), block(256);
  hipLaunchKernelGGL(mfma_rate_kernel, grid, block, 0, 0, out, 64, 1.0f);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(mfma_rate_kernel, grid, block, 0, 0, out, iters, 1.0f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  hipFree(out);
  if (ms <= 0) return -1;
  double waves = (double)grid.x * (block.x / 64);
  double flops = waves * iters * 4.0 * (2.0 * 32 * 32 * 16);
  return flops / (ms * 1e-3) / 1e12;
}

// 1 when device `a` can map device `b`'s memory (peer access over xGMI), 0 when not, -1 on error.
int gp_peer_access(int a, int b) {
  int ok = 0;
  if (hipDeviceCanAccessPeer(&ok, a, b) != hipSuccess) return -1;
  return ok ? 1 : 0;
}

// Device a -> device b copy bandwidth in GB/s (hipMemcpyPeerAsync on a stream of device a, peer
// access enabled both ways when possible), or -1 on error. On MI355X nodes this is an xGMI
// link; a pair far below the others is a degraded link or a copy staged through the host.
double gp_peer_copy_gbps(int a, int b, size_t bytes, int iters) {
  if (a == b || iters < 1 || bytes == 0) return -1;
  void *src = nullptr, *dst = nullptr;
  if (hipSetDevice(b) != hipSuccess || hipMalloc(&dst, bytes) != hipSuccess) return -1;
  int can = 0;
  hipDeviceCanAccessPeer(&can, b, a);
  if (can) hipDeviceEnablePeerAccess(a, 0);  // hipErrorPeerAccessAlreadyEnabled is fine
  (void)hipGetLastError();
  if (hipSetDevice(a) != hipSuccess || hipMalloc(&src, bytes) != hipSuccess) {
    hipSetDevice(b);
    hipFree(dst);
    return -1;
  }
  hipDeviceCanAccessPeer(&can, a, b);
  if (can) hipDeviceEnablePeerAccess(b, 0);
  (void)hipGetLastError();
  hipMemset(src, 1, bytes);
  hipStream_t st;
  hipEvent_t e0, e1;
  double gbps = -1;
  if (hipStreamCreate(&st) == hipSuccess) {
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipMemcpyPeerAsync(dst, b, src, a, bytes, st);  // warm-up (first touch, link training)
    hipEventRecord(e0, st);
    for (int i = 0; i < iters; ++i) hipMemcpyPeerAsync(dst, b, src, a, bytes, st);
    hipEventRecord(e1, st);
    if (hipEventSynchronize(e1) == hipSuccess) {
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms > 0) gbps = (double)bytes * iters / (ms * 1e-3) / 1e9;
    }
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    hipStreamDestroy(st);
  }
  hipFree(src);
  hipSetDevice(b);
  hipFree(dst);
  return gbps;
}

}  // extern "C"

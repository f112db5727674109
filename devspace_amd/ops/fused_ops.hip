// Fused training ops for MI355X dev-pod workloads (gfx950 / CDNA4, wave64), as a PyTorch
// extension: the hot non-GEMM ops of the rocm-pytorch example's training step
// (examples/rocm-pytorch/train.py), each one HBM pass instead of PyTorch's op chain.
//
//   rmsnorm_fwd / rmsnorm_bwd   y = x * rsqrt(mean(x^2) + eps) * w       (one wave per row)
//   swiglu_fwd / swiglu_bwd     y = silu(g) * u on h = [g | u]            (gate+up in one buffer:
//                               backward writes dh directly, no chunk/cat copies)
//   ce_fwd / ce_bwd             mean cross-entropy on bf16 logits          (online max/sum-exp per
//                               row in fp32, lse kept for the backward; no fp32 logits copy)
//
// Layout / design (cdna_hip_programming.md §6): every global access is a 16-byte vector
// (8 bf16 per lane, global_load/store_dwordx4) except SwiGLU rows whose width is not a
// multiple of 8 (bf16x2); row reductions are wave64 shuffles, block reductions go through
// LDS; math in fp32, one bf16 rounding per output (v_cvt_pk_bf16_f32). The reductions over
// rows (RMSNorm weight gradient, loss mean) are two-level (per-block partials + one column /
// block reduce kernel) instead of float atomics, so results are deterministic.
//
// Reference parity: this is workload-side code (the tool itself has no
// numeric path); numerics are tested against fp32 PyTorch in tests/test_fused_ops.py.
#include <hip/hip_runtime.h>
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <cmath>
#include <cstdint>

namespace {

typedef unsigned short u16;
template <int N>
using u16v = u16 __attribute__((ext_vector_type(N)));
typedef u16v<8> u16x8;

constexpr int kBlock = 256;  // 4 waves

__device__ __forceinline__ float b2f(u16 v) { return __uint_as_float((unsigned)v << 16); }
__device__ __forceinline__ u16 f2b(float f) {
  __bf16 b = (__bf16)f;  // v_cvt_pk_bf16_f32: RNE, NaN stays NaN
  return __builtin_bit_cast(u16, b);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// (m, s) pairs of an online log-sum-exp: s = sum exp(x - m)
__device__ __forceinline__ void lse_combine(float& m, float& s, float m2, float s2) {
  float M = fmaxf(m, m2);
  if (M == -INFINITY) return;
  s = s * __expf(m - M) + s2 * __expf(m2 - M);
  m = M;
}

__device__ __forceinline__ void wave_lse(float& m, float& s) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    lse_combine(m, s, m2, s2);
  }
}

// ------------------------------------------------------------------------------ RMSNorm

// One wave per row; lane l owns 16-byte vectors l, l+64, ... (VPL of them, the last ones
// masked when D/8 is not a multiple of 64) and keeps them in registers between the sum of
// squares and the scaled store, so x is read once.
template <int VPL>
__global__ void __launch_bounds__(kBlock) rmsnorm_fwd_kernel(const u16* __restrict__ x, const u16* __restrict__ w,
                                                            u16* __restrict__ y, float* __restrict__ rstd, int R,
                                                            int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const int nvec = D >> 3;
  const u16x8* xr = reinterpret_cast<const u16x8*>(x + (size_t)row * D);
  u16x8 v[VPL];
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
    const int i = lane + 64 * k;
    if (i < nvec) {
      v[k] = xr[i];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float f = b2f(v[k][j]);
        ss += f * f;
      }
    }
  }
  ss = wave_sum(ss);
  const float r = rsqrtf(ss / (float)D + eps);
  if (lane == 0) rstd[row] = r;
  const u16x8* wr = reinterpret_cast<const u16x8*>(w);
  u16x8* yr = reinterpret_cast<u16x8*>(y + (size_t)row * D);
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
    const int i = lane + 64 * k;
    if (i < nvec) {
      u16x8 wv = wr[i], o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2b(b2f(v[k][j]) * r * b2f(wv[j]));
      yr[i] = o;
    }
  }
}

// dx = r * (w*dy) - x * r^3 / D * sum(w*dy*x);  dw partial = sum_rows dy * x * r.
// A block owns `rows_per_block` consecutive rows (its 4 waves stride over them); each lane
// accumulates the weight-gradient of its columns in registers, the 4 waves are summed through
// LDS and the block writes one fp32 partial row (reduced by col_sum_kernel).
template <int VPL>
__global__ void __launch_bounds__(kBlock) rmsnorm_bwd_kernel(const u16* __restrict__ dy, const u16* __restrict__ x,
                                                            const u16* __restrict__ w, const float* __restrict__ rstd,
                                                            u16* __restrict__ dx, float* __restrict__ dw_part, int R,
                                                            int D, int rows_per_block) {
  extern __shared__ float sdw[];  // [4][D]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nvec = D >> 3;
  const u16x8* wr = reinterpret_cast<const u16x8*>(w);
  u16x8 wv[VPL];
  float acc[VPL][8];
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
    const int i = lane + 64 * k;
    if (i < nvec) wv[k] = wr[i];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[k][j] = 0.f;
  }
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(R, r0 + rows_per_block);
  const float inv_d = 1.0f / (float)D;
  // 2-deep software pipeline: the next row's dy/x loads are in flight while this row is
  // reduced and written (one row per wave step is a dependent load -> reduce -> store chain).
  u16x8 gv[VPL], xv[VPL];
  int row = r0 + wave;
  if (row < r1) {
    const u16x8* dyr = reinterpret_cast<const u16x8*>(dy + (size_t)row * D);
    const u16x8* xr = reinterpret_cast<const u16x8*>(x + (size_t)row * D);
#pragma unroll
    for (int k = 0; k < VPL; ++k) {
      const int i = lane + 64 * k;
      if (i < nvec) {
        gv[k] = dyr[i];
        xv[k] = xr[i];
      }
    }
  }
  for (; row < r1; row += 4) {
    const int nrow = row + 4;
    u16x8 gn[VPL], xn[VPL];
    if (nrow < r1) {
      const u16x8* dyr = reinterpret_cast<const u16x8*>(dy + (size_t)nrow * D);
      const u16x8* xr = reinterpret_cast<const u16x8*>(x + (size_t)nrow * D);
#pragma unroll
      for (int k = 0; k < VPL; ++k) {
        const int i = lane + 64 * k;
        if (i < nvec) {
          gn[k] = dyr[i];
          xn[k] = xr[i];
        }
      }
    }
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < VPL; ++k) {
      const int i = lane + 64 * k;
      if (i < nvec) {
#pragma unroll
        for (int j = 0; j < 8; ++j) dot += b2f(gv[k][j]) * b2f(wv[k][j]) * b2f(xv[k][j]);
      }
    }
    dot = wave_sum(dot);
    const float r = rstd[row];
    const float c = dot * r * r * r * inv_d;
    u16x8* dxr = reinterpret_cast<u16x8*>(dx + (size_t)row * D);
#pragma unroll
    for (int k = 0; k < VPL; ++k) {
      const int i = lane + 64 * k;
      if (i < nvec) {
        u16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float g = b2f(gv[k][j]), xf = b2f(xv[k][j]);
          o[j] = f2b(r * g * b2f(wv[k][j]) - xf * c);
          acc[k][j] += g * xf * r;
        }
        dxr[i] = o;
      }
    }
#pragma unroll
    for (int k = 0; k < VPL; ++k) {
      gv[k] = gn[k];
      xv[k] = xn[k];
    }
  }
  float* mine = sdw + wave * D;
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
    const int i = lane + 64 * k;
    if (i < nvec) {
#pragma unroll
      for (int j = 0; j < 8; ++j) mine[i * 8 + j] = acc[k][j];
    }
  }
  __syncthreads();
  float* part = dw_part + (size_t)blockIdx.x * D;
  for (int c = threadIdx.x; c < D; c += kBlock) part[c] = sdw[c] + sdw[D + c] + sdw[2 * D + c] + sdw[3 * D + c];
}

// out[c] = bf16(sum_r part[r][c]). 32 columns per 1024-thread block: each half-wave reads 32
// consecutive floats of one partial row, 32 row groups in flight, LDS combine.
__global__ void __launch_bounds__(1024) col_sum_kernel(const float* __restrict__ part, int nrows, int D,
                                                      u16* __restrict__ out) {
  __shared__ float red[32][33];
  const int cl = threadIdx.x & 31, g = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  float s0 = 0.f, s1 = 0.f;
  if (c < D) {
    int r = g;
    for (; r + 32 < nrows; r += 64) {
      s0 += part[(size_t)r * D + c];
      s1 += part[(size_t)(r + 32) * D + c];
    }
    for (; r < nrows; r += 32) s0 += part[(size_t)r * D + c];
  }
  red[g][cl] = s0 + s1;
  __syncthreads();
  if (threadIdx.x < 32 && c < D) {
    float t = 0.f;
#pragma unroll 8
    for (int k = 0; k < 32; ++k) t += red[k][cl];
    out[c] = f2b(t);
  }
}

// ------------------------------------------------------------------------------ SwiGLU

// One block per row of h = [g | u] (width 2H); V bf16 per access (8 when H % 8 == 0, else 2).
template <int V>
__global__ void __launch_bounds__(kBlock) swiglu_fwd_kernel(const u16* __restrict__ h, u16* __restrict__ y, int H) {
  const size_t row = blockIdx.x;
  const u16* hg = h + row * 2 * H;
  const u16* hu = hg + H;
  u16* yr = y + row * H;
  for (int c = threadIdx.x * V; c < H; c += kBlock * V) {
    u16v<V> g = *reinterpret_cast<const u16v<V>*>(hg + c);
    u16v<V> u = *reinterpret_cast<const u16v<V>*>(hu + c);
    u16v<V> o;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const float gf = b2f(g[j]);
      o[j] = f2b(gf / (1.0f + __expf(-gf)) * b2f(u[j]));
    }
    *reinterpret_cast<u16v<V>*>(yr + c) = o;
  }
}

template <int V>
__global__ void __launch_bounds__(kBlock) swiglu_bwd_kernel(const u16* __restrict__ dy, const u16* __restrict__ h,
                                                           u16* __restrict__ dh, int H) {
  const size_t row = blockIdx.x;
  const u16* hg = h + row * 2 * H;
  const u16* hu = hg + H;
  const u16* dyr = dy + row * H;
  u16* dg = dh + row * 2 * H;
  u16* du = dg + H;
  for (int c = threadIdx.x * V; c < H; c += kBlock * V) {
    u16v<V> g = *reinterpret_cast<const u16v<V>*>(hg + c);
    u16v<V> u = *reinterpret_cast<const u16v<V>*>(hu + c);
    u16v<V> d = *reinterpret_cast<const u16v<V>*>(dyr + c);
    u16v<V> og, ou;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const float gf = b2f(g[j]), uf = b2f(u[j]), df = b2f(d[j]);
      const float s = 1.0f / (1.0f + __expf(-gf));
      const float silu = gf * s;
      ou[j] = f2b(df * silu);
      og[j] = f2b(df * uf * s * (1.0f + gf * (1.0f - s)));
    }
    *reinterpret_cast<u16v<V>*>(dg + c) = og;
    *reinterpret_cast<u16v<V>*>(du + c) = ou;
  }
}

// ------------------------------------------------------------------------------ cross-entropy

// One block per row: online (max, sum-exp) over 16-byte vectors, wave64 shuffle combine,
// then the 4 waves through LDS. Writes lse[row] and loss[row] (0 for ignore_index).
__global__ void __launch_bounds__(kBlock) ce_fwd_kernel(const u16* __restrict__ logits, const int64_t* __restrict__ tgt,
                                                       float* __restrict__ lse_out, float* __restrict__ loss_out, int V,
                                                       int64_t ignore_index) {
  __shared__ float sm[4], ss[4];
  const size_t row = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const u16x8* lr = reinterpret_cast<const u16x8*>(logits + row * V);
  const int nvec = V >> 3;
  float m = -INFINITY, s = 0.f;
  for (int i = threadIdx.x; i < nvec; i += kBlock) {
    u16x8 v = lr[i];
    float f[8], mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      f[j] = b2f(v[j]);
      mx = fmaxf(mx, f[j]);
    }
    if (mx > m) {
      s = (m == -INFINITY) ? 0.f : s * __expf(m - mx);
      m = mx;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) s += __expf(f[j] - m);
  }
  wave_lse(m, s);
  if (lane == 0) {
    sm[wave] = m;
    ss[wave] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0], S = ss[0];
    for (int k = 1; k < 4; ++k) lse_combine(M, S, sm[k], ss[k]);
    const float lse = M + __logf(S);
    lse_out[row] = lse;
    const int64_t t = tgt[row];
    loss_out[row] = (t == ignore_index || t < 0 || t >= V) ? 0.f : lse - b2f(logits[row * V + t]);
  }
}

// Single block: out[0] = sum(loss) / count(valid targets), out[1] = count (fp32).
__global__ void __launch_bounds__(1024) ce_mean_kernel(const float* __restrict__ loss, const int64_t* __restrict__ tgt,
                                                      int R, int64_t ignore_index, float* __restrict__ out) {
  __shared__ float sl[16], sc[16];
  float l = 0.f, c = 0.f;
  for (int r = threadIdx.x; r < R; r += 1024) {
    l += loss[r];
    c += tgt[r] == ignore_index ? 0.f : 1.f;
  }
  l = wave_sum(l);
  c = wave_sum(c);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    sl[wave] = l;
    sc[wave] = c;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float L = 0.f, C = 0.f;
    for (int k = 0; k < 16; ++k) {
      L += sl[k];
      C += sc[k];
    }
    out[0] = L / C;
    out[1] = C;
  }
}

// dlogits = (softmax(logits) - onehot(t)) * grad / count, recomputed from lse (one read of
// the logits, one bf16 write).
__global__ void __launch_bounds__(kBlock) ce_bwd_kernel(const u16* __restrict__ logits, const int64_t* __restrict__ tgt,
                                                       const float* __restrict__ lse, const float* __restrict__ grad,
                                                       const float* __restrict__ stats, u16* __restrict__ dlogits,
                                                       int V, int64_t ignore_index) {
  const size_t row = blockIdx.x;
  const int64_t t = tgt[row];
  const bool valid = !(t == ignore_index || t < 0 || t >= V);
  const float scale = valid ? grad[0] / stats[1] : 0.f;
  const float l = lse[row];
  const u16x8* lr = reinterpret_cast<const u16x8*>(logits + row * V);
  u16x8* dr = reinterpret_cast<u16x8*>(dlogits + row * V);
  const int nvec = V >> 3;
  for (int i = threadIdx.x; i < nvec; i += kBlock) {
    u16x8 v = lr[i], o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float g = __expf(b2f(v[j]) - l) * scale;
      if (i * 8 + j == t) g -= scale;
      o[j] = f2b(g);
    }
    dr[i] = o;
  }
}

// ------------------------------------------------------------------------------ AdamW

// Multi-tensor AdamW (decoupled weight decay) on bf16 params / grads / moments, fp32 math:
// one launch updates up to kMaxT tensors; the tensor table travels in the kernel arguments
// (grad pointers change every step with zero_grad(set_to_none=True), so nothing is cached on
// the device). Each block owns kChunk elements of one tensor; 16-byte vectors, scalar tail.
constexpr int kMaxT = 48;
constexpr int kChunk = kBlock * 8 * 4;  // 8192 elements per block

struct AdamTable {
  u16* p[kMaxT];
  const u16* g[kMaxT];
  u16* m[kMaxT];
  u16* v[kMaxT];
  int64_t n[kMaxT];
  int blk_start[kMaxT + 1];
  int nt;
};

struct AdamScalars {
  float lr, b1, b2, eps, decay, step_size, bc2_sqrt;
};

__device__ __forceinline__ void adam_elem(float& p, float& m, float& v, float g, const AdamScalars& s) {
  p *= s.decay;
  m = s.b1 * m + (1.0f - s.b1) * g;
  v = s.b2 * v + (1.0f - s.b2) * g * g;
  p -= s.step_size * m / (sqrtf(v) / s.bc2_sqrt + s.eps);
}

__global__ void __launch_bounds__(kBlock) adamw_kernel(AdamTable t, AdamScalars s) {
  const int b = blockIdx.x;
  int ti = 0;
  while (ti + 1 < t.nt && t.blk_start[ti + 1] <= b) ++ti;
  const int64_t n = t.n[ti];
  const int64_t base = (int64_t)(b - t.blk_start[ti]) * kChunk;
  const int64_t end = min(n, base + (int64_t)kChunk);
  u16* P = t.p[ti];
  const u16* G = t.g[ti];
  u16* M = t.m[ti];
  u16* V = t.v[ti];
  for (int64_t e = base + threadIdx.x * 8; e < end; e += kBlock * 8) {
    if (e + 8 <= end) {
      u16x8 pv = *reinterpret_cast<const u16x8*>(P + e), gv = *reinterpret_cast<const u16x8*>(G + e);
      u16x8 mv = *reinterpret_cast<const u16x8*>(M + e), vv = *reinterpret_cast<const u16x8*>(V + e);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float pf = b2f(pv[j]), mf = b2f(mv[j]), vf = b2f(vv[j]);
        adam_elem(pf, mf, vf, b2f(gv[j]), s);
        pv[j] = f2b(pf);
        mv[j] = f2b(mf);
        vv[j] = f2b(vf);
      }
      *reinterpret_cast<u16x8*>(P + e) = pv;
      *reinterpret_cast<u16x8*>(M + e) = mv;
      *reinterpret_cast<u16x8*>(V + e) = vv;
    } else {
      for (int64_t i = e; i < end; ++i) {
        float pf = b2f(P[i]), mf = b2f(M[i]), vf = b2f(V[i]);
        adam_elem(pf, mf, vf, b2f(G[i]), s);
        P[i] = f2b(pf);
        M[i] = f2b(mf);
        V[i] = f2b(vf);
      }
    }
  }
}

// ------------------------------------------------------------------------------ host side

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_bf16(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, name, " must be bfloat16");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
}

#define LAUNCH_CHECK()                                                                         \
  do {                                                                                         \
    hipError_t e_ = hipGetLastError();                                                         \
    TORCH_CHECK(e_ == hipSuccess, "HIP launch failed: ", hipGetErrorString(e_));               \
  } while (0)

int vpl_for(int D) {
  const int nvec = D / 8;
  const int vpl = (nvec + 63) / 64;
  return vpl <= 1 ? 1 : vpl <= 2 ? 2 : vpl <= 4 ? 4 : vpl <= 8 ? 8 : -1;
}

bool rmsnorm_supported(int64_t D) { return D % 8 == 0 && D >= 8 && vpl_for((int)D) > 0; }

// x: [R, D] contiguous
std::vector<at::Tensor> rmsnorm_fwd(const at::Tensor& x, const at::Tensor& w, double eps) {
  check_bf16(x, "x");
  check_bf16(w, "weight");
  const int D = (int)x.size(-1);
  TORCH_CHECK(w.numel() == D, "weight size mismatch");
  TORCH_CHECK(rmsnorm_supported(D), "rmsnorm: hidden size must be a multiple of 8 and <= 4096");
  const int R = (int)(x.numel() / D);
  auto y = at::empty_like(x);
  auto rstd = at::empty({R}, x.options().dtype(at::kFloat));
  if (R == 0) return {y, rstd};
  dim3 grid((R + 3) / 4), block(kBlock);
  auto launch = [&](auto kernel) {
    hipLaunchKernelGGL(kernel, grid, block, 0, stream(), (const u16*)x.data_ptr(), (const u16*)w.data_ptr(),
                       (u16*)y.data_ptr(), rstd.data_ptr<float>(), R, D, (float)eps);
  };
  switch (vpl_for(D)) {
    case 1: launch(rmsnorm_fwd_kernel<1>); break;
    case 2: launch(rmsnorm_fwd_kernel<2>); break;
    case 4: launch(rmsnorm_fwd_kernel<4>); break;
    default: launch(rmsnorm_fwd_kernel<8>); break;
  }
  LAUNCH_CHECK();
  return {y, rstd};
}

std::vector<at::Tensor> rmsnorm_bwd(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& w,
                                    const at::Tensor& rstd) {
  check_bf16(dy, "grad");
  check_bf16(x, "x");
  check_bf16(w, "weight");
  const int D = (int)x.size(-1);
  const int R = (int)(x.numel() / D);
  TORCH_CHECK(rstd.numel() == R && rstd.scalar_type() == at::kFloat, "rstd mismatch");
  TORCH_CHECK(dy.numel() == x.numel(), "grad shape mismatch");
  auto dx = at::empty_like(x);
  auto dw = at::empty_like(w);
  if (R == 0) return {dx, dw.zero_()};
  // 2 rows per wave (8 per block): 512 blocks for the 4096-row case; partial rows stay <= 2 MB
  const int nblk = std::max(1, std::min(512, (R + 7) / 8));
  const int rpb = (R + nblk - 1) / nblk;
  auto part = at::empty({nblk, D}, x.options().dtype(at::kFloat));
  const size_t lds = (size_t)4 * D * sizeof(float);
  auto launch = [&](auto kernel) {
    hipLaunchKernelGGL(kernel, dim3(nblk), dim3(kBlock), lds, stream(), (const u16*)dy.data_ptr(),
                       (const u16*)x.data_ptr(), (const u16*)w.data_ptr(), rstd.data_ptr<float>(), (u16*)dx.data_ptr(),
                       part.data_ptr<float>(), R, D, rpb);
  };
  switch (vpl_for(D)) {
    case 1: launch(rmsnorm_bwd_kernel<1>); break;
    case 2: launch(rmsnorm_bwd_kernel<2>); break;
    case 4: launch(rmsnorm_bwd_kernel<4>); break;
    default: launch(rmsnorm_bwd_kernel<8>); break;
  }
  LAUNCH_CHECK();
  hipLaunchKernelGGL(col_sum_kernel, dim3((D + 31) / 32), dim3(1024), 0, stream(), part.data_ptr<float>(), nblk, D,
                     (u16*)dw.data_ptr());
  LAUNCH_CHECK();
  return {dx, dw};
}

at::Tensor swiglu_fwd(const at::Tensor& h) {
  check_bf16(h, "h");
  const int64_t W = h.size(-1);
  TORCH_CHECK(W % 4 == 0, "swiglu: last dim must be 2*H with H even");
  const int H = (int)(W / 2);
  const int R = (int)(h.numel() / W);
  auto sizes = h.sizes().vec();
  sizes.back() = H;
  auto y = at::empty(sizes, h.options());
  if (R == 0) return y;
  if (H % 8 == 0)
    hipLaunchKernelGGL(swiglu_fwd_kernel<8>, dim3(R), dim3(kBlock), 0, stream(), (const u16*)h.data_ptr(),
                       (u16*)y.data_ptr(), H);
  else
    hipLaunchKernelGGL(swiglu_fwd_kernel<2>, dim3(R), dim3(kBlock), 0, stream(), (const u16*)h.data_ptr(),
                       (u16*)y.data_ptr(), H);
  LAUNCH_CHECK();
  return y;
}

at::Tensor swiglu_bwd(const at::Tensor& dy, const at::Tensor& h) {
  check_bf16(dy, "grad");
  check_bf16(h, "h");
  const int64_t W = h.size(-1);
  const int H = (int)(W / 2);
  const int R = (int)(h.numel() / W);
  TORCH_CHECK(dy.numel() == (int64_t)R * H, "grad shape mismatch");
  auto dh = at::empty_like(h);
  if (R == 0) return dh;
  if (H % 8 == 0)
    hipLaunchKernelGGL(swiglu_bwd_kernel<8>, dim3(R), dim3(kBlock), 0, stream(), (const u16*)dy.data_ptr(),
                       (const u16*)h.data_ptr(), (u16*)dh.data_ptr(), H);
  else
    hipLaunchKernelGGL(swiglu_bwd_kernel<2>, dim3(R), dim3(kBlock), 0, stream(), (const u16*)dy.data_ptr(),
                       (const u16*)h.data_ptr(), (u16*)dh.data_ptr(), H);
  LAUNCH_CHECK();
  return dh;
}

// Returns (loss scalar, lse [R], stats [2] = {loss, count}).
std::vector<at::Tensor> ce_fwd(const at::Tensor& logits, const at::Tensor& tgt, int64_t ignore_index) {
  check_bf16(logits, "logits");
  TORCH_CHECK(logits.dim() == 2, "logits must be [N, V]");
  TORCH_CHECK(tgt.scalar_type() == at::kLong && tgt.is_contiguous() && tgt.is_cuda(), "targets must be int64 on GPU");
  const int R = (int)logits.size(0), V = (int)logits.size(1);
  TORCH_CHECK(V % 8 == 0, "vocab size must be a multiple of 8");
  TORCH_CHECK(tgt.numel() == R, "targets size mismatch");
  TORCH_CHECK(R > 0, "empty batch");
  auto fopt = logits.options().dtype(at::kFloat);
  auto lse = at::empty({R}, fopt);
  auto loss_rows = at::empty({R}, fopt);
  auto stats = at::empty({2}, fopt);
  hipLaunchKernelGGL(ce_fwd_kernel, dim3(R), dim3(kBlock), 0, stream(), (const u16*)logits.data_ptr(),
                     tgt.data_ptr<int64_t>(), lse.data_ptr<float>(), loss_rows.data_ptr<float>(), V, ignore_index);
  LAUNCH_CHECK();
  hipLaunchKernelGGL(ce_mean_kernel, dim3(1), dim3(1024), 0, stream(), loss_rows.data_ptr<float>(),
                     tgt.data_ptr<int64_t>(), R, ignore_index, stats.data_ptr<float>());
  LAUNCH_CHECK();
  return {stats.select(0, 0), lse, stats};
}

at::Tensor ce_bwd(const at::Tensor& grad, const at::Tensor& logits, const at::Tensor& tgt, const at::Tensor& lse,
                  const at::Tensor& stats, int64_t ignore_index) {
  check_bf16(logits, "logits");
  TORCH_CHECK(grad.scalar_type() == at::kFloat && grad.numel() == 1, "grad must be a float scalar");
  const int R = (int)logits.size(0), V = (int)logits.size(1);
  auto g = grad.contiguous();
  auto d = at::empty_like(logits);
  hipLaunchKernelGGL(ce_bwd_kernel, dim3(R), dim3(kBlock), 0, stream(), (const u16*)logits.data_ptr(),
                     tgt.data_ptr<int64_t>(), lse.data_ptr<float>(), g.data_ptr<float>(), stats.data_ptr<float>(),
                     (u16*)d.data_ptr(), V, ignore_index);
  LAUNCH_CHECK();
  return d;
}

// One optimizer step for a list of bf16 tensors sharing `step` (launches of <= kMaxT tensors).
void adamw_step(std::vector<at::Tensor> params, std::vector<at::Tensor> grads, std::vector<at::Tensor> exp_avgs,
                std::vector<at::Tensor> exp_avg_sqs, double lr, double beta1, double beta2, double eps,
                double weight_decay, int64_t step) {
  const size_t n = params.size();
  TORCH_CHECK(grads.size() == n && exp_avgs.size() == n && exp_avg_sqs.size() == n, "adamw: list sizes differ");
  TORCH_CHECK(step >= 1, "adamw: step must be >= 1");
  AdamScalars sc;
  sc.lr = (float)lr;
  sc.b1 = (float)beta1;
  sc.b2 = (float)beta2;
  sc.eps = (float)eps;
  sc.decay = (float)(1.0 - lr * weight_decay);
  sc.step_size = (float)(lr / (1.0 - std::pow(beta1, (double)step)));
  sc.bc2_sqrt = (float)std::sqrt(1.0 - std::pow(beta2, (double)step));
  AdamTable t;
  int nt = 0, blocks = 0;
  auto flush = [&]() {
    if (nt == 0) return;
    t.nt = nt;
    t.blk_start[nt] = blocks;
    hipLaunchKernelGGL(adamw_kernel, dim3(blocks), dim3(kBlock), 0, stream(), t, sc);
    LAUNCH_CHECK();
    nt = 0;
    blocks = 0;
  };
  for (size_t i = 0; i < n; ++i) {
    const at::Tensor* ts[4] = {&params[i], &grads[i], &exp_avgs[i], &exp_avg_sqs[i]};
    for (auto* x : ts) check_bf16(*x, "adamw tensor");
    const int64_t numel = params[i].numel();
    TORCH_CHECK(grads[i].numel() == numel && exp_avgs[i].numel() == numel && exp_avg_sqs[i].numel() == numel,
                "adamw: tensor sizes differ");
    if (numel == 0) continue;
    const int nb = (int)((numel + kChunk - 1) / kChunk);
    t.p[nt] = (u16*)params[i].data_ptr();
    t.g[nt] = (const u16*)grads[i].data_ptr();
    t.m[nt] = (u16*)exp_avgs[i].data_ptr();
    t.v[nt] = (u16*)exp_avg_sqs[i].data_ptr();
    t.n[nt] = numel;
    t.blk_start[nt] = blocks;
    blocks += nb;
    if (++nt == kMaxT) flush();
  }
  flush();
}

// ------------------------------------------------------------------------------ autograd
// C++ autograd nodes: one Python -> C++ call per op and no Python in the backward pass (a
// Python autograd.Function costs tens of microseconds of CPU per call, which shows on a
// launch-dense training step).

using torch::autograd::AutogradContext;
using torch::autograd::variable_list;

struct RMSNormFn : public torch::autograd::Function<RMSNormFn> {
  static at::Tensor forward(AutogradContext* ctx, const at::Tensor& x, const at::Tensor& w, double eps) {
    const int64_t D = x.size(-1);
    auto x2 = x.contiguous().view({-1, D});
    auto w2 = w.contiguous();
    auto r = rmsnorm_fwd(x2, w2, eps);
    ctx->save_for_backward({x2, w2, r[1]});
    ctx->saved_data["shape"] = x.sizes().vec();
    return r[0].view(x.sizes());
  }
  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    auto s = ctx->get_saved_variables();
    auto dy = grads[0].contiguous().view_as(s[0]);
    auto r = rmsnorm_bwd(dy, s[0], s[1], s[2]);
    auto shape = ctx->saved_data["shape"].toIntVector();
    return {r[0].view(shape), r[1], at::Tensor()};
  }
};

struct SwiGLUFn : public torch::autograd::Function<SwiGLUFn> {
  static at::Tensor forward(AutogradContext* ctx, const at::Tensor& h) {
    auto hc = h.contiguous();
    ctx->save_for_backward({hc});
    return swiglu_fwd(hc);
  }
  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    auto s = ctx->get_saved_variables();
    return {swiglu_bwd(grads[0].contiguous(), s[0])};
  }
};

struct CrossEntropyFn : public torch::autograd::Function<CrossEntropyFn> {
  static at::Tensor forward(AutogradContext* ctx, const at::Tensor& logits, const at::Tensor& tgt,
                            int64_t ignore_index) {
    auto lc = logits.contiguous();
    auto tc = tgt.contiguous();
    auto r = ce_fwd(lc, tc, ignore_index);
    ctx->save_for_backward({lc, tc, r[1], r[2]});
    ctx->saved_data["ignore"] = ignore_index;
    return r[0].clone();  // own storage: the autograd output must not alias the saved stats
  }
  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    auto s = ctx->get_saved_variables();
    auto g = grads[0].to(at::kFloat).reshape({1});
    return {ce_bwd(g, s[0], s[1], s[2], s[3], ctx->saved_data["ignore"].toInt()), at::Tensor(), at::Tensor()};
  }
};

at::Tensor rms_norm(const at::Tensor& x, const at::Tensor& w, double eps) { return RMSNormFn::apply(x, w, eps); }
at::Tensor swiglu(const at::Tensor& h) { return SwiGLUFn::apply(h); }
at::Tensor cross_entropy(const at::Tensor& logits, const at::Tensor& tgt, int64_t ignore_index) {
  return CrossEntropyFn::apply(logits, tgt, ignore_index);
}

}  // namespace

PYBIND11_MODULE(_fused_ops, m) {
  m.doc() = "gfx950 fused training ops (RMSNorm, SwiGLU, cross-entropy)";
  m.def("rmsnorm_supported", &rmsnorm_supported);
  // differentiable entry points (C++ autograd)
  m.def("rms_norm", &rms_norm);
  m.def("swiglu", &swiglu);
  m.def("cross_entropy", &cross_entropy);
  m.def("adamw_step", &adamw_step);
  // raw kernels (tests / custom graphs)
  m.def("rmsnorm_fwd", &rmsnorm_fwd);
  m.def("rmsnorm_bwd", &rmsnorm_bwd);
  m.def("swiglu_fwd", &swiglu_fwd);
  m.def("swiglu_bwd", &swiglu_bwd);
  m.def("ce_fwd", &ce_fwd);
  m.def("ce_bwd", &ce_bwd);
}

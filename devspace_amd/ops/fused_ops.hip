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
#include <ATen/Parallel.h>

#include <atomic>
#include <thread>
#include <vector>
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
// RES: fused residual add first, s = bf16(x + delta) is written to `sum` and normalised
// (the transformer's `x = x + f(x); h = norm(x)` in one pass instead of an add kernel + norm).
template <int VPL, bool RES>
__global__ void __launch_bounds__(kBlock) rmsnorm_fwd_kernel(const u16* __restrict__ x, const u16* __restrict__ delta,
                                                            const u16* __restrict__ w, u16* __restrict__ sum,
                                                            u16* __restrict__ y, float* __restrict__ rstd, int R,
                                                            int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const int nvec = D >> 3;
  const u16x8* xr = reinterpret_cast<const u16x8*>(x + (size_t)row * D);
  const u16x8* wr = reinterpret_cast<const u16x8*>(w);
  // w is loaded with the row, not after the reduction: the row's loads are its only memory
  // latency (the weight row is L2-resident, but a load issued after the shuffles still waits)
  u16x8 v[VPL], dv[VPL], wv[VPL];
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
    const int i = lane + 64 * k;
    if (i < nvec) {
      v[k] = xr[i];
      if (RES) dv[k] = reinterpret_cast<const u16x8*>(delta + (size_t)row * D)[i];
      wv[k] = wr[i];
    }
  }
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
    const int i = lane + 64 * k;
    if (i < nvec) {
      if (RES) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[k][j] = f2b(b2f(v[k][j]) + b2f(dv[k][j]));
        reinterpret_cast<u16x8*>(sum + (size_t)row * D)[i] = v[k];
      }
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
  u16x8* yr = reinterpret_cast<u16x8*>(y + (size_t)row * D);
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
    const int i = lane + 64 * k;
    if (i < nvec) {
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2b(b2f(v[k][j]) * r * b2f(wv[k][j]));
      yr[i] = o;
    }
  }
}

// dx = r * (w*dy) - x * r^3 / D * sum(w*dy*x);  dw partial = sum_rows dy * x * r.
// A block owns `rows_per_block` consecutive rows (its 4 waves stride over them); each lane
// accumulates the weight-gradient of its columns in registers, the 4 waves are summed through
// LDS and the block writes one fp32 partial row (reduced by col_sum_kernel).
// RES: the gradient arriving on the residual stream (dres) is added to dx before the single
// bf16 rounding (the fused add's backward: d(x) = d(delta) = dres + norm'(dy)).
template <int VPL, bool RES>
__global__ void __launch_bounds__(kBlock) rmsnorm_bwd_kernel(const u16* __restrict__ dy, const u16* __restrict__ x,
                                                            const u16* __restrict__ dres, const u16* __restrict__ w,
                                                            const float* __restrict__ rstd, u16* __restrict__ dx,
                                                            float* __restrict__ dw_part, int R, int D,
                                                            int rows_per_block) {
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
    const u16x8* drr = reinterpret_cast<const u16x8*>(dres + (size_t)row * D);
#pragma unroll
    for (int k = 0; k < VPL; ++k) {
      const int i = lane + 64 * k;
      if (i < nvec) {
        u16x8 o, rv;
        if (RES) rv = drr[i];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float g = b2f(gv[k][j]), xf = b2f(xv[k][j]);
          float d = r * g * b2f(wv[k][j]) - xf * c;
          if (RES) d += b2f(rv[j]);
          o[j] = f2b(d);
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
  // 8 loads in flight per thread (the reduction is latency-bound: 32 blocks read 2 MB for D = 1024)
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < D) {
    int r = g;
    for (; r + 7 * 32 < nrows; r += 8 * 32) {
#pragma unroll
      for (int u = 0; u < 8; ++u) s[u] += part[(size_t)(r + 32 * u) * D + c];
    }
    for (; r < nrows; r += 32) s[0] += part[(size_t)r * D + c];
  }
  red[g][cl] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
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

// ------------------------------------------------------------------------------ attention
//
// Flash attention (head dim 64, bf16 in/out, fp32 softmax/accumulators) on
// v_mfma_f32_32x32x16_bf16, reading Q/K/V straight from the packed qkv projection output
// [B, T, 3, H, 64] and writing O as [B, T, H, 64] (no transposes / stack copies around it).
//
// Forward (one workgroup = 128 queries of one (b, h), 4 waves x 32 queries; K/V tiles of 64
// keys double-buffered in LDS, register-staged: the next tile's global loads are issued before
// the current tile's MFMAs and written after them):
//   S^T = K Q^T      keys on the MFMA rows, the wave's 32 queries on the lanes, so the online
//                    softmax (max, exp2, sum) is lane-local plus one xor-32 exchange;
//   O^T += V^T P^T   the P^T accumulators are the B operand as they stand (k order permuted,
//                    cdna_hip_programming.md §3), V^T comes from ds_read_b64_tr_b16 reads of the
//                    row-major V tile; O^T keeps the query on the lane, so the per-query rescale
//                    is a scalar per lane.
// LDS tiles use 128-B rows with a 16-B chunk XOR swizzle, chunk ^ f(row) with
// f(row) = ((row >> 1) & 7) ^ ((row & 2) << 1). The ds_read_b128 row reads of the 32x32x16 A
// operand are conflict-free: the 8 rows of each parity in a 16-lane group get distinct f.
// The ds_read_b64_tr_b16 reads of the transposed operand are conflict-free too: a 32-lane half
// reads rows r0..r0+3 x one aligned quad of chunks, and the (row & 2) term flips bit 2 of f
// between rows r0 and r0+2, which sends their quads to the two halves of the 128-B row. With
// f = (row >> 1) & 7 alone those reads were 2-way (SQ_LDS_BANK_CONFLICT 294,912 per forward
// dispatch at B8 T512 H16, profiles/r1_attn_pmc.txt; bank model: scripts/attn_lds_banks.py).
// Backward (FlashAttention-2 split, no atomics): a dK/dV kernel (workgroup = 128 keys, loops over
// query tiles; S and dP with the key on the lane, dV^T += dO^T P and dK^T += Q^T dS from the
// accumulators) and a dQ kernel (workgroup = 128 queries, loops over key tiles like the forward;
// dQ^T += K^T dS^T), plus a rowsum(dO * O) preprocess.

constexpr int kHD = 64;     // head dim
constexpr int kQBlk = 128;  // queries (fwd / dQ) or keys (dK/dV) per workgroup
constexpr int kTile = 64;   // keys (fwd / dQ) or queries (dK/dV) per LDS tile
constexpr int kTileBytes = kTile * kHD * 2;

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((address_space(3))) unsigned char lds_u8;

__device__ __forceinline__ f32x16 mfma32(const u16x8& a, const u16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                 0, 0, 0);
}

// byte offset of 16-byte chunk `chunk` (0..7) of row `row` in a [64][64] bf16 LDS tile
__device__ __forceinline__ int tile_off(int row, int chunk) {
  return row * 128 + ((chunk ^ ((row >> 1) & 7) ^ ((row & 2) << 1)) << 4);
}

__device__ __forceinline__ u16x8 lds_row8(const unsigned char* tile, int row, int chunk) {
  return *reinterpret_cast<const u16x8*>(tile + tile_off(row, chunk));
}

// Transposed operand of a 32x32x16 MFMA from a row-major [rows][64] tile: lane (r = lane&31,
// h = lane>>5) gets column col0 + r of rows {r0 + 4h + 0..3} (elements 0..3) and
// {r0 + 8 + 4h + 0..3} (elements 4..7), i.e. the k order of an accumulator used as the other
// operand (§3 "An accumulator tile as the next MFMA's operand"). Two ds_read_b64_tr_b16.
__device__ __forceinline__ u16x8 lds_tr8(const unsigned char* tile, int r0, int col0, int lane) {
  const int g = lane >> 4, i = lane & 15, hh = lane >> 5;
  const int row = r0 + 4 * hh + (i >> 2);
  const int col = col0 + 16 * (g & 1) + 4 * (i & 3);
  const int off1 = tile_off(row, col >> 3) + ((col & 7) << 1);
  const int off2 = tile_off(row + 8, col >> 3) + ((col & 7) << 1);
  lds_u8* base = (lds_u8*)tile;
  s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + off1));
  s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + off2));
  return __builtin_bit_cast(u16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}

// 2^x on the transcendental unit (v_exp_f32): no denormal-range fix-up (exp2f adds a compare,
// a select and a v_ldexp per call); exp2(-inf) = 0, which the masked scores rely on.
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// accumulator registers 8s .. 8s+7 as a bf16 MFMA operand (k-step s of the accumulator's rows)
__device__ __forceinline__ u16x8 acc_to_op(const f32x16& acc, int s) {
  u16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = f2b(acc[8 * s + j]);
  return o;
}

// row (within a 32x32 accumulator tile) held by register `reg` of lane half `hh`
__device__ __forceinline__ int acc_row(int reg, int hh) { return (reg & 3) + 8 * (reg >> 2) + 4 * hh; }

struct AttnParams {
  const u16* q;
  const u16* k;
  const u16* v;
  const u16* o;
  const u16* dout;
  u16* out;            // fwd: O; bwd: dQ (dq kernel) / dK (dkdv kernel)
  u16* out2;           // bwd dkdv kernel: dV
  const float* lse;    // [B, H, T] log2-domain LSE of the scaled scores
  const float* delta;  // [B, H, T] rowsum(dO * O)
  float* stat_out;     // fwd: lse; bwd preprocess: delta
  int64_t sb, st, sh;  // q/k/v (and dq/dk/dv) strides in elements
  int64_t ob, ot, oh;  // o / dout strides
  int T, H;
  float scale_log2;  // softmax scale * log2(e)
  float scale;       // softmax scale
};

// 256 threads stage one [64][64] tile of two tensors (4 x 16 B per thread) through registers
struct Stage {
  u16x8 r[4];
  __device__ __forceinline__ void load(const u16* a, const u16* b, int64_t base, int64_t st, int row0) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = threadIdx.x + 256 * u;
      const int row = (c >> 3) & 63, ch = c & 7;
      const u16* src = ((c >> 9) ? b : a) + base + (int64_t)(row0 + row) * st + ch * 8;
      r[u] = *reinterpret_cast<const u16x8*>(src);
    }
  }
  __device__ __forceinline__ void store(unsigned char* ta, unsigned char* tb) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = threadIdx.x + 256 * u;
      const int row = (c >> 3) & 63, ch = c & 7;
      *reinterpret_cast<u16x8*>(((c >> 9) ? tb : ta) + tile_off(row, ch)) = r[u];
    }
  }
};

template <bool CAUSAL>
__global__ void __launch_bounds__(256, 2) attn_fwd_kernel(AttnParams p) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[2][2][kTileBytes];  // [buf][K|V]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int nqb = p.T / kQBlk;
  const int qb = CAUSAL ? nqb - 1 - (int)blockIdx.x : (int)blockIdx.x;  // heaviest blocks first
  const int h = blockIdx.y, b = blockIdx.z;
  const int64_t base = (int64_t)b * p.sb + (int64_t)h * p.sh;
  const int qw0 = qb * kQBlk + wave * 32;  // first query of this wave
  const int q = qw0 + r;
  u16x8 qf[4];
  {
    const u16* qrow = p.q + base + (int64_t)q * p.st;
#pragma unroll
    for (int s = 0; s < 4; ++s) qf[s] = *reinterpret_cast<const u16x8*>(qrow + 16 * s + 8 * hh);
  }
  f32x16 oacc[2];
#pragma unroll
  for (int nb = 0; nb < 2; ++nb)
#pragma unroll
    for (int i = 0; i < 16; ++i) oacc[nb][i] = 0.f;
  float m = -INFINITY, l = 0.f;
  const int ntiles = CAUSAL ? (qb + 1) * (kQBlk / kTile) : p.T / kTile;
  Stage stg;
  stg.load(p.k, p.v, base, p.st, 0);
  stg.store(smem[0][0], smem[0][1]);
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    if (t + 1 < ntiles) stg.load(p.k, p.v, base, p.st, (t + 1) * kTile);
    const unsigned char* Ks = smem[buf][0];
    const unsigned char* Vs = smem[buf][1];
    const int k0 = t * kTile;
    // wave-uniform causal classes of this tile: all keys after all of the wave's queries
    // (nothing to do), straddling the diagonal (mask), or fully visible (no per-element test)
    if (!(CAUSAL && k0 > qw0 + 31)) {
      f32x16 sacc[2];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int i = 0; i < 16; ++i) sacc[kb][i] = 0.f;
      // k-step outer, key block inner: two independent MFMA chains issue back to back
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) sacc[kb] = mfma32(lds_row8(Ks, kb * 32 + r, 2 * s + hh), qf[s], sacc[kb]);
      if (CAUSAL && k0 + kTile - 1 > qw0) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if (k0 + kb * 32 + acc_row(i, hh) > q) sacc[kb][i] = -INFINITY;
      }
      // raw-score max (scale > 0), then p = 2^(s * scale_log2 - m) as one FMA + v_exp. Tile 0
      // always holds key 0, so m is finite from the first tile on and no -inf guards are needed.
      float mt = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int i = 0; i < 16; ++i) mt = fmaxf(mt, sacc[kb][i]);
      mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
      const float mn = fmaxf(m, mt * p.scale_log2);
      const float alpha = fast_exp2(m - mn);
      float ls = 0.f;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float e = fast_exp2(__builtin_fmaf(sacc[kb][i], p.scale_log2, -mn));
          sacc[kb][i] = e;
          ls += e;
        }
      l = l * alpha + ls;
      m = mn;
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
#pragma unroll
        for (int i = 0; i < 16; ++i) oacc[nb][i] *= alpha;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const u16x8 pb = acc_to_op(sacc[ks >> 1], ks & 1);
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
          oacc[nb] = mfma32(lds_tr8(Vs, (ks >> 1) * 32 + 16 * (ks & 1), nb * 32, lane), pb, oacc[nb]);
      }
    }
    if (t + 1 < ntiles) stg.store(smem[buf ^ 1][0], smem[buf ^ 1][1]);
    __syncthreads();
  }
  const float lt = l + __shfl_xor(l, 32, 64);
  const float inv = 1.f / lt;
  u16* orow = p.out + (int64_t)b * p.ob + (int64_t)h * p.oh + (int64_t)q * p.ot;
#pragma unroll
  for (int nb = 0; nb < 2; ++nb)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      u16v<4> o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = f2b(oacc[nb][4 * g4 + j] * inv);
      *reinterpret_cast<u16v<4>*>(orow + nb * 32 + 8 * g4 + 4 * hh) = o;
    }
  if (hh == 0) p.stat_out[((int64_t)b * p.H + h) * p.T + q] = m + __log2f(lt);
}

// delta[b, h, t] = sum_d dO * O (fp32); 8 lanes per row
__global__ void __launch_bounds__(256) attn_bwd_pre_kernel(AttnParams p, int64_t rows) {
  const int64_t row = (int64_t)blockIdx.x * 32 + (threadIdx.x >> 3);
  const int c = threadIdx.x & 7;
  float s = 0.f;
  if (row < rows) {
    const int t = (int)(row % p.T);
    const int64_t bh = row / p.T;
    const int h = (int)(bh % p.H), b = (int)(bh / p.H);
    const int64_t off = (int64_t)b * p.ob + (int64_t)h * p.oh + (int64_t)t * p.ot + c * 8;
    u16x8 d = *reinterpret_cast<const u16x8*>(p.dout + off);
    u16x8 o = *reinterpret_cast<const u16x8*>(p.o + off);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += b2f(d[j]) * b2f(o[j]);
  }
  s += __shfl_xor(s, 1, 64);
  s += __shfl_xor(s, 2, 64);
  s += __shfl_xor(s, 4, 64);
  if (row < rows && c == 0) p.stat_out[row] = s;
}

// dK, dV: workgroup = 128 keys (4 waves x 32, key on the lane), loop over 64-query tiles.
template <bool CAUSAL>
__global__ void __launch_bounds__(256, 2) attn_bwd_dkdv_kernel(AttnParams p) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[2][2][kTileBytes];  // [buf][Q|dO]
  __shared__ __attribute__((aligned(16))) float sstat[2][2][kTile];             // [buf][lse|delta]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int kblk = blockIdx.x;  // key blocks near 0 see the most queries: launched first
  const int h = blockIdx.y, b = blockIdx.z;
  const int64_t base = (int64_t)b * p.sb + (int64_t)h * p.sh;
  const int64_t obase = (int64_t)b * p.ob + (int64_t)h * p.oh;
  const int64_t sbase = ((int64_t)b * p.H + h) * p.T;
  const int kw0 = kblk * kQBlk + wave * 32;  // first key of this wave
  const int key = kw0 + r;
  u16x8 kf[4], vf[4];
  {
    const u16* krow = p.k + base + (int64_t)key * p.st;
    const u16* vrow = p.v + base + (int64_t)key * p.st;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      kf[s] = *reinterpret_cast<const u16x8*>(krow + 16 * s + 8 * hh);
      vf[s] = *reinterpret_cast<const u16x8*>(vrow + 16 * s + 8 * hh);
    }
  }
  f32x16 dk[2], dv[2];
#pragma unroll
  for (int nb = 0; nb < 2; ++nb)
#pragma unroll
    for (int i = 0; i < 16; ++i) dk[nb][i] = dv[nb][i] = 0.f;
  const int t0 = CAUSAL ? kblk * (kQBlk / kTile) : 0;
  const int t1 = p.T / kTile;
  // Q (q strides) and dO (o strides) tiles + the tile's lse / delta values
  u16x8 rg[4];
  float sv = 0.f;
  auto load = [&](int t) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = threadIdx.x + 256 * u;
      const int row = (c >> 3) & 63, ch = c & 7;
      const int qrow = t * kTile + row;
      rg[u] = (c >> 9) ? *reinterpret_cast<const u16x8*>(p.dout + obase + (int64_t)qrow * p.ot + ch * 8)
                       : *reinterpret_cast<const u16x8*>(p.q + base + (int64_t)qrow * p.st + ch * 8);
    }
    if (threadIdx.x < 128) sv = (threadIdx.x < 64 ? p.lse : p.delta)[sbase + t * kTile + (threadIdx.x & 63)];
  };
  auto store = [&](int bufi) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = threadIdx.x + 256 * u;
      const int row = (c >> 3) & 63, ch = c & 7;
      *reinterpret_cast<u16x8*>(smem[bufi][c >> 9] + tile_off(row, ch)) = rg[u];
    }
    if (threadIdx.x < 128) sstat[bufi][threadIdx.x >> 6][threadIdx.x & 63] = sv;
  };
  if (t0 < t1) {
    load(t0);
    store(0);
  }
  __syncthreads();
  for (int t = t0; t < t1; ++t) {
    const int buf = (t - t0) & 1;
    if (t + 1 < t1) load(t + 1);
    const unsigned char* Qs = smem[buf][0];
    const unsigned char* Ds = smem[buf][1];
#pragma unroll
    for (int qs = 0; qs < 2; ++qs) {
      const int qa = t * kTile + qs * 32;  // first query of this 32-query slice
      if (CAUSAL && kw0 > qa + 31) continue;  // every key of the wave after every query: P = 0
      const bool diag = CAUSAL && kw0 + 31 > qa;
      f32x16 sacc, dpacc;
#pragma unroll
      for (int i = 0; i < 16; ++i) sacc[i] = dpacc[i] = 0.f;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        sacc = mfma32(lds_row8(Qs, qs * 32 + r, 2 * s + hh), kf[s], sacc);
        dpacc = mfma32(lds_row8(Ds, qs * 32 + r, 2 * s + hh), vf[s], dpacc);
      }
      // accumulator rows are queries qs*32 + acc_row(i, hh): 4 consecutive per register group
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int qi = qs * 32 + 8 * g4 + 4 * hh;
        const float4 lse4 = *reinterpret_cast<const float4*>(&sstat[buf][0][qi]);
        const float4 del4 = *reinterpret_cast<const float4*>(&sstat[buf][1][qi]);
        const float ls[4] = {lse4.x, lse4.y, lse4.z, lse4.w};
        const float dl[4] = {del4.x, del4.y, del4.z, del4.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int i = 4 * g4 + j;
          float pv = fast_exp2(__builtin_fmaf(sacc[i], p.scale_log2, -ls[j]));
          if (diag && key > t * kTile + qi + j) pv = 0.f;
          sacc[i] = pv;
          dpacc[i] = pv * (dpacc[i] - dl[j]);
        }
      }
#pragma unroll
      for (int kss = 0; kss < 2; ++kss) {
        const u16x8 pb = acc_to_op(sacc, kss);
        const u16x8 db = acc_to_op(dpacc, kss);
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
          dv[nb] = mfma32(lds_tr8(Ds, qs * 32 + 16 * kss, nb * 32, lane), pb, dv[nb]);
          dk[nb] = mfma32(lds_tr8(Qs, qs * 32 + 16 * kss, nb * 32, lane), db, dk[nb]);
        }
      }
    }
    if (t + 1 < t1) store(buf ^ 1);
    __syncthreads();
  }
  u16* dkrow = p.out + base + (int64_t)key * p.st;
  u16* dvrow = p.out2 + base + (int64_t)key * p.st;
#pragma unroll
  for (int nb = 0; nb < 2; ++nb)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      u16v<4> ok, ov;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        ok[j] = f2b(dk[nb][4 * g4 + j] * p.scale);
        ov[j] = f2b(dv[nb][4 * g4 + j]);
      }
      *reinterpret_cast<u16v<4>*>(dkrow + nb * 32 + 8 * g4 + 4 * hh) = ok;
      *reinterpret_cast<u16v<4>*>(dvrow + nb * 32 + 8 * g4 + 4 * hh) = ov;
    }
}

// dQ: workgroup = 128 queries (query on the lane), loop over 64-key tiles like the forward.
template <bool CAUSAL>
__global__ void __launch_bounds__(256, 2) attn_bwd_dq_kernel(AttnParams p) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[2][2][kTileBytes];  // [buf][K|V]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int nqb = p.T / kQBlk;
  const int qb = CAUSAL ? nqb - 1 - (int)blockIdx.x : (int)blockIdx.x;
  const int h = blockIdx.y, b = blockIdx.z;
  const int64_t base = (int64_t)b * p.sb + (int64_t)h * p.sh;
  const int qw0 = qb * kQBlk + wave * 32;
  const int q = qw0 + r;
  u16x8 qf[4], df[4];
  {
    const u16* qrow = p.q + base + (int64_t)q * p.st;
    const u16* drow = p.dout + (int64_t)b * p.ob + (int64_t)h * p.oh + (int64_t)q * p.ot;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      qf[s] = *reinterpret_cast<const u16x8*>(qrow + 16 * s + 8 * hh);
      df[s] = *reinterpret_cast<const u16x8*>(drow + 16 * s + 8 * hh);
    }
  }
  const int64_t sidx = ((int64_t)b * p.H + h) * p.T + q;
  const float lse = p.lse[sidx], del = p.delta[sidx];
  f32x16 dq[2];
#pragma unroll
  for (int nb = 0; nb < 2; ++nb)
#pragma unroll
    for (int i = 0; i < 16; ++i) dq[nb][i] = 0.f;
  const int ntiles = CAUSAL ? (qb + 1) * (kQBlk / kTile) : p.T / kTile;
  Stage stg;
  stg.load(p.k, p.v, base, p.st, 0);
  stg.store(smem[0][0], smem[0][1]);
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    if (t + 1 < ntiles) stg.load(p.k, p.v, base, p.st, (t + 1) * kTile);
    const unsigned char* Ks = smem[buf][0];
    const unsigned char* Vs = smem[buf][1];
    const int k0 = t * kTile;
    if (!(CAUSAL && k0 > qw0 + 31)) {  // same wave-uniform tile classes as the forward
      const bool diag = CAUSAL && k0 + kTile - 1 > qw0;
      f32x16 sacc[2], dpacc[2];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int i = 0; i < 16; ++i) sacc[kb][i] = dpacc[kb][i] = 0.f;
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          sacc[kb] = mfma32(lds_row8(Ks, kb * 32 + r, 2 * s + hh), qf[s], sacc[kb]);
          dpacc[kb] = mfma32(lds_row8(Vs, kb * 32 + r, 2 * s + hh), df[s], dpacc[kb]);
        }
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float pv = fast_exp2(__builtin_fmaf(sacc[kb][i], p.scale_log2, -lse));
          if (diag && k0 + kb * 32 + acc_row(i, hh) > q) pv = 0.f;
          dpacc[kb][i] = pv * (dpacc[kb][i] - del);
        }
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const u16x8 db = acc_to_op(dpacc[ks >> 1], ks & 1);
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
          dq[nb] = mfma32(lds_tr8(Ks, (ks >> 1) * 32 + 16 * (ks & 1), nb * 32, lane), db, dq[nb]);
      }
    }
    if (t + 1 < ntiles) stg.store(smem[buf ^ 1][0], smem[buf ^ 1][1]);
    __syncthreads();
  }
  u16* qrow = p.out + base + (int64_t)q * p.st;
#pragma unroll
  for (int nb = 0; nb < 2; ++nb)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      u16v<4> o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = f2b(dq[nb][4 * g4 + j] * p.scale);
      *reinterpret_cast<u16v<4>*>(qrow + nb * 32 + 8 * g4 + 4 * hh) = o;
    }
}

// ------------------------------------------------------------------------------ host side

// ------------------------------------------------------------------------------ state digest
// Content digest of training state for the rescue snapshots' de-duplication
// (devspace_amd/rescue.py digests): per row of up to 64 Ki int64 words w_i (i = the word's index
// in its tensor), S = sum w_i and M = sum mix(w_i ^ key(i)) mod 2^64, key(i) = (i + 1) * golden,
// mix = the splitmix64 finalizer (a bijection). M depends on every word's position: a swap of
// two words, or changes that keep the plain sum, give another M with probability 1 - 2^-64.
// One HBM read of the state (one block per row, 8-byte loads, wave64 + LDS reduction), one
// launch for all tensors (a row table), one small copy of (S, M) pairs to the host. The CPU
// path computes the same numbers with torch ops (rescue.py _digest_rows_torch).
struct DigestRow {
  const unsigned long long* p;  // the row's first word
  long long n;                  // words in this row (<= kDigestRowWords)
  long long base;               // index of the first word in its tensor
};
constexpr long long kDigestRowWords = 1 << 16;

__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z ^= z >> 30;
  z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 27;
  z *= 0x94D049BB133111EBull;
  z ^= z >> 31;
  return z;
}

__device__ __forceinline__ unsigned long long shfl_xor_u64(unsigned long long v, int o) {
  unsigned lo = __shfl_xor((unsigned)v, o, 64), hi = __shfl_xor((unsigned)(v >> 32), o, 64);
  return ((unsigned long long)hi << 32) | lo;
}

__global__ void __launch_bounds__(kBlock) state_digest_kernel(const DigestRow* __restrict__ rows,
                                                               long long* __restrict__ out) {
  const DigestRow r = rows[blockIdx.x];
  unsigned long long s = 0, m = 0;
  const unsigned long long kGolden = 0x9E3779B97F4A7C15ull;
  long long i = threadIdx.x;
  // 4 independent loads in flight per lane before the arithmetic that uses them
  for (; i + 3 * kBlock < r.n; i += 4 * kBlock) {
    unsigned long long v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(r.p + i + u * kBlock);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      s += v[u];
      m += mix64(v[u] ^ ((unsigned long long)(r.base + i + u * kBlock + 1) * kGolden));
    }
  }
  for (; i < r.n; i += kBlock) {
    unsigned long long v = __builtin_nontemporal_load(r.p + i);
    s += v;
    m += mix64(v ^ ((unsigned long long)(r.base + i + 1) * kGolden));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s += shfl_xor_u64(s, o);
    m += shfl_xor_u64(m, o);
  }
  __shared__ unsigned long long part[2][kBlock / 64];
  const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  if (lane == 0) {
    part[0][wave] = s;
    part[1][wave] = m;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long S = 0, M = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) {
      S += part[0][w];
      M += part[1][w];
    }
    out[2 * blockIdx.x] = (long long)S;
    out[2 * blockIdx.x + 1] = (long long)M;
  }
}

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

// x (and delta): [R, D] contiguous. Returns {y, rstd} or, with delta, {y, rstd, x + delta}.
std::vector<at::Tensor> rmsnorm_fwd_impl(const at::Tensor& x, const at::Tensor* delta, const at::Tensor& w, double eps) {
  check_bf16(x, "x");
  check_bf16(w, "weight");
  const int D = (int)x.size(-1);
  TORCH_CHECK(w.numel() == D, "weight size mismatch");
  TORCH_CHECK(rmsnorm_supported(D), "rmsnorm: hidden size must be a multiple of 8 and <= 4096");
  if (delta) {
    check_bf16(*delta, "delta");
    TORCH_CHECK(delta->sizes() == x.sizes(), "delta shape mismatch");
  }
  const int R = (int)(x.numel() / D);
  auto y = at::empty_like(x);
  auto rstd = at::empty({R}, x.options().dtype(at::kFloat));
  at::Tensor sum = delta ? at::empty_like(x) : at::Tensor();
  std::vector<at::Tensor> out = {y, rstd};
  if (delta) out.push_back(sum);
  if (R == 0) return out;
  dim3 grid((R + 3) / 4), block(kBlock);
  auto launch = [&](auto kernel) {
    hipLaunchKernelGGL(kernel, grid, block, 0, stream(), (const u16*)x.data_ptr(),
                       delta ? (const u16*)delta->data_ptr() : nullptr, (const u16*)w.data_ptr(),
                       delta ? (u16*)sum.data_ptr() : nullptr, (u16*)y.data_ptr(), rstd.data_ptr<float>(), R, D,
                       (float)eps);
  };
#define RMS_FWD_CASES(RES)                                \
  switch (vpl_for(D)) {                                   \
    case 1: launch(rmsnorm_fwd_kernel<1, RES>); break;    \
    case 2: launch(rmsnorm_fwd_kernel<2, RES>); break;    \
    case 4: launch(rmsnorm_fwd_kernel<4, RES>); break;    \
    default: launch(rmsnorm_fwd_kernel<8, RES>); break;   \
  }
  if (delta) {
    RMS_FWD_CASES(true)
  } else {
    RMS_FWD_CASES(false)
  }
#undef RMS_FWD_CASES
  LAUNCH_CHECK();
  return out;
}

std::vector<at::Tensor> rmsnorm_fwd(const at::Tensor& x, const at::Tensor& w, double eps) {
  return rmsnorm_fwd_impl(x, nullptr, w, eps);
}

std::vector<at::Tensor> add_rmsnorm_fwd(const at::Tensor& x, const at::Tensor& delta, const at::Tensor& w, double eps) {
  return rmsnorm_fwd_impl(x, &delta, w, eps);
}

// dres (optional): gradient already flowing on the residual stream, added into dx.
std::vector<at::Tensor> rmsnorm_bwd_impl(const at::Tensor& dy, const at::Tensor& x, const at::Tensor* dres,
                                         const at::Tensor& w, const at::Tensor& rstd) {
  check_bf16(dy, "grad");
  check_bf16(x, "x");
  check_bf16(w, "weight");
  const int D = (int)x.size(-1);
  const int R = (int)(x.numel() / D);
  TORCH_CHECK(rstd.numel() == R && rstd.scalar_type() == at::kFloat, "rstd mismatch");
  TORCH_CHECK(dy.numel() == x.numel(), "grad shape mismatch");
  if (dres) {
    check_bf16(*dres, "residual grad");
    TORCH_CHECK(dres->numel() == x.numel(), "residual grad shape mismatch");
  }
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
                       (const u16*)x.data_ptr(), dres ? (const u16*)dres->data_ptr() : nullptr,
                       (const u16*)w.data_ptr(), rstd.data_ptr<float>(), (u16*)dx.data_ptr(), part.data_ptr<float>(),
                       R, D, rpb);
  };
#define RMS_BWD_CASES(RES)                                \
  switch (vpl_for(D)) {                                   \
    case 1: launch(rmsnorm_bwd_kernel<1, RES>); break;    \
    case 2: launch(rmsnorm_bwd_kernel<2, RES>); break;    \
    case 4: launch(rmsnorm_bwd_kernel<4, RES>); break;    \
    default: launch(rmsnorm_bwd_kernel<8, RES>); break;   \
  }
  if (dres) {
    RMS_BWD_CASES(true)
  } else {
    RMS_BWD_CASES(false)
  }
#undef RMS_BWD_CASES
  LAUNCH_CHECK();
  hipLaunchKernelGGL(col_sum_kernel, dim3((D + 31) / 32), dim3(1024), 0, stream(), part.data_ptr<float>(), nblk, D,
                     (u16*)dw.data_ptr());
  LAUNCH_CHECK();
  return {dx, dw};
}

std::vector<at::Tensor> rmsnorm_bwd(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& w,
                                    const at::Tensor& rstd) {
  return rmsnorm_bwd_impl(dy, x, nullptr, w, rstd);
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

// packed qkv [B, T, 3, H, 64] bf16 -> (O [B, T, H, 64], lse [B, H, T] fp32 log2-domain)
bool attention_supported(const at::Tensor& qkv) {
  return qkv.dim() == 5 && qkv.size(2) == 3 && qkv.size(4) == kHD && qkv.size(1) % kQBlk == 0 && qkv.size(1) > 0;
}

AttnParams attn_params(const at::Tensor& qkv, double scale) {
  AttnParams p{};
  const int64_t T = qkv.size(1), H = qkv.size(3);
  const u16* base = (const u16*)qkv.data_ptr();
  p.q = base;
  p.k = base + H * kHD;
  p.v = base + 2 * H * kHD;
  p.sb = T * 3 * H * kHD;
  p.st = 3 * H * kHD;
  p.sh = kHD;
  p.ob = T * H * kHD;
  p.ot = H * kHD;
  p.oh = kHD;
  p.T = (int)T;
  p.H = (int)H;
  p.scale = (float)scale;
  p.scale_log2 = (float)(scale * 1.4426950408889634);
  return p;
}

std::vector<at::Tensor> attn_fwd(const at::Tensor& qkv, bool causal, double scale) {
  check_bf16(qkv, "qkv");
  TORCH_CHECK(attention_supported(qkv), "attention: qkv must be [B, T, 3, H, 64] with T % 128 == 0");
  const int64_t B = qkv.size(0), T = qkv.size(1), H = qkv.size(3);
  auto out = at::empty({B, T, H, kHD}, qkv.options());
  auto lse = at::empty({B, H, T}, qkv.options().dtype(at::kFloat));
  AttnParams p = attn_params(qkv, scale);
  p.out = (u16*)out.data_ptr();
  p.stat_out = lse.data_ptr<float>();
  dim3 grid((unsigned)(T / kQBlk), (unsigned)H, (unsigned)B);
  if (causal)
    hipLaunchKernelGGL(attn_fwd_kernel<true>, grid, dim3(256), 0, stream(), p);
  else
    hipLaunchKernelGGL(attn_fwd_kernel<false>, grid, dim3(256), 0, stream(), p);
  LAUNCH_CHECK();
  return {out, lse};
}

at::Tensor attn_bwd(const at::Tensor& dout, const at::Tensor& qkv, const at::Tensor& out, const at::Tensor& lse,
                    bool causal, double scale) {
  check_bf16(dout, "grad");
  check_bf16(qkv, "qkv");
  check_bf16(out, "out");
  TORCH_CHECK(dout.sizes() == out.sizes(), "attention: grad shape mismatch");
  const int64_t B = qkv.size(0), T = qkv.size(1), H = qkv.size(3);
  auto dqkv = at::empty_like(qkv);
  auto delta = at::empty({B, H, T}, qkv.options().dtype(at::kFloat));
  AttnParams p = attn_params(qkv, scale);
  p.o = (const u16*)out.data_ptr();
  p.dout = (const u16*)dout.data_ptr();
  p.stat_out = delta.data_ptr<float>();
  const int64_t rows = B * H * T;
  hipLaunchKernelGGL(attn_bwd_pre_kernel, dim3((unsigned)((rows + 31) / 32)), dim3(256), 0, stream(), p, rows);
  LAUNCH_CHECK();
  p.lse = lse.data_ptr<float>();
  p.delta = delta.data_ptr<float>();
  u16* dbase = (u16*)dqkv.data_ptr();
  dim3 grid((unsigned)(T / kQBlk), (unsigned)H, (unsigned)B);
  p.out = dbase + H * kHD;       // dK slot of the packed gradient
  p.out2 = dbase + 2 * H * kHD;  // dV slot
  if (causal)
    hipLaunchKernelGGL(attn_bwd_dkdv_kernel<true>, grid, dim3(256), 0, stream(), p);
  else
    hipLaunchKernelGGL(attn_bwd_dkdv_kernel<false>, grid, dim3(256), 0, stream(), p);
  LAUNCH_CHECK();
  p.out = dbase;  // dQ slot
  p.out2 = nullptr;
  if (causal)
    hipLaunchKernelGGL(attn_bwd_dq_kernel<true>, grid, dim3(256), 0, stream(), p);
  else
    hipLaunchKernelGGL(attn_bwd_dq_kernel<false>, grid, dim3(256), 0, stream(), p);
  LAUNCH_CHECK();
  return dqkv;
}

// (S, M) per row of every tensor in `words` (int64, contiguous, on one device): an int64
// [rows, 2] tensor, rows of each tensor in order (ceil(numel / 64 Ki) each).
at::Tensor state_digest(std::vector<at::Tensor> words) {
  TORCH_CHECK(!words.empty(), "state_digest: no tensors");
  const auto dev = words[0].device();
  std::vector<long long> table;
  for (auto& w : words) {
    TORCH_CHECK(w.scalar_type() == at::kLong && w.is_contiguous() && w.device() == dev,
                "state_digest: contiguous int64 tensors on one device");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(w.data_ptr()) % 8 == 0, "state_digest: 8-byte aligned data");
    const long long n = w.numel();
    const auto* p = reinterpret_cast<const unsigned long long*>(w.data_ptr());
    for (long long o = 0; o < n; o += kDigestRowWords) {
      table.push_back((long long)(uintptr_t)(p + o));
      table.push_back(std::min(kDigestRowWords, n - o));
      table.push_back(o);
    }
  }
  const long long rows = (long long)table.size() / 3;
  auto out = at::empty({rows, 2}, at::TensorOptions().dtype(at::kLong).device(dev));
  if (rows == 0) return out;
  static_assert(sizeof(DigestRow) == 3 * sizeof(long long), "row table layout");
  auto host = at::from_blob(table.data(), {rows * 3}, at::kLong).clone();
  auto dtab = host.to(dev, /*non_blocking=*/false);
  hipLaunchKernelGGL(state_digest_kernel, dim3((unsigned)rows), dim3(kBlock), 0, stream(),
                     reinterpret_cast<const DigestRow*>(dtab.data_ptr()), reinterpret_cast<long long*>(out.data_ptr()));
  LAUNCH_CHECK();
  return out;
}

// The same (S, M) pairs for int64 CPU tensors, one pass over the words, rows in parallel
// (torch's intra-op threads): what the rescue digests use for CPU-resident state when this
// extension is loaded (the torch-op formulation makes a dozen passes).
static inline unsigned long long mix64_host(unsigned long long z) {
  z ^= z >> 30;
  z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 27;
  z *= 0x94D049BB133111EBull;
  z ^= z >> 31;
  return z;
}

// one row: four words per iteration, independent chains (the multiplies overlap)
static void digest_row_host(const unsigned long long* p, long long b, long long e, unsigned long long* out) {
  const unsigned long long kGolden = 0x9E3779B97F4A7C15ull;
  unsigned long long S[4] = {0, 0, 0, 0}, M[4] = {0, 0, 0, 0};
  long long i = b;
  for (; i + 4 <= e; i += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const unsigned long long v = p[i + u];
      S[u] += v;
      M[u] += mix64_host(v ^ ((unsigned long long)(i + u + 1) * kGolden));
    }
  }
  for (; i < e; ++i) {
    S[0] += p[i];
    M[0] += mix64_host(p[i] ^ ((unsigned long long)(i + 1) * kGolden));
  }
  out[0] = S[0] + S[1] + S[2] + S[3];
  out[1] = M[0] + M[1] + M[2] + M[3];
}

at::Tensor state_digest_cpu(std::vector<at::Tensor> words) {
  struct Row {
    const unsigned long long* p;
    long long b, e;
  };
  std::vector<Row> rows;
  for (auto& w : words) {
    TORCH_CHECK(w.scalar_type() == at::kLong && w.is_contiguous() && w.device().is_cpu(),
                "state_digest_cpu: contiguous int64 CPU tensors");
    const auto* p = reinterpret_cast<const unsigned long long*>(w.data_ptr());
    const long long n = w.numel();
    for (long long o = 0; o < n; o += kDigestRowWords) rows.push_back({p, o, std::min(n, o + kDigestRowWords)});
  }
  auto out = at::empty({(long long)rows.size(), 2}, at::TensorOptions().dtype(at::kLong));
  auto* o = reinterpret_cast<unsigned long long*>(out.data_ptr());
  // rows over up to 8 threads (torch's intra-op thread count): a few threads saturate a socket's
  // memory bandwidth for this, and ranks of one pod digest at the same time
  const int nt = (int)std::max<long long>(1, std::min<long long>({(long long)rows.size(), 8LL,
                                                                   (long long)at::get_num_threads()}));
  std::atomic<size_t> next{0};
  auto work = [&]() {
    for (size_t r; (r = next.fetch_add(1)) < rows.size();) digest_row_host(rows[r].p, rows[r].b, rows[r].e, o + 2 * r);
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < nt; ++t) pool.emplace_back(work);
  work();
  for (auto& t : pool) t.join();
  return out;
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

// (s, y) = (x + delta, rmsnorm(x + delta) * w). Backward: d = ds + norm'(dy) for both x and
// delta (one kernel: the residual gradient is read inside the norm backward).
struct AddRMSNormFn : public torch::autograd::Function<AddRMSNormFn> {
  static variable_list forward(AutogradContext* ctx, const at::Tensor& x, const at::Tensor& delta, const at::Tensor& w,
                               double eps) {
    const int64_t D = x.size(-1);
    auto x2 = x.contiguous().view({-1, D});
    auto d2 = delta.contiguous().view({-1, D});
    auto w2 = w.contiguous();
    auto r = add_rmsnorm_fwd(x2, d2, w2, eps);
    ctx->save_for_backward({r[2], w2, r[1]});
    ctx->saved_data["shape"] = x.sizes().vec();
    return {r[2].view(x.sizes()), r[0].view(x.sizes())};
  }
  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    auto s = ctx->get_saved_variables();
    auto shape = ctx->saved_data["shape"].toIntVector();
    at::Tensor dy = grads[1].defined() ? grads[1].contiguous().view_as(s[0]) : at::zeros_like(s[0]);
    at::Tensor dres = grads[0].defined() ? grads[0].contiguous().view_as(s[0]) : at::Tensor();
    auto r = rmsnorm_bwd_impl(dy, s[0], dres.defined() ? &dres : nullptr, s[1], s[2]);
    auto dx = r[0].view(shape);
    return {dx, dx, r[1], at::Tensor()};
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

struct AttentionFn : public torch::autograd::Function<AttentionFn> {
  static at::Tensor forward(AutogradContext* ctx, const at::Tensor& qkv, bool causal, double scale) {
    auto qc = qkv.contiguous();
    auto r = attn_fwd(qc, causal, scale);
    ctx->save_for_backward({qc, r[0], r[1]});
    ctx->saved_data["causal"] = causal;
    ctx->saved_data["scale"] = scale;
    return r[0];
  }
  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    auto s = ctx->get_saved_variables();
    auto d = attn_bwd(grads[0].contiguous(), s[0], s[1], s[2], ctx->saved_data["causal"].toBool(),
                      ctx->saved_data["scale"].toDouble());
    return {d, at::Tensor(), at::Tensor()};
  }
};

at::Tensor attention(const at::Tensor& qkv, bool causal, double scale) {
  return AttentionFn::apply(qkv, causal, scale);
}

at::Tensor rms_norm(const at::Tensor& x, const at::Tensor& w, double eps) { return RMSNormFn::apply(x, w, eps); }

std::vector<at::Tensor> add_rms_norm(const at::Tensor& x, const at::Tensor& delta, const at::Tensor& w, double eps) {
  return AddRMSNormFn::apply(x, delta, w, eps);
}
at::Tensor swiglu(const at::Tensor& h) { return SwiGLUFn::apply(h); }
at::Tensor cross_entropy(const at::Tensor& logits, const at::Tensor& tgt, int64_t ignore_index) {
  return CrossEntropyFn::apply(logits, tgt, ignore_index);
}

}  // namespace

// SHA-256 of this file, passed by devspace_amd/ops/build.py: the loader checks the extension it
// imports was built from the source next to it (no stale kernels after an edit or a checkout)
#ifndef DEVSPACE_SOURCE_SHA
#define DEVSPACE_SOURCE_SHA "unknown"
#endif

PYBIND11_MODULE(_fused_ops, m) {
  m.doc() = "gfx950 fused training ops (RMSNorm, SwiGLU, cross-entropy)";
  m.attr("source_sha") = DEVSPACE_SOURCE_SHA;
  m.def("rmsnorm_supported", &rmsnorm_supported);
  // differentiable entry points (C++ autograd)
  m.def("rms_norm", &rms_norm);
  m.def("add_rms_norm", &add_rms_norm, "(x + delta, rmsnorm(x + delta) * w) with a fused backward");
  m.def("add_rmsnorm_fwd", &add_rmsnorm_fwd);
  m.def("swiglu", &swiglu);
  m.def("cross_entropy", &cross_entropy);
  m.def("adamw_step", &adamw_step);
  m.def("state_digest", &state_digest, "(sum, position-keyed mixed sum) per 64 Ki-word row of int64 tensors");
  m.def("state_digest_cpu", &state_digest_cpu, "state_digest for int64 CPU tensors (one pass, rows in parallel)");
  m.def("attention", &attention);
  m.def("attention_supported", &attention_supported);
  m.def("attn_fwd", &attn_fwd);
  m.def("attn_bwd", &attn_bwd);
  // raw kernels (tests / custom graphs)
  m.def("rmsnorm_fwd", &rmsnorm_fwd);
  m.def("rmsnorm_bwd", &rmsnorm_bwd);
  m.def("swiglu_fwd", &swiglu_fwd);
  m.def("swiglu_bwd", &swiglu_bwd);
  m.def("ce_fwd", &ce_fwd);
  m.def("ce_bwd", &ce_bwd);
}

// Norm / dot reductions for the regularisation + clipping terms of BiCNN
// (K11: f += λ1‖p‖₁, f += λ2‖p‖²/2, BiCNN/bicnn.lua:398-409) and for gradient-norm
// diagnostics. Deterministic two-pass: pass 1 = grid-stride float4 loads, per-wave
// shuffle reduction over 64 lanes, per-block LDS combine, one partial per block;
// pass 2 = one block folds the partials in a fixed order (no float atomics, so the
// result is bitwise reproducible — cdna_hip_programming.md Guideline 12).
#include "kernels.h"
#include "ew.h"
#include <algorithm>
#include <cmath>
#include <stdexcept>

namespace mpit {
namespace {

constexpr int kRB = 256;  // 4 waves

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

template <int NV>
__device__ __forceinline__ void block_reduce(float (&v)[NV], const bool (&is_max)[NV], float* lds) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = is_max[k] ? wave_max(v[k]) : wave_sum(v[k]);
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < NV; ++k) lds[wid * NV + k] = v[k];
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      float a = lds[k];
      for (int w = 1; w < kRB / 64; ++w) a = is_max[k] ? fmaxf(a, lds[w * NV + k]) : a + lds[w * NV + k];
      v[k] = a;
    }
  }
}

template <bool BF>
__global__ __launch_bounds__(kRB) void norms_pass1(const void* x, int64_t n, float* ws) {
  __shared__ float lds[(kRB / 64) * 3];
  float s1 = 0.f, s2 = 0.f, mx = 0.f;
  const int64_t n4 = n >> 2;
  const int64_t stride = int64_t(gridDim.x) * kRB;
  for (int64_t i = int64_t(blockIdx.x) * kRB + threadIdx.x; i < n4; i += stride) {
    float v[4];
    load4<BF>(x, i, v);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float a = fabsf(v[j]);
      s1 += a;
      s2 = fmaf(v[j], v[j], s2);
      mx = fmaxf(mx, a);
    }
  }
  if (blockIdx.x == 0) {
    const int64_t i = (n4 << 2) + threadIdx.x;
    if (i < n) {
      const float v = load1<BF>(x, i), a = fabsf(v);
      s1 += a; s2 = fmaf(v, v, s2); mx = fmaxf(mx, a);
    }
  }
  float r[3] = {s1, s2, mx};
  const bool im[3] = {false, false, true};
  block_reduce<3>(r, im, lds);
  if (threadIdx.x == 0) {
    ws[3 * blockIdx.x + 0] = r[0];
    ws[3 * blockIdx.x + 1] = r[1];
    ws[3 * blockIdx.x + 2] = r[2];
  }
}

__global__ __launch_bounds__(kRB) void norms_pass2(const float* ws, int nb, float* out) {
  __shared__ float lds[(kRB / 64) * 3];
  float r[3] = {0.f, 0.f, 0.f};
  for (int b = threadIdx.x; b < nb; b += kRB) {
    r[0] += ws[3 * b];
    r[1] += ws[3 * b + 1];
    r[2] = fmaxf(r[2], ws[3 * b + 2]);
  }
  const bool im[3] = {false, false, true};
  block_reduce<3>(r, im, lds);
  if (threadIdx.x == 0) { out[0] = r[0]; out[1] = r[1]; out[2] = r[2]; }
}

template <bool BF>
__global__ __launch_bounds__(kRB) void dot_pass1(const void* x, const void* y, int64_t n, float* ws) {
  __shared__ float lds[kRB / 64];
  float s = 0.f;
  const int64_t n4 = n >> 2;
  const int64_t stride = int64_t(gridDim.x) * kRB;
  for (int64_t i = int64_t(blockIdx.x) * kRB + threadIdx.x; i < n4; i += stride) {
    float a[4], b[4];
    load4<BF>(x, i, a);
    load4<BF>(y, i, b);
#pragma unroll
    for (int j = 0; j < 4; ++j) s = fmaf(a[j], b[j], s);
  }
  if (blockIdx.x == 0) {
    const int64_t i = (n4 << 2) + threadIdx.x;
    if (i < n) s = fmaf(load1<BF>(x, i), load1<BF>(y, i), s);
  }
  float r[1] = {s};
  const bool im[1] = {false};
  block_reduce<1>(r, im, lds);
  if (threadIdx.x == 0) ws[blockIdx.x] = r[0];
}

__global__ __launch_bounds__(kRB) void sum_pass2(const float* ws, int nb, float* out) {
  __shared__ float lds[kRB / 64];
  float r[1] = {0.f};
  for (int b = threadIdx.x; b < nb; b += kRB) r[0] += ws[b];
  const bool im[1] = {false};
  block_reduce<1>(r, im, lds);
  if (threadIdx.x == 0) out[0] = r[0];
}

int nblocks(int64_t n) {
  const int64_t n4 = std::max<int64_t>(1, n >> 2);
  return int(std::max<int64_t>(1, std::min<int64_t>((n4 + kRB - 1) / kRB, kNormMaxBlocks)));
}

bool aligned(const void* p, bool bf) { return reinterpret_cast<uintptr_t>(p) % (bf ? 8 : 16) == 0; }

// Clamped running sum over examples (K11 per example, BiCNN/bicnn.lua:398-409): every
// violating example adds its gradient and the regulariser to the accumulated gradient,
// which is then clamped — G = clamp(G + g_k + l1*sign(p) + l2*p, -c, c) for k = 0..n-1.
// Sequential in k, independent in the element: one thread owns 4 consecutive elements
// (float4 loads of every row g_k, coalesced across the wave), G stays in registers.
__device__ __forceinline__ float clampc(float v, float c) { return c > 0.f ? fminf(fmaxf(v, -c), c) : v; }

__global__ __launch_bounds__(kRB) void clamp_scan_kernel(float* __restrict__ G, const float* __restrict__ g,
                                                          const float* __restrict__ p, int64_t P, int64_t ldg, int n,
                                                          float l1, float l2, float c) {
  const int64_t i4 = int64_t(blockIdx.x) * kRB + threadIdx.x;
  const int64_t base = i4 * 4;
  if (base >= P) return;
  if (base + 4 <= P) {
    float4 acc = *reinterpret_cast<const float4*>(G + base);
    const float4 pv = *reinterpret_cast<const float4*>(p + base);
    const float r[4] = {l1 * ((pv.x > 0.f) - (pv.x < 0.f)) + l2 * pv.x, l1 * ((pv.y > 0.f) - (pv.y < 0.f)) + l2 * pv.y,
                        l1 * ((pv.z > 0.f) - (pv.z < 0.f)) + l2 * pv.z, l1 * ((pv.w > 0.f) - (pv.w < 0.f)) + l2 * pv.w};
    for (int k = 0; k < n; ++k) {
      const float4 v = *reinterpret_cast<const float4*>(g + int64_t(k) * ldg + base);
      acc.x = clampc(acc.x + v.x + r[0], c);
      acc.y = clampc(acc.y + v.y + r[1], c);
      acc.z = clampc(acc.z + v.z + r[2], c);
      acc.w = clampc(acc.w + v.w + r[3], c);
    }
    *reinterpret_cast<float4*>(G + base) = acc;
  } else {
    for (int64_t j = base; j < P; ++j) {
      float a = G[j];
      const float r = l1 * ((p[j] > 0.f) - (p[j] < 0.f)) + l2 * p[j];
      for (int k = 0; k < n; ++k) a = clampc(a + g[int64_t(k) * ldg + j] + r, c);
      G[j] = a;
    }
  }
}

}  // namespace

void clamp_scan(int dev, hipStream_t s, float* G, const float* g, const float* p, int64_t P, int64_t ldg, int n,
                float l1, float l2, float c) {
  if (n <= 0 || P <= 0) return;
  if (dev < 0) {
    for (int64_t j = 0; j < P; ++j) {
      float a = G[j];
      const float r = l1 * float((p[j] > 0.f) - (p[j] < 0.f)) + l2 * p[j];
      for (int k = 0; k < n; ++k) {
        a = a + g[int64_t(k) * ldg + j] + r;
        if (c > 0.f) a = std::min(std::max(a, -c), c);
      }
      G[j] = a;
    }
    return;
  }
  if (!aligned(G, false) || !aligned(g, false) || !aligned(p, false) || ldg % 4)
    throw std::invalid_argument("mpit.clamp_scan: fp32 operands must be 16-B aligned, ldg % 4 == 0");
  hip_check(hipSetDevice(dev), "hipSetDevice");
  const int64_t threads = (P + 3) / 4;
  hipLaunchKernelGGL(clamp_scan_kernel, dim3(unsigned((threads + kRB - 1) / kRB)), dim3(kRB), 0, s, G, g, p, P, ldg, n,
                     l1, l2, c);
  hip_check(hipGetLastError(), "clamp_scan launch");
}

void norms(int dev, hipStream_t s, const void* x, bool bf16, int64_t n, float* out, float* ws) {
  if (dev < 0) {
    double s1 = 0, s2 = 0;
    float mx = 0.f;
    for (int64_t i = 0; i < n; ++i) {
      const float v = bf16 ? load1<true>(x, i) : load1<false>(x, i);
      s1 += std::fabs(v); s2 += double(v) * v; mx = std::max(mx, std::fabs(v));
    }
    out[0] = float(s1); out[1] = float(s2); out[2] = mx;
    return;
  }
  if (!aligned(x, bf16)) throw std::invalid_argument("mpit.norms: operand must be 16-B (fp32) / 8-B (bf16) aligned");
  hip_check(hipSetDevice(dev), "hipSetDevice");
  const int nb = nblocks(n);
  if (bf16) hipLaunchKernelGGL(norms_pass1<true>, dim3(nb), dim3(kRB), 0, s, x, n, ws);
  else hipLaunchKernelGGL(norms_pass1<false>, dim3(nb), dim3(kRB), 0, s, x, n, ws);
  hipLaunchKernelGGL(norms_pass2, dim3(1), dim3(kRB), 0, s, ws, nb, out);
  hip_check(hipGetLastError(), "norms launch");
}

void dot(int dev, hipStream_t s, const void* x, const void* y, bool bf16, int64_t n, float* out, float* ws) {
  if (dev < 0) {
    double acc = 0;
    for (int64_t i = 0; i < n; ++i)
      acc += double(bf16 ? load1<true>(x, i) : load1<false>(x, i)) * (bf16 ? load1<true>(y, i) : load1<false>(y, i));
    out[0] = float(acc);
    return;
  }
  if (!aligned(x, bf16) || !aligned(y, bf16))
    throw std::invalid_argument("mpit.dot: operands must be 16-B (fp32) / 8-B (bf16) aligned");
  hip_check(hipSetDevice(dev), "hipSetDevice");
  const int nb = nblocks(n);
  if (bf16) hipLaunchKernelGGL(dot_pass1<true>, dim3(nb), dim3(kRB), 0, s, x, y, n, ws);
  else hipLaunchKernelGGL(dot_pass1<false>, dim3(nb), dim3(kRB), 0, s, x, y, n, ws);
  hipLaunchKernelGGL(sum_pass2, dim3(1), dim3(kRB), 0, s, ws, nb, out);
  hip_check(hipGetLastError(), "dot launch");
}

}  // namespace mpit

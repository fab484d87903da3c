// Norm / dot reductions for the regularisation + clipping terms of BiCNN
// (K11: f += λ1‖p‖₁, f += λ2‖p‖²/2, BiCNN/bicnn.lua:398-409) and for gradient-norm
// diagnostics. Deterministic two-pass: pass 1 = grid-stride float4 loads, per-wave
// shuffle reduction over 64 lanes, per-block LDS combine, one partial per block;
// pass 2 = one block folds the partials in a fixed order (no float atomics, so the
// result is bitwise reproducible — cdna_hip_programming.md Guideline 12).
#include "kernels.h"
#include "ew.h"
#include <cmath>

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

}  // namespace

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

// Softmax cross-entropy of the classifier's logits (ops/loss.py; the reference trains with
// nn.CrossEntropyCriterion / ClassNLLCriterion over LogSoftMax, asyncsgd/goot.lua): one block
// per row, three sweeps over the row's C logits (bf16 or fp32, math in fp32):
//   max m, sum s = sum exp(x - m)  (block reductions in a fixed order: deterministic),
//   loss[r] = log(s) + m - x[t]    (NaN for a target outside [0, C)),
//   d[r][c] = (exp(x[c] - m) / s - [c == t]) * scale   (fp32: the logits' gradient of the mean
//   loss for scale = 1 / rows, stashed by the forward so the backward is one multiply).
// Replaces PyTorch's log_softmax + nll_loss forward and their backward (six launches, plus the
// bf16 -> fp32 cast of bf16 logits) with one launch and a mean.
#include <hip/hip_runtime.h>

#include <cmath>
#include <stdexcept>

#include "ew.h"
#include "kernels.h"

namespace mpit {
namespace {

constexpr int kXentThreads = 256;

template <typename T>
__device__ __forceinline__ float ldx(const T* p, int64_t i) {
  if constexpr (sizeof(T) == 4) return p[i];
  else return bf2f(p[i]);
}

// every thread of the block gets the result; red: >= kXentThreads / 64 floats of LDS
template <bool MAX>
__device__ __forceinline__ float block_reduce(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float u = __shfl_xor(v, o);
    v = MAX ? fmaxf(v, u) : v + u;
  }
  const int w = threadIdx.x >> 6;
  __syncthreads();  // (an earlier reduction is done reading red)
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float r = red[0];
  for (int k = 1; k < kXentThreads / 64; ++k) r = MAX ? fmaxf(r, red[k]) : r + red[k];
  return r;
}

template <typename T>
__global__ __launch_bounds__(kXentThreads) void softmax_xent_kernel(const T* __restrict__ x, int64_t ldx_,
                                                                     const int64_t* __restrict__ tgt, int C,
                                                                     float scale, float* __restrict__ loss,
                                                                     float* __restrict__ d) {
  __shared__ float red[kXentThreads / 64];
  const int64_t r = blockIdx.x;
  const T* xr = x + r * ldx_;
  float m = -INFINITY;
  for (int c = threadIdx.x; c < C; c += kXentThreads) m = fmaxf(m, ldx(xr, c));
  m = block_reduce<true>(m, red);
  float s = 0.f;
  for (int c = threadIdx.x; c < C; c += kXentThreads) s += expf(ldx(xr, c) - m);
  s = block_reduce<false>(s, red);
  const int64_t t = tgt[r];
  const bool ok = t >= 0 && t < C;
  if (threadIdx.x == 0) loss[r] = ok ? logf(s) + m - ldx(xr, t) : NAN;
  const float inv = 1.f / s;
  float* dr = d + r * int64_t(C);
  for (int c = threadIdx.x; c < C; c += kXentThreads)
    dr[c] = (expf(ldx(xr, c) - m) * inv - (c == t ? 1.f : 0.f)) * scale;
}

}  // namespace

void softmax_xent(int dev, hipStream_t s, int64_t rows, int C, uintptr_t x, int64_t ldx, bool bf16, uintptr_t tgt,
                  float scale, uintptr_t loss, uintptr_t d) {
  if (rows <= 0 || C <= 0 || ldx < C) throw std::invalid_argument("softmax_xent: bad shape");
  if (rows > INT32_MAX) throw std::invalid_argument("softmax_xent: too many rows");
  if (!x || !tgt || !loss || !d) throw std::invalid_argument("softmax_xent: null pointer");
  hip_check(hipSetDevice(dev), "hipSetDevice");
  const dim3 g{unsigned(rows)}, b{unsigned(kXentThreads)};
  if (bf16)
    hipLaunchKernelGGL(softmax_xent_kernel<uint16_t>, g, b, 0, s, reinterpret_cast<const uint16_t*>(x), ldx,
                       reinterpret_cast<const int64_t*>(tgt), C, scale, reinterpret_cast<float*>(loss),
                       reinterpret_cast<float*>(d));
  else
    hipLaunchKernelGGL(softmax_xent_kernel<float>, g, b, 0, s, reinterpret_cast<const float*>(x), ldx,
                       reinterpret_cast<const int64_t*>(tgt), C, scale, reinterpret_cast<float*>(loss),
                       reinterpret_cast<float*>(d));
  hip_check(hipGetLastError(), "softmax_xent launch");
}

}  // namespace mpit

// fp16 planes of an fp32 tensor (the fp16x3 GEMM operands, gemm.hip FM 13): the producer of
// an activation or gradient writes h = f16(x 2^e) and l = f16(2^11 (x 2^e - h)) — gemm.hip
// split1h's arithmetic, both residual steps exact — h at element i and l at element numel + i
// of the tensor's 16-bit view (same 4 bytes per element as fp32). e comes from a bound of |x|
// known before the pass (kernels.h PlaneSpec), published in slot 0 of the planes' slotted
// bound so the consumers scale with the same e.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.h"

namespace mpit {

// the maximum a GEMM epilogue left in epoch slots (gemm.hip EpiArgs::omax): 64-bit (epoch,
// |value| bits) maxima, slot blockIdx % kBoundSlots; a slot of an older epoch holds nothing of ours
__device__ __forceinline__ float epoch_max(const unsigned long long* p, uint32_t ep) {
  float m = 0.f;
  if (p == nullptr) return m;
#pragma unroll
  for (int k = 0; k < kBoundSlots; ++k) {
    const unsigned long long v = __hip_atomic_load(p + k * (kBoundStride / 2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (uint32_t(v >> 32) == ep) m = fmaxf(m, __uint_as_float(uint32_t(v)));
  }
  return m;
}
// the same, one slot per lane and a wave reduction (no loop per thread): every lane of the
// wave must call it
__device__ __forceinline__ float epoch_max_wave(const unsigned long long* p, uint32_t ep) {
  float m = 0.f;
  const int l = threadIdx.x & 63;
  if (p != nullptr && l < kBoundSlots) {
    const unsigned long long v = __hip_atomic_load(p + l * (kBoundStride / 2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (uint32_t(v >> 32) == ep) m = __uint_as_float(uint32_t(v));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  return m;
}
// max |coefficient| over the C channels from the coefficients the apply threads already hold
// in registers (m[n] = the thread's max of row n): a wave's 64 lanes x 8 elements are 512
// consecutive elements and a block's 8 * blockDim >= C (bn_act.hip block_for), so a wave
// reduction covers every channel when C <= 512 and a block one otherwise. Replaces a loop of
// C / 64 coefficient loads per row and wave (the fp32 apply passes run one 512-element slot
// per wave: those loads outnumbered the pass's own). Every thread of the block must call it
// (C is block-uniform, so is the barrier).
template <int N>
__device__ __forceinline__ void coef_max_block(float (&m)[N], int C) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int n = 0; n < N; ++n) m[n] = fmaxf(m[n], __shfl_xor(m[n], o));
  if (C > 512) {
    __shared__ float sm[N][16];
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    if ((threadIdx.x & 63) == 0)
#pragma unroll
      for (int n = 0; n < N; ++n) sm[n][w] = m[n];
    __syncthreads();
#pragma unroll
    for (int n = 0; n < N; ++n) {
      float r = 0.f;
      for (int k = 0; k < nw; ++k) r = fmaxf(r, sm[n][k]);
      m[n] = r;
    }
  }
}
// a thread's max |v| over its 8 per-element coefficients
__device__ __forceinline__ float abs_max8(const float (&v)[8]) {
  float m = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) m = fmaxf(m, fabsf(v[k]));
  return m;
}
// slots_max with one slot per lane and a wave reduction (every lane of the wave calls it)
__device__ __forceinline__ float slots_max_wave(const float* p) {
  const int l = threadIdx.x & 63;
  float m = l < kBoundSlots ? p[l * kBoundStride] : 0.f;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  return m;
}
// the bound a slotted buffer holds (max over its slots)
__device__ __forceinline__ float slots_max(const float* p) {
  float a = p[0];
#pragma unroll
  for (int k = 1; k < kBoundSlots; ++k) a = fmaxf(a, p[k * kBoundStride]);
  return a;
}
// gemm.hip fp16_exp on a value: a * 2^e in [2^13, 2^14) (0 for a zero / non-finite bound)
__device__ __forceinline__ int plane_exp(float a) {
  if (!(a > 0.f) || !(a <= 3.0e38f)) return 0;
  int x;
  (void)frexpf(a, &x);
  return min(116, max(-126, 14 - x));
}
__device__ __forceinline__ float pexp2(int e) { return __uint_as_float(uint32_t(e + 127) << 23); }
struct PlaneScale {
  float s, s11;  // 2^e, 2^(e + 11)
};
// every block computes the same bound (same inputs; max is order-free): block 0 publishes it
__device__ __forceinline__ PlaneScale plane_scale(float bound, float* obound) {
  const int e = plane_exp(bound);
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < kBoundSlots)
    obound[threadIdx.x * kBoundStride] = threadIdx.x == 0 ? bound : 0.f;
  return {pexp2(e), pexp2(e + 11)};
}
typedef float pf32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 pf16x2 __attribute__((ext_vector_type(2)));
// two values -> (h, l) pairs as packed dwords
__device__ __forceinline__ void split_pair(float a, float b, PlaneScale ps, uint32_t& hw, uint32_t& lw) {
  const pf32x2 x = {a, b};
  const pf16x2 hp = __builtin_convertvector(x * ps.s, pf16x2);
  const pf32x2 r = x * ps.s11 - __builtin_convertvector(hp, pf32x2) * 2048.f;
  hw = __builtin_bit_cast(uint32_t, hp);
  lw = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, pf16x2));
}
// a packed (h, l) pair back to two floats: (h + l 2^-11) 2^-e, exact
__device__ __forceinline__ pf32x2 join_pair(uint32_t hw, uint32_t lw, float inv) {
  const pf32x2 hf = __builtin_convertvector(__builtin_bit_cast(pf16x2, hw), pf32x2);
  const pf32x2 lf = __builtin_convertvector(__builtin_bit_cast(pf16x2, lw), pf32x2);
  return (hf + lf * (1.f / 2048.f)) * inv;
}

}  // namespace mpit

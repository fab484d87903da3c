// The fp16x3 operand of the 7x7 stem's weight, in ONE launch per step.
//
// The stem convolution (gemm.hip conv_stem_*) reads its weight as a zero-extended
// [Co][8][8][4] image (kernel rows of 8 pixels x 4 channels). In an fp32 step that image
// goes to the fp16x3 GEMM as two fp16 planes (h, l) of the weight scaled by 2^e, e from the
// bound max |w|. Built from PyTorch ops that was ~15 small launches (copy into the
// zero-extended buffer, an inf-norm reduction, the slotted bound buffer, frexp / where /
// the plane arithmetic, stack) with host gaps between them at the very start of the step,
// while the GPU had nothing else queued (profiles/boundary_r04/README.md). Here one block
// reduces max |w| (the stem weight is small: 64 x 3 x 7 x 7), writes the slotted bound
// (slot 0 = max |w|, the others 0: the layout of ops/conv.py bound_of_value) and the two
// planes, with the arithmetic of ops/conv.py f16_planes (bitwise the same planes).
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <cmath>
#include <stdexcept>

#include "ew.h"
#include "kernels.h"
#include "stem_pack.h"

namespace mpit {
namespace {

constexpr int kSB = 1024;

// ops/conv.py _f16_exp: e with amax * 2^e in [2^13, 2^14), clamped; 0 for a zero / non-finite bound
__device__ __forceinline__ int f16_exp_of(float amax) {
  if (!(amax > 0.f) || !isfinite(amax)) return 0;
  int ex;
  (void)frexpf(amax, &ex);
  return min(max(14 - ex, -126), 116);
}

__device__ __forceinline__ float exp2i_f(int e) { return __int_as_float((e + 127) << 23); }

// w: [Co][R][S][C] (a channels_last [Co, C, R, S] weight); planes: [2][Co][8][8][4] fp16;
// bound: kBoundFloats fp32 (slotted)
__global__ __launch_bounds__(kSB) void stem_weight_planes_kernel(const float* __restrict__ w, int Co, int C, int R,
                                                                 int S, __half* __restrict__ planes,
                                                                 float* __restrict__ bound) {
  __shared__ float red[kSB / 64];
  const int t = threadIdx.x;
  const int n = Co * R * S * C;
  float m = 0.f;
  for (int i = t; i < n; i += kSB) m = fmaxf(m, fabsf(w[i]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((t & 63) == 0) red[t >> 6] = m;
  __syncthreads();
  float amax = red[0];
#pragma unroll
  for (int k = 1; k < kSB / 64; ++k) amax = fmaxf(amax, red[k]);
  for (int i = t; i < kBoundFloats; i += kSB) bound[i] = i == 0 ? amax : 0.f;
  const int e = f16_exp_of(amax);
  const float s = exp2i_f(e), s11 = exp2i_f(e + 11);
  const int np = Co * 8 * 8 * 4;
  for (int i = t; i < np; i += kSB) {
    const int c = i & 3, kw = (i >> 2) & 7, kh = (i >> 5) & 7, co = i >> 8;
    const float v = (c < C && kw < S && kh < R) ? w[((co * R + kh) * S + kw) * C + c] : 0.f;
    const __half h = __float2half_rn(v * s);
    // v * 2^(e+11) and h * 2^11 are exact: one rounding, as the PyTorch expression
    const float lo = v * s11 - __half2float(h) * 2048.f;
    planes[i] = h;
    planes[np + i] = __float2half_rn(lo);
  }
}

}  // namespace

void stem_weight_planes(int dev, hipStream_t s, uintptr_t w, int Co, int C, int R, int S, uintptr_t planes,
                        uintptr_t bound) {
  if (C > 4 || R > 8 || S > 8 || Co <= 0) throw std::invalid_argument("stem_weight_planes: the stem packs <= 8x8 taps of <= 4 channels");
  if (!w || !planes || !bound) throw std::invalid_argument("stem_weight_planes: null buffer");
  hip_check(hipSetDevice(dev), "hipSetDevice");
  hipLaunchKernelGGL(stem_weight_planes_kernel, dim3(1), dim3(kSB), 0, s, reinterpret_cast<const float*>(w), Co, C,
                     R, S, reinterpret_cast<__half*>(planes), reinterpret_cast<float*>(bound));
  hip_check(hipGetLastError(), "stem_weight_planes launch");
}

}  // namespace mpit

// NHWC bf16 / fp32 max pooling (ResNet stem: 3x3, stride 2, pad 1) with a one-byte argmax.
//
// Forward: one thread owns 8 channels (16 B bf16 / 32 B fp32) of one output pixel, reads its KxK window
// (16-B loads, channels contiguous), writes the max and the window index of the max
// (uint8, first maximum in scan order like PyTorch; a NaN wins and propagates).
// Backward: one thread owns 8 channels of one INPUT pixel and gathers the gradients of
// the (at most ceil(K/stride)^2) output windows that selected it — a gather, so no
// atomics and no zero-fill pass: dx is written exactly once. PyTorch's NHWC
// max_pool_backward walks the same windows but at ~6x the time (rocprof, profiles/).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <stdexcept>
#include <string>

#include "ew.h"
#include "kernels.h"
#include "planes.h"

namespace mpit {
namespace {

struct PoolGeo {
  int N, H, W, C, Ho, Wo, K, stride, pad;
};

// 8 channels of T as floats
__device__ __forceinline__ void ld8(const uint16_t* p, float (&f)[8]) {
  const uint4 v = *reinterpret_cast<const uint4*>(p);
  const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int e = 0; e < 8; ++e) f[e] = bf2f(uint16_t((u[e >> 1] >> (16 * (e & 1))) & 0xffff));
}
__device__ __forceinline__ void ld8(const float* p, float (&f)[8]) {
  const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w;
  f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}
__device__ __forceinline__ void st8(uint16_t* p, const float (&f)[8]) {
  uint4 o;
  uint32_t* op = &o.x;
#pragma unroll
  for (int e = 0; e < 4; ++e) op[e] = uint32_t(f2bf(f[2 * e])) | (uint32_t(f2bf(f[2 * e + 1])) << 16);
  *reinterpret_cast<uint4*>(p) = o;
}
__device__ __forceinline__ void st8(float* p, const float (&f)[8]) {
  reinterpret_cast<float4*>(p)[0] = make_float4(f[0], f[1], f[2], f[3]);
  reinterpret_cast<float4*>(p)[1] = make_float4(f[4], f[5], f[6], f[7]);
}

// I: index type of the pixel decomposition — uint32_t whenever the tensor allows (64-bit
// divisions are emulated and made these kernels 2.5x slower than their bytes)
template <typename T, typename I>
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                          uint8_t* __restrict__ idx, PoolGeo g,
                                                          const float* __restrict__ ibound, float* obound) {
  const I cv = I(g.C / 8);
  // fp16 planes output (fp32, obound != null): every output is one of the inputs, so the
  // input's bound is the output's (planes.h)
  [[maybe_unused]] PlaneScale ps{1.f, 2048.f};
  const int64_t nel = int64_t(g.N) * g.Ho * g.Wo * g.C;
  if constexpr (sizeof(T) == 4) {
    if (obound) ps = plane_scale(slots_max_wave(ibound), obound);
  }
  const I total = I(g.N) * I(g.Ho) * I(g.Wo) * cv;
  for (I t = I(blockIdx.x) * blockDim.x + threadIdx.x; t < total; t += I(gridDim.x) * blockDim.x) {
    const int c8 = int(t % cv);
    const I pix = t / cv;
    const int wo = int(pix % I(g.Wo));
    const I r = pix / I(g.Wo);
    const int ho = int(r % I(g.Ho));
    const int64_t n = int64_t(r / I(g.Ho));
    float best[8];
    uint8_t arg[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      best[e] = -__builtin_inff();
      arg[e] = 0;
    }
    const int h0 = ho * g.stride - g.pad, w0 = wo * g.stride - g.pad;
    for (int i = 0; i < g.K; ++i) {
      const int h = h0 + i;
      if (unsigned(h) >= unsigned(g.H)) continue;
      for (int j = 0; j < g.K; ++j) {
        const int w = w0 + j;
        if (unsigned(w) >= unsigned(g.W)) continue;
        float fv[8];
        ld8(x + ((n * g.H + h) * g.W + w) * g.C + c8 * 8, fv);
        const uint8_t k = uint8_t(i * g.K + j);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float f = fv[e];
          if (f > best[e] || (f != f && best[e] == best[e])) {
            best[e] = f;
            arg[e] = k;
          }
        }
      }
    }
    if (sizeof(T) == 4 && obound) {
      uint32_t hw[4], lw[4];
#pragma unroll
      for (int p = 0; p < 4; ++p) split_pair(best[2 * p], best[2 * p + 1], ps, hw[p], lw[p]);
      uint16_t* yh = reinterpret_cast<uint16_t*>(y) + int64_t(pix) * g.C + c8 * 8;
      *reinterpret_cast<uint4*>(yh) = make_uint4(hw[0], hw[1], hw[2], hw[3]);
      *reinterpret_cast<uint4*>(yh + nel) = make_uint4(lw[0], lw[1], lw[2], lw[3]);
    } else {
      st8(y + int64_t(pix) * g.C + c8 * 8, best);
    }
    uint2 a;
    a.x = uint32_t(arg[0]) | (uint32_t(arg[1]) << 8) | (uint32_t(arg[2]) << 16) | (uint32_t(arg[3]) << 24);
    a.y = uint32_t(arg[4]) | (uint32_t(arg[5]) << 8) | (uint32_t(arg[6]) << 16) | (uint32_t(arg[7]) << 24);
    *reinterpret_cast<uint2*>(idx + int64_t(pix) * g.C + c8 * 8) = a;
  }
}

// RB (a ReLU'd conv(+bias) below the pool, VGG / AlexNet): the gradient that reaches the
// pool's input is dz = dx * (y > 0) with y the pool's input; at a window's argmax y equals the
// pooled value, so the mask is ypool > 0, read per window. Each thread also accumulates the
// channel sums of what it writes (the conv's bias gradient): the grid-stride step is a
// multiple of C / 8 (host-checked), so a thread's 8 channels never change; per block the
// sums go through LDS into part[block][C].
template <typename T, typename I, bool RB>
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const T* __restrict__ dy,
                                                          const uint8_t* __restrict__ idx, T* __restrict__ dx,
                                                          PoolGeo g, const T* __restrict__ ypool,
                                                          float* __restrict__ part) {
  const I cv = I(g.C / 8);
  const I total = I(g.N) * I(g.H) * I(g.W) * cv;
  float bsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (I t = I(blockIdx.x) * blockDim.x + threadIdx.x; t < total; t += I(gridDim.x) * blockDim.x) {
    const int c8 = int(t % cv);
    const I pix = t / cv;
    const int w = int(pix % I(g.W));
    const I r = pix / I(g.W);
    const int h = int(r % I(g.H));
    const int64_t n = int64_t(r / I(g.H));
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // output windows containing h: ho*stride - pad <= h <= ho*stride - pad + K - 1
    const int hlo = max(0, (h + g.pad - g.K + g.stride) / g.stride), hhi = min(g.Ho - 1, (h + g.pad) / g.stride);
    const int wlo = max(0, (w + g.pad - g.K + g.stride) / g.stride), whi = min(g.Wo - 1, (w + g.pad) / g.stride);
    for (int ho = hlo; ho <= hhi; ++ho) {
      const int i = h - (ho * g.stride - g.pad);
      if (i < 0 || i >= g.K) continue;
      for (int wo = wlo; wo <= whi; ++wo) {
        const int j = w - (wo * g.stride - g.pad);
        if (j < 0 || j >= g.K) continue;
        const int64_t o = ((n * g.Ho + ho) * g.Wo + wo) * g.C + c8 * 8;
        const uint2 a = *reinterpret_cast<const uint2*>(idx + o);
        float gv[8];
        ld8(dy + o, gv);
        float yv[8];
        if constexpr (RB) ld8(ypool + o, yv);
        const uint8_t k = uint8_t(i * g.K + j);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint8_t ae = uint8_t(((e < 4 ? a.x : a.y) >> (8 * (e & 3))) & 0xff);
          bool take = ae == k;
          if constexpr (RB) take = take && yv[e] > 0.f;
          if (take) acc[e] += gv[e];
        }
      }
    }
    if constexpr (RB) {
      float q[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) q[e] = acc[e];
      st8(dx + int64_t(pix) * g.C + c8 * 8, q);
      if constexpr (sizeof(T) == 2) {  // the bias gradient of the values as stored
#pragma unroll
        for (int e = 0; e < 8; ++e) bsum[e] += bf2f(f2bf(acc[e]));
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) bsum[e] += acc[e];
      }
    } else {
      st8(dx + int64_t(pix) * g.C + c8 * 8, acc);
    }
  }
  if constexpr (RB) {
    __shared__ float red[256 * 8];
#pragma unroll
    for (int e = 0; e < 8; ++e) red[threadIdx.x * 8 + e] = bsum[e];
    // LDS hand-off only: a __syncthreads() fence would first wait for every dx store above
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int cvi = g.C / 8;
    for (int c = threadIdx.x; c < g.C; c += blockDim.x) {
      const int c8 = c / 8, e = c % 8;
      float sum = 0.f;
      // the threads whose channel group is c8: tid % cv == c8 (cv divides 256)
      for (int tid = c8; tid < 256; tid += cvi) sum += red[tid * 8 + e];
      part[int64_t(blockIdx.x) * g.C + c] = sum;
    }
  }
}

// Backward of a pool whose windows partition the input (K == stride, pad == 0: VGG's 2x2 / 2):
// one thread per OUTPUT window x 8 channels reads the window's argmax, gradient (and pooled
// value, RB) once and writes all K x K input pixels of the window (zeros off the argmax) —
// the input-pixel gather above reads each window K^2 times. Input rows / columns past the last
// full window (H % K) get zeros. RB as above: mask ypool > 0, channel sums of what is stored.
template <typename T, typename I, bool RB>
__global__ __launch_bounds__(256) void maxpool_bwd_part_kernel(const T* __restrict__ dy,
                                                               const uint8_t* __restrict__ idx, T* __restrict__ dx,
                                                               PoolGeo g, const T* __restrict__ ypool,
                                                               float* __restrict__ part) {
  const I cv = I(g.C / 8);
  const I total = I(g.N) * I(g.Ho) * I(g.Wo) * cv;
  float bsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (I t = I(blockIdx.x) * blockDim.x + threadIdx.x; t < total; t += I(gridDim.x) * blockDim.x) {
    const int c8 = int(t % cv);
    const I pix = t / cv;
    const int wo = int(pix % I(g.Wo));
    const I r = pix / I(g.Wo);
    const int ho = int(r % I(g.Ho));
    const int64_t n = int64_t(r / I(g.Ho));
    const int64_t o = int64_t(pix) * g.C + c8 * 8;
    const uint2 a = *reinterpret_cast<const uint2*>(idx + o);
    float gv[8];
    ld8(dy + o, gv);
    if constexpr (RB) {
      float yv[8];
      ld8(ypool + o, yv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if (!(yv[e] > 0.f)) gv[e] = 0.f;
        if constexpr (sizeof(T) == 2) bsum[e] += bf2f(f2bf(gv[e]));
        else bsum[e] += gv[e];
      }
    }
    for (int i = 0; i < g.K; ++i) {
      const int h = ho * g.K + i;
      for (int j = 0; j < g.K; ++j) {
        const int w = wo * g.K + j;
        const uint8_t k = uint8_t(i * g.K + j);
        float q[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint8_t ae = uint8_t(((e < 4 ? a.x : a.y) >> (8 * (e & 3))) & 0xff);
          q[e] = ae == k ? gv[e] : 0.f;
        }
        st8(dx + ((n * g.H + h) * g.W + w) * g.C + c8 * 8, q);
      }
    }
    // the rows / columns no window covers (H or W not a multiple of K) get zeros
    const float z[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (wo == g.Wo - 1)
      for (int i = 0; i < g.K; ++i)
        for (int w = g.Wo * g.K; w < g.W; ++w) st8(dx + ((n * g.H + ho * g.K + i) * g.W + w) * g.C + c8 * 8, z);
    if (ho == g.Ho - 1)
      for (int h = g.Ho * g.K; h < g.H; ++h)
        for (int w = wo * g.K; w < (wo == g.Wo - 1 ? g.W : wo * g.K + g.K); ++w)
          st8(dx + ((n * g.H + h) * g.W + w) * g.C + c8 * 8, z);
  }
  if constexpr (RB) {
    __shared__ float red[256 * 8];
#pragma unroll
    for (int e = 0; e < 8; ++e) red[threadIdx.x * 8 + e] = bsum[e];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int cvi = g.C / 8;
    for (int c = threadIdx.x; c < g.C; c += blockDim.x) {
      const int c8 = c / 8, e = c % 8;
      float sum = 0.f;
      for (int tid = c8; tid < 256; tid += cvi) sum += red[tid * 8 + e];
      part[int64_t(blockIdx.x) * g.C + c] = sum;
    }
  }
}

// Backward of a global average pool over an NHWC image: dx[n, p, c] = dy[n, c] / HW, one thread
// per 8 channels of one pixel (16-B bf16 / 32-B fp32 writes). PyTorch's expand + copy into the
// channels_last gradient ran at ~1 TB/s (~80-100 us per ResNet-50 step).
template <typename T>
__global__ __launch_bounds__(256) void avgpool_bwd_kernel(const T* __restrict__ dy, T* __restrict__ dx, int64_t total,
                                                          int HW, int C, float inv) {
  const int64_t cv = C / 8;
  for (int64_t t = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; t < total; t += int64_t(gridDim.x) * blockDim.x) {
    const int c8 = int(t % cv);
    const int64_t pix = t / cv;
    const int64_t n = pix / HW;
    float v[8];
    ld8(dy + n * C + c8 * 8, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= inv;
    st8(dx + pix * C + c8 * 8, v);
  }
}

PoolGeo pool_geo(int N, int H, int W, int C, int K, int stride, int pad) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || C % 8 || K <= 0 || K > 15 || stride <= 0 || pad < 0 || 2 * pad > K)
    throw std::invalid_argument("maxpool: unsupported geometry (C % 8 == 0, K <= 15, pad <= K/2)");
  PoolGeo g{N, H, W, C, (H + 2 * pad - K) / stride + 1, (W + 2 * pad - K) / stride + 1, K, stride, pad};
  if (g.Ho <= 0 || g.Wo <= 0) throw std::invalid_argument("maxpool: empty output");
  return g;
}

unsigned grid_for(int64_t work) { return unsigned(std::min<int64_t>((work + 255) / 256, 65536)); }

}  // namespace

template <typename T>
void maxpool_fwd_t(int dev, hipStream_t s, int N, int H, int W, int C, int K, int stride, int pad, uintptr_t x,
                   uintptr_t y, uintptr_t idx, uintptr_t ibound, uintptr_t obound) {
  const PoolGeo g = pool_geo(N, H, W, C, K, stride, pad);
  if ((x | y) % 16 || idx % 8) throw std::invalid_argument("maxpool_fwd: misaligned buffers");
  hip_check(hipSetDevice(dev), "hipSetDevice");
  const int64_t work = int64_t(N) * g.Ho * g.Wo * (C / 8);
  // 32-bit indexing while the grid-stride index cannot wrap (work + one grid < 2^32)
  const bool narrow = work + int64_t(grid_for(work)) * 256 < (int64_t(1) << 32);
  auto* k = narrow ? maxpool_fwd_kernel<T, uint32_t> : maxpool_fwd_kernel<T, int64_t>;
  hipLaunchKernelGGL(k, dim3(grid_for(work)), dim3(256), 0, s, reinterpret_cast<const T*>(x),
                     reinterpret_cast<T*>(y), reinterpret_cast<uint8_t*>(idx), g,
                     reinterpret_cast<const float*>(ibound), reinterpret_cast<float*>(obound));
  hip_check(hipGetLastError(), "maxpool_fwd launch");
}

constexpr int kPoolRbBlocks = 8192;  // partial rows of the fused bias gradient

template <typename T>
void maxpool_bwd_t(int dev, hipStream_t s, int N, int H, int W, int C, int K, int stride, int pad, uintptr_t dy,
                   uintptr_t idx, uintptr_t dx, uintptr_t ypool, uintptr_t db, uintptr_t ws) {
  const PoolGeo g = pool_geo(N, H, W, C, K, stride, pad);
  if ((dy | dx | ypool) % 16 || idx % 8) throw std::invalid_argument("maxpool_bwd: misaligned buffers");
  if (db && (!ypool || !ws)) throw std::invalid_argument("maxpool_bwd: the bias gradient needs ypool and ws");
  if (ypool && 256 % (C / 8)) throw std::invalid_argument("maxpool_bwd: the fused ReLU needs 256 % (C / 8) == 0");
  hip_check(hipSetDevice(dev), "hipSetDevice");
  const auto* y = reinterpret_cast<const T*>(ypool);
  float* part = reinterpret_cast<float*>(ws);
  // windows that partition the input (K == stride, no padding): one thread per window
  const bool part_win = K == stride && pad == 0 && std::getenv("MPIT_POOL_GATHER") == nullptr;
  const int64_t work = part_win ? int64_t(N) * g.Ho * g.Wo * (C / 8) : int64_t(N) * H * W * (C / 8);
  const unsigned grid = ypool ? unsigned(std::min<int64_t>((work + 255) / 256, kPoolRbBlocks)) : grid_for(work);
  const bool narrow = int64_t(N) * H * W * (C / 8) + int64_t(grid) * 256 < (int64_t(1) << 32);
  if (part_win) {
    auto* k = ypool ? (narrow ? maxpool_bwd_part_kernel<T, uint32_t, true> : maxpool_bwd_part_kernel<T, int64_t, true>)
                    : (narrow ? maxpool_bwd_part_kernel<T, uint32_t, false> : maxpool_bwd_part_kernel<T, int64_t, false>);
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, s, reinterpret_cast<const T*>(dy),
                       reinterpret_cast<const uint8_t*>(idx), reinterpret_cast<T*>(dx), g, y, part);
  } else if (ypool) {
    auto* k = narrow ? maxpool_bwd_kernel<T, uint32_t, true> : maxpool_bwd_kernel<T, int64_t, true>;
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, s, reinterpret_cast<const T*>(dy),
                       reinterpret_cast<const uint8_t*>(idx), reinterpret_cast<T*>(dx), g, y, part);
  } else {
    auto* k = narrow ? maxpool_bwd_kernel<T, uint32_t, false> : maxpool_bwd_kernel<T, int64_t, false>;
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, s, reinterpret_cast<const T*>(dy),
                       reinterpret_cast<const uint8_t*>(idx), reinterpret_cast<T*>(dx), g, y, part);
  }
  hip_check(hipGetLastError(), "maxpool_bwd launch");
  if (db) col_sums(s, part, grid, C, C, reinterpret_cast<float*>(db), part + int64_t(kPoolRbBlocks) * C);
}

int64_t maxpool_bwd_ws_floats(int C) { return int64_t(kPoolRbBlocks) * C + col_sums_ws_floats(C); }

void avgpool_bwd(int dev, hipStream_t s, int N, int HW, int C, uintptr_t dy, uintptr_t dx, bool f32) {
  if (N <= 0 || HW <= 0 || C <= 0 || C % 8) throw std::invalid_argument("avgpool_bwd: need C % 8 == 0");
  if ((dy | dx) % 16) throw std::invalid_argument("avgpool_bwd: misaligned buffers");
  hip_check(hipSetDevice(dev), "hipSetDevice");
  const int64_t total = int64_t(N) * HW * (C / 8);
  const float inv = 1.f / float(HW);
  if (f32)
    hipLaunchKernelGGL(avgpool_bwd_kernel<float>, dim3(grid_for(total)), dim3(256), 0, s,
                       reinterpret_cast<const float*>(dy), reinterpret_cast<float*>(dx), total, HW, C, inv);
  else
    hipLaunchKernelGGL(avgpool_bwd_kernel<uint16_t>, dim3(grid_for(total)), dim3(256), 0, s,
                       reinterpret_cast<const uint16_t*>(dy), reinterpret_cast<uint16_t*>(dx), total, HW, C, inv);
  hip_check(hipGetLastError(), "avgpool_bwd launch");
}

void maxpool_fwd(int dev, hipStream_t s, int N, int H, int W, int C, int K, int stride, int pad, uintptr_t x,
                 uintptr_t y, uintptr_t idx, bool f32, uintptr_t ibound, uintptr_t obound) {
  if (obound && (!f32 || !ibound)) throw std::invalid_argument("maxpool_fwd: fp16 planes need fp32 and the input's bound");
  if (f32) maxpool_fwd_t<float>(dev, s, N, H, W, C, K, stride, pad, x, y, idx, ibound, obound);
  else maxpool_fwd_t<uint16_t>(dev, s, N, H, W, C, K, stride, pad, x, y, idx, 0, 0);
}

void maxpool_bwd(int dev, hipStream_t s, int N, int H, int W, int C, int K, int stride, int pad, uintptr_t dy,
                 uintptr_t idx, uintptr_t dx, bool f32, uintptr_t ypool, uintptr_t db, uintptr_t ws) {
  if (f32) maxpool_bwd_t<float>(dev, s, N, H, W, C, K, stride, pad, dy, idx, dx, ypool, db, ws);
  else maxpool_bwd_t<uint16_t>(dev, s, N, H, W, C, K, stride, pad, dy, idx, dx, ypool, db, ws);
}

}  // namespace mpit

// ReLU + bias backward for the conv(+bias)(+ReLU) layers whose forward runs the bias and
// the ReLU in the GEMM epilogue (VGG / AlexNet on the MFMA implicit-GEMM path):
//   dz = dy * (y > 0)            (bf16 or fp32 [M, C], y = the layer's saved output)
//   db[c] = sum over rows of dz  (fp32, optional)
// One pass over dy and y (the masked gradient is what the dgrad / wgrad GEMMs consume, so
// it has to be written once anyway); the bias gradient rides along as a per-thread
// channel-group accumulation, combined per block in LDS and across blocks by a second
// tiny kernel in a fixed order (deterministic, no atomics).
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

#include "ew.h"
#include "kernels.h"

namespace mpit {
namespace {

constexpr int kMaxBlocks = 1024;

template <typename T>
__global__ __launch_bounds__(1024) void relu_bias_bwd_kernel(const T* __restrict__ dy,
                                                             const T* __restrict__ y,
                                                             T* __restrict__ dz, int64_t M, int C,
                                                             int64_t rows_per_block, float* __restrict__ part) {
  extern __shared__ float lds[];  // [R][C]
  const int G = C / 8;
  const int g = threadIdx.x % G, rs = threadIdx.x / G, R = blockDim.x / G;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int64_t r0 = int64_t(blockIdx.x) * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  for (int64_t r = r0 + rs; r < r1; r += R) {
    const int64_t o = r * C + g * 8;
    if constexpr (sizeof(T) == 4) {
      float4 a[2], b[2];
      a[0] = reinterpret_cast<const float4*>(dy + o)[0];
      a[1] = reinterpret_cast<const float4*>(dy + o)[1];
      b[0] = reinterpret_cast<const float4*>(y + o)[0];
      b[1] = reinterpret_cast<const float4*>(y + o)[1];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        a[k].x = b[k].x > 0.f ? a[k].x : 0.f;
        a[k].y = b[k].y > 0.f ? a[k].y : 0.f;
        a[k].z = b[k].z > 0.f ? a[k].z : 0.f;
        a[k].w = b[k].w > 0.f ? a[k].w : 0.f;
        acc[4 * k] += a[k].x;
        acc[4 * k + 1] += a[k].y;
        acc[4 * k + 2] += a[k].z;
        acc[4 * k + 3] += a[k].w;
        reinterpret_cast<float4*>(dz + o)[k] = a[k];
      }
      continue;
    } else {
    const uint4 a = *reinterpret_cast<const uint4*>(dy + o);
    const uint4 b = *reinterpret_cast<const uint4*>(y + o);
    const uint32_t av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w};
    uint32_t ov[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint32_t w = 0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint16_t yv = uint16_t(bv[k] >> (16 * h));
        const uint16_t gv = uint16_t(av[k] >> (16 * h));
        const bool pos = bf2f(yv) > 0.f;
        const uint16_t z = pos ? gv : uint16_t(0);
        acc[2 * k + h] += bf2f(z);
        w |= uint32_t(z) << (16 * h);
      }
      ov[k] = w;
    }
    *reinterpret_cast<uint4*>(dz + o) = make_uint4(ov[0], ov[1], ov[2], ov[3]);
    }
  }
  if (!part) return;
#pragma unroll
  for (int v = 0; v < 8; ++v) lds[rs * C + g * 8 + v] = acc[v];
  // LDS hand-off only: a __syncthreads() fence would first wait for every dz store above
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < R; ++k) s += lds[k * C + c];
    part[int64_t(blockIdx.x) * C + c] = s;
  }
}

// Combine the per-block partials: a block owns 64 channels, 16 lanes per channel stride
// over the partial rows (coalesced 256-B rows, many loads in flight), then fixed-order
// combine in LDS (deterministic).
// Two launches for many partial rows: blockIdx.y splits the rows into gridDim.y groups
// (level 1 writes [groups][C]), the second launch combines the groups.
constexpr int kSumCh = 64, kSumLanes = 16, kSumGroups = 16;
__global__ __launch_bounds__(kSumCh * kSumLanes) void sum_parts_kernel(const float* __restrict__ part, int nb, int C,
                                                                       float* __restrict__ out, int64_t ld) {
  __shared__ float sm[kSumLanes][kSumCh];
  const int cl = threadIdx.x % kSumCh, kl = threadIdx.x / kSumCh;
  const int c = blockIdx.x * kSumCh + cl;
  const int per = (nb + gridDim.y - 1) / gridDim.y, r0 = blockIdx.y * per, r1 = min(nb, r0 + per);
  float s = 0.f;
  if (c < C) {
#pragma unroll 8
    for (int k = r0 + kl; k < r1; k += kSumLanes) s += part[int64_t(k) * ld + c];
  }
  sm[kl][cl] = s;
  __syncthreads();
  if (kl != 0 || c >= C) return;
  for (int k = 1; k < kSumLanes; ++k) s += sm[k][cl];
  out[int64_t(blockIdx.y) * C + c] = s;
}

}  // namespace

int64_t relu_bias_bwd_ws_floats(int C) { return int64_t(kMaxBlocks + kSumGroups) * C; }

void relu_bias_bwd(int dev, hipStream_t s, int64_t M, int C, uintptr_t dy, uintptr_t y, uintptr_t dz, uintptr_t db,
                   uintptr_t ws, bool f32) {
  if (M <= 0 || C <= 0 || C % 8 || C / 8 > 1024) throw std::invalid_argument("relu_bias_bwd: need C % 8 == 0, C <= 8192");
  if ((dy | y | dz) % 16) throw std::invalid_argument("relu_bias_bwd: buffers must be 16-byte aligned");
  if (db && !ws) throw std::invalid_argument("relu_bias_bwd: bias gradient needs the workspace");
  hip_check(hipSetDevice(dev), "hipSetDevice");
  const int G = C / 8;
  const int blk = G >= 256 ? G : (256 / G) * G;
  const int R = blk / G;
  int64_t nb = std::min<int64_t>(kMaxBlocks, std::max<int64_t>(1, (M + R * 16 - 1) / (R * 16)));
  int64_t rpb = (M + nb - 1) / nb;
  nb = (M + rpb - 1) / rpb;
  float* part = db ? reinterpret_cast<float*>(ws) : nullptr;
  const size_t shm = db ? size_t(R) * C * sizeof(float) : 0;
  if (f32)
    hipLaunchKernelGGL(relu_bias_bwd_kernel<float>, dim3(unsigned(nb)), dim3(blk), shm, s,
                       reinterpret_cast<const float*>(dy), reinterpret_cast<const float*>(y),
                       reinterpret_cast<float*>(dz), M, C, rpb, part);
  else
    hipLaunchKernelGGL(relu_bias_bwd_kernel<uint16_t>, dim3(unsigned(nb)), dim3(blk), shm, s,
                       reinterpret_cast<const uint16_t*>(dy), reinterpret_cast<const uint16_t*>(y),
                       reinterpret_cast<uint16_t*>(dz), M, C, rpb, part);
  hip_check(hipGetLastError(), "relu_bias_bwd launch");
  if (db) col_sums(s, part, nb, C, C, reinterpret_cast<float*>(db), part + int64_t(kMaxBlocks) * C);
}

int64_t col_sums_ws_floats(int C) { return int64_t(kSumGroups) * C; }

void col_sums(hipStream_t s, const float* part, int64_t nb, int64_t ld, int C, float* out, float* mid) {
  if (nb <= 0 || C <= 0 || ld < C) throw std::invalid_argument("col_sums: bad shape");
  const dim3 cb((C + kSumCh - 1) / kSumCh);
  if (nb > 4 * kSumLanes) {  // level 1 into mid [kSumGroups][C], then the group combine
    if (!mid) throw std::invalid_argument("col_sums: many rows need the workspace");
    hipLaunchKernelGGL(sum_parts_kernel, dim3(cb.x, kSumGroups), dim3(kSumCh * kSumLanes), 0, s, part, int(nb), C, mid,
                       ld);
    hipLaunchKernelGGL(sum_parts_kernel, cb, dim3(kSumCh * kSumLanes), 0, s, mid, kSumGroups, C, out, int64_t(C));
  } else {
    hipLaunchKernelGGL(sum_parts_kernel, cb, dim3(kSumCh * kSumLanes), 0, s, part, int(nb), C, out, ld);
  }
  hip_check(hipGetLastError(), "col_sums launch");
}

void col_sums(int dev, hipStream_t s, uintptr_t part, int64_t nb, int64_t ld, int C, uintptr_t out, uintptr_t mid) {
  hip_check(hipSetDevice(dev), "hipSetDevice");
  col_sums(s, reinterpret_cast<const float*>(part), nb, ld, C, reinterpret_cast<float*>(out),
           reinterpret_cast<float*>(mid));
}

}  // namespace mpit

// Fused training-mode BatchNorm + (residual add) + ReLU for channels_last (NHWC)
// activations, forward and backward, bf16 or fp32 storage, fp32 math.
//
// Why: on MI355X the ResNet-50 step spends ~15 ms in MIOpen's NHWC batch-norm kernels and
// ~6.6 ms more in separate PyTorch add / ReLU / ReLU-backward passes (profiles/
// resnet50_n1_steady_kernels.md): 8 full passes over every activation in forward and 8 in
// backward, at ~2.8 TB/s. Memory-bound work belongs in as few HBM passes as possible:
//   forward : stats pass (read x) + apply pass (read x [, residual], write y [, ReLU bit mask])
//   backward: reduce pass (read dy, mask, x) + apply pass (read dy, mask, x, write dx [, dres])
// The ReLU mask is one bit per element (1/16 of a bf16 tensor), so the backward never
// re-reads the forward output y.
// Layout: the activation is a row-major [M = N*H*W, C] matrix. A thread owns VEC = 8
// channels (16 B bf16, 32 B fp32; the ReLU mask is one byte per 8 channels in both, the
// layout the GEMM epilogues read) and walks rows; since every block size and grid stride
// is a multiple of G = C/VEC, a thread keeps the same channels for its whole life, so
// per-channel coefficients stay in registers. The fp32 apply passes split a thread's 8
// elements into two coalesced float4 halves (Slot below).
// Statistics use shifted sums (shift = row 0 of each channel) accumulated in fp32 per
// thread, combined per block in LDS, then across blocks in fp64 by the finalize kernel:
// deterministic (no atomics) and free of the E[x^2]-E[x]^2 cancellation for |mean|>>std.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cmath>
#include <stdexcept>
#include <cstdlib>
#include <string>
#include <type_traits>

#include "ew.h"
#include "kernels.h"
#include "planes.h"

namespace mpit {
namespace {

constexpr int kMaxStatBlocks = 512;
constexpr int kFinCh = 64;   // channels per finalize block
constexpr int kFinK = 16;    // partial-lanes per channel in the finalize block (1024 threads)

template <typename T>
struct Vec;
template <>
struct Vec<uint16_t> {  // bf16
  static constexpr int N = 8;
  using raw = uint4;
  static __device__ __forceinline__ void load(const uint16_t* p, float (&v)[8]) {
    const uint4 r = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[2 * k] = bf2f(uint16_t(w[k] & 0xffff));
      v[2 * k + 1] = bf2f(uint16_t(w[k] >> 16));
    }
  }
  static __device__ __forceinline__ void store(uint16_t* p, const float (&v)[8]) {
    uint4 r;
    r.x = uint32_t(f2bf(v[0])) | (uint32_t(f2bf(v[1])) << 16);
    r.y = uint32_t(f2bf(v[2])) | (uint32_t(f2bf(v[3])) << 16);
    r.z = uint32_t(f2bf(v[4])) | (uint32_t(f2bf(v[5])) << 16);
    r.w = uint32_t(f2bf(v[6])) | (uint32_t(f2bf(v[7])) << 16);
    *reinterpret_cast<uint4*>(p) = r;
  }
};
template <>
struct Vec<float> {
  static constexpr int N = 8;
  static __device__ __forceinline__ void load(const float* p, float (&v)[8]) {
    const float4 r = reinterpret_cast<const float4*>(p)[0], q = reinterpret_cast<const float4*>(p)[1];
    v[0] = r.x; v[1] = r.y; v[2] = r.z; v[3] = r.w;
    v[4] = q.x; v[5] = q.y; v[6] = q.z; v[7] = q.w;
  }
  static __device__ __forceinline__ void store(float* p, const float (&v)[8]) {
    reinterpret_cast<float4*>(p)[0] = make_float4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<float4*>(p)[1] = make_float4(v[4], v[5], v[6], v[7]);
  }
};

// block size: the largest multiple of G that is <= 256 (G = channel groups per row)
inline int block_for(int G) { return G >= 256 ? G : (256 / G) * G; }

// ---------------------------------------------------------------- apply-pass lane layout
// Where the 8 elements of an apply-pass thread live. A thread owns vector slot i (global
// thread index, then + grid stride): bf16 — one 16-byte vector at element 8i, lanes
// contiguous. fp32 with SPLIT — two float4 at 4l and 256 + 4l of its wave's 512-float chunk
// (l = lane): each load instruction then reads 1 KiB contiguous across the wave, where one
// 32-byte vector per lane (the unsplit fp32 layout) leaves every cache line an instruction
// touches half used and needs a second instruction to the same lines. Element v = 4h + j is
// at off[h] + j; its ReLU-mask bit is bit sh[h] + j of byte mb[h] (the mask format is the
// same in both layouts: one byte per 8 consecutive elements). SPLIT needs 256-thread blocks
// and C | 2048, so that the grid stride (a multiple of 2048 elements) keeps every lane on the
// same channels for its life (split_ok).
template <bool SPLIT, bool CHK = false>
struct Slot {
  int64_t off[2], mb[2];
  int sh[2];
  int64_t lim;  // elements in the tensor (CHK)
  __device__ __forceinline__ Slot(int64_t i, int64_t nvec) : lim(nvec * 8) {
    if constexpr (SPLIT) {
      const int64_t w = i >> 6;
      const int l = int(i & 63);
      off[0] = w * 512 + 4 * l;
      off[1] = off[0] + 256;
      mb[0] = w * 64 + (l >> 1);
      mb[1] = mb[0] + 32;
      sh[0] = sh[1] = 4 * (l & 1);
    } else {
      off[0] = i * 8;
      off[1] = off[0] + 4;
      mb[0] = mb[1] = i;
      sh[0] = 0;
      sh[1] = 4;
    }
  }
  // half h holds data: only the last, partial wave chunk of a SPLIT pass checks (CHK)
  __device__ __forceinline__ bool valid(int h) const { return !(SPLIT && CHK) || off[h] < lim; }
  // channel of element v (constant over the thread's life); off[h] is a multiple of 4 and C
  // of 8, so the 4 elements of a half never wrap: 2 divisions per thread, not 8
  __device__ __forceinline__ void chans(int C, int (&c)[8]) const {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int b = int(off[h] % C);
#pragma unroll
      for (int j = 0; j < 4; ++j) c[4 * h + j] = b + j;
    }
  }
};

// MPIT_BN_SPLIT=0 keeps the unsplit fp32 layout (A/B knob)
inline bool split_ok(bool f32, int C, int blk) {
  static const bool on = [] {
    const char* e = std::getenv("MPIT_BN_SPLIT");
    return !(e && e[0] == '0');
  }();
  return on && f32 && blk == 256 && 2048 % C == 0;
}

// Walk over the thread's slots. U == 0: grid stride, body(Slot) for i, i + stride, ... while
// live. U > 0: one pass, exactly the U slots i + k * stride (k < U) with stride = the whole
// grid — no loop, so no wave waits for its own previous stores before its next loads
// (vmcnt counts both). SPLIT walks whole waves (the mask store's lane swap needs every
// lane): full chunks without checks (no branches between the loads), a partial chunk with
// per-half checks.
template <bool SPLIT, int U, class F>
__device__ __forceinline__ void for_slots(int64_t i, int64_t stride, int64_t nvec, F&& body) {
  if constexpr (U > 0) {
#pragma unroll
    for (int k = 0; k < U; ++k, i += stride) {
      if constexpr (SPLIT) {
        if ((i | 63) < nvec) body(Slot<true, false>(i, nvec));
        else if ((i & ~int64_t(63)) < nvec) body(Slot<true, true>(i, nvec));
      } else {
        if (i < nvec) body(Slot<false>(i, nvec));
      }
    }
  } else if constexpr (SPLIT) {
    for (; (i | 63) < nvec; i += stride) body(Slot<true, false>(i, nvec));
    if ((i & ~int64_t(63)) < nvec) body(Slot<true, true>(i, nvec));
  } else {
    for (; i < nvec; i += stride) body(Slot<false>(i, nvec));
  }
}

// Slots per thread of the apply passes: fp32 1, bf16 2 — measured per ResNet-50 shape against
// the grid-stride loop over <= 4096 blocks (0) and 4 (profiles/bn_apply_passes_r04.md);
// MPIT_BN_APPLY_U overrides (0, 1, 2).
inline int apply_u(bool f32) {
  static const int u = [] {
    const char* e = std::getenv("MPIT_BN_APPLY_U");
    return e ? std::atoi(e) : -1;
  }();
  return u >= 0 ? u : (f32 ? 1 : 2);
}

// launch a kernel instantiated for (SPLIT, U): l(bool_constant, int_constant)
template <bool F32, class L>
void with_mode(bool split, int u, L&& l) {
  auto go = [&](auto sp) {
    switch (u) {
      case 1: l(sp, std::integral_constant<int, 1>{}); break;
      case 2: l(sp, std::integral_constant<int, 2>{}); break;
      default: l(sp, std::integral_constant<int, 0>{});
    }
  };
  if constexpr (F32) {
    if (split) return go(std::true_type{});
  }
  go(std::false_type{});
}

// grid of an apply pass with u slots per thread (u == 0: grid stride)
inline int apply_grid_u(int64_t nvec, int block, int u) {
  if (u <= 0) return int(std::max<int64_t>(1, std::min<int64_t>((nvec + block - 1) / block, 4096)));
  return int(std::max<int64_t>(1, (nvec + int64_t(block) * u - 1) / (int64_t(block) * u)));
}

template <typename T, class S>
__device__ __forceinline__ void load8(const T* __restrict__ p, const S& s, float (&v)[8]) {
  if constexpr (sizeof(T) == 4) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
      if (s.valid(h)) r = *reinterpret_cast<const float4*>(p + s.off[h]);
      v[4 * h] = r.x; v[4 * h + 1] = r.y; v[4 * h + 2] = r.z; v[4 * h + 3] = r.w;
    }
  } else {
    Vec<T>::load(p + s.off[0], v);
  }
}

template <typename T, class S>
__device__ __forceinline__ void store8(T* __restrict__ p, const S& s, const float (&v)[8]) {
  if constexpr (sizeof(T) == 4) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
      if (s.valid(h))
        *reinterpret_cast<float4*>(p + s.off[h]) = make_float4(v[4 * h], v[4 * h + 1], v[4 * h + 2], v[4 * h + 3]);
  } else {
    Vec<T>::store(p + s.off[0], v);
  }
}

// the thread's 8 mask bits (bit v = element v)
template <bool SPLIT, bool CHK>
__device__ __forceinline__ uint32_t mask_bits(const uint8_t* __restrict__ m, const Slot<SPLIT, CHK>& s) {
  if constexpr (SPLIT) {
    uint32_t b = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h)
      if (s.valid(h)) b |= ((uint32_t(m[s.mb[h]]) >> s.sh[h]) & 15u) << (4 * h);
    return b;
  } else {
    return m[s.mb[0]];
  }
}

// store the thread's 8 mask bits; SPLIT: lanes 2k and 2k+1 share a byte — every lane of the
// wave must call this (the nibbles meet through a lane swap)
template <bool SPLIT, bool CHK>
__device__ __forceinline__ void mask_store(uint8_t* __restrict__ m, const Slot<SPLIT, CHK>& s, uint32_t bits) {
  if constexpr (SPLIT) {
    const uint32_t other = uint32_t(__shfl_xor(int(bits), 1));
    if (s.sh[0] == 0) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
        if (s.valid(h)) m[s.mb[h]] = uint8_t(((bits >> (4 * h)) & 15u) | (((other >> (4 * h)) & 15u) << 4));
    }
  } else {
    m[s.mb[0]] = uint8_t(bits);
  }
}

// ---------------------------------------------------------------- output bound (fp16x3)
// An apply kernel that produces the next convolution's fp32 GEMM operand also writes max|out|
// over the whole tensor: the fp16x3 GEMMs (gemm.hip FM 11) derive the operand's power-of-two
// scale from it. Each block reduces its maximum and issues ONE atomic max (no return value:
// nothing waits on it) into slot blockIdx % kBoundSlots of the bound (kernels.h; one address
// took 4096 serialised atomics per pass: +20 us a call), which the kernel that ran before the apply on the same
// stream set to zero — the finalize that wrote the apply coefficients (FinArgs::zero, the
// GEMM's folded finalize: EpiArgs::fzero) or, on the paths without one, a 4-byte memset.
// |out| >= 0, so the float bits order like unsigned integers.
struct AmaxOut {
  float* amax;  // null: not wanted
  // fp16 planes output (kernels.h PlaneSpec, fp32 passes only): obound != null
  float* obound = nullptr;
  const unsigned long long* xmax = nullptr;
  const unsigned long long* xmax2 = nullptr;
  const unsigned long long* gmax = nullptr;
  uint32_t xep = 0, xep2 = 0, gep = 0;
  const float* rbound = nullptr;
  int rplanes = 0;
};

AmaxOut amax_out(uintptr_t amax, const PlaneSpec* p) {
  AmaxOut o{reinterpret_cast<float*>(amax)};
  if (p) {
    o.obound = reinterpret_cast<float*>(p->obound);
    o.xmax = reinterpret_cast<const unsigned long long*>(p->xmax);
    o.xmax2 = reinterpret_cast<const unsigned long long*>(p->xmax2);
    o.gmax = reinterpret_cast<const unsigned long long*>(p->gmax);
    o.xep = p->xep;
    o.xep2 = p->xep2;
    o.gep = p->gep;
    o.rbound = reinterpret_cast<const float*>(p->rbound);
    o.rplanes = p->rplanes;
    if (o.obound) o.amax = nullptr;  // the planes' bound is known before the pass
  }
  return o;
}

// Barriers of an LDS hand-off only: the epilogues below run after the kernel's output
// stores, and __syncthreads()'s workgroup fence would wait for every one of them to retire
// (vmcnt(0)) before the block can finish.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ float block_max(float m, float* red /* >= 16 floats of LDS */) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  const int w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  lds_barrier();  // an earlier block_max of this kernel is done reading red
  if ((threadIdx.x & 63) == 0) red[w] = m;
  lds_barrier();
  float b = red[0];
  for (int k = 1; k < nw; ++k) b = fmaxf(b, red[k]);
  return b;  // every thread
}

__device__ __forceinline__ void amax_finish(float m, const AmaxOut& o) {
  __shared__ float red[16];
  const float b = block_max(m, red);
  if (threadIdx.x == 0)
    atomicMax(reinterpret_cast<unsigned int*>(o.amax + (blockIdx.x % kBoundSlots) * kBoundStride), __float_as_uint(b));
}

// ---------------------------------------------------------------- fp16 planes (FM 13 operands)
// (planes.h) the slot's 8 values as planes: h at element i, l at element nel + i of the
// 16-bit view
template <class S>
__device__ __forceinline__ void store_planes(float* __restrict__ y, int64_t nel, const S& s, const float (&v)[8],
                                             PlaneScale ps) {
  uint16_t* yh = reinterpret_cast<uint16_t*>(y);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (!s.valid(h)) continue;
    uint32_t hw[2], lw[2];
#pragma unroll
    for (int p = 0; p < 2; ++p) split_pair(v[4 * h + 2 * p], v[4 * h + 2 * p + 1], ps, hw[p], lw[p]);
    *reinterpret_cast<uint2*>(yh + s.off[h]) = make_uint2(hw[0], hw[1]);
    *reinterpret_cast<uint2*>(yh + nel + s.off[h]) = make_uint2(lw[0], lw[1]);
  }
}
// planes back to fp32 (exact, 22 significant bits)
template <class S>
__device__ __forceinline__ void load_planes(const float* __restrict__ r, int64_t nel, const S& s, float inv,
                                            float (&v)[8]) {
  const uint16_t* rh = reinterpret_cast<const uint16_t*>(r);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    uint2 a = make_uint2(0, 0), b = make_uint2(0, 0);
    if (s.valid(h)) {
      a = *reinterpret_cast<const uint2*>(rh + s.off[h]);
      b = *reinterpret_cast<const uint2*>(rh + nel + s.off[h]);
    }
    const pf32x2 x0 = join_pair(a.x, b.x, inv), x1 = join_pair(a.y, b.y, inv);
    v[4 * h] = x0.x;
    v[4 * h + 1] = x0.y;
    v[4 * h + 2] = x1.x;
    v[4 * h + 3] = x1.y;
  }
}

// ---------------------------------------------------------------- forward: statistics
template <typename T>
__global__ __launch_bounds__(1024) void bn_stats_kernel(const T* __restrict__ x, int64_t M, int C,
                                                        int64_t rows_per_block, float* __restrict__ part) {
  constexpr int V = Vec<T>::N;
  extern __shared__ float lds[];  // [R][2][C]
  const int G = C / V;
  const int g = threadIdx.x % G, rs = threadIdx.x / G, R = blockDim.x / G;
  float shift[V];
  Vec<T>::load(x + size_t(g) * V, shift);  // row 0
  float s1[V], s2[V];
#pragma unroll
  for (int v = 0; v < V; ++v) s1[v] = s2[v] = 0.f;
  const int64_t r0 = int64_t(blockIdx.x) * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  int64_t r = r0 + rs;
  for (; r + 3 * R < r1; r += 4 * R) {
    float a[4][V];
#pragma unroll
    for (int u = 0; u < 4; ++u) Vec<T>::load(x + (r + u * R) * C + g * V, a[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const float d = a[u][v] - shift[v];
        s1[v] += d;
        s2[v] = fmaf(d, d, s2[v]);
      }
  }
  for (; r < r1; r += R) {
    float a[V];
    Vec<T>::load(x + r * C + g * V, a);
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const float d = a[v] - shift[v];
      s1[v] += d;
      s2[v] = fmaf(d, d, s2[v]);
    }
  }
#pragma unroll
  for (int v = 0; v < V; ++v) {
    lds[(rs * 2 + 0) * C + g * V + v] = s1[v];
    lds[(rs * 2 + 1) * C + g * V + v] = s2[v];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float a = 0.f, b = 0.f;
    for (int k = 0; k < R; ++k) {
      a += lds[(k * 2 + 0) * C + c];
      b += lds[(k * 2 + 1) * C + c];
    }
    part[(size_t(blockIdx.x) * 2 + 0) * C + c] = a;
    part[(size_t(blockIdx.x) * 2 + 1) * C + c] = b;
  }
}

// Cross-block combine: a block owns kFinCh channels; kFinK lanes per channel stride over
// the partials (coalesced 256-B rows, independent loads in flight), then combine in LDS.
__device__ __forceinline__ bool fin_combine(const float* __restrict__ part, int nb, int C, double& a, double& b) {
  __shared__ double sa[kFinK][kFinCh], sb[kFinK][kFinCh];
  const int cl = threadIdx.x % kFinCh, kl = threadIdx.x / kFinCh;
  const int c = blockIdx.x * kFinCh + cl;
  double x = 0, y = 0;
  if (c < C) {
#pragma unroll 8
    for (int k = kl; k < nb; k += kFinK) {
      x += part[(size_t(k) * 2 + 0) * C + c];
      y += part[(size_t(k) * 2 + 1) * C + c];
    }
  }
  sa[kl][cl] = x;
  sb[kl][cl] = y;
  __syncthreads();
  if (kl != 0 || c >= C) return false;
  a = 0;
  b = 0;
  for (int k = 0; k < kFinK; ++k) {
    a += sa[k][cl];
    b += sb[k][cl];
  }
  return true;
}

template <typename T>
__device__ __forceinline__ void fin_fwd_channel(int c, double a, double b, int C, int64_t M, const T* __restrict__ x,
                                                const float* __restrict__ gamma, const float* __restrict__ beta,
                                                float eps, float momentum, float* __restrict__ rmean,
                                                float* __restrict__ rvar, float* __restrict__ save_mean,
                                                float* __restrict__ save_rstd, float* __restrict__ coef);

__device__ __forceinline__ void fin_bwd_channel(int c, double a, double b, int C, int64_t M,
                                                const float* __restrict__ gamma, const float* __restrict__ mean,
                                                const float* __restrict__ rstd, float* __restrict__ dgamma,
                                                float* __restrict__ dbeta, float* __restrict__ coef);

template <typename T>
__global__ __launch_bounds__(kFinCh * kFinK) void bn_finalize_fwd_kernel(
    const float* __restrict__ part, int nb, int C, int64_t M, const T* __restrict__ x, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, float momentum, float* __restrict__ rmean, float* __restrict__ rvar,
    float* __restrict__ save_mean, float* __restrict__ save_rstd, float* __restrict__ coef /*[2][C] scale, shift*/) {
  double a, b;
  if (!fin_combine(part, nb, C, a, b)) return;
  fin_fwd_channel(blockIdx.x * kFinCh + int(threadIdx.x % kFinCh), a, b, C, M, x, gamma, beta, eps, momentum, rmean,
                  rvar, save_mean, save_rstd, coef);
}

// channel c of the forward finalize from the fp64 sums (a, b) of (x - x[0][c]) and its square
template <typename T>
__device__ __forceinline__ void fin_fwd_channel(int c, double a, double b, int C, int64_t M, const T* __restrict__ x,
                                                const float* __restrict__ gamma, const float* __restrict__ beta,
                                                float eps, float momentum, float* __restrict__ rmean,
                                                float* __restrict__ rvar, float* __restrict__ save_mean,
                                                float* __restrict__ save_rstd, float* __restrict__ coef) {
  float k0;
  if constexpr (sizeof(T) == 2) k0 = bf2f(reinterpret_cast<const uint16_t*>(x)[c]);
  else k0 = reinterpret_cast<const float*>(x)[c];
  const double md = a / double(M);
  double var = b / double(M) - md * md;
  if (var < 0) var = 0;
  const double mean = double(k0) + md;
  const float rstd = float(1.0 / std::sqrt(var + double(eps)));
  const float sc = (gamma ? gamma[c] : 1.f) * rstd;
  coef[c] = sc;
  coef[C + c] = (beta ? beta[c] : 0.f) - float(mean) * sc;
  save_mean[c] = float(mean);
  save_rstd[c] = rstd;
  if (rmean) rmean[c] = (1.f - momentum) * rmean[c] + momentum * float(mean);
  if (rvar) rvar[c] = (1.f - momentum) * rvar[c] + momentum * float(var * double(M) / double(M > 1 ? M - 1 : 1));
}

// Partials emitted by a GEMM epilogue (gemm.hip), one row pair per 128-row tile — up to
// thousands of rows, too many for one finalize block per 64 channels. Level 1 folds
// groups of tile rows in parallel (grid: channel blocks x groups) into the [groups][2][C]
// layout the finalize kernels take:
//   CHAN (forward statistics): tile k holds (mean_k, M2_k) of n_k = min(128, M - 128k)
//        rows; out = sum n_k d_k, sum M2_k + n_k d_k^2 with d_k = mean_k - x[0][c] — the
//        shifted sums bn_finalize_fwd_kernel expects (shift = row 0 of x), fp64 inside;
//   plain (backward reductions): tile sums are added.
constexpr int kTileRows = 128;
// row lanes per channel of bn_tiles_finalize_kernel: 4 (64 channels x 4 = 256 threads) by
// default — in the backward the finalize shares the GPU with the side stream's weight-gradient
// GEMMs, and a 1024-thread block must wait for a whole CU's worth of free slots
// (profiles/bn_finalize_lanes_ab_r02.md); MPIT_BN_FIN_LANES=16 restores the wide block
constexpr int kFinLanesWide = 16;
constexpr int kFinLanesNarrow = 4;
constexpr int kTicketSlots = 64;  // rotating ticket sets (one per launch in flight)
constexpr int kMaxChBlocks = 32;  // C <= 2048

// Completion tickets of the fused level-1 + finalize kernel: one counter per channel
// block, reset to zero by the block that finalizes, so a set is reusable as soon as its
// launch retired; launches rotate over kTicketSlots sets.
__device__ uint32_t g_bn_tickets[kTicketSlots * kMaxChBlocks];

// finalize operands (forward or backward)
struct FinArgs {
  const float* gamma;
  const float* beta;
  float eps, momentum;
  float* rmean;
  float* rvar;
  float* save_mean;
  float* save_rstd;
  const float* mean;
  const float* rstd;
  float* dgamma;
  float* dbeta;
  float* coef;
  float* zero;  // set to 0 by the finalizing block (an output bound the apply pass then raises)
};

template <typename T, bool CHAN, int kTileLanes>
__global__ __launch_bounds__(64 * kTileLanes) void bn_tiles_finalize_kernel(const float* __restrict__ part, int nt,
                                                                            int C, int64_t M, const T* __restrict__ x,
                                                                            int rows_per_group, float* lvl,
                                                                            uint32_t* tickets, FinArgs fa) {
  __shared__ double sa[kTileLanes][64], sb[kTileLanes][64];
  __shared__ uint32_t prev;
  const int cl = threadIdx.x % 64, kl = threadIdx.x / 64;
  const int c = blockIdx.x * 64 + cl, grp = blockIdx.y;
  double a = 0, b = 0;
  if (c < C) {
    double k0 = 0;
    if constexpr (CHAN) {
      if constexpr (sizeof(T) == 2) k0 = bf2f(reinterpret_cast<const uint16_t*>(x)[c]);
      else k0 = reinterpret_cast<const float*>(x)[c];
    }
    const int r0 = grp * rows_per_group, r1 = min(nt, r0 + rows_per_group);
#pragma unroll 4
    for (int k = r0 + kl; k < r1; k += kTileLanes) {
      const float p0 = part[(size_t(k) * 2 + 0) * C + c], p1 = part[(size_t(k) * 2 + 1) * C + c];
      if constexpr (CHAN) {
        const double n = double(min<int64_t>(kTileRows, M - int64_t(k) * kTileRows));
        const double d = double(p0) - k0;
        a = fma(n, d, a);
        b += double(p1) + n * d * d;
      } else {
        a += p0;
        b += p1;
      }
    }
  }
  sa[kl][cl] = a;
  sb[kl][cl] = b;
  __syncthreads();
  if (kl == 0 && c < C) {
#pragma unroll
    for (int k = 1; k < kTileLanes; ++k) {
      a += sa[k][cl];
      b += sb[k][cl];
    }
    // write-through (sc1) stores: visible to a reader on any XCD without an L2 write-back
    __hip_atomic_store(&lvl[(size_t(grp) * 2 + 0) * C + c], float(a), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&lvl[(size_t(grp) * 2 + 1) * C + c], float(b), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // Hand-off (MI355X_MICROARCH.md, cross-workgroup table row 1): every storing wave waits
  // for its stores, a barrier, one agent-scope add per workgroup; the workgroup whose add
  // came last reads all groups with sc1 loads (L1 bypass) in group order — no fences.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) prev = atomicAdd(&tickets[blockIdx.x], 1u);
  __syncthreads();
  if (prev != gridDim.y - 1) return;
  // consumer: one agent acquire (invalidates this CU's L1), its wait, a barrier, then
  // plain loads the compiler can batch
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  a = b = 0;
  if (c < C) {
#pragma unroll 4
    for (int g = kl; g < int(gridDim.y); g += kTileLanes) {
      a += double(lvl[(size_t(g) * 2 + 0) * C + c]);
      b += double(lvl[(size_t(g) * 2 + 1) * C + c]);
    }
  }
  __syncthreads();
  sa[kl][cl] = a;
  sb[kl][cl] = b;
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(&tickets[blockIdx.x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (threadIdx.x < kBoundSlots && blockIdx.x == 0 && fa.zero) fa.zero[threadIdx.x * kBoundStride] = 0.f;
  if (kl != 0 || c >= C) return;
#pragma unroll
  for (int k = 1; k < kTileLanes; ++k) {
    a += sa[k][cl];
    b += sb[k][cl];
  }
  if constexpr (CHAN)
    fin_fwd_channel(c, a, b, C, M, x, fa.gamma, fa.beta, fa.eps, fa.momentum, fa.rmean, fa.rvar, fa.save_mean,
                    fa.save_rstd, fa.coef);
  else
    fin_bwd_channel(c, a, b, C, M, fa.gamma, fa.mean, fa.rstd, fa.dgamma, fa.dbeta, fa.coef);
}

// groups for level 1: >= 32 tile rows each (2 per lane), at most 128 (the last group
// combines them all, 8 per lane)
int tile_groups(int64_t nt, int* rows_per_group) {
  int g = int(std::min<int64_t>(128, std::max<int64_t>(1, (nt + 31) / 32)));
  *rows_per_group = int((nt + g - 1) / g);
  g = int((nt + *rows_per_group - 1) / *rows_per_group);
  return g;
}

// Partials emitted by a GEMM epilogue (gemm.hip), one row pair per 128-row tile — up to
// thousands of rows, too many for one finalize block per 64 channels. One launch: groups
// of tile rows are folded in parallel (grid: channel blocks x groups) into lvl[groups][2][C],
// and the last group to finish for a channel block (ticket) combines the groups and writes
// the BN coefficients (deterministic: fixed group order, fp64):
//   CHAN (forward statistics): tile k holds (mean_k, M2_k) of n_k = min(128, M - 128k)
//        rows; level 1 = sum n_k d_k, sum M2_k + n_k d_k^2 with d_k = mean_k - x[0][c], the
//        shifted sums of the stand-alone statistics pass;
//   plain (backward reductions): tile sums are added.
template <typename T, bool CHAN>
void launch_tiles_finalize(hipStream_t s, const float* part, int64_t nt, int C, int64_t M, const T* x, float* lvl,
                           const FinArgs& fa) {
  if (nt <= 0 || nt > INT32_MAX) throw std::invalid_argument("bn_act: bad partial count");
  const int nchb = (C + 63) / 64;
  if (nchb > kMaxChBlocks) throw std::invalid_argument("bn_act: too many channels for the tile reduction");
  static std::atomic<uint32_t> launches{0};
  uint32_t* base = nullptr;
  hip_check(hipGetSymbolAddress(reinterpret_cast<void**>(&base), HIP_SYMBOL(g_bn_tickets)), "ticket symbol");
  uint32_t* tick = base + size_t(launches.fetch_add(1) % kTicketSlots) * kMaxChBlocks;
  int rpg;
  const int g = tile_groups(nt, &rpg);
  static const bool wide = [] {
    const char* e = std::getenv("MPIT_BN_FIN_LANES");
    return e && std::atoi(e) == 16;
  }();
  if (wide)
    hipLaunchKernelGGL((bn_tiles_finalize_kernel<T, CHAN, kFinLanesWide>), dim3(nchb, g), dim3(64 * kFinLanesWide), 0,
                       s, part, int(nt), C, M, x, rpg, lvl, tick, fa);
  else
    hipLaunchKernelGGL((bn_tiles_finalize_kernel<T, CHAN, kFinLanesNarrow>), dim3(nchb, g), dim3(64 * kFinLanesNarrow),
                       0, s, part, int(nt), C, M, x, rpg, lvl, tick, fa);
}

// ---------------------------------------------------------------- forward: apply
// MASK: also store the ReLU mask, one byte per vector (bit v = element v of the vector is
// positive), so the backward never re-reads y (1/16 of its bytes for bf16, 1/32 for fp32).
template <typename T, bool RES, bool RELU, bool MASK, bool SPLIT, int U>
__global__ __launch_bounds__(1024) void bn_apply_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                        T* __restrict__ y, const float* __restrict__ coef, int64_t nvec,
                                                        int C, uint8_t* __restrict__ mask, AmaxOut am) {
  constexpr int V = Vec<T>::N;
  int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;  // multiple of G
  float sc[V], sh[V];
  {
    int ch[8];
    Slot<SPLIT>(i, nvec).chans(C, ch);
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const int c = ch[v];
      sc[v] = coef[c];
      sh[v] = coef[C + c];
    }
  }
  float mx = 0.f;
  // fp16 planes (fp32 passes): the output bound from the input's maximum and the coefficients,
  // |x sc + sh (+ res)| <= max|sc| max|x| + max|sh| (+ max|res|) (the fp16x3 split tolerates
  // values up to 4x the bound: its rounding is harmless); a block spans every channel
  [[maybe_unused]] PlaneScale ps{1.f, 2048.f};
  [[maybe_unused]] float rinv = 1.f;
  const int64_t nel = nvec * 8;
  if constexpr (sizeof(T) == 4) {
    const float rb = RES && am.rbound ? slots_max_wave(am.rbound) : 0.f;
    if (RES && am.rplanes) rinv = pexp2(-plane_exp(rb));
    if (am.obound) {  // (from the coefficients in registers)
      float m[2] = {abs_max8(sc), abs_max8(sh)};
      coef_max_block(m, C);
      float bound = fmaf(m[0], epoch_max_wave(am.xmax, am.xep), m[1]);
      if constexpr (RES) bound += rb;
      ps = plane_scale(bound, am.obound);
    }
  }
  for_slots<SPLIT, U>(i, stride, nvec, [&](const auto& s) {
    float a[V], rr[V];
    load8<T>(x, s, a);
    if constexpr (RES) {
      if (sizeof(T) == 4 && am.rplanes) load_planes(reinterpret_cast<const float*>(res), nel, s, rinv, rr);
      else load8<T>(res, s, rr);
    }
    uint32_t bits = 0;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      float t = fmaf(a[v], sc[v], sh[v]);
      if constexpr (RES) t += rr[v];
      if constexpr (RELU) t = fmaxf(t, 0.f);
      a[v] = t;
      if (s.valid(v >> 2)) mx = fmaxf(mx, fabsf(t));
    }
    if (sizeof(T) == 4 && am.obound) store_planes(reinterpret_cast<float*>(y), nel, s, a, ps);
    else store8<T>(y, s, a);
    if constexpr (MASK) {  // (rounding to bf16 never flips the sign of a normal number)
#pragma unroll
      for (int v = 0; v < V; ++v) bits |= uint32_t(a[v] > 0.f) << v;
      mask_store(mask, s, bits);
    }
  });
  if (am.amax) amax_finish(mx, am);
}

// ---------------------------------------------------------------- backward: reduce
// dz = dy (RELU: masked by the forward's bit mask); sums of dz and dz*(x - mean)
template <typename T, bool RELU>
__global__ __launch_bounds__(1024) void bn_bwd_reduce_kernel(const T* __restrict__ dy, const uint8_t* __restrict__ mask,
                                                             const T* __restrict__ x, const float* __restrict__ mean,
                                                             int64_t M, int C, int64_t rows_per_block,
                                                             float* __restrict__ part) {
  constexpr int V = Vec<T>::N;
  extern __shared__ float lds[];
  const int G = C / V;
  const int g = threadIdx.x % G, rs = threadIdx.x / G, R = blockDim.x / G;
  float mu[V], s1[V], s2[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    mu[v] = mean[g * V + v];
    s1[v] = s2[v] = 0.f;
  }
  const int64_t r0 = int64_t(blockIdx.x) * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  int64_t r = r0 + rs;
  for (; r + R < r1; r += 2 * R) {
    float d[2][V], xx[2][V];
    uint32_t mb[2] = {0xffu, 0xffu};
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int64_t o = (r + u * R) * C + g * V;
      Vec<T>::load(dy + o, d[u]);
      Vec<T>::load(x + o, xx[u]);
      if constexpr (RELU) mb[u] = mask[(r + u * R) * G + g];
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int v = 0; v < V; ++v) {
        float dz = d[u][v];
        if constexpr (RELU) dz = (mb[u] >> v) & 1u ? dz : 0.f;
        s1[v] += dz;
        s2[v] = fmaf(dz, xx[u][v] - mu[v], s2[v]);
      }
  }
  for (; r < r1; r += R) {
    float d[V], xx[V];
    const int64_t o = r * C + g * V;
    Vec<T>::load(dy + o, d);
    Vec<T>::load(x + o, xx);
    uint32_t mb = 0xffu;
    if constexpr (RELU) mb = mask[r * G + g];
#pragma unroll
    for (int v = 0; v < V; ++v) {
      float dz = d[v];
      if constexpr (RELU) dz = (mb >> v) & 1u ? dz : 0.f;
      s1[v] += dz;
      s2[v] = fmaf(dz, xx[v] - mu[v], s2[v]);
    }
  }
#pragma unroll
  for (int v = 0; v < V; ++v) {
    lds[(rs * 2 + 0) * C + g * V + v] = s1[v];
    lds[(rs * 2 + 1) * C + g * V + v] = s2[v];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float a = 0.f, b = 0.f;
    for (int k = 0; k < R; ++k) {
      a += lds[(k * 2 + 0) * C + c];
      b += lds[(k * 2 + 1) * C + c];
    }
    part[(size_t(blockIdx.x) * 2 + 0) * C + c] = a;
    part[(size_t(blockIdx.x) * 2 + 1) * C + c] = b;
  }
}

__global__ __launch_bounds__(kFinCh * kFinK) void bn_finalize_bwd_kernel(
    const float* __restrict__ part, int nb, int C, int64_t M, const float* __restrict__ gamma,
    const float* __restrict__ mean, const float* __restrict__ rstd, float* __restrict__ dgamma, float* __restrict__ dbeta,
    float* __restrict__ coef /*[3][C] a c b*/) {
  double a, b;
  if (!fin_combine(part, nb, C, a, b)) return;
  fin_bwd_channel(blockIdx.x * kFinCh + int(threadIdx.x % kFinCh), a, b, C, M, gamma, mean, rstd, dgamma, dbeta, coef);
}

// channel c of the backward finalize from the sums a = sum dz, b = sum dz (x - mean)
__device__ __forceinline__ void fin_bwd_channel(int c, double a, double b, int C, int64_t M,
                                                const float* __restrict__ gamma, const float* __restrict__ mean,
                                                const float* __restrict__ rstd, float* __restrict__ dgamma,
                                                float* __restrict__ dbeta, float* __restrict__ coef) {
  const float rs = rstd[c];
  if (dgamma) dgamma[c] = float(b) * rs;
  if (dbeta) dbeta[c] = float(a);
  const float A = (gamma ? gamma[c] : 1.f) * rs;
  const float mdz = float(a / double(M)), mdx = float(b / double(M));
  const float Cc = -A * rs * rs * mdx;
  coef[c] = A;
  coef[C + c] = Cc;
  coef[2 * C + c] = -A * mdz - Cc * mean[c];
}

template <typename T, bool RELU, bool RESGRAD, bool SPLIT, int U>
__global__ __launch_bounds__(1024) void bn_bwd_apply_kernel(const T* __restrict__ dy, const uint8_t* __restrict__ mask,
                                                            const T* __restrict__ x, const float* __restrict__ coef,
                                                            T* __restrict__ dx, T* __restrict__ dres, int64_t nvec,
                                                            int C, AmaxOut am) {
  constexpr int V = Vec<T>::N;
  int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  float A[V], Cc[V], B[V];
  {
    int ch[8];
    Slot<SPLIT>(i, nvec).chans(C, ch);
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const int c = ch[v];
      A[v] = coef[c];
      Cc[v] = coef[C + c];
      B[v] = coef[2 * C + c];
    }
  }
  float mx = 0.f;
  // fp16 planes: |A dz + Cc x + B| <= max|A| max|dy| + max|Cc| max|x| + max|B|
  [[maybe_unused]] PlaneScale ps{1.f, 2048.f};
  const int64_t nel = nvec * 8;
  if constexpr (sizeof(T) == 4) {
    if (am.obound) {  // (from the coefficients in registers)
      float m[3] = {abs_max8(A), abs_max8(Cc), abs_max8(B)};
      coef_max_block(m, C);
      ps = plane_scale(fmaf(m[0], epoch_max_wave(am.gmax, am.gep), fmaf(m[1], epoch_max_wave(am.xmax, am.xep), m[2])),
                       am.obound);
    }
  }
  for_slots<SPLIT, U>(i, stride, nvec, [&](const auto& s) {
    float d[V], xx[V];
    load8<T>(dy, s, d);
    load8<T>(x, s, xx);
    uint32_t mb = 0xffu;
    if constexpr (RELU) mb = mask_bits(mask, s);
#pragma unroll
    for (int v = 0; v < V; ++v) {
      float dz = d[v];
      if constexpr (RELU) dz = (mb >> v) & 1u ? dz : 0.f;
      d[v] = dz;
      xx[v] = fmaf(A[v], dz, fmaf(Cc[v], xx[v], B[v]));
      if (s.valid(v >> 2)) mx = fmaxf(mx, fabsf(xx[v]));
    }
    if (sizeof(T) == 4 && am.obound) store_planes(reinterpret_cast<float*>(dx), nel, s, xx, ps);
    else store8<T>(dx, s, xx);
    if constexpr (RESGRAD) store8<T>(dres, s, d);
  });
  if (am.amax) amax_finish(mx, am);
}

// ---------------------------------------------------------------- BN pair (ResNet downsample)
// y = relu(x1*sc1 + sh1 + x2*sc2 + sh2): a block's last BN plus its downsample shortcut's BN
// (no ReLU on the shortcut), one pass over (x1, x2) instead of materialising bn2(x2).
template <typename T, bool SPLIT, int U>
__global__ __launch_bounds__(1024) void bn_pair_apply_kernel(const T* __restrict__ x1,
                                                             const T* __restrict__ x2,
                                                             T* __restrict__ y, const float* __restrict__ coef1,
                                                             const float* __restrict__ coef2, int64_t nvec, int C,
                                                             uint8_t* __restrict__ mask, AmaxOut am) {
  constexpr int V = 8;
  int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;  // multiple of G
  float a1[V], b1[V], a2[V], b2[V];
  {
    int ch[8];
    Slot<SPLIT>(i, nvec).chans(C, ch);
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const int c = ch[v];
      a1[v] = coef1[c];
      b1[v] = coef1[C + c];
      a2[v] = coef2[c];
      b2[v] = coef2[C + c];
    }
  }
  float mx = 0.f;
  [[maybe_unused]] PlaneScale ps{1.f, 2048.f};
  const int64_t nel = nvec * 8;
  if constexpr (sizeof(T) == 4) {
    if (am.obound) {  // |y| <= max|a1| max|x1| + max|b1| + max|a2| max|x2| + max|b2|
      float m[4] = {abs_max8(a1), abs_max8(b1), abs_max8(a2), abs_max8(b2)};
      coef_max_block(m, C);
      ps = plane_scale(fmaf(m[0], epoch_max_wave(am.xmax, am.xep), m[1]) +
                           fmaf(m[2], epoch_max_wave(am.xmax2, am.xep2), m[3]),
                       am.obound);
    }
  }
  for_slots<SPLIT, U>(i, stride, nvec, [&](const auto& s) {
    float p[V], q[V];
    load8<T>(x1, s, p);
    load8<T>(x2, s, q);
    uint32_t bits = 0;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const float t = fmaxf(fmaf(p[v], a1[v], b1[v]) + fmaf(q[v], a2[v], b2[v]), 0.f);
      p[v] = t;
      bits |= uint32_t(t > 0.f) << v;
      if (s.valid(v >> 2)) mx = fmaxf(mx, t);
    }
    if (sizeof(T) == 4 && am.obound) store_planes(reinterpret_cast<float*>(y), nel, s, p, ps);
    else store8<T>(y, s, p);
    mask_store(mask, s, bits);
  });
  if (am.amax) amax_finish(mx, am);
}

// dz = dy * mask; dx1 = A1 dz + C1 x1 + B1, dx2 = A2 dz + C2 x2 + B2 (coef [3][C] each)
template <typename T, bool SPLIT, int U>
__global__ __launch_bounds__(1024) void bn_pair_bwd_apply_kernel(
    const T* __restrict__ dy, const uint8_t* __restrict__ mask, const T* __restrict__ x1,
    const float* __restrict__ coef1, T* __restrict__ dx1, const T* __restrict__ x2,
    const float* __restrict__ coef2, T* __restrict__ dx2, int64_t nvec, int C, AmaxOut am1, AmaxOut am2) {
  constexpr int V = 8;
  int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  float A1[V], C1[V], B1[V], A2[V], C2[V], B2[V];
  {
    int ch[8];
    Slot<SPLIT>(i, nvec).chans(C, ch);
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const int c = ch[v];
      A1[v] = coef1[c];
      C1[v] = coef1[C + c];
      B1[v] = coef1[2 * C + c];
      A2[v] = coef2[c];
      C2[v] = coef2[C + c];
      B2[v] = coef2[2 * C + c];
    }
  }
  float m1 = 0.f, m2 = 0.f;
  [[maybe_unused]] PlaneScale ps1{1.f, 2048.f}, ps2{1.f, 2048.f};
  const int64_t nel = nvec * 8;
  if constexpr (sizeof(T) == 4) {
    // |dx_k| <= max|A_k| max|dy| + max|C_k| max|x_k| + max|B_k| (coefficients in registers)
    if (am1.obound || am2.obound) {
      float m[6] = {abs_max8(A1), abs_max8(C1), abs_max8(B1), abs_max8(A2), abs_max8(C2), abs_max8(B2)};
      coef_max_block(m, C);
      if (am1.obound)
        ps1 = plane_scale(fmaf(m[0], epoch_max_wave(am1.gmax, am1.gep), fmaf(m[1], epoch_max_wave(am1.xmax, am1.xep), m[2])),
                          am1.obound);
      if (am2.obound)
        ps2 = plane_scale(fmaf(m[3], epoch_max_wave(am2.gmax, am2.gep), fmaf(m[4], epoch_max_wave(am2.xmax, am2.xep), m[5])),
                          am2.obound);
    }
  }
  for_slots<SPLIT, U>(i, stride, nvec, [&](const auto& s) {
    float d[V], p[V], q[V];
    load8<T>(dy, s, d);
    load8<T>(x1, s, p);
    load8<T>(x2, s, q);
    const uint32_t mb = mask_bits(mask, s);
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const float dz = (mb >> v) & 1u ? d[v] : 0.f;
      p[v] = fmaf(A1[v], dz, fmaf(C1[v], p[v], B1[v]));
      q[v] = fmaf(A2[v], dz, fmaf(C2[v], q[v], B2[v]));
      if (s.valid(v >> 2)) {
        m1 = fmaxf(m1, fabsf(p[v]));
        m2 = fmaxf(m2, fabsf(q[v]));
      }
    }
    if (sizeof(T) == 4 && am1.obound) store_planes(reinterpret_cast<float*>(dx1), nel, s, p, ps1);
    else store8<T>(dx1, s, p);
    if (sizeof(T) == 4 && am2.obound) store_planes(reinterpret_cast<float*>(dx2), nel, s, q, ps2);
    else store8<T>(dx2, s, q);
  });
  if (am1.amax) amax_finish(m1, am1);
  if (am2.amax) amax_finish(m2, am2);
}

void check_shape(int64_t M, int C, int V, uintptr_t ptr) {
  if (M <= 0 || C <= 0) throw std::invalid_argument("bn_act: empty tensor");
  if (C % V) throw std::invalid_argument("bn_act: channels must be a multiple of " + std::to_string(V));
  if (C / V > 1024) throw std::invalid_argument("bn_act: too many channels");
  if (ptr % 16) throw std::invalid_argument("bn_act: tensors must be 16-byte aligned");
}

int stat_blocks(int64_t M, int R, int64_t* rows_per_block) {
  int64_t nb = std::min<int64_t>(kMaxStatBlocks, std::max<int64_t>(1, (M + R * 8 - 1) / (R * 8)));
  int64_t rpb = (M + nb - 1) / nb;
  rpb = (rpb + R - 1) / R * R;
  nb = (M + rpb - 1) / rpb;
  *rows_per_block = rpb;
  return int(nb);
}

template <typename T>
void launch_apply(hipStream_t s, const T* x, const T* res, T* y, int64_t M, int C, const float* coef, bool relu,
                  uint8_t* mask, AmaxOut am = {}) {
  constexpr int V = Vec<T>::N;
  const int G = C / V;
  const int blk = block_for(G);
  const int64_t nvec = M * G;
  const int u = apply_u(sizeof(T) == 4);
  const dim3 g(apply_grid_u(nvec, blk, u)), b(blk);
  with_mode<sizeof(T) == 4>(split_ok(sizeof(T) == 4, C, blk), u, [&](auto sp, auto uu) {
    constexpr bool SP = decltype(sp)::value;
    constexpr int U = decltype(uu)::value;
    if (relu && mask) {
      if (res) hipLaunchKernelGGL((bn_apply_kernel<T, true, true, true, SP, U>), g, b, 0, s, x, res, y, coef, nvec, C, mask, am);
      else hipLaunchKernelGGL((bn_apply_kernel<T, false, true, true, SP, U>), g, b, 0, s, x, res, y, coef, nvec, C, mask, am);
    } else if (relu) {
      if (res) hipLaunchKernelGGL((bn_apply_kernel<T, true, true, false, SP, U>), g, b, 0, s, x, res, y, coef, nvec, C, mask, am);
      else hipLaunchKernelGGL((bn_apply_kernel<T, false, true, false, SP, U>), g, b, 0, s, x, res, y, coef, nvec, C, mask, am);
    } else {
      if (res) hipLaunchKernelGGL((bn_apply_kernel<T, true, false, false, SP, U>), g, b, 0, s, x, res, y, coef, nvec, C, mask, am);
      else hipLaunchKernelGGL((bn_apply_kernel<T, false, false, false, SP, U>), g, b, 0, s, x, res, y, coef, nvec, C, mask, am);
    }
  });
}

template <typename T>
void fwd_impl(int dev, hipStream_t s, const T* x, const T* res, T* y, int64_t M, int C, const float* gamma,
              const float* beta, float* rmean, float* rvar, float* save_mean, float* save_rstd, float* ws,
              float momentum, float eps, bool relu, uint8_t* mask, const float* tstats, int64_t nstat,
              uintptr_t amax, const PlaneSpec* planes) {
  constexpr int V = Vec<T>::N;
  // amax: zeroed by the finalize below (tile statistics) or a memset, raised by the apply pass;
  // with y == nullptr (coefficients only, bn_pair) only the zeroing happens
  const AmaxOut am = amax_out(y ? amax : 0, planes);
  check_shape(M, C, V, reinterpret_cast<uintptr_t>(x));
  const int G = C / V;
  const int blk = block_for(G);
  float* coef = ws;  // [2][C]
  if (tstats) {  // statistics from the producing GEMM's epilogue: no pass over x
    if (nstat != (M + kTileRows - 1) / kTileRows) throw std::invalid_argument("bn_act: stats tiles do not match M");
    FinArgs fa{};
    fa.gamma = gamma;
    fa.beta = beta;
    fa.eps = eps;
    fa.momentum = momentum;
    fa.rmean = rmean;
    fa.rvar = rvar;
    fa.save_mean = save_mean;
    fa.save_rstd = save_rstd;
    fa.coef = coef;
    fa.zero = reinterpret_cast<float*>(amax);
    launch_tiles_finalize<T, true>(s, tstats, nstat, C, M, x, ws + 2 * C, fa);
    if (y) launch_apply<T>(s, x, res, y, M, C, coef, relu, mask, am);
    hip_check(hipGetLastError(), "bn_act forward launch");
    return;
  }
  const int R = blk / G;
  int64_t rpb;
  const int nb = stat_blocks(M, R, &rpb);
  float* part = ws + 2 * C;
  const size_t shm = size_t(R) * 2 * C * sizeof(float);
  hipLaunchKernelGGL(bn_stats_kernel<T>, dim3(nb), dim3(blk), shm, s, x, M, C, rpb, part);
  hipLaunchKernelGGL(bn_finalize_fwd_kernel<T>, dim3((C + kFinCh - 1) / kFinCh), dim3(kFinCh * kFinK), 0, s, part, nb,
                     C, M, x, gamma, beta, eps, momentum, rmean, rvar, save_mean, save_rstd, coef);
  if (amax) hip_check(hipMemsetAsync(reinterpret_cast<void*>(amax), 0, kBoundFloats * sizeof(float), s), "amax zero");
  if (y) launch_apply<T>(s, x, res, y, M, C, coef, relu, mask, am);  // y == nullptr: coefficients only
  hip_check(hipGetLastError(), "bn_act forward launch");
}

template <typename T>
void bwd_impl(hipStream_t s, const T* dy, const uint8_t* mask, const T* x, T* dx, T* dres, int64_t M, int C,
              const float* gamma, const float* mean, const float* rstd, float* dgamma, float* dbeta, float* ws,
              bool relu, const float* gpart, int64_t npart, const float* coef_in, uintptr_t amax,
              const PlaneSpec* planes) {
  constexpr int V = Vec<T>::N;
  // amax: zeroed by the finalize (or, given coefficients, by the GEMM that folded it), raised
  // by the apply pass; dx == nullptr: coefficients (and the zeroing) only
  const AmaxOut am = amax_out(dx ? amax : 0, planes);
  check_shape(M, C, V, reinterpret_cast<uintptr_t>(x));
  if (relu && !mask) throw std::invalid_argument("bn_act backward: ReLU needs the forward mask");
  const int G = C / V;
  const int blk = block_for(G);
  const int R = blk / G;
  int64_t rpb;
  const int nb = stat_blocks(M, R, &rpb);
  const float* coef = coef_in ? coef_in : ws;  // [3][C]
  float* part = ws + 3 * C;
  const size_t shm = size_t(R) * 2 * C * sizeof(float);
  if (coef_in) {
    // coefficients, dgamma and dbeta already written by the GEMM that produced dy
  } else if (gpart) {  // reductions already produced by the GEMM that wrote dy (gemm.hip EPI_BNRED)
    FinArgs fa{};
    fa.gamma = gamma;
    fa.mean = mean;
    fa.rstd = rstd;
    fa.dgamma = dgamma;
    fa.dbeta = dbeta;
    fa.coef = ws;
    fa.zero = reinterpret_cast<float*>(amax);
    launch_tiles_finalize<T, false>(s, gpart, npart, C, M, x, part, fa);
  } else {
    if (relu)
      hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, true>), dim3(nb), dim3(blk), shm, s, dy, mask, x, mean, M, C, rpb,
                         part);
    else
      hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, false>), dim3(nb), dim3(blk), shm, s, dy, mask, x, mean, M, C, rpb,
                         part);
    hipLaunchKernelGGL(bn_finalize_bwd_kernel, dim3((C + kFinCh - 1) / kFinCh), dim3(kFinCh * kFinK), 0, s, part, nb,
                       C, M, gamma, mean, rstd, dgamma, dbeta, ws);
    if (amax) hip_check(hipMemsetAsync(reinterpret_cast<void*>(amax), 0, kBoundFloats * sizeof(float), s), "amax zero");
  }
  const int64_t nvec = M * G;
  const int u = apply_u(sizeof(T) == 4);
  const dim3 g(apply_grid_u(nvec, blk, u)), b(blk);
  if (!dx) {  // coefficients only (ws[0, 3C)), dgamma / dbeta
    hip_check(hipGetLastError(), "bn_act backward launch");
    return;
  }
  with_mode<sizeof(T) == 4>(split_ok(sizeof(T) == 4, C, blk), u, [&](auto sp, auto uu) {
    constexpr bool SP = decltype(sp)::value;
    constexpr int U = decltype(uu)::value;
    if (relu) {
      if (dres) hipLaunchKernelGGL((bn_bwd_apply_kernel<T, true, true, SP, U>), g, b, 0, s, dy, mask, x, coef, dx, dres, nvec, C, am);
      else hipLaunchKernelGGL((bn_bwd_apply_kernel<T, true, false, SP, U>), g, b, 0, s, dy, mask, x, coef, dx, dres, nvec, C, am);
    } else {
      if (dres) hipLaunchKernelGGL((bn_bwd_apply_kernel<T, false, true, SP, U>), g, b, 0, s, dy, mask, x, coef, dx, dres, nvec, C, am);
      else hipLaunchKernelGGL((bn_bwd_apply_kernel<T, false, false, SP, U>), g, b, 0, s, dy, mask, x, coef, dx, dres, nvec, C, am);
    }
  });
  hip_check(hipGetLastError(), "bn_act backward launch");
}

}  // namespace

int64_t bn_workspace_floats(int C) { return int64_t(3) * C + int64_t(2) * kMaxStatBlocks * C; }

int64_t bn_mask_bytes(bool bf16, int64_t M, int C) { (void)bf16; return M * (C / 8); }

void bn_act_fwd(int dev, hipStream_t s, bool bf16, uintptr_t x, uintptr_t res, uintptr_t y, int64_t M, int C,
                uintptr_t gamma, uintptr_t beta, uintptr_t rmean, uintptr_t rvar, uintptr_t save_mean,
                uintptr_t save_rstd, uintptr_t ws, float momentum, float eps, bool relu, uintptr_t mask,
                uintptr_t stats, int64_t nstat, uintptr_t amax, uintptr_t coef, const PlaneSpec* planes) {
  hip_check(hipSetDevice(dev), "hipSetDevice");
  if (planes && (bf16 || (planes->obound && !y) || (planes->rplanes && !(res && planes->rbound)) ||
                 (planes->obound && res && !planes->rbound)))
    throw std::invalid_argument("bn_act forward: fp16 planes are for fp32 passes with the bounds of their inputs");
  auto F = [](uintptr_t p) { return reinterpret_cast<float*>(p); };
  auto* mk = reinterpret_cast<uint8_t*>(mask);
  if (coef) {  // finalize folded into the producing GEMM (gemm.hip stats_fold): the apply pass only
    if (!y) throw std::invalid_argument("bn_act forward: given coefficients need y");
    if (bf16) {
      check_shape(M, C, 8, x);
      launch_apply<uint16_t>(s, reinterpret_cast<const uint16_t*>(x), reinterpret_cast<const uint16_t*>(res),
                             reinterpret_cast<uint16_t*>(y), M, C, F(coef), relu, mk, AmaxOut{F(amax)});
    } else {
      check_shape(M, C, 8, x);
      launch_apply<float>(s, reinterpret_cast<const float*>(x), reinterpret_cast<const float*>(res),
                          reinterpret_cast<float*>(y), M, C, F(coef), relu, mk, amax_out(amax, planes));
    }
    hip_check(hipGetLastError(), "bn_act forward launch");
    return;
  }
  if (bf16)
    fwd_impl<uint16_t>(dev, s, reinterpret_cast<const uint16_t*>(x), reinterpret_cast<const uint16_t*>(res),
                       reinterpret_cast<uint16_t*>(y), M, C, F(gamma), F(beta), F(rmean), F(rvar), F(save_mean),
                       F(save_rstd), F(ws), momentum, eps, relu, mk, F(stats), nstat, amax, nullptr);
  else
    fwd_impl<float>(dev, s, reinterpret_cast<const float*>(x), reinterpret_cast<const float*>(res),
                    reinterpret_cast<float*>(y), M, C, F(gamma), F(beta), F(rmean), F(rvar), F(save_mean), F(save_rstd),
                    F(ws), momentum, eps, relu, mk, F(stats), nstat, amax, planes);
}

void bn_act_apply(int dev, hipStream_t s, bool bf16, uintptr_t x, uintptr_t res, uintptr_t y, int64_t M, int C,
                  uintptr_t coef, bool relu) {
  hip_check(hipSetDevice(dev), "hipSetDevice");
  if (bf16) {
    check_shape(M, C, 8, x);
    launch_apply<uint16_t>(s, reinterpret_cast<const uint16_t*>(x), reinterpret_cast<const uint16_t*>(res),
                           reinterpret_cast<uint16_t*>(y), M, C, reinterpret_cast<const float*>(coef), relu, nullptr);
  } else {
    check_shape(M, C, 8, x);
    launch_apply<float>(s, reinterpret_cast<const float*>(x), reinterpret_cast<const float*>(res),
                        reinterpret_cast<float*>(y), M, C, reinterpret_cast<const float*>(coef), relu, nullptr);
  }
  hip_check(hipGetLastError(), "bn_act apply launch");
}

void bn_act_bwd(int dev, hipStream_t s, bool bf16, uintptr_t dy, uintptr_t mask, uintptr_t x, uintptr_t dx,
                uintptr_t dres, int64_t M, int C, uintptr_t gamma, uintptr_t mean, uintptr_t rstd, uintptr_t dgamma,
                uintptr_t dbeta, uintptr_t ws, bool relu, uintptr_t part, int64_t npart, uintptr_t coef,
                uintptr_t amax, const PlaneSpec* planes) {
  hip_check(hipSetDevice(dev), "hipSetDevice");
  if (planes && planes->obound && (bf16 || !dx || dres))
    throw std::invalid_argument("bn_act backward: fp16 planes are for fp32 dx passes without a residual gradient");
  auto F = [](uintptr_t p) { return reinterpret_cast<float*>(p); };
  const auto* mk = reinterpret_cast<const uint8_t*>(mask);
  if (coef && !dx) throw std::invalid_argument("bn_act backward: given coefficients need dx");
  if (bf16)
    bwd_impl<uint16_t>(s, reinterpret_cast<const uint16_t*>(dy), mk, reinterpret_cast<const uint16_t*>(x),
                       reinterpret_cast<uint16_t*>(dx), reinterpret_cast<uint16_t*>(dres), M, C, F(gamma), F(mean),
                       F(rstd), F(dgamma), F(dbeta), F(ws), relu, F(part), npart, F(coef), amax, nullptr);
  else
    bwd_impl<float>(s, reinterpret_cast<const float*>(dy), mk, reinterpret_cast<const float*>(x),
                    reinterpret_cast<float*>(dx), reinterpret_cast<float*>(dres), M, C, F(gamma), F(mean), F(rstd),
                    F(dgamma), F(dbeta), F(ws), relu, F(part), npart, F(coef), amax, planes);
}

template <typename T>
static void pair_apply_t(hipStream_t s, uintptr_t x1, uintptr_t coef1, uintptr_t x2, uintptr_t coef2, uintptr_t y,
                         int64_t M, int C, uintptr_t mask, uintptr_t amax, uintptr_t scratch, const PlaneSpec* planes) {
  const int G = C / 8, blk = block_for(G);
  const int64_t nvec = M * G;
  const int u = apply_u(sizeof(T) == 4);
  with_mode<sizeof(T) == 4>(split_ok(sizeof(T) == 4, C, blk), u, [&](auto sp, auto uu) {
  hipLaunchKernelGGL((bn_pair_apply_kernel<T, decltype(sp)::value, decltype(uu)::value>), dim3(apply_grid_u(nvec, blk, u)), dim3(blk), 0, s,
                     reinterpret_cast<const T*>(x1), reinterpret_cast<const T*>(x2), reinterpret_cast<T*>(y),
                     reinterpret_cast<const float*>(coef1), reinterpret_cast<const float*>(coef2), nvec, C,
                     reinterpret_cast<uint8_t*>(mask), amax_out(amax, planes));
  });
}

template <typename T>
static void pair_bwd_t(hipStream_t s, uintptr_t dy, uintptr_t mask, uintptr_t x1, uintptr_t coef1, uintptr_t dx1,
                       uintptr_t x2, uintptr_t coef2, uintptr_t dx2, int64_t M, int C, uintptr_t amax1, uintptr_t amax2,
                       uintptr_t scratch, const PlaneSpec* p1, const PlaneSpec* p2) {
  const int G = C / 8, blk = block_for(G);
  const int64_t nvec = M * G;
  const int u = apply_u(sizeof(T) == 4);
  with_mode<sizeof(T) == 4>(split_ok(sizeof(T) == 4, C, blk), u, [&](auto sp, auto uu) {
  hipLaunchKernelGGL((bn_pair_bwd_apply_kernel<T, decltype(sp)::value, decltype(uu)::value>), dim3(apply_grid_u(nvec, blk, u)), dim3(blk), 0, s,
                     reinterpret_cast<const T*>(dy), reinterpret_cast<const uint8_t*>(mask),
                     reinterpret_cast<const T*>(x1), reinterpret_cast<const float*>(coef1), reinterpret_cast<T*>(dx1),
                     reinterpret_cast<const T*>(x2), reinterpret_cast<const float*>(coef2), reinterpret_cast<T*>(dx2),
                     nvec, C, amax_out(amax1, p1), amax_out(amax2, p2));
  });
}

void bn_pair_apply(int dev, hipStream_t s, uintptr_t x1, uintptr_t coef1, uintptr_t x2, uintptr_t coef2, uintptr_t y,
                   int64_t M, int C, uintptr_t mask, bool f32, uintptr_t amax, uintptr_t scratch,
                   const PlaneSpec* planes) {
  hip_check(hipSetDevice(dev), "hipSetDevice");
  if (planes && planes->obound && !f32) throw std::invalid_argument("bn_pair_apply: fp16 planes are for fp32 passes");
  check_shape(M, C, 8, x1);
  check_shape(M, C, 8, x2);
  if (!mask) throw std::invalid_argument("bn_pair_apply: needs the ReLU mask buffer");
  if (f32) pair_apply_t<float>(s, x1, coef1, x2, coef2, y, M, C, mask, amax, scratch, planes);
  else pair_apply_t<uint16_t>(s, x1, coef1, x2, coef2, y, M, C, mask, amax, scratch, nullptr);
  hip_check(hipGetLastError(), "bn_pair_apply launch");
}

void bn_pair_bwd_apply(int dev, hipStream_t s, uintptr_t dy, uintptr_t mask, uintptr_t x1, uintptr_t coef1,
                       uintptr_t dx1, uintptr_t x2, uintptr_t coef2, uintptr_t dx2, int64_t M, int C, bool f32,
                       uintptr_t amax1, uintptr_t amax2, uintptr_t scratch, const PlaneSpec* p1,
                       const PlaneSpec* p2) {
  hip_check(hipSetDevice(dev), "hipSetDevice");
  if (((p1 && p1->obound) || (p2 && p2->obound)) && !f32)
    throw std::invalid_argument("bn_pair_bwd_apply: fp16 planes are for fp32 passes");
  check_shape(M, C, 8, x1);
  check_shape(M, C, 8, x2);
  if (f32) pair_bwd_t<float>(s, dy, mask, x1, coef1, dx1, x2, coef2, dx2, M, C, amax1, amax2, scratch, p1, p2);
  else pair_bwd_t<uint16_t>(s, dy, mask, x1, coef1, dx1, x2, coef2, dx2, M, C, amax1, amax2, scratch, nullptr, nullptr);
  hip_check(hipGetLastError(), "bn_pair_bwd_apply launch");
}

}  // namespace mpit

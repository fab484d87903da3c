// Multi-array fused elementwise engine for CDNA4 (gfx950) + an identical host path.
//
// Every parameter-server / worker update rule of mpiT (SURVEY.md §2.7, K1–K14) is a
// flat, memory-bound, one-pass elementwise op over a shard of length S. The reference
// runs each of them as a chain of 3–8 separate Torch7 tensor calls
// (e.g. BiCNN/pserver.lua:130-136 for RMSProp); here every rule is ONE kernel that
// reads each operand once and writes each result once.
//
// Design (cdna_hip_programming.md Guideline 11/13, Appendix B "Element-wise"):
//   * 256-thread blocks (4 wave64s), 16-B per lane per array (float4 / 4×bf16 in 8 B),
//     U independent float4 per array in flight per thread (ILP for HBM latency).
//   * tile = 256 lanes × 4 elems × U; lane t of tile u reads base+u*1024+4t so
//     every wave-instruction is a fully coalesced 1 KiB access.
//   * U and the grid follow the shard size (pick_shape): a PS shard of an 8-way sharded
//     ResNet-50 (3.2 M elements, ~5 us of traffic) needs every CU busy from the first
//     wave, so small shards get U = 1 and one tile per block (up to 8 blocks per CU
//     resident at once); large ones U = 4 with a grid-stride over 2 waves of 2048 blocks.
//   * arrays may be fp32 or bf16 (per-array bit in the BF mask); math is fp32.
//   * read-only arrays are never stored, write-only arrays are never loaded, so the
//     HBM bytes equal the "fused B/elem" column of SURVEY §2.7.
// The same functor runs on the host (CPU servers, gloo plumbing config) through
// run_host(), so CPU and GPU share one definition of each rule.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>
#include <algorithm>

#define MPIT_HD __host__ __device__ __forceinline__

namespace mpit {

MPIT_HD float bf2f(uint16_t h) {
  uint32_t u = uint32_t(h) << 16;
  return __builtin_bit_cast(float, u);
}
MPIT_HD uint16_t f2bf(float f) {
  // plain cast: v_cvt_pk_bf16_f32 on gfx950 (RNE, keeps NaN a NaN; MI355X_MICROARCH
  // "Correctness boundaries"), software RNE on the host.
  return __builtin_bit_cast(uint16_t, static_cast<__bf16>(f));
}

template <int NA>
struct Arrays {
  void* p[NA];
};

template <bool BF>
__device__ __forceinline__ void load4(const void* base, int64_t i4, float (&x)[4]) {
  if constexpr (BF) {
    const uint2 v = reinterpret_cast<const uint2*>(base)[i4];
    x[0] = bf2f(uint16_t(v.x & 0xffff));
    x[1] = bf2f(uint16_t(v.x >> 16));
    x[2] = bf2f(uint16_t(v.y & 0xffff));
    x[3] = bf2f(uint16_t(v.y >> 16));
  } else {
    const float4 v = reinterpret_cast<const float4*>(base)[i4];
    x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
  }
}

template <bool BF>
__device__ __forceinline__ void store4(void* base, int64_t i4, const float (&x)[4]) {
  if constexpr (BF) {
    uint2 v;
    v.x = uint32_t(f2bf(x[0])) | (uint32_t(f2bf(x[1])) << 16);
    v.y = uint32_t(f2bf(x[2])) | (uint32_t(f2bf(x[3])) << 16);
    reinterpret_cast<uint2*>(base)[i4] = v;
  } else {
    reinterpret_cast<float4*>(base)[i4] = make_float4(x[0], x[1], x[2], x[3]);
  }
}

template <bool BF>
MPIT_HD float load1(const void* base, int64_t i) {
  if constexpr (BF) return bf2f(reinterpret_cast<const uint16_t*>(base)[i]);
  else return reinterpret_cast<const float*>(base)[i];
}
template <bool BF>
MPIT_HD void store1(void* base, int64_t i, float v) {
  if constexpr (BF) reinterpret_cast<uint16_t*>(base)[i] = f2bf(v);
  else reinterpret_cast<float*>(base)[i] = v;
}

constexpr int kBlock = 256;
constexpr int kMaxGrid = 2048;

template <int NA, uint32_t RD, uint32_t WR, uint32_t BF, int kUnroll, class F>
__global__ __launch_bounds__(kBlock) void ew_vec_kernel(Arrays<NA> a, int64_t n, F f) {
  const int64_t n4 = n >> 2;
  const int64_t tile = int64_t(kBlock) * kUnroll;
  const int64_t ntiles = (n4 + tile - 1) / tile;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    float x[kUnroll][NA][4];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int64_t i4 = t * tile + u * kBlock + threadIdx.x;
      if (i4 < n4) {
#pragma unroll
        for (int k = 0; k < NA; ++k) {
          if ((RD >> k) & 1) {
            if ((BF >> k) & 1) load4<true>(a.p[k], i4, x[u][k]);
            else load4<false>(a.p[k], i4, x[u][k]);
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int64_t i4 = t * tile + u * kBlock + threadIdx.x;
      if (i4 < n4) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float e[NA];
#pragma unroll
          for (int k = 0; k < NA; ++k) e[k] = x[u][k][j];
          f(e);
#pragma unroll
          for (int k = 0; k < NA; ++k) x[u][k][j] = e[k];
        }
#pragma unroll
        for (int k = 0; k < NA; ++k) {
          if ((WR >> k) & 1) {
            if ((BF >> k) & 1) store4<true>(a.p[k], i4, x[u][k]);
            else store4<false>(a.p[k], i4, x[u][k]);
          }
        }
      }
    }
  }
  // scalar tail (n % 4 elements), one block
  if (blockIdx.x == 0) {
    const int64_t i = (n4 << 2) + threadIdx.x;
    if (i < n) {
      float e[NA];
#pragma unroll
      for (int k = 0; k < NA; ++k)
        if ((RD >> k) & 1) e[k] = ((BF >> k) & 1) ? load1<true>(a.p[k], i) : load1<false>(a.p[k], i);
      f(e);
#pragma unroll
      for (int k = 0; k < NA; ++k)
        if ((WR >> k) & 1) {
          if ((BF >> k) & 1) store1<true>(a.p[k], i, e[k]);
          else store1<false>(a.p[k], i, e[k]);
        }
    }
  }
}

// Fallback for pointers that are not 16-B (fp32) / 8-B (bf16) aligned: shard views at
// arbitrary offsets (reference shards start at any element, asyncsgd/pclient.lua:116-128).
template <int NA, uint32_t RD, uint32_t WR, uint32_t BF, class F>
__global__ __launch_bounds__(kBlock) void ew_scalar_kernel(Arrays<NA> a, int64_t n, F f) {
  const int64_t stride = int64_t(gridDim.x) * kBlock;
  for (int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride) {
    float e[NA];
#pragma unroll
    for (int k = 0; k < NA; ++k)
      if ((RD >> k) & 1) e[k] = ((BF >> k) & 1) ? load1<true>(a.p[k], i) : load1<false>(a.p[k], i);
    f(e);
#pragma unroll
    for (int k = 0; k < NA; ++k)
      if ((WR >> k) & 1) {
        if ((BF >> k) & 1) store1<true>(a.p[k], i, e[k]);
        else store1<false>(a.p[k], i, e[k]);
      }
  }
}

inline void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess)
    throw std::runtime_error(std::string("mpit HIP error in ") + what + ": " + hipGetErrorString(e));
}

template <int NA, uint32_t RD, uint32_t WR, uint32_t BF, class F>
void run_host(const Arrays<NA>& a, int64_t n, const F& f) {
  auto body = [&](int64_t lo, int64_t hi) {
    for (int64_t i = lo; i < hi; ++i) {
      float e[NA];
      for (int k = 0; k < NA; ++k)
        if ((RD >> k) & 1) e[k] = ((BF >> k) & 1) ? load1<true>(a.p[k], i) : load1<false>(a.p[k], i);
      f(e);
      for (int k = 0; k < NA; ++k)
        if ((WR >> k) & 1) {
          if ((BF >> k) & 1) store1<true>(a.p[k], i, e[k]);
          else store1<false>(a.p[k], i, e[k]);
        }
    }
  };
  const int64_t kPar = int64_t(1) << 20;
  if (n < kPar) {
    body(0, n);
    return;
  }
  int nt = int(std::min<int64_t>(8, n / kPar));
  std::vector<std::thread> th;
  int64_t chunk = (n + nt - 1) / nt;
  for (int t = 0; t < nt; ++t) {
    int64_t lo = t * chunk, hi = std::min(n, lo + chunk);
    if (lo < hi) th.emplace_back(body, lo, hi);
  }
  for (auto& x : th) x.join();
}

// (unroll, grid cap) for n4 float4 groups; MPIT_EW_UNROLL / MPIT_EW_GRID override (A/B).
inline void pick_shape(int64_t n4, int& unroll, int64_t& cap) {
  static const int env_u = [] { const char* e = std::getenv("MPIT_EW_UNROLL"); return e ? std::atoi(e) : 0; }();
  static const int64_t env_g = [] { const char* e = std::getenv("MPIT_EW_GRID"); return e ? std::atoll(e) : 0; }();
  unroll = n4 <= (int64_t(1) << 21) ? 1 : (n4 <= (int64_t(1) << 23) ? 2 : 4);
  cap = n4 <= (int64_t(1) << 21) ? int64_t(1) << 30 : kMaxGrid;
  if (env_u == 1 || env_u == 2 || env_u == 4) unroll = env_u;
  if (env_g > 0) cap = env_g;
}

// ---- multi-segment form: ONE launch over up to kMaxSegs independent operand sets ----
// (a parameter server applying several due shard pieces at once: 8 pieces of 3.2 M
// elements are launch- and tail-bound one by one, one wave of the whole chip together).
// Segments must be disjoint; every segment's operands 16-B (fp32) / 8-B (bf16) aligned.
constexpr int kMaxSegs = 16;
template <int NA>
struct SegArrays {
  void* p[kMaxSegs][NA];
  int64_t n[kMaxSegs];
  int64_t t0[kMaxSegs + 1];  // first block (one tile of kBlock float4) of each segment
  int nseg;
};

template <int NA, uint32_t RD, uint32_t WR, uint32_t BF, class F>
__global__ __launch_bounds__(kBlock) void ew_multi_kernel(SegArrays<NA> sa, F f) {
  const int64_t b = blockIdx.x;
  int s = 0;
  while (s + 1 < sa.nseg && b >= sa.t0[s + 1]) ++s;
  const int64_t n = sa.n[s], n4 = n >> 2;
  const int64_t i4 = (b - sa.t0[s]) * kBlock + threadIdx.x;
  float x[NA][4];
  if (i4 < n4) {
#pragma unroll
    for (int k = 0; k < NA; ++k)
      if ((RD >> k) & 1) {
        if ((BF >> k) & 1) load4<true>(sa.p[s][k], i4, x[k]);
        else load4<false>(sa.p[s][k], i4, x[k]);
      }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float e[NA];
#pragma unroll
      for (int k = 0; k < NA; ++k) e[k] = x[k][j];
      f(e);
#pragma unroll
      for (int k = 0; k < NA; ++k) x[k][j] = e[k];
    }
#pragma unroll
    for (int k = 0; k < NA; ++k)
      if ((WR >> k) & 1) {
        if ((BF >> k) & 1) store4<true>(sa.p[s][k], i4, x[k]);
        else store4<false>(sa.p[s][k], i4, x[k]);
      }
  }
  // the segment's n % 4 tail: its last block
  if (b + 1 == sa.t0[s + 1]) {
    const int64_t i = (n4 << 2) + threadIdx.x;
    if (i < n) {
      float e[NA];
#pragma unroll
      for (int k = 0; k < NA; ++k)
        if ((RD >> k) & 1) e[k] = ((BF >> k) & 1) ? load1<true>(sa.p[s][k], i) : load1<false>(sa.p[s][k], i);
      f(e);
#pragma unroll
      for (int k = 0; k < NA; ++k)
        if ((WR >> k) & 1) {
          if ((BF >> k) & 1) store1<true>(sa.p[s][k], i, e[k]);
          else store1<false>(sa.p[s][k], i, e[k]);
        }
    }
  }
}

// Segment list of the current ew_update_multi call on this thread (see updates.hip): the
// rule dispatch below is shared, and run_ew takes the segments from here when set.
struct MultiSegs {
  std::vector<std::vector<uintptr_t>> ptrs;
  std::vector<int64_t> ns;
};
inline thread_local const MultiSegs* t_multi = nullptr;

template <int NA, uint32_t RD, uint32_t WR, uint32_t BF, class F>
void run_ew(const Arrays<NA>& a, int64_t n, const F& f, int dev, hipStream_t stream);

template <int NA, uint32_t RD, uint32_t WR, uint32_t BF, class F>
void run_ew_multi(const MultiSegs& ms, const F& f, int dev, hipStream_t stream) {
  const size_t ns = ms.ns.size();
  auto seg = [&](size_t i) {
    Arrays<NA> a;
    for (int k = 0; k < NA; ++k) a.p[k] = reinterpret_cast<void*>(ms.ptrs[i][size_t(k)]);
    return a;
  };
  bool ok = dev >= 0 && ns <= size_t(kMaxSegs);
  for (size_t i = 0; ok && i < ns; ++i) {
    if (ms.ptrs[i].size() != size_t(NA)) throw std::invalid_argument("mpit: wrong number of operands");
    for (int k = 0; k < NA; ++k) {
      if (!(((RD | WR) >> k) & 1)) continue;
      const uintptr_t al = ((BF >> k) & 1) ? 8 : 16;
      if (ms.ptrs[i][size_t(k)] % al) ok = false;
    }
  }
  if (!ok) {  // host, too many segments or unaligned: one pass per segment
    for (size_t i = 0; i < ns; ++i) run_ew<NA, RD, WR, BF, F>(seg(i), ms.ns[i], f, dev, stream);
    return;
  }
  SegArrays<NA> sa{};
  int64_t t = 0;
  int m = 0;
  for (size_t i = 0; i < ns; ++i) {
    if (ms.ns[i] <= 0) continue;
    for (int k = 0; k < NA; ++k) sa.p[m][k] = reinterpret_cast<void*>(ms.ptrs[i][size_t(k)]);
    sa.n[m] = ms.ns[i];
    sa.t0[m] = t;
    t += std::max<int64_t>(1, ((ms.ns[i] >> 2) + kBlock - 1) / kBlock);
    ++m;
  }
  if (m == 0) return;
  sa.t0[m] = t;
  sa.nseg = m;
  hipLaunchKernelGGL((ew_multi_kernel<NA, RD, WR, BF, F>), dim3(unsigned(t)), dim3(kBlock), 0, stream, sa, f);
  hip_check(hipGetLastError(), "ew multi launch");
}

// dev < 0: host; otherwise launch on `stream` (which belongs to the current device).
template <int NA, uint32_t RD, uint32_t WR, uint32_t BF, class F>
void run_ew(const Arrays<NA>& a, int64_t n, const F& f, int dev, hipStream_t stream) {
  if (const MultiSegs* ms = t_multi) {  // ew_update_multi: the segment list replaces (a, n)
    t_multi = nullptr;
    run_ew_multi<NA, RD, WR, BF, F>(*ms, f, dev, stream);
    return;
  }
  if (n <= 0) return;
  if (dev < 0) {
    run_host<NA, RD, WR, BF>(a, n, f);
    return;
  }
  bool aligned = true;
  for (int k = 0; k < NA; ++k) {
    if (!(((RD | WR) >> k) & 1)) continue;
    const uintptr_t al = ((BF >> k) & 1) ? 8 : 16;
    if (reinterpret_cast<uintptr_t>(a.p[k]) % al) aligned = false;
  }
  if (aligned) {
    const int64_t n4 = n >> 2;
    int unroll;
    int64_t cap;
    pick_shape(n4, unroll, cap);
    const int64_t tile = int64_t(kBlock) * unroll;
    int64_t grid = std::max<int64_t>(1, std::min<int64_t>((n4 + tile - 1) / tile, cap));
    if (unroll == 1)
      hipLaunchKernelGGL((ew_vec_kernel<NA, RD, WR, BF, 1, F>), dim3(grid), dim3(kBlock), 0, stream, a, n, f);
    else if (unroll == 2)
      hipLaunchKernelGGL((ew_vec_kernel<NA, RD, WR, BF, 2, F>), dim3(grid), dim3(kBlock), 0, stream, a, n, f);
    else
      hipLaunchKernelGGL((ew_vec_kernel<NA, RD, WR, BF, 4, F>), dim3(grid), dim3(kBlock), 0, stream, a, n, f);
  } else {
    int64_t grid = std::max<int64_t>(1, std::min<int64_t>((n + kBlock - 1) / kBlock, kMaxGrid));
    hipLaunchKernelGGL((ew_scalar_kernel<NA, RD, WR, BF, F>), dim3(grid), dim3(kBlock), 0, stream, a, n, f);
  }
  hip_check(hipGetLastError(), "ew launch");
}

}  // namespace mpit

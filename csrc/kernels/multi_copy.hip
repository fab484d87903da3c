// K12: gradient bucketing / unbucketing — many tensors <-> one contiguous shard in ONE
// launch, with fp32<->bf16 cast and an optional scale (the K14 "g /= B" fused in).
//
// The reference gets a flat parameter vector from nn's getParameters() and then shard
// views as sub-storages (asyncsgd/goot.lua:41, asyncsgd/pclient.lua:51-53). Here model
// parameters normally live directly in a registered flat window (zero-copy, see
// mpit_amd/utils/flat.py); this kernel serves models that are not flat (bucketed
// all-reduce, bf16 model copies of an fp32 master).
//
// Work list: the host splits every tensor into chunks of <= kChunk elements; one
// workgroup per chunk (grid-stride over chunks), so 161 ResNet-50 tensors of very
// different sizes still give a balanced grid of thousands of workgroups. Within a chunk
// lanes move 16 B (fp32) / 8 B (bf16) per access when both ends are aligned, else
// scalar; the branch is uniform per workgroup.
#include "kernels.h"
#include "ew.h"

namespace mpit {
namespace {

constexpr int kCB = 256;

template <bool SB, bool DB>
__device__ void copy_chunk(const CopyChunk& c, float scale) {
  const void* src = reinterpret_cast<const void*>(c.src);
  void* dst = reinterpret_cast<void*>(c.dst);
  const bool vec = (c.src % (SB ? 8 : 16) == 0) && (c.dst % (DB ? 8 : 16) == 0);
  int64_t done = 0;
  if (vec) {
    const int64_t n4 = c.n >> 2;
    for (int64_t i = threadIdx.x; i < n4; i += kCB) {
      float v[4];
      load4<SB>(src, i, v);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] *= scale;
      store4<DB>(dst, i, v);
    }
    done = n4 << 2;
  }
  for (int64_t i = done + threadIdx.x; i < c.n; i += kCB) store1<DB>(dst, i, scale * load1<SB>(src, i));
}

__global__ __launch_bounds__(kCB) void multi_copy_kernel(const CopyChunk* table, int64_t nchunks, float scale) {
  for (int64_t b = blockIdx.x; b < nchunks; b += gridDim.x) {
    const CopyChunk c = table[b];
    switch (c.flags & 3) {
      case 0: copy_chunk<false, false>(c, scale); break;
      case 1: copy_chunk<true, false>(c, scale); break;
      case 2: copy_chunk<false, true>(c, scale); break;
      default: copy_chunk<true, true>(c, scale); break;
    }
  }
}

}  // namespace

void multi_copy(int dev, hipStream_t s, const CopyChunk* table, int64_t nchunks, float scale) {
  if (nchunks <= 0) return;
  if (dev < 0) {
    for (int64_t b = 0; b < nchunks; ++b) {
      const CopyChunk& c = table[b];
      const void* src = reinterpret_cast<const void*>(c.src);
      void* dst = reinterpret_cast<void*>(c.dst);
      const bool sb = c.flags & 1, db = c.flags & 2;
      for (int64_t i = 0; i < c.n; ++i) {
        const float v = scale * (sb ? load1<true>(src, i) : load1<false>(src, i));
        if (db) store1<true>(dst, i, v);
        else store1<false>(dst, i, v);
      }
    }
    return;
  }
  hip_check(hipSetDevice(dev), "hipSetDevice");
  const int64_t grid = std::min<int64_t>(nchunks, 8192);
  hipLaunchKernelGGL(multi_copy_kernel, dim3(grid), dim3(kCB), 0, s, table, nchunks, scale);
  hip_check(hipGetLastError(), "multi_copy launch");
}

}  // namespace mpit

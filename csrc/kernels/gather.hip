// K12 + K9 fused: gather a model's per-parameter gradient tensors into one flat push
// buffer with the Downpour scale (and optional weight decay) applied on the way:
//     dst[off_t + i] = a * g_t[i] + b * aux[off_t + i]
// in ONE launch, with the tensor table passed by value in the kernel arguments (no
// per-step host->device table copy, safe under graph capture).
//
// Why: with gradients accumulated into a pre-zeroed flat buffer, autograd issues one
// "grad += new" kernel per parameter (161 for ResNet-50) plus a memset; letting autograd
// hand over its freshly allocated gradient tensors and gathering them once removes
// those passes — the push buffer is written exactly once, by this kernel.
#include "ew.h"
#include "kernels.h"

namespace mpit {
namespace {

constexpr int kGB = 256;
constexpr int64_t kGChunk = int64_t(kGB) * 4 * 8;  // elements per workgroup item

struct GatherTable {
  uint64_t src[kGatherMaxT];
  int64_t off[kGatherMaxT];
  int32_t n[kGatherMaxT];
  int32_t cstart[kGatherMaxT + 1];  // prefix sum of chunks per tensor
  int32_t nt;
};

template <bool AUX>
__global__ __launch_bounds__(kGB) void gather_scale_kernel(GatherTable tab, float* __restrict__ dst,
                                                           const float* __restrict__ aux, float a, float b) {
  const int nchunks = tab.cstart[tab.nt];
  for (int c = blockIdx.x; c < nchunks; c += gridDim.x) {
    // tensor owning chunk c (uniform binary search over the prefix table)
    int lo = 0, hi = tab.nt - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (tab.cstart[mid] <= c) lo = mid;
      else hi = mid - 1;
    }
    const int t = lo;
    const int64_t begin = int64_t(c - tab.cstart[t]) * kGChunk;
    const int64_t end = min(int64_t(tab.n[t]), begin + kGChunk);
    const float* src = reinterpret_cast<const float*>(tab.src[t]);
    float* d = dst + tab.off[t];
    const float* x = AUX ? aux + tab.off[t] : nullptr;
    const bool vec = ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(d)) & 15) == 0 &&
                     (!AUX || (reinterpret_cast<uintptr_t>(x) & 15) == 0) && (begin & 3) == 0;
    int64_t i = begin;
    if (vec) {
      const int64_t vend = begin + ((end - begin) & ~int64_t(3));
      for (int64_t k = begin + 4 * threadIdx.x; k < vend; k += 4 * kGB) {
        const float4 g = *reinterpret_cast<const float4*>(src + k);
        float4 r = make_float4(a * g.x, a * g.y, a * g.z, a * g.w);
        if constexpr (AUX) {
          const float4 w = *reinterpret_cast<const float4*>(x + k);
          r.x = fmaf(b, w.x, r.x); r.y = fmaf(b, w.y, r.y); r.z = fmaf(b, w.z, r.z); r.w = fmaf(b, w.w, r.w);
        }
        *reinterpret_cast<float4*>(d + k) = r;
      }
      i = vend;
    }
    for (int64_t k = i + threadIdx.x; k < end; k += kGB) {
      float r = a * src[k];
      if constexpr (AUX) r = fmaf(b, x[k], r);
      d[k] = r;
    }
  }
}

}  // namespace

void gather_scale(int dev, hipStream_t s, const std::vector<uintptr_t>& srcs, const std::vector<int64_t>& offs,
                  const std::vector<int64_t>& ns, uintptr_t dst, uintptr_t aux, float a, float b) {
  const size_t T = srcs.size();
  if (offs.size() != T || ns.size() != T) throw std::invalid_argument("gather_scale: table size mismatch");
  if (dev < 0) {
    for (size_t t = 0; t < T; ++t) {
      const float* src = reinterpret_cast<const float*>(srcs[t]);
      float* d = reinterpret_cast<float*>(dst) + offs[t];
      const float* x = aux ? reinterpret_cast<const float*>(aux) + offs[t] : nullptr;
      for (int64_t i = 0; i < ns[t]; ++i) d[i] = a * src[i] + (x ? b * x[i] : 0.f);
    }
    return;
  }
  hip_check(hipSetDevice(dev), "hipSetDevice");
  for (size_t base = 0; base < T; base += kGatherMaxT) {
    GatherTable tab{};
    const int nt = int(std::min<size_t>(kGatherMaxT, T - base));
    tab.nt = nt;
    int32_t c = 0;
    for (int k = 0; k < nt; ++k) {
      if (ns[base + k] > INT32_MAX) throw std::invalid_argument("gather_scale: tensor too large");
      tab.src[k] = srcs[base + k];
      tab.off[k] = offs[base + k];
      tab.n[k] = int32_t(ns[base + k]);
      tab.cstart[k] = c;
      c += int32_t((ns[base + k] + kGChunk - 1) / kGChunk);
    }
    tab.cstart[nt] = c;
    if (c == 0) continue;
    const int grid = std::min(c, 8192);
    if (aux)
      hipLaunchKernelGGL(gather_scale_kernel<true>, dim3(grid), dim3(kGB), 0, s, tab, reinterpret_cast<float*>(dst),
                         reinterpret_cast<const float*>(aux), a, b);
    else
      hipLaunchKernelGGL(gather_scale_kernel<false>, dim3(grid), dim3(kGB), 0, s, tab, reinterpret_cast<float*>(dst),
                         nullptr, a, b);
    hip_check(hipGetLastError(), "gather_scale launch");
  }
}

}  // namespace mpit

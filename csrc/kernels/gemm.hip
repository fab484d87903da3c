// MFMA GEMMs for NHWC 1x1 convolutions (bf16 operands, fp32 accumulate), gfx950.
//
// A stride-1 1x1 convolution over a channels_last activation is a plain GEMM over the
// [M = N*H*W, C] row-major matrix view:
//   forward  Y[M,Co]  = X[M,Ci] . W[Co,Ci]^T        -> gemm_nt  (A = X,  B = W)
//   dgrad    dX[M,Ci] = dY[M,Co] . W[Co,Ci]         -> gemm_nt  (A = dY, B = W^T)
//   wgrad    dW[Co,Ci] = dY[M,Co]^T . X[M,Ci]       -> gemm_tn  (reduction over M, split-K)
// The ResNet-50 shapes are tall and skinny (M up to 802816, Ci/Co 64..2048), so most of
// them are HBM-bound: the kernels below stream A once, keep the weight tile resident in
// LDS/L2, and (forward) can emit the per-channel batch-norm statistics of the output
// from the accumulators, which saves the separate statistics pass over Y.
//
// gemm_nt: C[M,N] = A[M,K] . B[N,K]^T, both operands K-contiguous. 256 threads = 4 waves
// in a 2x2 arrangement; each wave owns a (BM/2)x(BN/2) sub-tile built from 32x32x16 bf16
// MFMAs. Tiles of BK=64 are staged global->VGPR->LDS with 16-byte loads, double buffered
// (one barrier per k-tile; the loads of tile k+1 are in flight during the MFMAs of tile
// k). LDS rows are 128 B with the 16-byte chunk XOR-swizzled by (row>>1)&7, so the
// ds_read_b128 fragment reads of any 16 consecutive rows hit 64 distinct banks. The MFMA
// is issued with the operands swapped (D = B.A^T) so each lane ends up holding 4
// consecutive output channels of one row: the epilogue packs them into 8-byte stores
// without an LDS round trip. Block -> tile mapping is XCD-aware: the blocks that share
// an A row-panel are dispatched to the same XCD so the panel is fetched into one L2.
//
// gemm_tn (wgrad): both operands are M-major, the reduction runs over rows. Tiles of 64
// rows x 128 (or 64) columns are staged row-major in LDS (row stride padded by 64 B) and
// the MFMA fragments (8 consecutive rows of one column) are read with the gfx950
// transposing LDS read ds_read_b64_tr_b16. M is split over blocks; each split writes an
// fp32 partial tile and a vectorised reduce sums the splits (deterministic, no atomics).
//
// RxS convolutions (3x3 in ResNet / VGG / AlexNet) run on the same two kernels as
// implicit GEMMs over an NHWC input (template flag CONV, geometry in ConvGeo): the GEMM
// K index is (tap, channel) with the weight stored [Co][R][S][C] (channels_last), so a
// 32-wide k-tile of gemm_nt (or a TBK-wide column tile of gemm_tn) is one tap and a
// contiguous run of channels of one input pixel. Each lane's LDS DMA source is that
// pixel's row, or a zero line in global memory when the tap falls in the padding — the
// im2col matrix is never materialised. forward = gemm_nt on (X, W); backward-data of a
// stride-1 conv = gemm_nt on (dY, W flipped and transposed); backward-weight = gemm_tn on
// (dY, implicit X) straight into the fp32 master-weight gradient.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <array>
#include <map>
#include <mutex>
#include <vector>
#include <stdexcept>
#include <string>

#include "ew.h"
#include "kernels.h"

namespace mpit {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int kBK = 32;  // k-depth of one staged bf16 tile (gemm_nt): 64-B LDS rows
constexpr int kStemTap = 32;  // row-tap stem: 8 pixels x 4 channels per kernel row

// Element types: uint16_t = bf16 operands on v_mfma_f32_32x32x16_bf16; float = fp32
// operands on v_mfma_f32_32x32x2_f32 (exact fp32 products, fp32 accumulate: the
// reference's fp32 training precision). Staging, LDS images and the epilogue are written
// in bytes / 16-byte chunks, so both share them: a chunk is 8 bf16 or 4 fp32.
template <typename T>
__host__ __device__ constexpr int epc() { return 16 / int(sizeof(T)); }  // elements per 16-B chunk
template <typename T>
__host__ __device__ constexpr int nt_bk_of() { return 64 / int(sizeof(T)); }  // k of one 64-B LDS row

// 8 consecutive elements of T held raw in registers (loads issued ahead of their use)
template <typename T>
struct V8;
template <>
struct V8<uint16_t> {
  uint4 r;
  __device__ __forceinline__ void load(const uint16_t* p, int = 4) { r = *reinterpret_cast<const uint4*>(p); }
  __device__ __forceinline__ void zero() { r = make_uint4(0, 0, 0, 0); }
  __device__ __forceinline__ float get(int e) const {
    const uint32_t w = e < 2 ? r.x : e < 4 ? r.y : e < 6 ? r.z : r.w;
    return bf2f(uint16_t((e & 1) ? (w >> 16) : (w & 0xffff)));
  }
};
template <>
struct V8<float> {
  float4 a, b;
  __device__ __forceinline__ void load(const float* p, int h = 4) {  // elements 4..7 at p + h
    a = *reinterpret_cast<const float4*>(p);
    b = *reinterpret_cast<const float4*>(p + h);
  }
  __device__ __forceinline__ void zero() { a = b = make_float4(0.f, 0.f, 0.f, 0.f); }
  __device__ __forceinline__ float get(int e) const {
    const float4& q = e < 4 ? a : b;
    const int k = e & 3;
    return k == 0 ? q.x : k == 1 ? q.y : k == 2 ? q.z : q.w;
  }
};
__device__ __forceinline__ void store8(uint16_t* p, const float (&v)[8], int = 4) {
  uint4 r;
  r.x = uint32_t(f2bf(v[0])) | (uint32_t(f2bf(v[1])) << 16);
  r.y = uint32_t(f2bf(v[2])) | (uint32_t(f2bf(v[3])) << 16);
  r.z = uint32_t(f2bf(v[4])) | (uint32_t(f2bf(v[5])) << 16);
  r.w = uint32_t(f2bf(v[6])) | (uint32_t(f2bf(v[7])) << 16);
  *reinterpret_cast<uint4*>(p) = r;
}
__device__ __forceinline__ void store8(float* p, const float (&v)[8], int h = 4) {  // elements 4..7 at p + h
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(p + h) = make_float4(v[4], v[5], v[6], v[7]);
}
// value as stored in T (the epilogue's statistics see exactly what is written)
template <typename T>
__device__ __forceinline__ float rnd(float v) {
  if constexpr (sizeof(T) == 2) return bf2f(f2bf(v));
  else return v;
}

// fp32 GEMMs on the bf16 matrix cores ("bf16x6", FM = 1): every fp32 operand is split
// exactly into three bf16 terms, x = h + m + l (round-to-nearest h = bf16(x), m =
// bf16(x - h), l = bf16(x - h - m); for normal numbers the three carry all 24 significant
// bits), and a product is the sum of the six partial products whose order sum is <= 2:
// hh + (hm + mh + mm + hl + lh). The dropped ml, lm, ll are below 2^-25 relative, and
// bf16 x bf16 products are exact in the fp32 accumulators, so the result carries fp32
// accuracy at 6 bf16 MFMAs per product (2.5 PF / 6 = 417 TF peak, against 157 TF for the
// fp32-input MFMA). hh accumulates in its own registers, the five small terms in a second
// set, so the big running sum is rounded once per 16-deep MFMA, not six times.
//
// The split runs on element pairs so every step is one packed instruction: v_cvt_pk_bf16_f32
// rounds two floats into one dword, the rounded pair is unpacked by a shift and a mask, and
// v_pk_add_f32 forms both residuals — 9 VALU per pair (4.5 per element) and the bf16 planes
// come out as whole dwords of the MFMA operand registers (no element inserts).
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t pk_bf16(f32x2 x) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(x, bf16x2));
}
__device__ __forceinline__ f32x2 unpk_bf16(uint32_t u) {
  return f32x2{__builtin_bit_cast(float, u << 16), __builtin_bit_cast(float, u & 0xffff0000u)};
}
__device__ __forceinline__ void split3(const float (&v)[8], bf16x8& h, bf16x8& m, bf16x8& l) {
  u32x4 hu, mu, lu;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const f32x2 x = {v[2 * p], v[2 * p + 1]};
    const uint32_t hp = pk_bf16(x);
    const f32x2 r = x - unpk_bf16(hp);
    const uint32_t mp = pk_bf16(r);
    const f32x2 q = r - unpk_bf16(mp);
    hu[p] = hp;
    mu[p] = mp;
    lu[p] = pk_bf16(q);
  }
  h = __builtin_bit_cast(bf16x8, hu);
  m = __builtin_bit_cast(bf16x8, mu);
  l = __builtin_bit_cast(bf16x8, lu);
}
// fp32 GEMMs on the fp16 matrix cores ("fp16x3", FM = 11): an operand with a power-of-two
// scale 2^e (per tensor, from a device-side upper bound amax of |x|: amax * 2^e in [2^13,
// 2^14), fp16_exp) splits exactly into two fp16 terms, s = x * 2^e = h + l * 2^-11 with h =
// f16(s) (round to nearest: 11 significant bits) and l = f16((s - h) * 2^11) (the next 11).
// s - h and (s - h) * 2^11 are exact in fp32, so x is carried to 22 bits (relative error
// <= 2^-22) wherever s >= 2^-14 (|x| within 2^27 of amax: fp16 normals); smaller values are
// carried to an absolute error below 2^-48 * amax. A product takes three fp16 MFMAs,
// hh into one accumulator and hl + lh into a second (scaled back by 2^-11 once, in the
// epilogue, with the operand scales 2^-(ea + eb)); the dropped ll is < 2^-22 relative — the
// same order as the bf16x6 split's dropped terms, at half its MFMA count (2.5 PF / 3 = 833 TF
// peak). Numerics against fp64: tests/test_fp32_path.py.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
// e with amax * 2^e in [2^13, 2^14) (0 for a zero / non-finite bound), clamped to a normal 2^e
__device__ __forceinline__ int fp16_exp(const float* amax) {
  float a = amax[0];  // the bound: max over its kBoundSlots slots (kernels.h)
#pragma unroll
  for (int k = 1; k < kBoundSlots; ++k) a = fmaxf(a, amax[k * kBoundStride]);
  if (!(a > 0.f) || !(a <= 3.0e38f)) return 0;
  int x;
  (void)frexpf(a, &x);  // a = f * 2^x, f in [0.5, 1)
  return min(116, max(-126, 14 - x));  // 2^(e + 11) stays a normal float
}
__device__ __forceinline__ float exp2i(int e) { return __builtin_bit_cast(float, uint32_t(e + 127) << 23); }
// the lane's 8 fp32 values -> fp16 planes h, l of x * 2^e (s = 2^e, s11 = 2^(e + 11));
// per pair: v_pk_mul x2, v_cvt_pk_f16_f32 x2, v_cvt_f32_f16 x2, v_pk_fma: 7 VALU
__device__ __forceinline__ void split2h(const float (&v)[8], float s, float s11, f16x8& h, f16x8& l) {
  u32x4 hu, lu;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const f32x2 x = {v[2 * p], v[2 * p + 1]};
    const f16x2 hp = __builtin_convertvector(x * s, f16x2);
    const f32x2 hf = __builtin_convertvector(hp, f32x2);
    const f32x2 r = x * s11 - hf * 2048.f;  // 2^11 (x s - h), exact
    hu[p] = __builtin_bit_cast(uint32_t, hp);
    lu[p] = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, f16x2));
  }
  h = __builtin_bit_cast(f16x8, hu);
  l = __builtin_bit_cast(f16x8, lu);
}
// one fp32 value -> (h, l) fp16 bits of v * s (split2h's arithmetic; weight plans)
__device__ __forceinline__ void split1h(float v, float s, float s11, uint16_t& h, uint16_t& l) {
  const _Float16 hh = _Float16(v * s);
  h = __builtin_bit_cast(uint16_t, hh);
  l = __builtin_bit_cast(uint16_t, _Float16(v * s11 - float(hh) * 2048.f));
}

template <int TM, int TN>
__device__ __forceinline__ void mfma_x3(f32x16 (&hi)[TM][TN], f32x16 (&lo)[TM][TN], const bf16x8 (&ah)[TM],
                                        const bf16x8 (&am)[TM], const bf16x8 (&al)[TM], const bf16x8 (&bh)[TN],
                                        const bf16x8 (&bm)[TN], const bf16x8 (&bl)[TN], bool swap) {
  // swap: D = B.A^T (the NT kernel's lane -> row-of-C layout), else D = A.B^T
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const bf16x8 &x0 = swap ? bh[j] : ah[i], &y0 = swap ? ah[i] : bh[j];
      const bf16x8 &x1 = swap ? bm[j] : am[i], &y1 = swap ? am[i] : bm[j];
      const bf16x8 &x2 = swap ? bl[j] : al[i], &y2 = swap ? al[i] : bl[j];
      hi[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x0, y0, hi[i][j], 0, 0, 0);
      lo[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x1, y0, lo[i][j], 0, 0, 0);
      lo[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x0, y1, lo[i][j], 0, 0, 0);
      lo[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x1, y1, lo[i][j], 0, 0, 0);
      lo[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x2, y0, lo[i][j], 0, 0, 0);
      lo[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x0, y2, lo[i][j], 0, 0, 0);
    }
}

// NHWC convolution geometry for the implicit-GEMM (CONV) kernel variants
struct ConvGeo {
  int H, W, C;     // input image
  int Ho, Wo;      // output (GEMM row) grid
  int S;           // kernel width (taps are r*S + s)
  int stride, pad, padw;
  // output row mapping (gemm_nt epilogue): ostr > 1 writes grid pixel (i, j) to pixel
  // (i*ostr + oph, j*ostr + opw) of an OH x OW image (one parity class of a strided conv's
  // backward-data); ozero also writes zeros to the other three parities (stride 2 only)
  int ostr, oph, opw, OH, OW, ozero;
  // elements per input pixel when a tap is not one pixel's channels (0: C). The "row tap"
  // stem conv (conv_stem_*) reads C = 32 contiguous elements = 8 pixels of 4 channels per
  // kernel row: a 7x7 / 3-channel stem as an 8-row implicit GEMM over a padded NHWC4 image
  int pitch;
};

enum { EPI_NONE = 0, EPI_STATS = 1, EPI_BNRED = 2, EPI_BNRED2 = 3, EPI_RELUB = 4 };

// column-reduction epilogue operands (see gemm_nt_kernel)
struct EpiArgs {
  float* part;                 // [row0 + tiles][2][N] fp32 partials
  const void* x;               // EPI_BNRED: the BN's input (element type of C), laid out like C (ldc == N)
  const uint8_t* mask;         // EPI_BNRED: the BN's ReLU bit mask (1 byte / 8 channels) or null
  const float* mean;           // EPI_BNRED: the BN's batch mean [N]
  int64_t row0;                // first partial row of this launch
  float* part2;                // EPI_BNRED2: the second BN of a bn_pair (same gradient and mask)
  const void* x2;
  const float* mean2;
  // EPI_BNRED fold (fcoef != null): the BN backward's finalize runs in this GEMM's last
  // blocks (see the end of gemm_nt_kernel's epilogue) instead of a separate launch
  const float* fgamma;         // BN weight [N] or null (1)
  const float* frstd;          // BN 1/std [N]
  float* fdgamma;              // outputs [N] (or null)
  float* fdbeta;
  float* fcoef;                // [3][N] the BN backward's apply coefficients
  float* flvl;                 // [groups][2][N] group sums
  uint32_t* ftick;             // this launch's tickets [ntn][groups + 1]
  int fgroup;                  // M-tiles per group
  float* fzero;                // set to 0 by the finalizing block of column tile 0 (or null)
  // fp16x3 (FM 11): device upper bounds of |A| and |B| that set the operand scales
  const float* amax_a;
  const float* amax_b;
  // FM 13 (fp16x3, A planes): A is two fp16 planes h, l of A * 2^ea (ea from amax_a), the
  // l plane aps elements after the h plane — written by A's producer (the BN apply passes),
  // so the kernel splits nothing
  int64_t aps;
  // max |C| of this launch (the input of the BN that writes fp16 planes from it, planes.h):
  // one 64-bit (epoch, value bits) atomic max per block into slot blockIdx % kBoundSlots of
  // omax; a slot of an older launch (smaller epoch) is replaced, so the buffer is never zeroed
  unsigned long long* omax;
  uint32_t oepoch;
  // EPI_STATS fold (scoef != null): the BN forward's finalize runs in this GEMM's last
  // blocks (stats_fold): the statistics of the output become the BN's scale / shift
  // [2][N], save_mean / save_rstd and running-statistics update; flvl ([groups][3][N]),
  // ftick, fgroup and fzero as for the backward fold
  float* scoef;
  const float* sgamma;
  const float* sbeta;
  float* srmean;
  float* srvar;
  float* smean;
  float* srstd;
  float seps, smom;
  // tagged fold protocol (fepoch != 0, both folds): the fold ticket is taken before the
  // block's output stores and every partial value is written as one 8-byte (value, epoch)
  // store; the folding block spins on the epochs instead of every block draining its own
  // output stores before its ticket (see stats_fold)
  uint32_t fepoch;
};

// write-through (sc1) store: visible to a reader on any XCD without an L2 write-back
__device__ __forceinline__ void st_wt(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// tagged partials: element i of a [rows][2][N] table of (value, epoch) pairs
__device__ __forceinline__ void st_tag(float* part, int64_t i, float v, uint32_t epoch) {
  __hip_atomic_store(reinterpret_cast<uint64_t*>(part) + i, (uint64_t(epoch) << 32) | __float_as_uint(v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the value once its writer's epoch is visible. The writer took its ticket before the folding
// block took the last one and stores the pair right after its output rows, so the wait is
// short; it is bounded (~1 s) so that a protocol error shows as wrong statistics, not a hang.
__device__ __forceinline__ float ld_tag(const float* part, int64_t i, uint32_t epoch) {
  const uint64_t* p = reinterpret_cast<const uint64_t*>(part) + i;
  uint64_t v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (int spin = 0; uint32_t(v >> 32) != epoch && spin < (1 << 20); ++spin) {
    __builtin_amdgcn_s_sleep(2);
    v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return __uint_as_float(uint32_t(v));
}

// source line for padding taps: LDS DMA of zeros (any chunk of a 256-B row, either type)
__device__ __attribute__((aligned(256))) uint16_t g_zero_line[256] = {};

// 16-B chunk swizzle of a 64-B LDS row: any 16 consecutive rows read at one logical chunk
// hit 16 distinct (row%4, chunk) bank groups = all 64 banks.
__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 2) & 3); }
// the same for 128-B rows (8 chunks): 16 rows at one logical chunk hit 16 distinct
// (row%2, chunk) bank groups. BKB = bytes per LDS row.
template <int BKB>
__device__ __forceinline__ int swzk(int row, int chunk) {
  if constexpr (BKB == 64) return swz(row, chunk);
  else return chunk ^ ((row >> 1) & 7);
}

// bytes of one staged row of gemm_nt: the 256x256 tile (1 block/CU) stages 128-B rows
// (64 bf16: 16 MFMAs per wave between fragment refills, half the barriers per FLOP)
// fp32 bf16x6 with FM = 3 stages 32-deep k-tiles (128-B rows of 32 floats: two k16 MFMA steps
// per barrier) instead of FM = 1's 16-deep ones.
__host__ __device__ constexpr int nt_bkb(int BM, int BN, int FM = 0) {
  return (BM == 256 && BN == 256) || FM == 3 || FM == 4 || FM >= 5 ? 128 : 64;
}

typedef __attribute__((address_space(3))) void lds_void;

// 16-byte global -> LDS DMA; the LDS address must be wave-uniform (lane data lands at
// lds + 16*lane).
__device__ __forceinline__ void glds16(const void* src, void* lds) {
  __builtin_amdgcn_global_load_lds(src, (lds_void*)lds, 16, 0, 0);
}

// ds_read_b64_tr_b16 (T10): lane 4q+p of each 16-lane group addresses row q, columns
// 4p..4p+3 of a 4x16 block; lane i receives column i.
__device__ __forceinline__ s16x4 ds_tr16(const uint16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p);
}

// The same LDS DMA issued from inline asm. hipcc treats a builtin LDS DMA as aliasing
// every later ds_read_b64_tr_b16 and drains it (vmcnt(0)) before each transposed read,
// which serialises the ring; issued from asm it is invisible to that tracking and the
// kernel's own counted vmcnt waits order it. m0 carries the wave-uniform LDS base; no
// other instruction of the kernels using this helper reads m0.
// (s_nop 0: an SALU write of M0 needs one wait state before an LDS DMA reads it)
__device__ __forceinline__ void glds16_asm(const void* src, void* lds) {
  const uint32_t l = __builtin_amdgcn_readfirstlane(uint32_t(reinterpret_cast<uintptr_t>((lds_void*)lds)));
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(l), "v"(src) : "memory", "m0");
}

// The same DMA through a buffer descriptor: 16 B per lane from (descriptor base + voff) to
// LDS byte address lds + 16 * lane. The descriptor is raw (stride 0) with num_records =
// 2^31, so a lane offset >= 2^31 is out of range and DMAs zeros (padding taps). The base
// and the LDS address are wave-uniform SGPR values built by SALU arithmetic.
typedef int i32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kBufOob = 0x80000000u;
__device__ __forceinline__ i32x4 buf_rsrc(uint64_t base, uint32_t nrec = kBufOob) {
  return i32x4{int(uint32_t(base)), int(uint32_t(base >> 32) & 0xffffu), int(nrec), 0x00020000};
}
__device__ __forceinline__ void blds16(i32x4 rsrc, uint32_t voff, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rsrc),
               "s"(lds)
               : "memory", "m0");
}
// For descriptors the compiler cannot prove wave-uniform (gemm_nt's bf16 256 x 256 tiles):
// each word through v_readfirstlane (a no-op for SGPR values), and the 5 wait states a VALU
// write of an SGPR needs before a VMEM instruction reads it
__device__ __forceinline__ void blds16u(i32x4 rsrc, uint32_t voff, uint32_t lds) {
  const i32x4 r = {__builtin_amdgcn_readfirstlane(rsrc[0]), __builtin_amdgcn_readfirstlane(rsrc[1]),
                   __builtin_amdgcn_readfirstlane(rsrc[2]), __builtin_amdgcn_readfirstlane(rsrc[3])};
  const uint32_t l = __builtin_amdgcn_readfirstlane(lds);
  asm volatile("s_nop 4\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff),
               "s"(r), "s"(l)
               : "memory", "m0");
}
// FM 13 wave grid: 4 x 1 (FM 11's, where it made one wave split each A row) or, built with
// -DMPIT_FM13_W22 (A/B variant), 2 x 2: with both operands ready-made a 64 x 64 wave reads 8
// fragments per 12 MFMAs instead of 10
#ifdef MPIT_FM13_W22
constexpr bool kFm13W22 = true;
#else
constexpr bool kFm13W22 = false;
#endif
#ifdef MPIT_FM13_PF
constexpr bool kFm13Pf = true;
#else
constexpr bool kFm13Pf = false;
#endif
// MPIT_GLOBAL_DMA (build define, A/B only): gemm_nt's bf16 and fp16x3 kernels and gemm_tn
// stage through per-lane 64-bit global addresses as before round 5 instead of the buffer
// descriptors; MPIT_F11_GLOBAL_DMA only the fp16x3 gemm_nt ones
#if defined(MPIT_GLOBAL_DMA) || defined(MPIT_F11_GLOBAL_DMA)
constexpr bool kF11Buf = false;
#else
constexpr bool kF11Buf = true;
#endif
#ifdef MPIT_GLOBAL_DMA
constexpr bool kBf16Buf = false, kTnBuf = false;
#else
constexpr bool kBf16Buf = true, kTnBuf = true;
#endif

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Workgroup barrier for an LDS hand-off only: this wave's LDS operations complete, then the
// barrier. __syncthreads()'s workgroup fence also waits vmcnt(0) — every global store the
// wave has issued must retire first — which in an epilogue that has just stored its output
// tile stalls the whole block for a write round trip before it can reduce and exit.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Map a linear block id to a tile id so that consecutive tile ids (which share the A
// row-panel, or the rows of a wgrad split) land on one XCD: blocks are dispatched
// round-robin over the 8 XCDs, so XCD x runs blocks x, x+8, ...; it is given the x-th
// contiguous range of tile ids (ranges differ in length by one when nb % 8 != 0).
__device__ __forceinline__ int xcd_tile(int bid, int nb) {
  const int x = bid % 8, q = nb / 8, r = nb % 8;
  return x * q + min(x, r) + bid / 8;
}

// BN backward finalize folded into the EPI_BNRED GEMM (replaces the separate
// bn_tiles_finalize launch, which in the backward waits for CU slots behind the side
// stream's weight-gradient GEMMs): tickets per (column tile, group of fgroup M-tiles) —
// the group's last block sums the group's partial rows (fp64, row order) into flvl; the
// last group-folder of the column tile sums the groups in group order and writes dgamma,
// dbeta and the apply coefficients (bn_act.hip fin_bwd_channel's math). Deterministic; the
// hand-off is bn_tiles_finalize_kernel's: write-through stores, s_waitcnt, barrier, one
// agent-scope ticket add per workgroup, agent acquire in the consumer.
constexpr int kFoldSlots = 32;  // kFoldStreams groups of kFoldPerStream ticket sets
constexpr int kFoldPerStream = 4;
constexpr int kFoldStreams = kFoldSlots / kFoldPerStream;
constexpr int kFoldMax = 8192;
constexpr int kFoldMaxGroups = 128;
__device__ uint32_t g_fold_tickets[kFoldSlots * kFoldMax];

// The fold's row loops read one value per row and lane; issued one dependent load at a time
// they are latency-bound (~1 us each: a folding block held its CU slot for ~100 us, and the
// level-2 fold is the GEMM's tail). ld_batch issues NB loads (n of them valid) before using
// any; the callers add the values in the original row order, so the sums are bitwise the
// one-at-a-time ones. epoch != 0: tagged pairs (ld_tag's spin only for a pair not yet there).
template <int NB>
__device__ __forceinline__ void ld_batch(const float* part, const int64_t (&idx)[NB], int n, float (&out)[NB],
                                         uint32_t epoch) {
  if (epoch) {
    uint64_t raw[NB];
#pragma unroll
    for (int u = 0; u < NB; ++u)
      if (u < n)
        raw[u] = __hip_atomic_load(reinterpret_cast<const uint64_t*>(part) + idx[u], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int u = 0; u < NB; ++u)
      if (u < n)
        out[u] = uint32_t(raw[u] >> 32) == epoch ? __uint_as_float(uint32_t(raw[u])) : ld_tag(part, idx[u], epoch);
  } else {
#pragma unroll
    for (int u = 0; u < NB; ++u)
      if (u < n) out[u] = part[idx[u]];
  }
}

// this block's level-1 fold ticket: per (column tile, group of fgroup M-tiles)
template <int HALVES>
__device__ __forceinline__ uint32_t* fold_ticket(const EpiArgs& ep, int64_t M, int mt, int nt) {
  const int64_t mtn = (M + HALVES * 128 - 1) / (HALVES * 128);
  const int ngr = int((mtn + ep.fgroup - 1) / ep.fgroup);
  return ep.ftick + size_t(nt) * size_t(ngr + 1) + mt / ep.fgroup;
}

template <int BN, int HALVES>
__device__ __forceinline__ void bnred_fold(const EpiArgs& ep, void* smem, int64_t M, int N, int mt, int nt, int n0,
                                           uint32_t ftk) {
  constexpr int NT = 256, L = NT / BN;  // lanes per column
  const int t = threadIdx.x, cl = t % BN, kl = t / BN;
  const int64_t mtn = (M + HALVES * 128 - 1) / (HALVES * 128);
  const int fg = ep.fgroup;
  const int ngr = int((mtn + fg - 1) / fg);
  const int grp = mt / fg;
  const int gsz = int(min<int64_t>(fg, mtn - int64_t(grp) * fg));
  uint32_t* tk = ep.ftick + size_t(nt) * size_t(ngr + 1);
  uint32_t* flag = reinterpret_cast<uint32_t*>(smem);
  double* sd = reinterpret_cast<double*>(smem) + 2;  // [2][L][BN]
  const uint32_t ep_tag = ep.fepoch;
  if (ep_tag) {  // tagged: the ticket was taken before the output stores (ftk, block-uniform)
    if (ftk != uint32_t(gsz - 1)) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    __syncthreads();  // (LDS: phase B's reduction table is read; sd reuses it)
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // every partial store of this block issued and retired; LDS reads done
    if (t == 0) flag[0] = atomicAdd(&tk[grp], 1u);
    __syncthreads();
    if (flag[0] != uint32_t(gsz - 1)) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  const int64_t nparts = (M + 127) / 128;
  const int64_t r0 = int64_t(grp) * fg * HALVES, r1 = min(nparts, r0 + int64_t(gsz) * HALVES);
  double a = 0, b = 0;
  for (int64_t rb = r0 + kl; rb < r1; rb += 8 * L) {
    const int n = int(min<int64_t>(8, (r1 - rb + L - 1) / L));
    int64_t ix[16];
    float v[16];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      ix[2 * u] = ((rb + u * L) * 2) * N + n0 + cl;
      ix[2 * u + 1] = ix[2 * u] + N;
    }
    ld_batch<16>(ep.part, ix, 2 * n, v, ep_tag);
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (u < n) {
        a += double(v[2 * u]);
        b += double(v[2 * u + 1]);
      }
  }
  sd[kl * BN + cl] = a;
  sd[(L + kl) * BN + cl] = b;
  __syncthreads();
  if (kl == 0) {
#pragma unroll
    for (int k = 1; k < L; ++k) {
      a += sd[k * BN + cl];
      b += sd[(L + k) * BN + cl];
    }
    st_wt(ep.flvl + (int64_t(grp) * 2) * N + n0 + cl, float(a));
    st_wt(ep.flvl + (int64_t(grp) * 2 + 1) * N + n0 + cl, float(b));
  }
  if (t == 0) __hip_atomic_store(&tk[grp], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) flag[0] = atomicAdd(&tk[ngr], 1u);
  __syncthreads();
  if (flag[0] != uint32_t(ngr - 1)) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  a = b = 0;
  for (int gb = kl; gb < ngr; gb += 8 * L) {
    const int n = min(8, (ngr - gb + L - 1) / L);
    int64_t ix[16];
    float v[16];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      ix[2 * u] = (int64_t(gb + u * L) * 2) * N + n0 + cl;
      ix[2 * u + 1] = ix[2 * u] + N;
    }
    ld_batch<16>(ep.flvl, ix, 2 * n, v, 0u);
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (u < n) {
        a += double(v[2 * u]);
        b += double(v[2 * u + 1]);
      }
  }
  sd[kl * BN + cl] = a;
  sd[(L + kl) * BN + cl] = b;
  __syncthreads();
  if (t == 0) __hip_atomic_store(&tk[ngr], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (t < kBoundSlots && nt == 0 && ep.fzero) ep.fzero[t * kBoundStride] = 0.f;
  if (kl != 0) return;
  a = b = 0;
#pragma unroll
  for (int k = 0; k < L; ++k) {  // lane order, as the finalize kernel's LDS combine
    a += sd[k * BN + cl];
    b += sd[(L + k) * BN + cl];
  }
  const int c = n0 + cl;
  const float rs = ep.frstd[c];
  if (ep.fdgamma) ep.fdgamma[c] = float(b) * rs;
  if (ep.fdbeta) ep.fdbeta[c] = float(a);
  const float A = (ep.fgamma ? ep.fgamma[c] : 1.f) * rs;
  const float mdz = float(a / double(M)), mdx = float(b / double(M));
  const float Cc = -A * rs * rs * mdx;
  ep.fcoef[c] = A;
  ep.fcoef[N + c] = Cc;
  ep.fcoef[2 * N + c] = -A * mdz - Cc * ep.mean[c];
}

// BN forward finalize folded into the EPI_STATS GEMM (replaces the bn_tiles_finalize launch
// of the BN forward, bn_act.hip): the partial rows hold (mean_k, M2_k) of n_k = min(128,
// M - 128k) rows. Level 1: the last block of a group of fgroup M-tiles (ticket) merges the
// group's rows in fp64, shifted by the group's first row mean, into (mean_g as a float pair,
// M2_g) in flvl[g][3][N]; level 2: the last group-folder of the column tile merges the groups
// shifted by mean_0 (the first tile's mean) and writes what the finalize wrote: scale / shift,
// save_mean / save_rstd, the running statistics (unbiased variance, momentum), and zeroes
// the BN output's fp16x3 bound. Deterministic (fixed orders); the hand-off is bnred_fold's.
template <int BN, int HALVES>
__device__ __forceinline__ void stats_fold(const EpiArgs& ep, void* smem, int64_t M, int N, int mt, int nt, int n0,
                                           uint32_t ftk) {
  constexpr int NT = 256, L = NT / BN;
  const int t = threadIdx.x, cl = t % BN, kl = t / BN;
  const int64_t mtn = (M + HALVES * 128 - 1) / (HALVES * 128);
  const int fg = ep.fgroup;
  const int ngr = int((mtn + fg - 1) / fg);
  const int grp = mt / fg;
  const int gsz = int(min<int64_t>(fg, mtn - int64_t(grp) * fg));
  uint32_t* tk = ep.ftick + size_t(nt) * size_t(ngr + 1);
  uint32_t* flag = reinterpret_cast<uint32_t*>(smem);
  double* sd = reinterpret_cast<double*>(smem) + 2;  // [3][L][BN]
  const uint32_t ep_tag = ep.fepoch;
  if (ep_tag) {  // tagged: the ticket was taken before the output stores (ftk, block-uniform)
    if (ftk != uint32_t(gsz - 1)) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    __syncthreads();  // (LDS: phase B's reduction table is read; sd reuses it)
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // every partial store of this block issued and retired; LDS reads done
    if (t == 0) flag[0] = atomicAdd(&tk[grp], 1u);
    __syncthreads();
    if (flag[0] != uint32_t(gsz - 1)) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  auto pv = [&](int64_t i) -> double {
    return ep_tag ? double(ld_tag(ep.part, i, ep_tag)) : double(ep.part[i]);
  };
  const int64_t nparts = (M + 127) / 128;
  const int64_t r0 = int64_t(grp) * fg * HALVES, r1 = min(nparts, r0 + int64_t(gsz) * HALVES);
  const int c = n0 + cl;
  const double kg = pv((r0 * 2) * N + c);  // the group's shift: its first row's mean
  double a = 0, b = 0;
  for (int64_t rb = r0 + kl; rb < r1; rb += 8 * L) {
    const int n = int(min<int64_t>(8, (r1 - rb + L - 1) / L));
    int64_t ix[16];
    float v[16];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      ix[2 * u] = ((rb + u * L) * 2) * N + c;
      ix[2 * u + 1] = ix[2 * u] + N;
    }
    ld_batch<16>(ep.part, ix, 2 * n, v, ep_tag);
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (u < n) {
        const int64_t r = rb + u * L;
        const double nk = double(min<int64_t>(128, M - r * 128));
        const double d = double(v[2 * u]) - kg;
        a = fma(nk, d, a);
        b += double(v[2 * u + 1]) + nk * d * d;
      }
  }
  sd[kl * BN + cl] = a;
  sd[(L + kl) * BN + cl] = b;
  __syncthreads();
  if (kl == 0) {
#pragma unroll
    for (int k = 1; k < L; ++k) {
      a += sd[k * BN + cl];
      b += sd[(L + k) * BN + cl];
    }
    const double ng = double(min<int64_t>(M, r1 * 128) - r0 * 128);
    const double mg = kg + a / ng;
    const float mh = float(mg);
    st_wt(ep.flvl + (int64_t(grp) * 3) * N + c, mh);
    st_wt(ep.flvl + (int64_t(grp) * 3 + 1) * N + c, float(mg - double(mh)));
    st_wt(ep.flvl + (int64_t(grp) * 3 + 2) * N + c, float(fmax(b - a * a / ng, 0.0)));
  }
  if (t == 0) __hip_atomic_store(&tk[grp], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) flag[0] = atomicAdd(&tk[ngr], 1u);
  __syncthreads();
  if (flag[0] != uint32_t(ngr - 1)) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const double k0 = pv(c);  // tile 0's mean
  a = b = 0;
  for (int gb = kl; gb < ngr; gb += 8 * L) {
    const int n = min(8, (ngr - gb + L - 1) / L);
    int64_t ix[24];
    float v[24];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      ix[3 * u] = (int64_t(gb + u * L) * 3) * N + c;
      ix[3 * u + 1] = ix[3 * u] + N;
      ix[3 * u + 2] = ix[3 * u] + 2 * N;
    }
    ld_batch<24>(ep.flvl, ix, 3 * n, v, 0u);
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (u < n) {
        const int g = gb + u * L;
        const int64_t g0 = int64_t(g) * fg * HALVES, g1 = min(nparts, g0 + int64_t(fg) * HALVES);
        const double ng = double(min<int64_t>(M, g1 * 128) - g0 * 128);
        const double d = double(v[3 * u]) + double(v[3 * u + 1]) - k0;
        a = fma(ng, d, a);
        b += double(v[3 * u + 2]) + ng * d * d;
      }
  }
  sd[kl * BN + cl] = a;
  sd[(L + kl) * BN + cl] = b;
  __syncthreads();
  if (t == 0) __hip_atomic_store(&tk[ngr], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (t < kBoundSlots && nt == 0 && ep.fzero) ep.fzero[t * kBoundStride] = 0.f;
  if (kl != 0) return;
  a = b = 0;
#pragma unroll
  for (int k = 0; k < L; ++k) {  // lane order
    a += sd[k * BN + cl];
    b += sd[(L + k) * BN + cl];
  }
  // bn_act.hip fin_fwd_channel's math with the shift k0
  const double md = a / double(M);
  double var = b / double(M) - md * md;
  if (var < 0) var = 0;
  const double mean = k0 + md;
  const float rstd = float(1.0 / sqrt(var + double(ep.seps)));
  const float sc = (ep.sgamma ? ep.sgamma[c] : 1.f) * rstd;
  ep.scoef[c] = sc;
  ep.scoef[N + c] = (ep.sbeta ? ep.sbeta[c] : 0.f) - float(mean) * sc;
  ep.smean[c] = float(mean);
  ep.srstd[c] = rstd;
  const float mom = ep.smom;
  if (ep.srmean) ep.srmean[c] = (1.f - mom) * ep.srmean[c] + mom * float(mean);
  if (ep.srvar) ep.srvar[c] = (1.f - mom) * ep.srvar[c] + mom * float(var * double(M) / double(M > 1 ? M - 1 : 1));
}

// ------------------------------------------------------------------------------ NT GEMM
// Column-reduction epilogues (EPI), one fp32 partial row pair per 128-row M-tile written to
// ep.part[ep.row0 + mt][2][N] (deterministic, no atomics; reduced by the consumer):
//   EPI_STATS  forward batch-norm statistics of the output: (mean, M2) of the tile's rows
//              per column (Chan form: each 64-row half is summed shifted by its own first
//              row, the halves are merged exactly), so no E[y^2]-E[y]^2 cancellation;
//   EPI_BNRED  backward batch-norm reduction for the BN whose OUTPUT gradient this GEMM
//              produces (a convolution's backward-data): dz = round(C) * relu_mask,
//              (sum dz, sum dz*(x - mean)) per column with x the BN's input — the separate
//              reduction pass over (dz, x) of the BN backward disappears.
// The epilogue stages the bf16 tile in LDS and runs row-major (see phase B), so every
// global access of a wave covers whole row segments; the column partials of the rows a
// thread walks are combined through LDS.
//
// Waves: 2 x 2, each owning a BM/2 x BN/2 sub-tile. 128x128 (64x64 per wave, 4 MFMAs per
// k16 step, up to 5 resident blocks per CU) for the memory-bound short-K GEMMs; 256x128 and
// 256x256 (128x64 / 128x128 per wave: 8 / 16 MFMAs per k16 between barriers, half the LDS
// fragment reads per MFMA, 2 / 1 blocks per CU) for the compute-bound deep-K ones — the
// shape of tile the library GEMMs run at ~1 PFLOP/s on these problems (see launch_nt).
//
// Staging: global_load_lds (16-B LDS DMA, no VGPRs) into a ring of STAGES buffers with
// STAGES-1 k-tiles in flight; a counted s_waitcnt vmcnt + raw s_barrier retires exactly
// the tile about to be used (a __syncthreads() would drain the whole ring). The LDS image
// is lane-linear per wave instruction (16 rows x 64 B); the swizzle is applied on the
// global source address.
template <typename T, int BM, int BN, int STAGES, int EPI, bool CONV, int FM = 0>
__global__ __launch_bounds__(256, sizeof(T) == 4 ? (BM == 256 ? (BN == 64 ? 2 : 1) : (BN == 64 ? 3 : 2)) : (BM == 256 ? (BN == 256 ? 1 : 2) : (STAGES == 2 ? (CONV || EPI == 3 ? 4 : 5) : 2))) void gemm_nt_kernel(const T* __restrict__ A, int64_t lda,
                                                         const T* __restrict__ B, int64_t ldb,
                                                         T* C, int64_t ldc, int64_t M, int N, int K,
                                                         int ntn, EpiArgs ep, const T* Cin,
                                                         const uint8_t* __restrict__ Cmask,
                                                         const float* __restrict__ bias, int relu, ConvGeo geo,
                                                         int64_t bps) {
  constexpr int NW = 4, NT = NW * 64;  // waves, threads
  // wave grid over the tile: 2 x 2 (each wave 64 x 64 of a 128 x 128 tile), or for FM 9
  // (pre-split B) 4 x 1: each wave owns 32 rows x all 128 columns, so every A row is split in
  // registers by exactly one wave (the ready-made B planes are the shared operand)
  constexpr int WGM = (sizeof(T) == 4 && (FM == 9 || FM == 10 || FM == 11 || (FM == 13 && !kFm13W22))) ? 4 : 2,
                WGN = NW / WGM;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int EPC = epc<T>();                          // elements per 16-B chunk
  constexpr int BKB = nt_bkb(BM, BN, FM), BK = BKB / int(sizeof(T));
  constexpr int CPK = BKB / 16, RPI = 64 / CPK;          // 16-B chunks per row, rows per glds
  constexpr int IA = BM / RPI / NW, IB = BN / RPI / NW;  // glds instructions per wave per tile
  constexpr bool F32 = sizeof(T) == 4;
  // FM 4 (fp32, B pre-split): B arrives as three bf16 planes (h, m, l; plane stride bps
  // elements, made once per step by the weight plan), staged as three 64-B-row images of
  // 32 bf16 per row — the A operand alone is split in registers
  // FM 11 (fp32, fp16x3): B arrives as two fp16 planes (h, l) of the scaled weight, staged the
  // same way (two 64-B-row images); A is scaled and split in registers (split2h)
  constexpr bool BSPLIT = F32 && (FM == 4 || FM == 9 || FM == 10 || FM == 11 || FM == 13);
  constexpr int NPL = FM == 11 || FM == 13 ? 2 : 3;  // B planes
  constexpr int IBP = BSPLIT ? BN / 16 / NW : 0;  // glds per wave per B plane (16 rows x 64 B)
  // FM 13: A arrives as two fp16 planes too (h, l of A * 2^ea; plane stride ep.aps), staged
  // like B's (two 64-B-row images of 32 halves per row): nothing is split in the kernel
  constexpr bool ASPLIT = F32 && FM == 13;
  constexpr int IAP = ASPLIT ? BM / 16 / NW : 0;  // glds per wave per A plane
  static_assert(!ASPLIT || (IAP >= 1 && kF11Buf), "FM 13 stages A planes through buffer descriptors");
  constexpr int NI = BSPLIT ? (ASPLIT ? 2 * IAP : IA) + NPL * IBP : IA + IB;
  // elements (T) per stage: A rows, then B (fp32 rows, or NPL 16-bit plane images)
  constexpr int BTILE = BSPLIT ? NPL * BN * 32 / 2 : BN * BK;
  constexpr int TILE = BM * BK + BTILE;
  static_assert(IA >= 1 && IB >= 1, "tile too small");
  static_assert(!F32 || BKB == 64 || FM == 3 || FM == 4 || FM >= 5, "fp32 tiles stage 64-B rows (FM 3: 128-B)");
  extern __shared__ __attribute__((aligned(16))) uint16_t smem_raw[];
  T* smem = reinterpret_cast<T*>(smem_raw);
  const T* zline = reinterpret_cast<const T*>(g_zero_line);

  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int mt = tile / ntn, nt = tile % ntn;
  const int64_t m0 = int64_t(mt) * BM;
  const int n0 = nt * BN;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wm = w / WGN, wn = w % WGN;

  // source of this lane for each of the wave's glds instructions (k offset added per tile);
  // CONV: the output pixel of the row (first input pixel of its window) instead
  const T* pa[IA];
  const T* pb[IB];
  constexpr int NAR = ASPLIT ? IAP : IA;  // per-lane A row sources
  int hi0[NAR], wi0[NAR], ca[NAR], img[NAR];
#pragma unroll
  for (int i = 0; i < NAR; ++i) {
    // (FM 13: a plane row is 64 B = 4 chunks of 8 halves, 16 rows per wave instruction)
    const int row = ASPLIT ? (w * IAP + i) * 16 + lane / 4 : (w * IA + i) * RPI + lane / CPK;
    const int c = ASPLIT ? swz(row, lane % 4) : swzk<BKB>(row, lane % CPK);
    const int64_t gm = min(m0 + row, M - 1);  // clamp: tail rows compute garbage, never stored
    if constexpr (CONV) {
      const int hw = geo.Ho * geo.Wo;
      const int64_t n = gm / hw;
      const int rem = int(gm - n * hw), ho = rem / geo.Wo, wo = rem - ho * geo.Wo;
      hi0[i] = ho * geo.stride - geo.pad;
      wi0[i] = wo * geo.stride - geo.padw;
      img[i] = int(n) * geo.H;
      ca[i] = c * (ASPLIT ? 8 : EPC);
    } else if constexpr (!ASPLIT) {
      pa[i] = A + gm * lda + c * EPC;
    }
  }
  int kc = 0, kr = 0, ks = 0;  // CONV: channel offset and tap of the next tile issued
  const int pitch = geo.pitch ? geo.pitch : geo.C;
#pragma unroll
  for (int i = 0; i < IB; ++i) {
    const int row = (w * IB + i) * RPI + lane / CPK, c = swzk<BKB>(row, lane % CPK);
    pb[i] = B + int64_t(n0 + row) * ldb + c * EPC;
  }
  const uint16_t* pbp[BSPLIT ? IBP : 1];
  if constexpr (BSPLIT) {
    const uint16_t* Bh = reinterpret_cast<const uint16_t*>(B);
#pragma unroll
    for (int i = 0; i < IBP; ++i) {
      const int row = (w * IBP + i) * 16 + lane / 4, c = swz(row, lane % 4);
      pbp[i] = Bh + int64_t(n0 + row) * ldb + c * 8;
    }
  }
  // bf16 and FM 11 staging through buffer descriptors (blds16): each lane keeps 32-bit byte
  // offsets from block-uniform bases — A: the block's first row (plain) or first image (CONV,
  // offsets re-made once per tap, out-of-range for padding taps); B: the block's first
  // column row (of each plane) — and a tile's k offset moves the descriptor base (SALU), so
  // issuing a tile costs no per-lane 64-bit address arithmetic, no padding branches and no
  // readfirstlane of the LDS address. The host checks that every offset stays below 2^31.
  constexpr bool F11B = (F32 && (FM == 11 || FM == 13) && kF11Buf) || (!F32 && FM == 0 && kBf16Buf);
  constexpr int NVB = BSPLIT ? IBP : IB;
  [[maybe_unused]] uint32_t voa[F11B ? NAR : 1], vob[F11B ? NVB : 1];
  constexpr int AES = ASPLIT ? 2 : int(sizeof(T));  // bytes per A element in global memory
  [[maybe_unused]] uint64_t abase = 0, bbase = 0;
  [[maybe_unused]] uint32_t lds0 = 0;
  [[maybe_unused]] int ih0 = 0;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  if constexpr (F11B) {
    lds0 = __builtin_amdgcn_readfirstlane(uint32_t(reinterpret_cast<uintptr_t>((lds_void*)smem)));
    if constexpr (CONV) {
      const int64_t img0 = m0 / (int64_t(geo.Ho) * geo.Wo);
      ih0 = int(img0) * geo.H;
      abase = reinterpret_cast<uint64_t>(A) + uint64_t(img0 * geo.H * geo.W) * uint64_t(pitch) * uint64_t(AES);
    } else {
      abase = reinterpret_cast<uint64_t>(A) + uint64_t(m0) * uint64_t(lda) * uint64_t(AES);
#pragma unroll
      for (int i = 0; i < NAR; ++i) {
        const int row = ASPLIT ? (w * IAP + i) * 16 + lane / 4 : (w * IA + i) * RPI + lane / CPK;
        const int c = ASPLIT ? swz(row, lane % 4) : swzk<BKB>(row, lane % CPK);
        const int64_t gm = min(m0 + row, M - 1);
        voa[i] = uint32_t(((gm - m0) * lda + c * (ASPLIT ? 8 : EPC)) * AES);
      }
    }
    bbase = reinterpret_cast<uint64_t>(B) + uint64_t(n0) * uint64_t(ldb) * (BSPLIT ? 2u : sizeof(T));
    if constexpr (BSPLIT) {
#pragma unroll
      for (int i = 0; i < IBP; ++i) {
        const int row = (w * IBP + i) * 16 + lane / 4, c = swz(row, lane % 4);
        vob[i] = uint32_t((row * ldb + c * 8) * 2);
      }
    } else {
#pragma unroll
      for (int i = 0; i < IB; ++i) {
        const int row = (w * IB + i) * RPI + lane / CPK, c = swzk<BKB>(row, lane % CPK);
        vob[i] = uint32_t((row * ldb + c * EPC) * int(sizeof(T)));
      }
    }
  }
  // fp32 tiles issue their LDS DMA from inline asm: with the builtin, hipcc cannot tell
  // that the next stage's DMA targets the other ring buffer and drains it (vmcnt(0)) before
  // the first fragment read of the current stage, so the load of stage kt + 1 never
  // overlaps the MFMAs of stage kt (seen in the gfx950 disassembly of the STAGES = 2 loop).
  // The counted wait_vmcnt + barrier at the top of each iteration orders the ring.
  auto glds = [](const void* src, void* lds) {
    if constexpr (sizeof(T) == 4) glds16_asm(src, lds);
    else glds16(src, lds);
  };
  auto issue = [&](int kt, int buf) {
    T* As = smem + buf * TILE;
    T* Bs = As + BM * BK;
    if constexpr (F11B) {
      // (the compiler keeps the descriptors in SGPRs except in the bf16 256 x 256 kernels,
      // where they go through v_readfirstlane: blds16u)
      auto bl = [](i32x4 r, uint32_t v, uint32_t l) {
        if constexpr (!F32 && BM == 256 && BN == 256) blds16u(r, v, l);
        else blds16(r, v, l);
      };
      // (the prologue's descriptors may come straight from a v_readfirstlane: a VALU write of
      // an SGPR needs 5 wait states before a VMEM instruction reads it)
      if (kt < STAGES - 1) asm volatile("s_nop 4" ::: "memory");
      uint64_t ab;
      if constexpr (CONV) {
        if (kc == 0) {  // first tile of the tap (kr, ks): this lane's pixel offsets for it
#pragma unroll
          for (int i = 0; i < NAR; ++i) {
            const int hi = hi0[i] + kr, wi = wi0[i] + ks;
            const bool ok = unsigned(hi) < unsigned(geo.H) && unsigned(wi) < unsigned(geo.W);
            voa[i] = ok ? uint32_t((((img[i] - ih0) + hi) * geo.W + wi) * pitch + ca[i]) * uint32_t(AES)
                        : kBufOob;
          }
        }
        ab = abase + uint64_t(kc) * uint64_t(AES);
      } else {
        ab = abase + uint64_t(kt) * uint64_t(BK * AES);
      }
      constexpr int TB = int(sizeof(T));
      if constexpr (ASPLIT) {  // two 64-B-row plane images (h, l) of BM rows, like B's
        const uint32_t la = lds0 + uint32_t(buf * TILE * TB + wu * IAP * 16 * 32 * 2);
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const i32x4 ra = buf_rsrc(ab + uint64_t(p) * uint64_t(ep.aps) * 2u);
#pragma unroll
          for (int i = 0; i < IAP; ++i) bl(ra, voa[i], la + uint32_t(p * BM * 32 * 2 + i * 16 * 32 * 2));
        }
      } else {
        const i32x4 ra = buf_rsrc(ab);
        const uint32_t la = lds0 + uint32_t((buf * TILE + wu * IA * RPI * BK) * TB);
#pragma unroll
        for (int i = 0; i < IA; ++i) bl(ra, voa[i], la + uint32_t(i * RPI * BK * TB));
      }
      if constexpr (BSPLIT) {
        const uint32_t lb = lds0 + uint32_t((buf * TILE + BM * BK) * TB + wu * IBP * 16 * 32 * 2);
#pragma unroll
        for (int p = 0; p < NPL; ++p) {
          const i32x4 rb = buf_rsrc(bbase + (uint64_t(p) * uint64_t(bps) + uint64_t(kt) * 32u) * 2u);
#pragma unroll
          for (int i = 0; i < IBP; ++i) bl(rb, vob[i], lb + uint32_t(p * BN * 32 * 2 + i * 16 * 32 * 2));
        }
      } else {
        const i32x4 rb = buf_rsrc(bbase + uint64_t(kt) * uint64_t(BK * TB));
        const uint32_t lb = lds0 + uint32_t((buf * TILE + BM * BK + wu * IB * RPI * BK) * TB);
#pragma unroll
        for (int i = 0; i < IB; ++i) bl(rb, vob[i], lb + uint32_t(i * RPI * BK * TB));
      }
    } else {
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      if constexpr (CONV) {
        const int hi = hi0[i] + kr, wi = wi0[i] + ks;
        const bool ok = unsigned(hi) < unsigned(geo.H) && unsigned(wi) < unsigned(geo.W);
        const T* src = ok ? A + (((img[i] + hi) * geo.W + wi) * pitch + kc + ca[i]) : zline + ca[i];
        glds(src, As + (w * IA + i) * RPI * BK);
      } else {
        glds(pa[i] + kt * BK, As + (w * IA + i) * RPI * BK);
      }
    }
    if constexpr (BSPLIT) {
      uint16_t* Bp = reinterpret_cast<uint16_t*>(Bs);
#pragma unroll
      for (int p = 0; p < NPL; ++p)
#pragma unroll
        for (int i = 0; i < IBP; ++i)
          glds(pbp[i] + p * bps + kt * 32, Bp + p * (BN * 32) + (w * IBP + i) * 16 * 32);
    } else {
#pragma unroll
      for (int i = 0; i < IB; ++i)
        glds(pb[i] + kt * BK, Bs + (w * IB + i) * RPI * BK);
    }
    }
    if constexpr (CONV) {  // tiles are issued in k order: step to the next (tap, channel) slab
      kc += BK;
      if (kc == geo.C) {
        kc = 0;
        if (++ks == geo.S) {
          ks = 0;
          ++kr;
        }
      }
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;

  // fp32: the running chain of the current block of tiles (native fp32 MFMA, see the MFMA
  // loop) or the small-term accumulators of the split products (FM = 1)
  f32x16 tacc[F32 ? TM : 1][F32 ? TN : 1];
#pragma unroll
  for (int i = 0; i < (F32 ? TM : 1); ++i)
#pragma unroll
    for (int j = 0; j < (F32 ? TN : 1); ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) tacc[i][j][v] = 0.f;

  const int fr = lane & 31, fh = lane >> 5;
  const int nk = K / BK;
  // FM 11: operand scales 2^ea (A, applied in the split) and 2^eb (B, applied by the plan)
  [[maybe_unused]] int ea = 0, eb = 0;
  [[maybe_unused]] float sa = 1.f, sa11 = 2048.f;
  if constexpr (F32 && (FM == 11 || FM == 13)) {
    ea = fp16_exp(ep.amax_a);
    eb = fp16_exp(ep.amax_b);
    sa = exp2i(ea);
    sa11 = exp2i(ea + 11);
  }
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) issue(s, s);
  for (int kt = 0; kt < nk; ++kt) {
    // tiles issued after kt that may stay in flight
    const int after = min(nk, kt + STAGES - 1) - (kt + 1);
    if (STAGES >= 4 && after >= 2) wait_vmcnt<2 * NI>();
    else if (STAGES >= 3 && after >= 1) wait_vmcnt<NI>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + STAGES - 1 < nk) issue(kt + STAGES - 1, (kt + STAGES - 1) % STAGES);
    const T* As = smem + (kt % STAGES) * TILE;
    const T* Bs = As + BM * BK;
    if constexpr (F32 && FM == 10) {
      // FM 10 (experiment, MPIT_F32_NT=acc1): FM 9 with the six products accumulated in ONE
      // register set (standard fp32 accumulation instead of the separate small-term sum) and
      // the fragments of step kk + 1 read before the split + MFMAs of step kk (the 64
      // registers of the second accumulator hold the prefetched fragments)
      const uint16_t* Bp = reinterpret_cast<const uint16_t*>(Bs);
      constexpr int KK = BK / 16;
      bf16x8 ph[2][TN], pm[2][TN], pl[2][TN];
      float4 pa[2][TM][2];
      auto rd = [&](int kk, int sl) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int r = wn * WN + j * 32 + fr;
          const int o = r * 32 + swz(r, 2 * kk + fh) * 8;
          ph[sl][j] = *reinterpret_cast<const bf16x8*>(Bp + o);
          pm[sl][j] = *reinterpret_cast<const bf16x8*>(Bp + BN * 32 + o);
          pl[sl][j] = *reinterpret_cast<const bf16x8*>(Bp + 2 * BN * 32 + o);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int r = wm * WM + i * 32 + fr;
          pa[sl][i][0] = *reinterpret_cast<const float4*>(As + r * BK + swzk<BKB>(r, 4 * kk + 2 * fh) * 4);
          pa[sl][i][1] = *reinterpret_cast<const float4*>(As + r * BK + swzk<BKB>(r, 4 * kk + 2 * fh + 1) * 4);
        }
      };
      rd(0, 0);
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        if (kk + 1 < KK) rd(kk + 1, (kk + 1) & 1);
        const int sl = kk & 1;
        bf16x8 ah[TM], am[TM], al[TM];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const float4 x0 = pa[sl][i][0], x1 = pa[sl][i][1];
          const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
          split3(v, ah[i], am[i], al[i]);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pm[sl][j], ah[i], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ph[sl][j], am[i], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pm[sl][j], am[i], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pl[sl][j], ah[i], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ph[sl][j], al[i], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ph[sl][j], ah[i], acc[i][j], 0, 0, 0);
          }
      }
      continue;
    } else if constexpr (F32 && FM == 13) {
      // fp16x3 on planes: A's h, l read ready-made like B's (chunk 2kk + fh of a 64-B plane
      // row); hh -> acc, hl + lh -> tacc — FM 11's products on the same planes, no split
      const uint16_t* Bp = reinterpret_cast<const uint16_t*>(Bs);
      const uint16_t* Ap = reinterpret_cast<const uint16_t*>(As);
      // MPIT_FM13_PF (A/B build define): every fragment of the stage read before its first
      // MFMA (KK sets of fragment registers), instead of per k16 step
      constexpr int KK = BK / 16, KS = kFm13Pf ? KK : 1;
      f16x8 ah[KS][TM], al[KS][TM], bh[KS][TN], bl[KS][TN];
      auto rd = [&](int kk, int sl) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int r = wn * WN + j * 32 + fr;
          const int o = r * 32 + swz(r, 2 * kk + fh) * 8;
          bh[sl][j] = *reinterpret_cast<const f16x8*>(Bp + o);
          bl[sl][j] = *reinterpret_cast<const f16x8*>(Bp + BN * 32 + o);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int r = wm * WM + i * 32 + fr;
          const int o = r * 32 + swz(r, 2 * kk + fh) * 8;
          ah[sl][i] = *reinterpret_cast<const f16x8*>(Ap + o);
          al[sl][i] = *reinterpret_cast<const f16x8*>(Ap + BM * 32 + o);
        }
      };
      if constexpr (kFm13Pf) {
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) rd(kk, kk);
      }
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        const int sl = kFm13Pf ? kk : 0;
        if constexpr (!kFm13Pf) rd(kk, 0);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bh[sl][j], ah[sl][i], acc[i][j], 0, 0, 0);
            tacc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bl[sl][j], ah[sl][i], tacc[i][j], 0, 0, 0);
            tacc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bh[sl][j], al[sl][i], tacc[i][j], 0, 0, 0);
          }
      }
      continue;
    } else if constexpr (F32 && FM == 11) {
      // fp16x3: B planes h, l read ready-made; the lane's 8 A floats of k16 step kk (chunks
      // 4kk + 2fh, +1) scaled and split in registers; hh -> acc, hl + lh -> tacc
      const uint16_t* Bp = reinterpret_cast<const uint16_t*>(Bs);
#pragma unroll
      for (int kk = 0; kk < BK / 16; ++kk) {
        f16x8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int r = wn * WN + j * 32 + fr;
          const int o = r * 32 + swz(r, 2 * kk + fh) * 8;
          bh[j] = *reinterpret_cast<const f16x8*>(Bp + o);
          bl[j] = *reinterpret_cast<const f16x8*>(Bp + BN * 32 + o);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int r = wm * WM + i * 32 + fr;
          const float4 x0 = *reinterpret_cast<const float4*>(As + r * BK + swzk<BKB>(r, 4 * kk + 2 * fh) * 4);
          const float4 x1 = *reinterpret_cast<const float4*>(As + r * BK + swzk<BKB>(r, 4 * kk + 2 * fh + 1) * 4);
#if defined(MPIT_ABLATE_PLANES) || defined(MPIT_ABLATE_PLANES_NT)  // timing ablation: A as if it arrived as fp16 planes (no split)
          ah[i] = __builtin_bit_cast(f16x8, x0);
          al[i] = __builtin_bit_cast(f16x8, x1);
#else
          const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
          split2h(v, sa, sa11, ah[i], al[i]);
#endif
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bh[j], ah[i], acc[i][j], 0, 0, 0);
            tacc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bl[j], ah[i], tacc[i][j], 0, 0, 0);
            tacc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bh[j], al[i], tacc[i][j], 0, 0, 0);
          }
      }
      continue;
    } else if constexpr (BSPLIT) {
      // A: the lane's 8 floats of k16 step kk (chunks 4kk + 2fh, +1) split in registers;
      // B: the same k (chunk 2kk + fh of a 64-B plane row) read ready-made from each plane
      const uint16_t* Bp = reinterpret_cast<const uint16_t*>(Bs);
#pragma unroll
      for (int kk = 0; kk < BK / 16; ++kk) {
        bf16x8 ah[TM], am[TM], al[TM], bh[TN], bm[TN], bl[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int r = wn * WN + j * 32 + fr;
          const int o = r * 32 + swz(r, 2 * kk + fh) * 8;
          bh[j] = *reinterpret_cast<const bf16x8*>(Bp + o);
          bm[j] = *reinterpret_cast<const bf16x8*>(Bp + BN * 32 + o);
          bl[j] = *reinterpret_cast<const bf16x8*>(Bp + 2 * BN * 32 + o);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int r = wm * WM + i * 32 + fr;
          const float4 x0 = *reinterpret_cast<const float4*>(As + r * BK + swzk<BKB>(r, 4 * kk + 2 * fh) * 4);
          const float4 x1 = *reinterpret_cast<const float4*>(As + r * BK + swzk<BKB>(r, 4 * kk + 2 * fh + 1) * 4);
          const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
          split3(v, ah[i], am[i], al[i]);
        }
        mfma_x3<TM, TN>(acc, tacc, ah, am, al, bh, bm, bl, true);
      }
      continue;
    } else if constexpr (F32 && FM >= 5 && FM <= 7) {
      // TIMING ABLATION ONLY (MPIT_F32_ABLATE=nosplit): FM 3's loop with the operand split
      // replaced by a reinterpretation of the raw fp32 bits (wrong numbers, zero VALU) — how
      // fast the kernel would be if its operands arrived pre-split
#pragma unroll
      for (int kk = 0; kk < BK / 16; ++kk) {
        bf16x8 ah[TM], am[TM], al[TM], bh[TN], bm[TN], bl[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int r = wm * WM + i * 32 + fr;
          const float4 x0 = *reinterpret_cast<const float4*>(As + r * BK + swzk<BKB>(r, 4 * kk + 2 * fh) * 4);
          const float4 x1 = *reinterpret_cast<const float4*>(As + r * BK + swzk<BKB>(r, 4 * kk + 2 * fh + 1) * 4);
          if constexpr (FM == 6) {  // ablation 6: A split, B raw
            const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
            split3(v, ah[i], am[i], al[i]);
          } else {
            ah[i] = __builtin_bit_cast(bf16x8, x0);
            am[i] = __builtin_bit_cast(bf16x8, x1);
            al[i] = ah[i];
          }
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int r = wn * WN + j * 32 + fr;
          const float4 x0 = *reinterpret_cast<const float4*>(Bs + r * BK + swzk<BKB>(r, 4 * kk + 2 * fh) * 4);
          const float4 x1 = *reinterpret_cast<const float4*>(Bs + r * BK + swzk<BKB>(r, 4 * kk + 2 * fh + 1) * 4);
          if constexpr (FM == 7) {  // ablation 7: A raw, B split
            const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
            split3(v, bh[j], bm[j], bl[j]);
          } else {
            bh[j] = __builtin_bit_cast(bf16x8, x0);
            bm[j] = __builtin_bit_cast(bf16x8, x1);
            bl[j] = bh[j];
          }
        }
        mfma_x3<TM, TN>(acc, tacc, ah, am, al, bh, bm, bl, true);
      }
      continue;
    } else if constexpr (F32 && (FM == 1 || FM == 3)) {
      // bf16x6: the lane's 8 floats of a row in k16 step kk (chunks 4kk + 2fh, +1 of the row)
      // are exactly the k = 8fh + j operand of one v_mfma_f32_32x32x16_bf16; split each
      // fragment in registers
#pragma unroll
      for (int kk = 0; kk < BK / 16; ++kk) {
        bf16x8 ah[TM], am[TM], al[TM], bh[TN], bm[TN], bl[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int r = wm * WM + i * 32 + fr;
          const float4 x0 = *reinterpret_cast<const float4*>(As + r * BK + swzk<BKB>(r, 4 * kk + 2 * fh) * 4);
          const float4 x1 = *reinterpret_cast<const float4*>(As + r * BK + swzk<BKB>(r, 4 * kk + 2 * fh + 1) * 4);
          const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
          split3(v, ah[i], am[i], al[i]);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int r = wn * WN + j * 32 + fr;
          const float4 x0 = *reinterpret_cast<const float4*>(Bs + r * BK + swzk<BKB>(r, 4 * kk + 2 * fh) * 4);
          const float4 x1 = *reinterpret_cast<const float4*>(Bs + r * BK + swzk<BKB>(r, 4 * kk + 2 * fh + 1) * 4);
          const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
          split3(v, bh[j], bm[j], bl[j]);
        }
        mfma_x3<TM, TN>(acc, tacc, ah, am, al, bh, bm, bl, true);
      }
      continue;
    } else if constexpr (F32) {
      // v_mfma_f32_32x32x2_f32: lane (fr, fh) supplies A[row fr][k] and B[col fr][k] of one
      // k per instruction. The 16-deep tile is split by lane half: half fh runs k = 8fh + s
      // in step s (any bijection onto the tile's k works when A and B use the same one), so
      // a lane's 8 values of a row are two contiguous chunks: 2 ds_read_b128 per fragment.
      float4 af[TM][2], bfg[TN][2];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wm * WM + i * 32 + fr;
        af[i][0] = *reinterpret_cast<const float4*>(As + r * BK + swzk<BKB>(r, 2 * fh) * 4);
        af[i][1] = *reinterpret_cast<const float4*>(As + r * BK + swzk<BKB>(r, 2 * fh + 1) * 4);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = wn * WN + j * 32 + fr;
        bfg[j][0] = *reinterpret_cast<const float4*>(Bs + r * BK + swzk<BKB>(r, 2 * fh) * 4);
        bfg[j][1] = *reinterpret_cast<const float4*>(Bs + r * BK + swzk<BKB>(r, 2 * fh + 1) * 4);
      }
      auto el = [](const float4 (&q)[2], int s) -> float {
        const float4& h = q[s >> 2];
        const int k = s & 3;
        return k == 0 ? h.x : k == 1 ? h.y : k == 2 ? h.z : h.w;
      };
      // Blocked accumulation: the MFMA is a k-ordered fmaf chain, so a 4608-deep K summed
      // in one chain loses ~sqrt(K) ulps; chains of 32 (two tiles) into tacc, folded into
      // acc once per block, keep the error at the level of a blocked fp32 library GEMM.
#pragma unroll
      for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            tacc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(el(bfg[j], s), el(af[i], s), tacc[i][j], 0, 0, 0);
      if ((kt & 1) || kt == nk - 1) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            acc[i][j] += tacc[i][j];
#pragma unroll
            for (int v = 0; v < 16; ++v) tacc[i][j][v] = 0.f;
          }
      }
      continue;
    } else {
    if constexpr (TM * TN >= 8) {
      // big wave tiles run one or two waves per SIMD, so nothing else hides a fragment read:
      // the fragments of k16 step kk+1 are read while step kk's MFMAs run (two register
      // sets), pinned so the scheduler does not re-serialise read -> wait -> MFMAs
      constexpr int KK = BK / 16;
      bf16x8 af[2][TM], bfg[2][TN];
      auto frag = [&](int kk, int slot) {
        const int c = 2 * kk + fh;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int r = wm * WM + i * 32 + fr;
          af[slot][i] = *reinterpret_cast<const bf16x8*>(As + r * BK + swzk<BKB>(r, c) * 8);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int r = wn * WN + j * 32 + fr;
          bfg[slot][j] = *reinterpret_cast<const bf16x8*>(Bs + r * BK + swzk<BKB>(r, c) * 8);
        }
      };
      frag(0, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, TM + TN, 0);
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        if (kk + 1 < KK) {
          frag(kk + 1, (kk + 1) & 1);
          __builtin_amdgcn_sched_group_barrier(0x100, TM + TN, 0);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfg[kk & 1][j], af[kk & 1][i], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, TM * TN, 0);
      }
      continue;
    }
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      bf16x8 af[TM], bfg[TN];
      const int c = 2 * kk + fh;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wm * WM + i * 32 + fr;
        af[i] = *reinterpret_cast<const bf16x8*>(As + r * BK + swzk<BKB>(r, c) * 8);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = wn * WN + j * 32 + fr;
        bfg[j] = *reinterpret_cast<const bf16x8*>(Bs + r * BK + swzk<BKB>(r, c) * 8);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfg[j], af[i], acc[i][j], 0, 0, 0);
    }
    }
  }

  if constexpr (F32 && (FM == 11 || FM == 13)) {  // (hh + 2^-11 (hl + lh)) 2^-(ea + eb), exact scalings
    const float ia = exp2i(-ea), ib = exp2i(-eb);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[i][j][v] = fmaf(tacc[i][j][v], 1.f / 2048.f, acc[i][j][v]) * ia * ib;
  } else if constexpr (F32 && FM != 0) {  // hh + the five small terms
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] += tacc[i][j];
  }

  // ---- epilogue, phase A: accumulators (+ bias, ReLU) -> T tile in LDS. Lane holds
  // D[n][m] with m = lane&31, n = (v&3) + 8*(v>>2) + 4*(lane>>5): 4 consecutive columns of
  // one row, one 8-B (bf16) / 16-B (fp32) LDS store each (the C/D layout of both MFMAs).
  // Unpadded rows (the bf16 tile fits in the 2-slot ring, keeping 5 blocks/CU possible); the
  // 16-B chunk index is XOR-swizzled by the row so phase A's column writes spread over banks
  constexpr int LDT = BN, CPRS = BN / EPC;
  auto tsw = [](int row, int n) { return row * LDT + (((n / EPC) ^ (row % CPRS)) * EPC) + (n % EPC); };
  // tagged BN fold (ep.fepoch): the fold ticket is taken now, before any output store, so
  // its return does not queue behind them (vmcnt retires in issue order)
  [[maybe_unused]] uint32_t ftk = 0;
  __shared__ uint32_t s_ftk;
  if constexpr (EPI == EPI_STATS || EPI == EPI_BNRED) {
    if (ep.fepoch && (EPI == EPI_STATS ? ep.scoef != nullptr : ep.fcoef != nullptr) && t == 0)
      ftk = atomicAdd(fold_ticket<BM / 128>(ep, M, mt, nt), 1u);
  }
  T* tl = smem;                // reuses the ring
  __syncthreads();             // every wave is done reading the ring
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int nl = wn * WN + j * 32 + 8 * g + 4 * fh;
        if (bias != nullptr) {  // conv bias (+ ReLU) (VGG / AlexNet)
          const float4 b4 = *reinterpret_cast<const float4*>(bias + n0 + nl);
          acc[i][j][4 * g + 0] += b4.x;
          acc[i][j][4 * g + 1] += b4.y;
          acc[i][j][4 * g + 2] += b4.z;
          acc[i][j][4 * g + 3] += b4.w;
        }
        if (relu) {
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[i][j][4 * g + e] = fmaxf(acc[i][j][4 * g + e], 0.f);
        }
        if constexpr (F32) {
          *reinterpret_cast<float4*>(tl + tsw(wm * WM + i * 32 + fr, nl)) =
              make_float4(acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]);
        } else {
          const uint32_t lo = uint32_t(f2bf(acc[i][j][4 * g])) | (uint32_t(f2bf(acc[i][j][4 * g + 1])) << 16);
          const uint32_t hi = uint32_t(f2bf(acc[i][j][4 * g + 2])) | (uint32_t(f2bf(acc[i][j][4 * g + 3])) << 16);
          *reinterpret_cast<uint2*>(tl + tsw(wm * WM + i * 32 + fr, nl)) = make_uint2(lo, hi);
        }
      }
  if constexpr (EPI == EPI_STATS || EPI == EPI_BNRED) {
    if (t == 0) s_ftk = ftk;  // (read by the fold after phase B's barriers)
  }
  __syncthreads();

  // ---- phase B: row-major. A thread owns 8 channels (one bf16 / two fp32 16-B chunks) of a
  // row and walks the rows RPP apart, so every global access of a wave covers whole row
  // segments: the C store, the Cin / Cmask / BN x / BN mask loads.
  // Partials are per 128-row tile whatever BM is: with BM = 256 the row-threads split into
  // two halves of 128 rows (HALVES = BM / 128), each thread staying in one.
  constexpr int CPR = BN / 8, RPP = NT / CPR, NP = BM / RPP;
  constexpr int HALVES = BM / 128, RPH = RPP / HALVES;  // row-threads per 128-row half
  const int ch = t % CPR, rg = t / CPR;
  const int rr = (rg / RPH) * 128 + rg % RPH;  // first row of this thread; rows rr + p*RPH
  // fp32: the thread's 8 channels are two float4 halves HOFF = BN/2 apart (columns 4ch.. and
  // BN/2 + 4ch..), so each access instruction of a wave covers 256-B row segments instead of
  // 32-B lane strides that leave every cache line it touches half used; bf16: 8 consecutive
  // channels, one 16-B chunk
  constexpr int HOFF = F32 ? BN / 2 : 4;
  const int cl0 = F32 ? ch * 4 : ch * 8;  // tile column of element 0; element e at ecol(e)
  auto ecol = [&](int e) { return cl0 + (e < 4 ? e : HOFF + e - 4); };
  const int nc = n0 + cl0;  // first global column of this thread
  // the 8 mask bits of the thread's elements at offset o (one mask byte per 8 channels)
  auto mbits = [](const uint8_t* mk, int64_t o) -> uint32_t {
    if constexpr (HOFF == 4) return mk[o >> 3];
    else return ((uint32_t(mk[o >> 3]) >> (o & 7)) & 15u) | (((uint32_t(mk[(o + HOFF) >> 3]) >> ((o + HOFF) & 7)) & 15u) << 4);
  };
  float s1[8], s2[8], sf[8], mu[8];
  float om = 0.f;  // max |C| over this thread's stores (ep.omax)
  int nv = 0;
#pragma unroll
  for (int e = 0; e < 8; ++e) s1[e] = s2[e] = sf[e] = mu[e] = 0.f;
  constexpr bool BNRED = EPI == EPI_BNRED || EPI == EPI_BNRED2, DUAL = EPI == EPI_BNRED2, RELUB = EPI == EPI_RELUB;
  float s3[8], mu2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s3[e] = mu2[e] = 0.f;
  if constexpr (BNRED) {
    const float4 a0 = *reinterpret_cast<const float4*>(ep.mean + nc);
    const float4 a1 = *reinterpret_cast<const float4*>(ep.mean + nc + HOFF);
    mu[0] = a0.x; mu[1] = a0.y; mu[2] = a0.z; mu[3] = a0.w;
    mu[4] = a1.x; mu[5] = a1.y; mu[6] = a1.z; mu[7] = a1.w;
  }
  if constexpr (DUAL) {
    const float4 a0 = *reinterpret_cast<const float4*>(ep.mean2 + nc);
    const float4 a1 = *reinterpret_cast<const float4*>(ep.mean2 + nc + HOFF);
    mu2[0] = a0.x; mu2[1] = a0.y; mu2[2] = a0.z; mu2[3] = a0.w;
    mu2[4] = a1.x; mu2[5] = a1.y; mu2[6] = a1.z; mu2[7] = a1.w;
  }
  const T* epx = reinterpret_cast<const T*>(ep.x);
  const T* epx2 = reinterpret_cast<const T*>(ep.x2);
  // Rows go in batches of PB: all loads of a batch are issued before its first store (C
  // may alias Cin, so the compiler would otherwise serialise load -> store per row), and
  // batches keep the live registers low enough for 5 resident blocks per CU.
  constexpr int PB = NP < 4 ? NP : 4;
#pragma unroll
  for (int pb = 0; pb < NP; pb += PB) {
  int64_t orow[PB];
  V8<T> cv[PB], xq[PB], xq2[PB];
  uint32_t cmb[PB], xmb[PB];
#pragma unroll
  for (int q = 0; q < PB; ++q) {
    const int p = pb + q;
    const int64_t m = m0 + rr + p * RPH;
    orow[q] = m;  // output row (pixel) of GEMM row m
    if constexpr (CONV) {
      if (geo.ostr > 1) {
        const int hw = geo.Ho * geo.Wo;
        const int64_t nimg = m / hw;
        const int rem = int(m - nimg * hw), gi = rem / geo.Wo, gj = rem - gi * geo.Wo;
        orow[q] = (nimg * geo.OH + gi * geo.ostr + geo.oph) * geo.OW + gj * geo.ostr + geo.opw;
      }
    }
    const bool ok = m < M;
    const int64_t o = orow[q] * ldc + nc;
    if (Cin != nullptr) {
      if (ok) cv[q].load(Cin + o, HOFF);
      else cv[q].zero();
      cmb[q] = Cmask ? (ok ? mbits(Cmask, o) : 0u) : 0xffu;
    }
    if constexpr (BNRED) {
      if (ok) xq[q].load(epx + o, HOFF);
      else xq[q].zero();
      xmb[q] = ok ? (ep.mask ? mbits(ep.mask, o) : 0xffu) : 0u;
    }
    if constexpr (RELUB) {
      if (ok) xq[q].load(epx + o, HOFF);
      else xq[q].zero();
    }
    if constexpr (DUAL) {
      if (ok) xq2[q].load(epx2 + o, HOFF);
      else xq2[q].zero();
    }
  }
#pragma unroll
  for (int q = 0; q < PB; ++q) {
    const int rl = rr + (pb + q) * RPH;
    if (m0 + rl >= M) continue;
    const int64_t o = orow[q] * ldc + nc;
    float v[8];
    if constexpr (F32) {
      const float4 h0 = *reinterpret_cast<const float4*>(tl + tsw(rl, cl0));
      const float4 h1 = *reinterpret_cast<const float4*>(tl + tsw(rl, cl0 + HOFF));
      v[0] = h0.x; v[1] = h0.y; v[2] = h0.z; v[3] = h0.w;
      v[4] = h1.x; v[5] = h1.y; v[6] = h1.z; v[7] = h1.w;
    } else {
      V8<uint16_t> hv;
      hv.load(tl + tsw(rl, cl0));
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = hv.get(e);
    }
    if (Cin != nullptr) {  // C = A.B^T + Cin
      // Cmask: Cin is a ReLU'd gradient given as (dy, forward bit mask: one byte per 8
      // channels, bit e = channel 8k+e positive) — dy*mask is never materialised
      const uint32_t mb = cmb[q];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = rnd<T>(v[e] + ((mb >> e) & 1u ? cv[q].get(e) : 0.f));
    }
    if constexpr (RELUB) {  // dz = dy * (y > 0) of the layer below, as stored
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v[e] = xq[q].get(e) > 0.f ? rnd<T>(v[e]) : 0.f;
        s1[e] += v[e];
      }
    }
    store8(C + o, v, HOFF);
    if (ep.omax != nullptr) {
#pragma unroll
      for (int e = 0; e < 8; ++e) om = fmaxf(om, fabsf(v[e]));
    }
    if constexpr (CONV) {
      if (geo.ozero) {  // class (0,0) of a stride-2 conv whose other parities have no taps
        const int64_t pix = orow[q] % (int64_t(geo.OH) * geo.OW);
        const int oh = int(pix / geo.OW), ow = int(pix % geo.OW);
        const float z[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (ow + 1 < geo.OW) store8(C + o + ldc, z, HOFF);
        if (oh + 1 < geo.OH) {
          store8(C + o + int64_t(geo.OW) * ldc, z, HOFF);
          if (ow + 1 < geo.OW) store8(C + o + int64_t(geo.OW + 1) * ldc, z, HOFF);
        }
      }
    }
    if constexpr (EPI == EPI_STATS) {  // shifted by this thread's first row
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float y = v[e];
        if (nv == 0) sf[e] = y;
        const float d = y - sf[e];
        s1[e] += d;
        s2[e] = fmaf(d, d, s2[e]);
      }
      ++nv;
    } else if constexpr (BNRED) {  // dz = C * mask; (sum dz, sum dz (x - mean) [, sum dz (x2 - mean2)])
      const uint32_t xb = xmb[q];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float dz = (xb >> e) & 1u ? v[e] : 0.f;
        s1[e] += dz;
        s2[e] = fmaf(dz, xq[q].get(e) - mu[e], s2[e]);
        if constexpr (DUAL) s3[e] = fmaf(dz, xq2[q].get(e) - mu2[e], s3[e]);
      }
    }
  }
  }
  if (ep.omax != nullptr) {  // the block's max |C|: one (epoch, value) atomic max
    __shared__ float s_om[NW];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) om = fmaxf(om, __shfl_xor(om, o));
    if (lane == 0) s_om[w] = om;
    lds_barrier();
    if (t == 0) {
      float b = s_om[0];
#pragma unroll
      for (int k = 1; k < NW; ++k) b = fmaxf(b, s_om[k]);
      atomicMax(ep.omax + (blockIdx.x % kBoundSlots) * (kBoundStride / 2),
                (static_cast<unsigned long long>(ep.oepoch) << 32) | __float_as_uint(b));
    }
  }
  if constexpr (EPI != EPI_NONE) {
    // combine the RPP threads of each chunk through LDS: [RPP][3][BN] floats
    float* red = reinterpret_cast<float*>(smem);
    lds_barrier();  // phase B is done reading the tile (its C stores stay in flight)
    if constexpr (EPI == EPI_STATS) {  // this thread's (n, mean, M2)
      const float n = float(nv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = nv ? s1[e] / n : 0.f;
        red[(rg * 3 + 0) * BN + ecol(e)] = n;
        red[(rg * 3 + 1) * BN + ecol(e)] = nv ? sf[e] + d : 0.f;
        red[(rg * 3 + 2) * BN + ecol(e)] = nv ? fmaxf(s2[e] - s1[e] * d, 0.f) : 0.f;
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[(rg * 3 + 0) * BN + ecol(e)] = s1[e];
        red[(rg * 3 + 1) * BN + ecol(e)] = s2[e];
        if constexpr (DUAL) red[(rg * 3 + 2) * BN + ecol(e)] = s3[e];
      }
    }
    lds_barrier();
    for (int q = t; q < BN * HALVES; q += NT) {
      const int hf = q / BN, n = q % BN;
      const int64_t tile = int64_t(mt) * HALVES + hf;  // 128-row partial row
      if (tile * 128 >= M) continue;
      float* prow = ep.part + (ep.row0 + tile) * 2 * int64_t(N) + n0;
      if constexpr (EPI == EPI_STATS) {  // merge the half's (n, mean, M2) triples (Chan et al.)
        float na = 0.f, mean = 0.f, m2 = 0.f;
        for (int k = hf * RPH; k < (hf + 1) * RPH; ++k) {
          const float nb = red[(k * 3 + 0) * BN + n];
          if (nb == 0.f) continue;
          const float mb = red[(k * 3 + 1) * BN + n], tot = na + nb, d = mb - mean;
          mean += d * (nb / tot);
          m2 += red[(k * 3 + 2) * BN + n] + d * d * (na * nb / tot);
          na = tot;
        }
        if (ep.scoef != nullptr && ep.fepoch) {  // (value, epoch) pairs
          const int64_t i = (ep.row0 + tile) * 2 * int64_t(N) + n0 + n;
          st_tag(ep.part, i, mean, ep.fepoch);
          st_tag(ep.part, i + N, m2, ep.fepoch);
        } else if (ep.scoef != nullptr) {  // read by the folding blocks (any XCD)
          st_wt(prow + n, mean);
          st_wt(prow + N + n, m2);
        } else {
          prow[n] = mean;
          prow[N + n] = m2;
        }
      } else {
        float a = 0.f, b = 0.f, c3 = 0.f;
        for (int k = hf * RPH; k < (hf + 1) * RPH; ++k) {
          a += red[(k * 3 + 0) * BN + n];
          b += red[(k * 3 + 1) * BN + n];
          if constexpr (DUAL) c3 += red[(k * 3 + 2) * BN + n];
        }
        if constexpr (RELUB) {
          prow[n] = a;  // (the second row is unused)
        } else if (EPI == EPI_BNRED && ep.fcoef != nullptr && ep.fepoch) {  // (value, epoch) pairs
          const int64_t i = (ep.row0 + tile) * 2 * int64_t(N) + n0 + n;
          st_tag(ep.part, i, a, ep.fepoch);
          st_tag(ep.part, i + N, b, ep.fepoch);
        } else if (EPI == EPI_BNRED && ep.fcoef != nullptr) {  // read by the folding block (any XCD)
          st_wt(prow + n, a);
          st_wt(prow + N + n, b);
        } else {
          prow[n] = a;
          prow[N + n] = b;
        }
        if constexpr (DUAL) {
          float* prow2 = ep.part2 + (ep.row0 + tile) * 2 * int64_t(N) + n0;
          prow2[n] = a;
          prow2[N + n] = c3;
        }
      }
    }
  }
  if constexpr (EPI == EPI_BNRED) {
    if (ep.fcoef != nullptr) bnred_fold<BN, HALVES>(ep, smem, M, N, mt, nt, n0, s_ftk);
  }
  if constexpr (EPI == EPI_STATS) {
    if (ep.scoef != nullptr) stats_fold<BN, HALVES>(ep, smem, M, N, mt, nt, n0, s_ftk);
  }
}

// ------------------------------------------------------------------------------ TN GEMM
// part[split][N][K] = sum over rows m of this split of dY[m][n] * X[m][k]
//
// Staging: global_load_lds into a ring of STAGES tiles of kRows rows (same counted-vmcnt
// scheme as gemm_nt). LDS rows are the plain data rows (128 B or 256 B) with a 16-B chunk
// XOR swizzle chosen so the ds_read_b64_tr_b16 fragment reads of a 32-lane half (4 rows x
// 32 columns) hit 64 distinct banks; glds is lane-linear, so the swizzle is applied to the
// global source address. A partial last step (M % kRows) is zero-filled in LDS.
constexpr int kRows = 32;  // rows (reduction) per staged step

// 16-B chunk swizzle of a row of CPR chunks (bf16: CPR = 16: 256-B rows, 8: 128-B rows).
// fp32 fragments are read one element per lane (ds_read_b32, 32 consecutive columns per
// half-wave): conflict-free on the plain row-major image, no swizzle.
template <typename T, int CPR>
__device__ __forceinline__ int tswz(int row, int ch) {
  if constexpr (sizeof(T) == 4) return ch;
  else if constexpr (CPR == 16) return ch ^ (((row & 3) << 2) | ((row >> 2) & 3));
  else return ch ^ (((row >> 1) & 1) << 2);
}

// In-kernel split reduction (replaces split_reduce_kernel launches): every split writes its
// partial tile write-through, takes a ticket for its (tile, group of kReduceGroup splits);
// the block whose ticket comes last sums the group's partials in split order, and when
// there is more than one group the last group-reducer of the tile sums the group sums in
// group order into out (out = beta*out + sum) — the same additions in the same order as
// the two split_reduce levels, so the result is bitwise the one of the separate launches.
// Hand-off as in bn_tiles_finalize_kernel (bn_act.hip): sc1 stores, s_waitcnt, barrier,
// one agent-scope ticket add per workgroup; the consumer: agent acquire, then plain loads.
constexpr int kReduceGroup = 32;
constexpr int kTnTicketSlots = 16;
constexpr int kTnMaxTickets = 8192;
__device__ uint32_t g_tn_tickets[kTnTicketSlots * kTnMaxTickets];

struct TnRed {
  float* out;      // final [N][K] (null: separate split_reduce launches)
  float* mid;      // [groups][N][K] group sums (groups > 1)
  uint32_t* tick;  // this launch's tickets: [tiles][groups + 1]
  float beta;
  int ns, groups;
  const float* amax_y;  // FM 11 (fp16x3): device bounds of |Y| and |X| (operand scales)
  const float* amax_x;
  // FM 13 (fp16x3 on planes, 16-bit kernel): Y and X are each two fp16 planes h, l of the
  // operand times 2^e (e from its bound), the l plane yps / xps elements after the h plane
  int64_t yps, xps;
};

// sum rows n0..n0+TBN, cols k0..k0+TBK of nsrc [N][K] slices starting at src (slice stride
// N*K) in slice order; 256 threads, float4 per element group
template <int TBN, int TBK>
__device__ __forceinline__ void tn_tile_sum(const float* src, int nsrc, int64_t slice, int N, int K, int n0, int k0,
                                            float* dst, bool final_store, float beta, bool wt) {
  constexpr int C4 = TBK / 4;
  for (int e = threadIdx.x; e < TBN * C4; e += 256) {
    const int n = n0 + e / C4, k = k0 + (e % C4) * 4;
    const int64_t o = int64_t(n) * K + k;
    float4 a = *reinterpret_cast<const float4*>(src + o);
    for (int q = 1; q < nsrc; ++q) {
      const float4 b = *reinterpret_cast<const float4*>(src + int64_t(q) * slice + o);
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    if (final_store) {
      if (beta != 0.f) {
        const float4 c = *reinterpret_cast<const float4*>(dst + o);
        a.x += beta * c.x; a.y += beta * c.y; a.z += beta * c.z; a.w += beta * c.w;
      }
      *reinterpret_cast<float4*>(dst + o) = a;
    } else if (wt) {
      st_wt(dst + o, a.x); st_wt(dst + o + 1, a.y); st_wt(dst + o + 2, a.z); st_wt(dst + o + 3, a.w);
    } else {
      *reinterpret_cast<float4*>(dst + o) = a;
    }
  }
}

template <typename T, int TBN, int TBK, int STAGES, bool CONV, int FM = 0, int KR = kRows>
__global__ __launch_bounds__(256, 2) void gemm_tn_kernel(const T* __restrict__ Y, int64_t ldy,
                                                         const T* __restrict__ X, int64_t ldx,
                                                         float* __restrict__ part, int64_t M, int N, int K,
                                                         int64_t rows_per_split, int ntk, int ntiles, ConvGeo geo,
                                                         TnRed red) {
  // rows per staged step (KR = 64, bf16 only, MPIT_TN_KROWS=64: half the barriers and ring
  // turns per row for the memory-bound wgrads)
  constexpr int kRows = KR;
  constexpr int WN = TBN / 2, WK = TBK / 2;
  constexpr int TM = WN / 32, TN = WK / 32;
  constexpr int EPC = epc<T>();
  constexpr int CY = TBN / EPC, CX = TBK / EPC;        // 16-B chunks per row
  constexpr int RY = 64 / CY, RX = 64 / CX;           // rows per glds wave-instruction
  constexpr int IY = kRows / RY / 4, IX = kRows / RX / 4;  // glds per wave per tile
  // FM 13: 16-bit staging of TWO planes (h, l) per operand: images YH, YL, XH, XL
  constexpr bool P13 = FM == 13;
  constexpr int NPLT = P13 ? 2 : 1;
  constexpr int NI = (IY + IX) * NPLT;
  constexpr int TILE = kRows * (TBN + TBK) * NPLT;
  constexpr bool F32 = sizeof(T) == 4;
  static_assert(IY >= 1 && IX >= 1, "tile too small");
  static_assert(!P13 || (sizeof(T) == 2 && kTnBuf), "FM 13 is the 16-bit kernel on buffer descriptors");
  extern __shared__ __attribute__((aligned(16))) uint16_t smem_raw[];
  T* smem = reinterpret_cast<T*>(smem_raw);
  const T* zline = reinterpret_cast<const T*>(g_zero_line);

  const int id = xcd_tile(blockIdx.x, gridDim.x);
  const int tile = id % ntiles, split = id / ntiles;
  const int n0 = (tile / ntk) * TBN, k0 = (tile % ntk) * TBK;
  const int64_t r0 = int64_t(split) * rows_per_split;
  const int64_t r1 = min(M, r0 + rows_per_split);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wn = w >> 1, wk = w & 1;

  // Per-lane sources of each glds. Addresses advance incrementally by one step of kRows
  // rows (no per-step 64-bit multiplies: the VALU work between the MFMAs stays within
  // their issue shadow); rows past the split's end read the split's last row (the LDS
  // copy is zeroed before use). CONV: the column tile is channels [xc, xc + TBK) of tap
  // (xr, xs) and each lane tracks the output pixel (pn, pho, pwo) of its rows, advanced
  // by the step's (dn, dh, dw) decomposition of kRows with at most one carry per digit.
  const int nrows = int(r1 - r0);
  int ry[IY], rx[IX], ox[IX];
  const T* py[IY];
  const T* pyl[IY];
  const T* px[IX];
  const T* pxl[IX];
#pragma unroll
  for (int i = 0; i < IY; ++i) {
    ry[i] = (w * IY + i) * RY + lane / CY;
    const int oy = n0 + tswz<T, CY>(ry[i], lane % CY) * EPC;
    py[i] = Y + (r0 + ry[i]) * ldy + oy;
    pyl[i] = Y + (r1 - 1) * ldy + oy;
  }
#pragma unroll
  for (int i = 0; i < IX; ++i) {
    rx[i] = (w * IX + i) * RX + lane / CX;
    ox[i] = tswz<T, CX>(rx[i], lane % CX) * EPC;  // channel offset inside the tile
    if constexpr (!CONV) {
      px[i] = X + (r0 + rx[i]) * ldx + k0 + ox[i];
      pxl[i] = X + (r1 - 1) * ldx + k0 + ox[i];
    }
  }
  const int64_t ystep = int64_t(kRows) * ldy, xstep = int64_t(kRows) * ldx;
  int dn = 0, dh = 0, dw = 0;
  // CONV: tap (xr, xs) and element offset xc inside the tap of each lane's chunk
  // (per lane: a column tile may span taps when a tap is narrower than the tile, stem)
  int pn[IX], pho[IX], pwo[IX], xr[IX], xs[IX], xc[IX];
  const int pitch = geo.pitch ? geo.pitch : geo.C;
  if constexpr (CONV) {
#pragma unroll
    for (int i = 0; i < IX; ++i) {
      const int kcol = k0 + ox[i], tap = kcol / geo.C;
      xc[i] = kcol - tap * geo.C;
      xr[i] = tap / geo.S;
      xs[i] = tap - xr[i] * geo.S;
    }
    const int hw = geo.Ho * geo.Wo;
    dn = kRows / hw;
    dh = (kRows - dn * hw) / geo.Wo;
    dw = kRows - dn * hw - dh * geo.Wo;
#pragma unroll
    for (int i = 0; i < IX; ++i) {
      const int64_t m = r0 + rx[i];
      pn[i] = int(m / hw);
      const int rem = int(m - int64_t(pn[i]) * hw);
      pho[i] = rem / geo.Wo;
      pwo[i] = rem - pho[i] * geo.Wo;
    }
  }
  const int64_t nsteps = r1 > r0 ? (r1 - r0 + kRows - 1) / kRows : 0;
  // Buffer-descriptor staging (blds16, as gemm_nt): 32-bit lane offsets from uniform bases —
  // Y and plain X: the step's first row (the base moves per step in SALU; the descriptor
  // ends at the split's last row, so rows past it read zeros instead of re-reading that
  // row); CONV X: the split's first image, padding taps and rows past the split out of range.
  constexpr bool TBUF = kTnBuf;
  constexpr int TB = int(sizeof(T));
  [[maybe_unused]] uint32_t voy[TBUF ? IY : 1], vox[TBUF ? IX : 1];
  [[maybe_unused]] uint32_t lds0 = 0;
  [[maybe_unused]] uint64_t xbase = 0;
  [[maybe_unused]] int pn0 = 0;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  if constexpr (TBUF) {
    lds0 = __builtin_amdgcn_readfirstlane(uint32_t(reinterpret_cast<uintptr_t>((lds_void*)smem)));
#pragma unroll
    for (int i = 0; i < IY; ++i) voy[i] = uint32_t((ry[i] * ldy + tswz<T, CY>(ry[i], lane % CY) * EPC) * TB);
    if constexpr (CONV) {
      pn0 = int(r0 / (int64_t(geo.Ho) * geo.Wo));
      xbase = reinterpret_cast<uint64_t>(X) + uint64_t(int64_t(pn0) * geo.H * geo.W) * uint64_t(pitch) * TB;
    } else {
#pragma unroll
      for (int i = 0; i < IX; ++i) vox[i] = uint32_t((rx[i] * ldx + ox[i]) * TB);
    }
  }
  auto issue = [&](int64_t st, int buf) {
    T* Ys = smem + buf * TILE;
    T* Xs = Ys + kRows * TBN * NPLT;
    const int rs = int(st) * kRows;  // first row of the step, relative to r0
    if constexpr (TBUF) {
      // (the prologue's descriptors may come straight from a v_readfirstlane: 5 wait states)
      if (st < STAGES - 1) asm volatile("s_nop 4" ::: "memory");
      const int64_t left = int64_t(nrows - rs);
      const uint32_t ly = lds0 + uint32_t((buf * TILE + wu * IY * RY * TBN) * TB);
      const uint32_t ny = uint32_t(min<int64_t>(left * ldy * TB, int64_t(kBufOob)));
#pragma unroll
      for (int pl = 0; pl < NPLT; ++pl) {  // (FM 13: the h plane, then the l plane yps later)
        const i32x4 ry4 =
            buf_rsrc(reinterpret_cast<uint64_t>(Y) + uint64_t(((r0 + rs) * ldy + n0 + (P13 ? pl * red.yps : 0)) * TB), ny);
#pragma unroll
        for (int i = 0; i < IY; ++i) blds16(ry4, voy[i], ly + uint32_t((pl * kRows * TBN + i * RY * TBN) * TB));
      }
      const uint32_t lx = lds0 + uint32_t((buf * TILE + kRows * TBN * NPLT + wu * IX * RX * TBK) * TB);
      if constexpr (CONV) {
#pragma unroll
        for (int i = 0; i < IX; ++i) {
          const int hi = pho[i] * geo.stride - geo.pad + xr[i], wi = pwo[i] * geo.stride - geo.padw + xs[i];
          const bool ok = rs + rx[i] < nrows && unsigned(hi) < unsigned(geo.H) && unsigned(wi) < unsigned(geo.W);
          const uint32_t off = uint32_t(((((pn[i] - pn0) * geo.H + hi) * geo.W + wi) * pitch + xc[i]) * TB);
#pragma unroll
          for (int pl = 0; pl < NPLT; ++pl)
            blds16(buf_rsrc(xbase + uint64_t(P13 ? pl * red.xps : 0) * TB), ok ? off : kBufOob,
                   lx + uint32_t((pl * kRows * TBK + i * RX * TBK) * TB));
          pwo[i] += dw;  // next step's rows (issued strictly in order)
          const int cw = pwo[i] >= geo.Wo;
          pwo[i] -= cw ? geo.Wo : 0;
          pho[i] += dh + cw;
          const int ch = pho[i] >= geo.Ho;
          pho[i] -= ch ? geo.Ho : 0;
          pn[i] += dn + ch;
        }
      } else {
        const uint32_t nx = uint32_t(min<int64_t>(left * ldx * TB, int64_t(kBufOob)));
#pragma unroll
        for (int pl = 0; pl < NPLT; ++pl) {
          const i32x4 rx4 =
              buf_rsrc(reinterpret_cast<uint64_t>(X) + uint64_t(((r0 + rs) * ldx + k0 + (P13 ? pl * red.xps : 0)) * TB), nx);
#pragma unroll
          for (int i = 0; i < IX; ++i) blds16(rx4, vox[i], lx + uint32_t((pl * kRows * TBK + i * RX * TBK) * TB));
        }
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < IY; ++i) {
      glds16_asm(rs + ry[i] < nrows ? py[i] : pyl[i], Ys + (w * IY + i) * RY * TBN);
      py[i] += ystep;
    }
#pragma unroll
    for (int i = 0; i < IX; ++i) {
      if constexpr (CONV) {
        const int hi = pho[i] * geo.stride - geo.pad + xr[i], wi = pwo[i] * geo.stride - geo.padw + xs[i];
        const bool ok = rs + rx[i] < nrows && unsigned(hi) < unsigned(geo.H) && unsigned(wi) < unsigned(geo.W);
        const int off = ((pn[i] * geo.H + hi) * geo.W + wi) * pitch + xc[i];  // < 2^31 (host-checked)
        glds16_asm(ok ? X + off : zline + (ox[i] & (128 / int(sizeof(T)) - 1)), Xs + (w * IX + i) * RX * TBK);
        pwo[i] += dw;  // next step's rows (issued strictly in order)
        const int cw = pwo[i] >= geo.Wo;
        pwo[i] -= cw ? geo.Wo : 0;
        pho[i] += dh + cw;
        const int ch = pho[i] >= geo.Ho;
        pho[i] -= ch ? geo.Ho : 0;
        pn[i] += dn + ch;
      } else {
        glds16_asm(rs + rx[i] < nrows ? px[i] : pxl[i], Xs + (w * IX + i) * RX * TBK);
        px[i] += xstep;
      }
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;

  // transposed-read lane geometry: 16-lane group g, lane i = 4q + p of the group
  const int g = lane >> 4, gi = lane & 15, q = gi >> 2, p = gi & 3;
  const int h = g >> 1;
  const int cbase = 2 * (g & 1) + (p >> 1), cbyte = 4 * (p & 1);  // chunk / element offset in it
  const int fr = lane & 31, fh = lane >> 5;
  // fp32 split products (FM = 1, 11, 12, 13): the small-term accumulators
  constexpr bool LACC = F32 || P13;
  f32x16 lacc[LACC ? TM : 1][LACC ? TN : 1];
  [[maybe_unused]] int ey = 0, ex = 0;
  [[maybe_unused]] float sy = 1.f, sy11 = 2048.f, sx = 1.f, sx11 = 2048.f;
  if constexpr ((F32 && (FM == 11 || FM == 12)) || P13) {
    ey = fp16_exp(red.amax_y);
    ex = fp16_exp(red.amax_x);
    sy = exp2i(ey);
    sy11 = exp2i(ey + 11);
    sx = exp2i(ex);
    sx11 = exp2i(ex + 11);
  }
#pragma unroll
  for (int i = 0; i < (LACC ? TM : 1); ++i)
#pragma unroll
    for (int j = 0; j < (LACC ? TN : 1); ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) lacc[i][j][v] = 0.f;

#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nsteps) issue(s, s);
  for (int64_t st = 0; st < nsteps; ++st) {
    const int64_t after = min(nsteps, st + STAGES - 1) - (st + 1);
    if (STAGES >= 4 && after >= 2) wait_vmcnt<2 * NI>();
    else if (STAGES >= 3 && after >= 1) wait_vmcnt<NI>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int buf = int(st % STAGES);
    T* Ys = smem + buf * TILE;
    T* Xs = Ys + kRows * TBN * NPLT;
    const int64_t valid = r1 - (r0 + st * kRows);
    if (valid < kRows) {  // last, partial step of this split (nothing else in flight)
      constexpr int NYC = kRows * CY, NXC = kRows * CX;  // 16-B chunks of one Y / X image
      for (int e = t; e < NPLT * (NYC + NXC); e += 256) {
        const int row = e < NPLT * NYC ? (e % NYC) / CY : ((e - NPLT * NYC) % NXC) / CX;
        if (row >= valid) reinterpret_cast<uint4*>(Ys)[e] = make_uint4(0, 0, 0, 0);  // Xs follows Ys
      }
      __syncthreads();
    }
    if (st + STAGES - 1 < nsteps) issue(st + STAGES - 1, int((st + STAGES - 1) % STAGES));
    if constexpr (F32 && FM == 1) {
      // bf16x6 (see split3): lane (fr, fh) of a 16-row step holds Y[16kk + 8fh + j][n0' + fr]
      // and X[16kk + 8fh + j][k0' + fr], j = 0..7 — the k = 8fh + j operands of one
      // v_mfma_f32_32x32x16_bf16, read down a column (ds_read_b32, 32 consecutive floats
      // per half-wave: conflict-free) and split in registers
#pragma unroll
      for (int kk = 0; kk < kRows / 16; ++kk) {
        const int r0 = 16 * kk + 8 * fh;
        bf16x8 ah[TM], am[TM], al[TM], bh[TN], bm[TN], bl[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          float v[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = Ys[(r0 + e) * TBN + wn * WN + i * 32 + fr];
          split3(v, ah[i], am[i], al[i]);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          float v[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = Xs[(r0 + e) * TBK + wk * WK + j * 32 + fr];
          split3(v, bh[j], bm[j], bl[j]);
        }
        mfma_x3<TM, TN>(acc, lacc, ah, am, al, bh, bm, bl, false);
      }
    } else if constexpr (F32 && FM == 11) {
      // fp16x3 (see split2h): the same column reads, each operand scaled and split into fp16
      // h, l; hh -> acc, hl + lh -> lacc
#pragma unroll
      for (int kk = 0; kk < kRows / 16; ++kk) {
        const int r0 = 16 * kk + 8 * fh;
        f16x8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          float v[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = Ys[(r0 + e) * TBN + wn * WN + i * 32 + fr];
          split2h(v, sy, sy11, ah[i], al[i]);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          float v[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = Xs[(r0 + e) * TBK + wk * WK + j * 32 + fr];
          split2h(v, sx, sx11, bh[j], bl[j]);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
            lacc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], lacc[i][j], 0, 0, 0);
            lacc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], lacc[i][j], 0, 0, 0);
          }
      }
    } else if constexpr (F32 && FM == 12) {
      // fp16x3, split ONCE per element (FM 11 splits every element in each of the two waves
      // that read it, after 8 ds_read_b32 column reads per fragment): every thread takes its
      // share of this stage's fp32 rows (row-contiguous float4), the block barriers, and the
      // fp16 h / l planes of Y and X are written over the same ring slot in the bf16 kernel's
      // 16-bit image layout (swizzled 256-B rows); after a second barrier the fragments are
      // read exactly as the bf16 path reads them (ds_read_b64_tr_b16, two per fragment and
      // plane) — no per-use split, no column reads. Same planes as FM 11 (split2h's
      // arithmetic), so the same products; only the k order inside an MFMA differs.
      constexpr int NY4 = kRows * TBN / 4, NF4 = kRows * (TBN + TBK) / 4 / 256;
      constexpr int CY16 = TBN / 8, CX16 = TBK / 8;  // 16-B chunks per row of the 16-bit images
      static_assert(kRows * (TBN + TBK) % 1024 == 0, "the stage splits evenly over 256 threads");
#if !defined(MPIT_ABLATE_PLANES) && !defined(MPIT_ABLATE_PLANES_TN)  // (timing ablation: the staged rows taken as if they were the planes)
      float4 v4[NF4];
      const float4* src4 = reinterpret_cast<const float4*>(Ys);
#pragma unroll
      for (int u = 0; u < NF4; ++u) v4[u] = src4[t + 256 * u];
      // every thread holds its fp32 values: the slot takes the planes. LDS-only barriers:
      // a __syncthreads() here waits vmcnt(0), i.e. for the next stage's LDS DMA issued at
      // the top of this step, and the ring never overlaps a load with the MFMAs
      lds_barrier();
      uint16_t* YH = reinterpret_cast<uint16_t*>(Ys);
      uint16_t* YL = YH + kRows * TBN;
      uint16_t* XH = YL + kRows * TBN;
      uint16_t* XL = XH + kRows * TBK;
#pragma unroll
      for (int u = 0; u < NF4; ++u) {
        const int e = t + 256 * u;
        const bool isy = e < NY4;  // (uniform per wave: NY4 is a multiple of 64)
        const int e2 = isy ? e : e - NY4;
        const int cpr = (isy ? TBN : TBK) / 4;  // float4 per row
        const int row = e2 / cpr, c4 = e2 - row * cpr;
        const float sc = isy ? sy : sx, sc11 = isy ? sy11 : sx11;
        const float4 x = v4[u];
        const f32x2 x01 = {x.x, x.y}, x23 = {x.z, x.w};
        const f16x2 h01 = __builtin_convertvector(x01 * sc, f16x2), h23 = __builtin_convertvector(x23 * sc, f16x2);
        const f32x2 r01 = x01 * sc11 - __builtin_convertvector(h01, f32x2) * 2048.f;
        const f32x2 r23 = x23 * sc11 - __builtin_convertvector(h23, f32x2) * 2048.f;
        const f16x2 l01 = __builtin_convertvector(r01, f16x2), l23 = __builtin_convertvector(r23, f16x2);
        uint2 hw, lw;
        hw.x = __builtin_bit_cast(uint32_t, h01);
        hw.y = __builtin_bit_cast(uint32_t, h23);
        lw.x = __builtin_bit_cast(uint32_t, l01);
        lw.y = __builtin_bit_cast(uint32_t, l23);
        const int o = isy ? row * TBN + tswz<uint16_t, CY16>(row, c4 >> 1) * 8 + (c4 & 1) * 4
                          : row * TBK + tswz<uint16_t, CX16>(row, c4 >> 1) * 8 + (c4 & 1) * 4;
        *reinterpret_cast<uint2*>((isy ? YH : XH) + o) = hw;
        *reinterpret_cast<uint2*>((isy ? YL : XL) + o) = lw;
      }
      lds_barrier();
#else
      uint16_t* YH = reinterpret_cast<uint16_t*>(Ys);
      uint16_t* YL = YH + kRows * TBN;
      uint16_t* XH = YL + kRows * TBN;
      uint16_t* XL = XH + kRows * TBK;
#endif
#pragma unroll
      for (int kk = 0; kk < kRows / 16; ++kk) {
        const int rr = 16 * kk + 8 * h + q;  // row of this lane in the first 4-row block
        f16x8 ah[TM], al[TM], bh[TN], bl[TN];
        auto frag = [&](const uint16_t* img, int ld, int ch, auto cy) -> f16x8 {
          constexpr int CPR = decltype(cy)::value;
          const s16x4 lo = ds_tr16(img + rr * ld + tswz<uint16_t, CPR>(rr, ch) * 8 + cbyte);
          const s16x4 hi = ds_tr16(img + (rr + 4) * ld + tswz<uint16_t, CPR>(rr + 4, ch) * 8 + cbyte);
          return __builtin_bit_cast(f16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        };
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int ch = (wn * WN + i * 32) / 8 + cbase;
          ah[i] = frag(YH, TBN, ch, std::integral_constant<int, CY16>{});
          al[i] = frag(YL, TBN, ch, std::integral_constant<int, CY16>{});
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int ch = (wk * WK + j * 32) / 8 + cbase;
          bh[j] = frag(XH, TBK, ch, std::integral_constant<int, CX16>{});
          bl[j] = frag(XL, TBK, ch, std::integral_constant<int, CX16>{});
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
            lacc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], lacc[i][j], 0, 0, 0);
            lacc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], lacc[i][j], 0, 0, 0);
          }
      }
    } else if constexpr (P13) {
      // fp16x3 on planes: the staged images are FM 12's after its split (same layout, same
      // transposed fragment reads), DMA'd straight from the producers' planes
      const uint16_t* YH = Ys;
      const uint16_t* YL = YH + kRows * TBN;
      const uint16_t* XH = Xs;
      const uint16_t* XL = XH + kRows * TBK;
#pragma unroll
      for (int kk = 0; kk < kRows / 16; ++kk) {
        const int rr = 16 * kk + 8 * h + q;  // row of this lane in the first 4-row block
        f16x8 ah[TM], al[TM], bh[TN], bl[TN];
        auto frag = [&](const uint16_t* img, int ld, int ch, auto cy) -> f16x8 {
          constexpr int CPR = decltype(cy)::value;
          const s16x4 lo = ds_tr16(img + rr * ld + tswz<uint16_t, CPR>(rr, ch) * 8 + cbyte);
          const s16x4 hi = ds_tr16(img + (rr + 4) * ld + tswz<uint16_t, CPR>(rr + 4, ch) * 8 + cbyte);
          return __builtin_bit_cast(f16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        };
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int ch = (wn * WN + i * 32) / 8 + cbase;
          ah[i] = frag(YH, TBN, ch, std::integral_constant<int, CY>{});
          al[i] = frag(YL, TBN, ch, std::integral_constant<int, CY>{});
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int ch = (wk * WK + j * 32) / 8 + cbase;
          bh[j] = frag(XH, TBK, ch, std::integral_constant<int, CX>{});
          bl[j] = frag(XL, TBK, ch, std::integral_constant<int, CX>{});
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
            lacc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], lacc[i][j], 0, 0, 0);
            lacc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], lacc[i][j], 0, 0, 0);
          }
      }
    } else if constexpr (F32) {
      // v_mfma_f32_32x32x2_f32: lane (fr, fh) supplies Y[row][n0' + fr] and X[row][k0' + fr]
      // of row 2s + fh in step s (32 consecutive floats per half-wave: ds_read_b32, no
      // conflicts). Each staged step is one fresh 32-long fmaf chain folded into acc (blocked
      // accumulation, as gemm_nt's fp32 loop).
      f32x16 tacc[TM][TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int v = 0; v < 16; ++v) tacc[i][j][v] = 0.f;
#pragma unroll
      for (int s = 0; s < kRows / 2; ++s) {
        const int rrow = 2 * s + fh;
        float af[TM], bfg[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = Ys[rrow * TBN + wn * WN + i * 32 + fr];
#pragma unroll
        for (int j = 0; j < TN; ++j) bfg[j] = Xs[rrow * TBK + wk * WK + j * 32 + fr];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) tacc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bfg[j], tacc[i][j], 0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] += tacc[i][j];
    } else {
#pragma unroll
    for (int kk = 0; kk < kRows / 16; ++kk) {
      const int rr = 16 * kk + 8 * h + q;  // row of this lane in the first 4-row block
      bf16x8 af[TM], bfg[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int ch = (wn * WN + i * 32) / 8 + cbase;
        const s16x4 lo = ds_tr16(Ys + rr * TBN + tswz<T, CY>(rr, ch) * 8 + cbyte);
        const s16x4 hi = ds_tr16(Ys + (rr + 4) * TBN + tswz<T, CY>(rr + 4, ch) * 8 + cbyte);
        af[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int ch = (wk * WK + j * 32) / 8 + cbase;
        const s16x4 lo = ds_tr16(Xs + rr * TBK + tswz<T, CX>(rr, ch) * 8 + cbyte);
        const s16x4 hi = ds_tr16(Xs + (rr + 4) * TBK + tswz<T, CX>(rr + 4, ch) * 8 + cbyte);
        bfg[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfg[j], acc[i][j], 0, 0, 0);
    }
    }
  }
  if constexpr (F32 && FM == 1) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] += lacc[i][j];
  } else if constexpr ((F32 && (FM == 11 || FM == 12)) || P13) {
    const float iy = exp2i(-ey), ix = exp2i(-ex);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[i][j][v] = fmaf(lacc[i][j][v], 1.f / 2048.f, acc[i][j][v]) * iy * ix;
  }
  // D[n][k]: column k = lane&31, row n = (v&3) + 8*(v>>2) + 4*(lane>>5)
  float* out = part + int64_t(split) * N * K;
  const bool fused = red.tick != nullptr;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int n = n0 + wn * WN + i * 32 + (v & 3) + 8 * (v >> 2) + 4 * fh;
        const int k = k0 + wk * WK + j * 32 + fr;
        if (fused) st_wt(out + int64_t(n) * K + k, acc[i][j][v]);
        else out[int64_t(n) * K + k] = acc[i][j][v];
      }
  if (!fused) return;
  __shared__ uint32_t prev;
  const int64_t slice = int64_t(N) * K;
  const int grp = split / kReduceGroup, g0 = grp * kReduceGroup, gn = min(red.ns, g0 + kReduceGroup) - g0;
  uint32_t* tk = red.tick + int64_t(tile) * (red.groups + 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) prev = atomicAdd(&tk[grp], 1u);
  __syncthreads();
  if (prev != uint32_t(gn - 1)) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(&tk[grp], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (red.groups == 1) {  // one level: the group sum is the result
    tn_tile_sum<TBN, TBK>(part + int64_t(g0) * slice, gn, slice, N, K, n0, k0, red.out, true, red.beta, false);
    return;
  }
  tn_tile_sum<TBN, TBK>(part + int64_t(g0) * slice, gn, slice, N, K, n0, k0, red.mid + int64_t(grp) * slice, false,
                        0.f, true);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) prev = atomicAdd(&tk[red.groups], 1u);
  __syncthreads();
  if (prev != uint32_t(red.groups - 1)) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(&tk[red.groups], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  tn_tile_sum<TBN, TBK>(red.mid, red.groups, slice, N, K, n0, k0, red.out, true, red.beta, false);
}

// fp32 backward-weight GEMM with the operand split done ONCE per element (round 3):
// dW[n][k] = sum_m Y[m][n] X[m][k] over a 128 x 128 tile, rows in steps of 16.
// The fp32 rows of the next step are staged in registers (each thread: 8 consecutive rows x
// 2 adjacent columns, float2 loads — a wave covers 512 contiguous bytes per row), split
// into the three bf16 planes h, m, l (split3: x = h + m + l) and written k-contiguous into
// an LDS image [plane][column][16 k] — the transposition the MFMA fragments need (8
// consecutive rows of one column) happens in that write, so every fragment is one
// ds_read_b128 per plane. gemm_tn_kernel's fp32 path instead splits each element twice (two
// waves read it) and reads each fragment with 8 ds_read_b32. Two LDS images alternate: the
// split of step s + 1 and the MFMAs of step s run between the same pair of barriers.
// MEASURED SLOWER than gemm_tn_kernel (profiles/wgrad_split_once_r03.md), so opt-in:
// MPIT_TN_F32S=1.
// Same planes, same MFMA sequence per output tile (mfma_x3), same k order: bitwise equal
// to gemm_tn_kernel's bf16x6 path. CONV: X is the implicit im2col of an NHWC image, one tap
// per column tile (C % 128 == 0); each thread tracks the output pixel of its first row.
constexpr int kTsR = 16;  // rows per step
// bf16 offset of (column c, k-half kh) in one plane of the image: 16-B chunk ch = 2c + kh,
// bits 0..2 XORed with bits 2..4. Conflict-free both ways (exhaustive check over the lane
// groups of MI355X_MICROARCH's LDS table): a ds_write_b128 group of 8 consecutive lanes
// (chunks 4l + d) hits 8 distinct 16-B slots of 128 B, and a ds_read_b128 group of 16
// fragment lanes (chunks 2(c0 + fr) + kh) 16 distinct slots of 256 B.
__device__ __forceinline__ int tsc(int c, int kh) {
  const int ch = 2 * c + kh;
  return (ch ^ ((ch >> 2) & 7)) * 8;
}
template <bool CONV>
__global__ __launch_bounds__(256, 2) void gemm_tn_f32s_kernel(const float* __restrict__ Y, int64_t ldy,
                                                              const float* __restrict__ X, int64_t ldx,
                                                              float* __restrict__ part, int64_t M, int N, int K,
                                                              int64_t rows_per_split, int ntk, int ntiles, ConvGeo geo) {
  constexpr int TB = 128, TM = 2, TN = 2, WN = 64, WK = 64;
  constexpr int IMG = 3 * 256 * kTsR;  // bf16 elements of one LDS image
  extern __shared__ __attribute__((aligned(16))) uint16_t smem_raw[];
  const int id = xcd_tile(blockIdx.x, gridDim.x);
  const int tile = id % ntiles, split = id / ntiles;
  const int n0 = (tile / ntk) * TB, k0 = (tile % ntk) * TB;
  const int64_t r0 = int64_t(split) * rows_per_split;
  const int64_t r1 = min(M, r0 + rows_per_split);
  const int nrows = int(max<int64_t>(0, r1 - r0));
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wn = w >> 1, wk = w & 1;
  const int fr = lane & 31, fh = lane >> 5;
  // staging role: waves 0, 1 stage Y, waves 2, 3 stage X; rows 8*(w & 1) .. +7 of a step;
  // columns 2*lane, 2*lane + 1 of the tile
  const bool isx = w >= 2;
  const int rh = w & 1;
  const int col = 2 * lane;
  const float* src = isx ? (X + (CONV ? 0 : k0 + col)) : (Y + n0 + col);
  const int64_t ld = isx ? ldx : ldy;
  // CONV: this column tile's tap (xr, xs) and channel offset, and the output pixel of the
  // thread's first row of the current step
  int xr = 0, xs = 0, xc = 0, pn = 0, pho = 0, pwo = 0, dn = 0, dh = 0, dw = 0;
  if constexpr (CONV) {
    const int tap = k0 / geo.C;
    xc = k0 - tap * geo.C + col;
    xr = tap / geo.S;
    xs = tap - xr * geo.S;
    const int hw = geo.Ho * geo.Wo;
    const int64_t m = r0 + 8 * rh;
    pn = int(m / hw);
    const int rem = int(m - int64_t(pn) * hw);
    pho = rem / geo.Wo;
    pwo = rem - pho * geo.Wo;
    dn = kTsR / hw;
    dh = (kTsR - dn * hw) / geo.Wo;
    dw = kTsR - dn * hw - dh * geo.Wo;
  }
  const int64_t nsteps = (nrows + kTsR - 1) / kTsR;

  // the thread's 8 rows of step st (zeros past the split's end / for padding taps)
  auto load = [&](int64_t st, f32x2 (&rg)[8]) {
    const int rb = int(st) * kTsR + 8 * rh;
    if constexpr (CONV) {
      if (isx) {
        int n = pn, ho = pho, wo = pwo;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int hi = ho * geo.stride - geo.pad + xr, wi = wo * geo.stride - geo.padw + xs;
          const bool ok = rb + e < nrows && unsigned(hi) < unsigned(geo.H) && unsigned(wi) < unsigned(geo.W);
          rg[e] = ok ? *reinterpret_cast<const f32x2*>(src + ((int64_t(n) * geo.H + hi) * geo.W + wi) * geo.C + xc)
                     : f32x2{0.f, 0.f};
          if (++wo == geo.Wo) {
            wo = 0;
            if (++ho == geo.Ho) {
              ho = 0;
              ++n;
            }
          }
        }
        // next step's first row: + kTsR rows (at most one carry per digit)
        pwo += dw;
        const int cw = pwo >= geo.Wo;
        pwo -= cw ? geo.Wo : 0;
        pho += dh + cw;
        const int ch = pho >= geo.Ho;
        pho -= ch ? geo.Ho : 0;
        pn += dn + ch;
        return;
      }
    }
    const float* p = src + (r0 + rb) * ld;
#pragma unroll
    for (int e = 0; e < 8; ++e)
      rg[e] = rb + e < nrows ? *reinterpret_cast<const f32x2*>(p + int64_t(e) * ld) : f32x2{0.f, 0.f};
  };
  // split the staged rows and write both columns' planes (k-contiguous) into image `buf`
  auto store = [&](const f32x2 (&rg)[8], int buf) {
    uint16_t* img = smem_raw + buf * IMG;
    const int cc = (isx ? 128 : 0) + col;  // image column of the first of the two
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = rg[e][j];
      bf16x8 h, m, l;
      split3(v, h, m, l);
      const int o = tsc(cc + j, rh);
      *reinterpret_cast<bf16x8*>(img + o) = h;
      *reinterpret_cast<bf16x8*>(img + 256 * kTsR + o) = m;
      *reinterpret_cast<bf16x8*>(img + 2 * 256 * kTsR + o) = l;
    }
  };
  f32x16 acc[TM][TN], lacc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][j][v] = lacc[i][j][v] = 0.f;
  // the 24 MFMAs of step st from image `buf`
  auto mma = [&](int buf) {
    const uint16_t* img = smem_raw + buf * IMG;
    bf16x8 ah[TM], am[TM], al[TM], bh[TN], bm[TN], bl[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int o = tsc(wn * WN + i * 32 + fr, fh);
      ah[i] = *reinterpret_cast<const bf16x8*>(img + o);
      am[i] = *reinterpret_cast<const bf16x8*>(img + 256 * kTsR + o);
      al[i] = *reinterpret_cast<const bf16x8*>(img + 2 * 256 * kTsR + o);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int o = tsc(128 + wk * WK + j * 32 + fr, fh);
      bh[j] = *reinterpret_cast<const bf16x8*>(img + o);
      bm[j] = *reinterpret_cast<const bf16x8*>(img + 256 * kTsR + o);
      bl[j] = *reinterpret_cast<const bf16x8*>(img + 2 * 256 * kTsR + o);
    }
    mfma_x3<TM, TN>(acc, lacc, ah, am, al, bh, bm, bl, false);
  };
  auto sync = [] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // three register sets: the rows of step s + 3 are requested while step s computes, so a
  // load has two steps (two barriers) to arrive before its split; images alternate per step
  f32x2 q0[8], q1[8], q2[8];
  if (nsteps > 0) load(0, q0);
  if (nsteps > 1) load(1, q1);
  if (nsteps > 2) load(2, q2);
  if (nsteps > 0) store(q0, 0);
  sync();
  auto phase = [&](int64_t s, f32x2 (&rl)[8], const f32x2 (&rs)[8], int ib) {
    if (s + 3 < nsteps) load(s + 3, rl);
    mma(ib);
    if (s + 1 < nsteps) store(rs, ib ^ 1);
    sync();
  };
  // unrolled by 6 so the register sets keep static names: step s uses set s % 3, image s % 2
  for (int64_t st = 0; st < nsteps; st += 6) {
    phase(st, q0, q1, 0);
    if (st + 1 >= nsteps) break;
    phase(st + 1, q1, q2, 1);
    if (st + 2 >= nsteps) break;
    phase(st + 2, q2, q0, 0);
    if (st + 3 >= nsteps) break;
    phase(st + 3, q0, q1, 1);
    if (st + 4 >= nsteps) break;
    phase(st + 4, q1, q2, 0);
    if (st + 5 >= nsteps) break;
    phase(st + 5, q2, q0, 1);
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] += lacc[i][j];
  // D[n][k]: column k = lane&31, row n = (v&3) + 8*(v>>2) + 4*(lane>>5) (gemm_tn_kernel's map)
  float* out = part + int64_t(split) * N * K;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int n = n0 + wn * WN + i * 32 + (v & 3) + 8 * (v >> 2) + 4 * fh;
        const int k = k0 + wk * WK + j * 32 + fr;
        out[int64_t(n) * K + k] = acc[i][j][v];
      }
}

// Split reduction, one level: block (x, y) sums splits [y*G, y*G+G) of its float4
// lanes into out2[y] (or, when gridDim.y == 1, into out with out = beta*out + sum).
__global__ __launch_bounds__(256) void split_reduce_kernel(const float4* __restrict__ part, int nsplit, int64_t n4,
                                                           float4* __restrict__ out, float beta) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const int s0 = blockIdx.y * kReduceGroup, s1 = min(nsplit, s0 + kReduceGroup);
  float4 a = part[int64_t(s0) * n4 + i];
#pragma unroll 8
  for (int s = s0 + 1; s < s1; ++s) {
    const float4 b = part[int64_t(s) * n4 + i];
    a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
  }
  if (gridDim.y > 1) {
    out[int64_t(blockIdx.y) * n4 + i] = a;
    return;
  }
  if (beta != 0.f) {
    const float4 o = out[i];
    a.x += beta * o.x; a.y += beta * o.y; a.z += beta * o.z; a.w += beta * o.w;
  }
  out[i] = a;
}

// fp32 w[R][T][Cc] -> bf16 copy wb[R][T][Cc] and a bf16 transpose wt with the taps
// rearranged by `map`: tap t goes to wt[base[t] + (c*tc[t] + dt[t])*R + r]. The default
// map (base 0, tc T, dt T-1-t) is the tap-flipped transpose [Cc][T][R] of a stride-1
// backward-data; the parity classes of a strided one get one block each.
// Tap t = blockIdx.z.
constexpr int kMaxTaps = 49;
struct TapMap {
  int64_t base[kMaxTaps];
  int16_t tc[kMaxTaps], dt[kMaxTaps];
};

// one 32 x 32 (channel x row) tile of tap `tap`, 256 threads. O = output element type:
// uint16_t (bf16 cast + transpose) or float (fp32 transpose; the plain copy is the master
// weight itself, so wb is null).
template <typename O>
__device__ __forceinline__ O cvt_out(float v) {
  if constexpr (sizeof(O) == 2) return f2bf(v);
  else return v;
}
template <typename O>
__device__ __forceinline__ void cast_tile(const float* __restrict__ w, int R, int Cc, int T, O* __restrict__ wb,
                                          O* __restrict__ wt, const TapMap& map, int cx, int ry, int tap, int ldt) {
  __shared__ O tile[32][33];
  const int c0 = cx * 32, r0 = ry * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 8 rows per pass
  for (int y = ty; y < 32; y += 8) {
    const int r = r0 + y, c = c0 + tx;
    if (r < R && c < Cc) {
      const int64_t i = (int64_t(r) * T + tap) * Cc + c;
      const O b = cvt_out<O>(w[i]);
      if (wb) wb[i] = b;
      tile[y][tx] = b;
    }
  }
  __syncthreads();
  if (!wt) return;
  const int64_t base = map.base[tap];
  const int tc = map.tc[tap], dt = map.dt[tap];
  for (int y = ty; y < 32; y += 8) {
    const int c = c0 + y, r = r0 + tx;
    if (r < R && c < Cc) wt[base + (int64_t(c) * tc + dt) * ldt + r] = tile[tx][y];
  }
}

// A large 1-tap weight's bf16 transpose only (the classifier layers, ops/linear.py): one
// 128 (rows of w) x 64 (columns) tile per block. Eight float4 row reads in flight per thread
// (256-B row segments), 8-byte packed bf16 writes covering 256-B output row segments. The
// 32 x 32 scalar tile above moves VGG-16's 411 MB fc1 weight at ~1.2 TB/s, a 64 x 64 vector
// tile with 4 reads in flight at ~1.7 TB/s (r05i). Host-checked: R % 128, Cc % 64, w 16-B aligned.
__device__ __forceinline__ void cast_tile64_t(const float* __restrict__ w, int R, int Cc, uint16_t* __restrict__ wt,
                                              int cx, int ry) {
  __shared__ float tile[128][65];
  const int c0 = cx * 64, r0 = ry * 128;
  const int t = threadIdx.x;
  {
    const int cc = (t & 15) * 4, rr = t >> 4;
    float4 v[8];
#pragma unroll
    for (int p = 0; p < 8; ++p)
      v[p] = *reinterpret_cast<const float4*>(w + int64_t(r0 + rr + 16 * p) * Cc + c0 + cc);
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int r = rr + 16 * p;
      tile[r][cc] = v[p].x;
      tile[r][cc + 1] = v[p].y;
      tile[r][cc + 2] = v[p].z;
      tile[r][cc + 3] = v[p].w;
    }
  }
  __syncthreads();
  const int rc = (t & 31) * 4, cr = t >> 5;
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int c = cr + 8 * p;
    const uint32_t lo = uint32_t(f2bf(tile[rc][c])) | (uint32_t(f2bf(tile[rc + 1][c])) << 16);
    const uint32_t hi = uint32_t(f2bf(tile[rc + 2][c])) | (uint32_t(f2bf(tile[rc + 3][c])) << 16);
    *reinterpret_cast<uint2*>(wt + int64_t(c0 + c) * R + r0 + rc) = make_uint2(lo, hi);
  }
}

// The bf16x6 operand split of one fp32 value: h = bf16(v), m = bf16(v - h), l = bf16(v - h - m)
// (round to nearest; for normal numbers v == h + m + l exactly) — split3's arithmetic.
__device__ __forceinline__ void split1(float v, uint16_t& h, uint16_t& m, uint16_t& l) {
  h = f2bf(v);
  const float r = v - bf2f(h);
  m = f2bf(r);
  l = f2bf(r - bf2f(m));
}

// cast_tile for the pre-split fp32 path: the same copy / transpose, written as three bf16
// planes (h at p, m at p + plane, l at p + 2 * plane) for the FM 4 GEMMs. wb: planes or
// null; wt: planes (pt > 0) or plain fp32 (pt == 0: the GEMM reading it splits in registers)
// f16 (fp16x3 plans): two fp16 planes h, l of the weight scaled by s = 2^e (s11 = 2^(e + 11)),
// split1h's arithmetic, instead of the three bf16 ones.
__device__ __forceinline__ void cast_tile_planes(const float* __restrict__ w, int R, int Cc, int T,
                                                 uint16_t* __restrict__ wb, int64_t pb, void* __restrict__ wt_,
                                                 int64_t pt, const TapMap& map, int cx, int ry, int tap, bool f16,
                                                 float s, float s11) {
  __shared__ float tile[32][33];
  const int c0 = cx * 32, r0 = ry * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int y = ty; y < 32; y += 8) {
    const int r = r0 + y, c = c0 + tx;
    if (r < R && c < Cc) {
      const int64_t i = (int64_t(r) * T + tap) * Cc + c;
      const float v = w[i];
      if (wb && f16) {
        uint16_t h, l;
        split1h(v, s, s11, h, l);
        wb[i] = h;
        wb[pb + i] = l;
      } else if (wb) {
        uint16_t h, m, l;
        split1(v, h, m, l);
        wb[i] = h;
        wb[pb + i] = m;
        wb[2 * pb + i] = l;
      }
      tile[y][tx] = v;
    }
  }
  __syncthreads();
  if (!wt_) return;
  const int64_t base = map.base[tap];
  const int tc = map.tc[tap], dt = map.dt[tap];
  for (int y = ty; y < 32; y += 8) {
    const int c = c0 + y, r = r0 + tx;
    if (r < R && c < Cc) {
      const int64_t o = base + (int64_t(c) * tc + dt) * R + r;
      if (pt == 0) {
        static_cast<float*>(wt_)[o] = tile[tx][y];
        continue;
      }
      uint16_t* wt = static_cast<uint16_t*>(wt_);
      if (f16) {
        uint16_t h, l;
        split1h(tile[tx][y], s, s11, h, l);
        wt[o] = h;
        wt[pt + o] = l;
        continue;
      }
      uint16_t h, m, l;
      split1(tile[tx][y], h, m, l);
      wt[o] = h;
      wt[pt + o] = m;
      wt[2 * pt + o] = l;
    }
  }
}

template <typename O>
__global__ __launch_bounds__(256) void cast_transpose_kernel(const float* __restrict__ w, int R, int Cc, int T,
                                                             O* __restrict__ wb, O* __restrict__ wt, TapMap map) {
  cast_tile<O>(w, R, Cc, T, wb, wt, map, blockIdx.x, blockIdx.y, blockIdx.z, R);
}

// Every convolution weight of a model in one launch (the per-step bf16 casts of the fp32
// master weights, or the fp32 transposes of an fp32 step): block b belongs to the job whose
// block0 is the largest <= b.
struct CastJob {
  const float* w;
  void* wb;
  void* wt;
  int R, Cc, T, tcx, tcy;  // tiles along Cc and R
  int big;                 // cast_tile64_t (64 x 64 tiles: a large 1-tap bf16 transpose only)
  int f32;                 // outputs: 0 bf16, 1 fp32 (no plain copy), 2 pre-split planes
  int f16;                 // (f32 == 2) planes are fp16 h, l of the weight scaled by amax's 2^e
  const float* amax;       // (f16) device upper bound of |w| over the plan
  int64_t block0;
  int64_t pb, pt;          // plane strides (elements) of wb / wt when f32 == 2
  int ldt;                 // row length of a plain transpose wt (R, or a padded classifier's Np)
  TapMap map;
};

// The fp16-plane jobs' bound, max |w| over every such weight of the plan (one pass before
// cast_batch_kernel, which derives the planes' scale from it): block b of job j (the same
// block -> job map) strides over the job's R * Cc * T weights, reduces its maximum and issues
// ONE fire-and-forget atomic max into slot b % kBoundSlots of J.amax (zeroed by the launch).
// Replaces the per-step torch _foreach_norm + stack + amax chain (several launches with host
// gaps between them at the step boundary).
__global__ __launch_bounds__(256) void cast_amax_kernel(const CastJob* __restrict__ jobs, int njobs, int64_t nblocks) {
  __shared__ int jsel;
  __shared__ float red[4];
  if (threadIdx.x == 0) {
    int lo = 0, hi = njobs - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (jobs[mid].block0 <= int64_t(blockIdx.x)) lo = mid;
      else hi = mid - 1;
    }
    jsel = lo;
  }
  __syncthreads();
  const CastJob& J = jobs[jsel];
  if (!(J.f32 == 2 && J.f16)) return;  // uniform per block
  const int64_t nbj = (jsel + 1 < njobs ? jobs[jsel + 1].block0 : nblocks) - J.block0;
  const int64_t n = int64_t(J.R) * J.Cc * J.T;
  float m = 0.f;
  for (int64_t i = (int64_t(blockIdx.x) - J.block0) * 256 + threadIdx.x; i < n; i += nbj * 256)
    m = fmaxf(m, fabsf(J.w[i]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float b = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    atomicMax(reinterpret_cast<unsigned int*>(const_cast<float*>(J.amax) + (blockIdx.x % kBoundSlots) * kBoundStride),
              __float_as_uint(b));
  }
}

__global__ __launch_bounds__(256) void cast_batch_kernel(const CastJob* __restrict__ jobs, int njobs) {
  __shared__ int jsel;
  if (threadIdx.x == 0) {
    int lo = 0, hi = njobs - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (jobs[mid].block0 <= int64_t(blockIdx.x)) lo = mid;
      else hi = mid - 1;
    }
    jsel = lo;
  }
  __syncthreads();
  const CastJob& J = jobs[jsel];
  const int64_t local = int64_t(blockIdx.x) - J.block0;
  const int per_tap = J.tcx * J.tcy;
  const int tap = int(local / per_tap), rem = int(local % per_tap);
  if (J.big) {
    // row bands fastest: the blocks in flight together read 64-column strips of every input
    // row and write whole 8-KB output rows (column tiles fastest scattered the writes over
    // every output row: ~1.8 TB/s for VGG-16's fc1 weight, r05j)
    cast_tile64_t(J.w, J.R, J.Cc, static_cast<uint16_t*>(J.wt), rem / J.tcy, rem % J.tcy);
  } else if (J.f32 == 2) {
    float sc = 1.f, sc11 = 2048.f;
    if (J.f16) {
      const int e = fp16_exp(J.amax);
      sc = exp2i(e);
      sc11 = exp2i(e + 11);
    }
    cast_tile_planes(J.w, J.R, J.Cc, J.T, static_cast<uint16_t*>(J.wb), J.pb, J.wt, J.pt, J.map, rem % J.tcx,
                     rem / J.tcx, tap, J.f16 != 0, sc, sc11);
  }
  else if (J.f32)
    cast_tile<float>(J.w, J.R, J.Cc, J.T, static_cast<float*>(J.wb), static_cast<float*>(J.wt), J.map, rem % J.tcx,
                     rem / J.tcx, tap, J.ldt);
  else
    cast_tile<uint16_t>(J.w, J.R, J.Cc, J.T, static_cast<uint16_t*>(J.wb), static_cast<uint16_t*>(J.wt), J.map,
                        rem % J.tcx, rem / J.tcx, tap, J.ldt);
}

void check_ptr(uintptr_t p, const char* what) {
  if (p % 16) throw std::invalid_argument(std::string("gemm: ") + what + " must be 16-byte aligned");
}

int cu_count(int dev) {
  static int cached[64] = {0};
  if (dev < 0 || dev >= 64) return 256;
  if (!cached[dev]) {
    int v = 0;
    hip_check(hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev), "hipDeviceGetAttribute");
    cached[dev] = v > 0 ? v : 256;
  }
  return cached[dev];
}

}  // namespace

int device_cu_count(int dev) { return cu_count(dev); }

// A stream whose dispatches only use the CUs set in `mask` (bit i of word i / 32 = CU i).
// The backward-weight side stream runs on such a stream so a few CUs stay free for the
// critical path's small kernels (BN finalize / apply) instead of queueing behind
// side-stream GEMM blocks that hold every CU's registers (ops/conv.py WgradStream).
uintptr_t stream_create_cu_masked(int dev, const std::vector<uint32_t>& mask) {
  if (mask.empty()) throw std::invalid_argument("stream_create_cu_masked: empty mask");
  hip_check(hipSetDevice(dev), "hipSetDevice");
  hipStream_t s = nullptr;
  hip_check(hipExtStreamCreateWithCUMask(&s, uint32_t(mask.size()), mask.data()), "hipExtStreamCreateWithCUMask");
  return reinterpret_cast<uintptr_t>(s);
}

bool gemm_nt_supported(int64_t M, int N, int K, bool f32) {
  return M > 0 && N > 0 && K > 0 && N % 64 == 0 && K % (f32 ? 16 : kBK) == 0;
}

int64_t gemm_nt_stats_floats(int64_t M, int N) { return gemm_nt_tiles(M) * 2 * int64_t(N); }

int64_t gemm_nt_tiles(int64_t M) { return (M + 127) / 128; }

int64_t gemm_nt_fold_lvl_floats(int N) { return int64_t(kFoldMaxGroups) * 3 * N; }

// Block tile of gemm_nt: 0 = 128 x (128 | 64), 1 = 256 x 128, 2 = 256 x 256;
// MPIT_GEMM_TILE=128|256x128|256 selects one (A/B runs, large plain GEMMs). fp32 runs the
// 128-row tiles only (its MFMA is 16x slower per FLOP: LDS-bound tile shapes do not matter).
static int nt_tile_config(int64_t M, int N, int K, bool conv, int cin_conv, bool f32) {
  static const int forced = [] {
    const char* e = std::getenv("MPIT_GEMM_TILE");
    if (!e) return -1;
    const std::string v(e);
    return v == "256" ? 2 : v == "256x128" ? 1 : v == "128" ? 0 : -1;
  }();
  if (f32) {
    // MPIT_F32_TILE=256x128: 256 x 128 blocks (1 per CU, 128 x 64 per wave) for the bf16x6
    // fp32 GEMMs, whose 6 MFMAs per product make them compute-bound
    static const int f32_forced = [] {
      const char* e = std::getenv("MPIT_F32_TILE");
      return e && std::string(e) == "256x128" ? 1 : 0;
    }();
    return f32_forced == 1 && N % 128 == 0 ? 1 : 0;
  }
  // Measured (profiles/gemm_big_tile_ab_r01.jsonl, gemm_bk64_128tile_ab_r01.jsonl): 256x256
  // (BK 64) beats 128x128 on large square GEMMs (8192^3: 944 vs 611 TFLOP/s) and 256x128 on
  // 50176x256x2304 (+18 %), yet inside the models all-256 tiles lose end to end (round 1:
  // ResNet-50 -1.6 %, VGG-16 -2.7 %; round 4: ResNet-50 bf16 -3 %): one or two blocks per CU
  // leave the epilogue and the other streams nothing to overlap with. Round 4: 256x128 only
  // where K is deep (>= 1024) AND the grid still has >= 4 blocks per CU — VGG-16's 112/56-
  // pixel 3x3 convolutions and their backward-data, no ResNet-50 shape — VGG-16 bf16 EASGD
  // +3.5 % (4,944 vs 4,774 / 4,824 img/s with every GEMM on 256x128, gpurun_out/r04vgg).
  // MPIT_GEMM_DEEPK=k: 256 x 128 for every GEMM with K >= k, whatever its grid (default 2304:
  // VGG-16 bf16 5,319 vs 5,239 img/s, r05i; ResNet-50 bf16 within noise, r05d; 0 = off)
  static const int deepk = [] {
    const char* e = std::getenv("MPIT_GEMM_DEEPK");
    return e ? std::atoi(e) : 2304;
  }();
  int cfg = forced >= 0 ? forced
                        : (K >= 1024 && N % 128 == 0 && ((M + 255) / 256) * int64_t(N / 128) >= 1024 ? 1 : 0);
  if (forced < 0 && deepk > 0 && K >= deepk && N % 128 == 0) cfg = 1;
  if (cfg == 2 && (N % 256 || K % 64 || (conv && cin_conv % 64))) cfg = N % 128 ? 0 : 1;
  if (cfg == 1 && N % 128) cfg = 0;
  return cfg;
}

// fp32 GEMM mode: 1 = bf16x6 split products on the bf16 MFMA (default), 0 = the fp32-input
// MFMA (exact fmaf chains, 1/2.7 of the split path's peak). MPIT_F32_MFMA=native selects 0.
static int f32_mode() {
  static const int m = [] {
    const char* e = std::getenv("MPIT_F32_MFMA");
    return e && std::string(e) == "native" ? 0 : 1;
  }();
  return m;
}

// MPIT_GEMM_LOG=1: one stderr line per GEMM launch (kind, M, N, K, conv, epilogue / splits),
// in issue order — scripts/gemm_calls.py joins it with a kernel trace for per-call TFLOP/s
static bool gemm_log() {
  static const bool on = [] {
    const char* e = std::getenv("MPIT_GEMM_LOG");
    return e && std::string(e) == "1";
  }();
  return on;
}

// group size (M-tiles) and ticket set of a folded BN finalize: <= kFoldMaxGroups groups of
// >= 16 M-tiles. Ticket counters are reset to zero by their last user, so a set is free
// once its launch retired — guaranteed only for launches of the SAME stream (stream
// order). Each (device, stream) therefore owns its own kFoldPerStream sets (the first
// kFoldStreams streams of a device in the static table, later ones in a zeroed allocation
// of their own: no process-lifetime cap on the streams a process may fold from, e.g. one
// priority stream per Trainer) and rotates within them; two folded GEMMs in flight on
// different streams never share a set.
static void fold_plan(EpiArgs& ep, int dev, hipStream_t s, int64_t mtn, int ntn) {
  const int64_t fg = std::max<int64_t>(16, (mtn + kFoldMaxGroups - 1) / kFoldMaxGroups);
  const int64_t ngr = (mtn + fg - 1) / fg;
  if (int64_t(ntn) * (ngr + 1) > kFoldMax) throw std::invalid_argument("gemm_nt: BN fold ticket table too small");
  struct Group {
    uint32_t* sets;  // kFoldPerStream * kFoldMax counters
    uint32_t next;
  };
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, Group> groups;
  static std::map<int, int> used;  // static-table groups handed out per device
  uint32_t* set = nullptr;
  {
    std::lock_guard<std::mutex> g(mu);
    auto it = groups.find({dev, s});
    if (it == groups.end()) {
      int& u = used[dev];
      uint32_t* sets = nullptr;
      if (u < kFoldStreams) {
        uint32_t* base = nullptr;
        hip_check(hipGetSymbolAddress(reinterpret_cast<void**>(&base), HIP_SYMBOL(g_fold_tickets)), "fold ticket symbol");
        sets = base + size_t(u++) * kFoldPerStream * kFoldMax;
      } else {
        const size_t bytes = size_t(kFoldPerStream) * kFoldMax * sizeof(uint32_t);
        hip_check(hipMalloc(reinterpret_cast<void**>(&sets), bytes), "fold ticket sets");
        hip_check(hipMemsetAsync(sets, 0, bytes, s), "fold ticket sets zero");
      }
      it = groups.emplace(std::make_pair(dev, s), Group{sets, 0}).first;
    }
    set = it->second.sets + size_t(it->second.next++ % kFoldPerStream) * kFoldMax;
  }
  ep.ftick = set;
  ep.fgroup = int(fg);
  if (ep.fepoch) {  // tagged protocol requested: a fresh epoch per launch (never 0)
    static std::atomic<uint32_t> epochs{0};
    uint32_t e;
    do e = epochs.fetch_add(1) + 1; while (e == 0);
    ep.fepoch = e;
  }
}

template <typename T>
static void launch_nt_t(int dev, hipStream_t s, int64_t M, int N, int K, uintptr_t A, int64_t lda, uintptr_t B,
                        int64_t ldb, uintptr_t C, int64_t ldc, uintptr_t cin, uintptr_t cmask, const ConvGeo* geo,
                        const EpiArgs& ep_in, int epi, uintptr_t bias, bool relu, int64_t bps) {
  constexpr bool F32 = sizeof(T) == 4;
  EpiArgs ep = ep_in;  // the fold's group size and ticket set are filled in per launch
  constexpr int EPC = epc<T>();
  if (!gemm_nt_supported(M, N, K, F32))
    throw std::invalid_argument(std::string("gemm_nt: need N % 64 == 0 and K % ") + (F32 ? "16" : "32") +
                                " == 0 (M=" + std::to_string(M) + " N=" + std::to_string(N) + " K=" + std::to_string(K) +
                                ")");
  check_ptr(A, "A");
  check_ptr(B, "B");
  check_ptr(C, "C");
  if (lda % EPC || ldb % EPC || ldc % 8 || (!geo && lda < K) || ldb < K || ldc < N)
    throw std::invalid_argument("gemm_nt: bad leading dimensions");
  if (epi != EPI_NONE) {
    if (!ep.part) throw std::invalid_argument("gemm_nt: reduction epilogue needs a partials buffer");
    if (epi == EPI_BNRED2 && geo) throw std::invalid_argument("gemm_nt: paired BN reduction is for 1x1 GEMMs");
    if (ep.fcoef && (epi != EPI_BNRED || ep.row0 != 0 || !ep.frstd || !ep.flvl))
      throw std::invalid_argument("gemm_nt: the BN finalize fold needs a single-launch EPI_BNRED with rstd and lvl");
    if (ep.scoef && (epi != EPI_STATS || ep.row0 != 0 || !ep.smean || !ep.srstd || !ep.flvl))
      throw std::invalid_argument("gemm_nt: the BN forward fold needs a single-launch EPI_STATS with mean, rstd and lvl");
    if (epi == EPI_RELUB) {
      if (!geo || geo->ostr != 1) throw std::invalid_argument("gemm_nt: the fused ReLU epilogue is for stride-1 convolutions");
      if (!ep.x || ldc != N) throw std::invalid_argument("gemm_nt: the fused ReLU epilogue needs x and ldc == N");
      check_ptr(reinterpret_cast<uintptr_t>(ep.x), "ReLU y");
    }
    if (epi == EPI_BNRED || epi == EPI_BNRED2) {
      if (!ep.x || !ep.mean || ldc != N) throw std::invalid_argument("gemm_nt: BN reduction needs x, mean, ldc == N");
      check_ptr(reinterpret_cast<uintptr_t>(ep.x), "BN x");
      check_ptr(reinterpret_cast<uintptr_t>(ep.mean), "BN mean");
    }
  }
  hip_check(hipSetDevice(dev), "hipSetDevice");
  if (gemm_log())
    std::fprintf(stderr, "MPIT_GEMM nt %lld %d %d conv=%d epi=%d f32=%d\n", (long long)M, N, K, geo ? 1 : 0, epi,
                 F32 ? 1 : 0);
  const auto* a = reinterpret_cast<const T*>(A);
  const auto* b = reinterpret_cast<const T*>(B);
  auto* c = reinterpret_cast<T*>(C);
  const auto* ci = reinterpret_cast<const T*>(cin);
  if (cin) check_ptr(cin, "Cin");
  if (cmask && (!cin || ldc != N)) throw std::invalid_argument("gemm_nt: cmask needs cin with ldc == N");
  const auto* cm = reinterpret_cast<const uint8_t*>(cmask);
  if (bias) check_ptr(bias, "bias");
  const auto* bs = reinterpret_cast<const float*>(bias);
  const int rl = relu ? 1 : 0;
  const ConvGeo g = geo ? *geo : ConvGeo{};
  // fp32 variant: 0 native fp32 MFMA, 1 bf16x6 on 16-deep k-tiles, 3 bf16x6 on 32-deep ones
  // (default where K and the conv's channels are multiples of 32; MPIT_F32_BK=16 forces 1).
  // Same-box ResNet-50 fp32 bench: 32-deep 4075 vs 16-deep 4016 img/s (profiles/gemm_fp32_variants_ab_r02.md)
  static const int f32_bk = [] {
    const char* e = std::getenv("MPIT_F32_BK");
    return e && std::atoi(e) == 16 ? 16 : 32;
  }();
  static const int ablate = [] {
    const char* e = std::getenv("MPIT_F32_ABLATE");
    if (!e) return 0;
    const std::string v(e);
    return v == "nosplit" ? 5 : v == "splitA" ? 6 : v == "splitB" ? 7 : 0;
  }();
  int fm = !F32 || f32_mode() != 1 ? 0
           : (f32_bk == 32 && K % 32 == 0 && (!geo || (geo->C % 32 == 0 && (!geo->pitch || bps > 0))) ? 3 : 1);
  if (fm == 3 && ablate) fm = ablate;
  if (bps > 0) {  // B is three pre-split bf16 planes: only the FM 4 kernels read that
    if (!F32 || fm != 3 || ablate || bps < int64_t(N) * ldb || ldb % 8)
      throw std::invalid_argument("gemm_nt: pre-split B planes need the fp32 bf16x6 path with K % 32 == 0 "
                                  "(and conv channels % 32 == 0), ldb % 8 == 0 and a plane stride >= N * ldb");
    check_ptr(B + uintptr_t(bps) * 2, "B plane 1");
    if (N % 64) throw std::invalid_argument("gemm_nt: pre-split B planes need N % 64 == 0");
    // MPIT_F32_WAVES=2x2: the 2 x 2 wave grid (FM 4); default 4 x 1 (FM 9);
    // MPIT_F32_NT=acc1: FM 10 (one accumulator, fragment prefetch; experiment)
    static const bool w22 = [] {
      const char* e = std::getenv("MPIT_F32_WAVES");
      return e && std::string(e) == "2x2";
    }();
    static const bool acc1 = [] {
      const char* e = std::getenv("MPIT_F32_NT");
      return e && std::string(e) == "acc1";
    }();
    fm = w22 ? 4 : (acc1 ? 10 : 9);
    if (ep.amax_b) {  // fp16 planes h, l of the scaled weight (fp16x3): A needs its bound too
      if (!ep.amax_a) throw std::invalid_argument("gemm_nt: fp16 B planes need the A operand's amax bound");
      check_ptr(B + uintptr_t(bps) * 2, "B plane 1");
      fm = 11;
      if (ep.aps > 0) {  // A as fp16 planes too (FM 13)
        if (!kF11Buf || lda % 8 || (geo && geo->pitch)) throw std::invalid_argument("gemm_nt: bad A planes");
        check_ptr(A + uintptr_t(ep.aps) * 2, "A plane 1");
        fm = 13;
      }
    }
  } else if (ep.amax_b) {
    throw std::invalid_argument("gemm_nt: amax_b is the scale of fp16 B planes (bps > 0)");
  }
  if (ep.aps > 0 && fm != 13) throw std::invalid_argument("gemm_nt: A planes need fp16 B planes (fp16x3)");
  if ((F32 && (fm == 11 || fm == 13) && kF11Buf) || (!F32 && kBf16Buf)) {
    // the buffer-descriptor staging keeps every lane offset below 2^31 bytes of its block base
    const int64_t lim = int64_t(1) << 31, esz = fm == 13 ? 2 : int64_t(sizeof(T));
    int64_t aspan;
    if (geo) {
      const int64_t hw = int64_t(geo->Ho) * geo->Wo;
      const int64_t imgs = std::min<int64_t>((M + hw - 1) / hw, (256 + hw - 1) / hw + 1);
      aspan = imgs * geo->H * geo->W * int64_t(geo->pitch ? geo->pitch : geo->C) * esz;
    } else {
      aspan = (int64_t(256) * lda + K) * esz;
    }
    if (aspan >= lim || (int64_t(256) * ldb + K) * esz >= lim)
      throw std::invalid_argument("gemm_nt: operand rows (or images) span >= 2 GiB per block");
  }
  const int nk = K / (fm >= 3 ? 32 : nt_bk_of<T>());
  // MPIT_GEMM_STAGES caps the ring depth (A/B measurements). fp32: the 64 KB epilogue tile
  // of a 128x128 block holds a 4-deep 16-deep ring (or a 2-deep 32-deep one) for free.
  static const int max_stages = [] {
    const char* e = std::getenv("MPIT_GEMM_STAGES");
    return e ? std::max(2, std::min(4, std::atoi(e))) : 2;
  }();
  static const int f32_stages = [] {
    const char* e = std::getenv("MPIT_F32_STAGES");
    return e ? std::max(2, std::min(4, std::atoi(e))) : 0;
  }();
  int cap = F32 && N % 128 == 0 ? (fm >= 3 ? 2 : 4) : max_stages;
  if (F32 && f32_stages) cap = f32_stages;
  // (the pre-split kernels, FM >= 4, are built for the 2-deep ring of 128-row tiles only)
  const int stages = fm >= 4 ? 2 : std::min(cap, nk >= 4 ? 4 : (nk == 3 ? 3 : 2));
  // (kernel templates are named at a non-template call site so their host stubs are emitted)
#define MPIT_NT_OPT_IN(BM, BN, ST, EPI, CONV, FMV)                                                                 \
  do {                                                                                                             \
    static const bool opted = (hip_check(hipFuncSetAttribute(reinterpret_cast<const void*>(                       \
                                                             &gemm_nt_kernel<T, BM, BN, ST, EPI, CONV, FMV>),     \
                                                         hipFuncAttributeMaxDynamicSharedMemorySize, int(shm)),    \
                                     "hipFuncSetAttribute"),                                                       \
                               true);                                                                              \
    (void)opted;                                                                                                   \
  } while (0)
#define MPIT_NT_LAUNCH1(BM, BN, ST, EPI, CONV)                                                                       \
  do {                                                                                                             \
    if constexpr (F32 && BM == 256 && BN == 64) { /* fp16x3 only (MPIT_F32_TILE=256x64) */                      \
      if (fm != 11) throw std::logic_error("gemm_nt: 256 x 64 fp32 tiles are for the fp16x3 kernels (FM 11)");    \
      MPIT_NT_OPT_IN(BM, BN, ST, EPI, CONV, 11);                                                                   \
      hipLaunchKernelGGL((gemm_nt_kernel<T, BM, BN, ST, EPI, CONV, 11>), dim3(unsigned(nb)), dim3(256), shm, s, a,   \
                         lda, b, ldb, c, ldc, M, N, K, ntn, ep, ci, cm, bs, rl, g, bps);                            \
      break;                                                                                                       \
    } else {                                                                                                       \
    if constexpr (F32 && BM == 128 && ST == 2) {                                                                 \
      if (fm == 13) {                                                                                              \
        if (shm > 65536) MPIT_NT_OPT_IN(BM, BN, ST, EPI, CONV, 13);                                                 \
        hipLaunchKernelGGL((gemm_nt_kernel<T, BM, BN, ST, EPI, CONV, 13>), dim3(unsigned(nb)), dim3(256), shm, s, a, \
                           lda, b, ldb, c, ldc, M, N, K, ntn, ep, ci, cm, bs, rl, g, bps);                          \
        break;                                                                                                     \
      }                                                                                                            \
      if (fm == 11) {                                                                                              \
        if (shm > 65536) MPIT_NT_OPT_IN(BM, BN, ST, EPI, CONV, 11);                                                 \
        hipLaunchKernelGGL((gemm_nt_kernel<T, BM, BN, ST, EPI, CONV, 11>), dim3(unsigned(nb)), dim3(256), shm, s, a, \
                           lda, b, ldb, c, ldc, M, N, K, ntn, ep, ci, cm, bs, rl, g, bps);                          \
        break;                                                                                                     \
      }                                                                                                            \
      if (fm >= 5 && fm <= 7) { /* timing ablations (MPIT_F32_ABLATE) */                                        \
        if (fm == 5) {                                                                                             \
          if (shm > 65536) MPIT_NT_OPT_IN(BM, BN, ST, EPI, CONV, 5);                                                \
          hipLaunchKernelGGL((gemm_nt_kernel<T, BM, BN, ST, EPI, CONV, 5>), dim3(unsigned(nb)), dim3(256), shm, s, \
                             a, lda, b, ldb, c, ldc, M, N, K, ntn, ep, ci, cm, bs, rl, g, bps);                          \
        } else if (fm == 6) {                                                                                      \
          if (shm > 65536) MPIT_NT_OPT_IN(BM, BN, ST, EPI, CONV, 6);                                                \
          hipLaunchKernelGGL((gemm_nt_kernel<T, BM, BN, ST, EPI, CONV, 6>), dim3(unsigned(nb)), dim3(256), shm, s, \
                             a, lda, b, ldb, c, ldc, M, N, K, ntn, ep, ci, cm, bs, rl, g, bps);                          \
        } else {                                                                                                   \
          if (shm > 65536) MPIT_NT_OPT_IN(BM, BN, ST, EPI, CONV, 7);                                                \
          hipLaunchKernelGGL((gemm_nt_kernel<T, BM, BN, ST, EPI, CONV, 7>), dim3(unsigned(nb)), dim3(256), shm, s, \
                             a, lda, b, ldb, c, ldc, M, N, K, ntn, ep, ci, cm, bs, rl, g, bps);                          \
        }                                                                                                          \
        break;                                                                                                     \
      }                                                                                                            \
      if (fm == 4) {                                                                                               \
        if (shm > 65536) MPIT_NT_OPT_IN(BM, BN, ST, EPI, CONV, 4);                                                  \
        hipLaunchKernelGGL((gemm_nt_kernel<T, BM, BN, ST, EPI, CONV, 4>), dim3(unsigned(nb)), dim3(256), shm, s, a, \
                           lda, b, ldb, c, ldc, M, N, K, ntn, ep, ci, cm, bs, rl, g, bps);                          \
        break;                                                                                                     \
      }                                                                                                            \
      if (fm == 9) {                                                                                               \
        if (shm > 65536) MPIT_NT_OPT_IN(BM, BN, ST, EPI, CONV, 9);                                                  \
        hipLaunchKernelGGL((gemm_nt_kernel<T, BM, BN, ST, EPI, CONV, 9>), dim3(unsigned(nb)), dim3(256), shm, s, a, \
                           lda, b, ldb, c, ldc, M, N, K, ntn, ep, ci, cm, bs, rl, g, bps);                          \
        break;                                                                                                     \
      }                                                                                                            \
      if (fm == 10) {                                                                                              \
        if (shm > 65536) MPIT_NT_OPT_IN(BM, BN, ST, EPI, CONV, 10);                                                 \
        hipLaunchKernelGGL((gemm_nt_kernel<T, BM, BN, ST, EPI, CONV, 10>), dim3(unsigned(nb)), dim3(256), shm, s, a, \
                           lda, b, ldb, c, ldc, M, N, K, ntn, ep, ci, cm, bs, rl, g, bps);                          \
        break;                                                                                                     \
      }                                                                                                            \
    }                                                                                                              \
    if constexpr (F32) {                                                                                           \
      if (fm >= 4) throw std::logic_error("gemm_nt: pre-split kernels run 128-row tiles on a 2-deep ring");        \
      if (fm == 3) {                                                                                               \
        if (shm > 65536) MPIT_NT_OPT_IN(BM, BN, ST, EPI, CONV, 3);                                                  \
        hipLaunchKernelGGL((gemm_nt_kernel<T, BM, BN, ST, EPI, CONV, 3>), dim3(unsigned(nb)), dim3(256), shm, s, a, \
                           lda, b, ldb, c, ldc, M, N, K, ntn, ep, ci, cm, bs, rl, g, bps);                               \
        break;                                                                                                     \
      }                                                                                                            \
      if (fm == 1) {                                                                                               \
        if (shm > 65536) MPIT_NT_OPT_IN(BM, BN, ST, EPI, CONV, 1);                                                  \
        hipLaunchKernelGGL((gemm_nt_kernel<T, BM, BN, ST, EPI, CONV, 1>), dim3(unsigned(nb)), dim3(256), shm, s, a, \
                           lda, b, ldb, c, ldc, M, N, K, ntn, ep, ci, cm, bs, rl, g, bps);                               \
        break;                                                                                                     \
      }                                                                                                            \
    }                                                                                                              \
    if (shm > 65536) MPIT_NT_OPT_IN(BM, BN, ST, EPI, CONV, 0);                                                      \
    hipLaunchKernelGGL((gemm_nt_kernel<T, BM, BN, ST, EPI, CONV>), dim3(unsigned(nb)), dim3(256), shm, s, a, lda, b, \
                       ldb, c, ldc, M, N, K, ntn, ep, ci, cm, bs, rl, g, bps);                                           \
    }                                                                                                              \
  } while (0)
#define MPIT_NT_LAUNCH2(BM, BN, ST, CONV)                                                         \
  do {                                                                                              \
    if (epi == EPI_STATS) MPIT_NT_LAUNCH1(BM, BN, ST, EPI_STATS, CONV);                        \
    else if (epi == EPI_BNRED) MPIT_NT_LAUNCH1(BM, BN, ST, EPI_BNRED, CONV);                   \
    else if (epi == EPI_BNRED2 && !CONV) MPIT_NT_LAUNCH1(BM, BN, ST, EPI_BNRED2, false);       \
    else if (epi == EPI_RELUB && CONV) MPIT_NT_LAUNCH1(BM, BN, ST, EPI_RELUB, true);           \
    else MPIT_NT_LAUNCH1(BM, BN, ST, EPI_NONE, CONV);                                          \
  } while (0)
#define MPIT_NT_LAUNCH(BM, BN, ST)                                                                             \
  do {                                                                                                         \
    const int64_t mtn = (M + BM - 1) / BM;                                                                     \
    const int ntn = N / BN;                                                                                    \
    const int64_t nb = mtn * ntn;                                                                              \
    if (nb > INT32_MAX) throw std::invalid_argument("gemm_nt: too many tiles");                               \
    if (ep.fcoef || ep.scoef) fold_plan(ep, dev, s, mtn, ntn);                                                                 \
    /* LDS: the k-tile ring, reused by the epilogue's output tile and reduction table */                      \
    const size_t shm = std::max({size_t(ST) * (size_t(BM) * nt_bkb(BM, BN, fm) +                               \
                                                (fm == 11 || fm == 13 ? size_t(BN) * 128 : fm == 4 || fm >= 9 ? size_t(BN) * 192 : size_t(BN) * nt_bkb(BM, BN, fm))), \
                                 size_t(BM) * BN * sizeof(T), size_t(256) * 8 * 3 * sizeof(float)});          \
    if (geo) MPIT_NT_LAUNCH2(BM, BN, ST, true);                                                           \
    else MPIT_NT_LAUNCH2(BM, BN, ST, false);                                                              \
  } while (0)
  const int tcfg = fm == 4 || fm >= 9 ? 0 : nt_tile_config(M, N, K, geo != nullptr, geo ? geo->C : 0, F32);
  if constexpr (F32) {
    // MPIT_F32_TILE=256x64: the fp16x3 GEMMs with N == 64 on 256 x 64 blocks (each wave 64 x 64
    // instead of 32 x 64: twice the MFMAs per barrier and per A fragment split, 2 blocks/CU)
    static const bool t256x64 = [] {
      const char* e = std::getenv("MPIT_F32_TILE");
      return e && std::string(e) == "256x64";
    }();
    if (fm == 11 && N == 64 && t256x64) {  // (FM 13 runs 128-row tiles)
      MPIT_NT_LAUNCH(256, 64, 2);
      hip_check(hipGetLastError(), "gemm_nt launch");
      return;
    }
    if (tcfg == 1) {
      MPIT_NT_LAUNCH(256, 128, 3);
      hip_check(hipGetLastError(), "gemm_nt launch");
      return;
    }
  } else {
    if (tcfg == 2) {
      MPIT_NT_LAUNCH(256, 256, 2);  // 2 x 64-deep stages = the 128 KB epilogue tile
      hip_check(hipGetLastError(), "gemm_nt launch");
      return;
    }
    if (tcfg == 1) {
      MPIT_NT_LAUNCH(256, 128, 3);
      hip_check(hipGetLastError(), "gemm_nt launch");
      return;
    }
  }
  // MPIT_F32_BN64=1: fp32 GEMMs on 128x64 tiles (3 blocks per CU instead of 2) — A/B knob
  static const bool f32_bn64 = [] {
    const char* e = std::getenv("MPIT_F32_BN64");
    return e && std::string(e) == "1";
  }();
  if (N % 128 == 0 && !(F32 && f32_bn64)) {
    if (stages == 4) MPIT_NT_LAUNCH(128, 128, 4);
    else if (stages == 3) MPIT_NT_LAUNCH(128, 128, 3);
    else MPIT_NT_LAUNCH(128, 128, 2);
  } else {
    if (stages == 4) MPIT_NT_LAUNCH(128, 64, 4);
    else if (stages == 3) MPIT_NT_LAUNCH(128, 64, 3);
    else MPIT_NT_LAUNCH(128, 64, 2);
  }
#undef MPIT_NT_LAUNCH
#undef MPIT_NT_LAUNCH2
#undef MPIT_NT_LAUNCH1
#undef MPIT_NT_OPT_IN
  hip_check(hipGetLastError(), "gemm_nt launch");
}

// bps > 0: B is three pre-split bf16 planes (h, m, l) of plane stride bps elements (fp32 only)
static void launch_nt(int dev, hipStream_t s, int64_t M, int N, int K, uintptr_t A, int64_t lda, uintptr_t B,
                      int64_t ldb, uintptr_t C, int64_t ldc, uintptr_t cin, uintptr_t cmask, const ConvGeo* geo,
                      const EpiArgs& ep, int epi, bool f32, uintptr_t bias = 0, bool relu = false, int64_t bps = 0) {
  if (f32) launch_nt_t<float>(dev, s, M, N, K, A, lda, B, ldb, C, ldc, cin, cmask, geo, ep, epi, bias, relu, bps);
  else launch_nt_t<uint16_t>(dev, s, M, N, K, A, lda, B, ldb, C, ldc, cin, cmask, geo, ep, epi, bias, relu, bps);
}

// the reduction epilogue selected by the (stats, BN reduction) operands
static EpiArgs epi_args(uintptr_t stats, const BnRed* r, int* mode) {
  EpiArgs ep{};
  *mode = EPI_NONE;
  if (r) {
    ep.amax_a = reinterpret_cast<const float*>(r->amax_a);
    ep.amax_b = reinterpret_cast<const float*>(r->amax_b);
    ep.aps = r->aps;
    ep.omax = reinterpret_cast<unsigned long long*>(r->omax);
    ep.oepoch = r->oepoch;
  }
  if (stats && r && r->part) throw std::invalid_argument("gemm_nt: stats and BN reduction are exclusive");
  if (stats) {
    ep.part = reinterpret_cast<float*>(stats);
    *mode = EPI_STATS;
    if (r && r->scoef) {
      ep.scoef = reinterpret_cast<float*>(r->scoef);
      ep.sgamma = reinterpret_cast<const float*>(r->sgamma);
      ep.sbeta = reinterpret_cast<const float*>(r->sbeta);
      ep.srmean = reinterpret_cast<float*>(r->srmean);
      ep.srvar = reinterpret_cast<float*>(r->srvar);
      ep.smean = reinterpret_cast<float*>(r->smean);
      ep.srstd = reinterpret_cast<float*>(r->srstd);
      ep.flvl = reinterpret_cast<float*>(r->slvl);
      ep.fzero = reinterpret_cast<float*>(r->szero);
      ep.seps = r->seps;
      ep.smom = r->smom;
      ep.fepoch = r->ftag ? 1u : 0u;  // (the launch assigns the epoch: fold_plan)
    }
  } else if (r && r->part && r->relu_y) {
    if (r->mask || r->mean || r->part2 || r->fcoef) throw std::invalid_argument("gemm_nt: relu_y excludes a BN reduction");
    ep.part = reinterpret_cast<float*>(r->part);
    ep.x = reinterpret_cast<const void*>(r->x);
    ep.row0 = r->row0;
    *mode = EPI_RELUB;
  } else if (r && r->part) {
    ep.part = reinterpret_cast<float*>(r->part);
    ep.x = reinterpret_cast<const void*>(r->x);
    ep.mask = reinterpret_cast<const uint8_t*>(r->mask);
    ep.mean = reinterpret_cast<const float*>(r->mean);
    ep.row0 = r->row0;
    *mode = EPI_BNRED;
    if (r->fcoef) {
      ep.fcoef = reinterpret_cast<float*>(r->fcoef);
      ep.fgamma = reinterpret_cast<const float*>(r->fgamma);
      ep.frstd = reinterpret_cast<const float*>(r->frstd);
      ep.fdgamma = reinterpret_cast<float*>(r->fdgamma);
      ep.fdbeta = reinterpret_cast<float*>(r->fdbeta);
      ep.flvl = reinterpret_cast<float*>(r->flvl);
      ep.fzero = reinterpret_cast<float*>(r->fzero);
      ep.fepoch = r->ftag ? 1u : 0u;
    }
    if (r->part2) {
      if (!r->x2 || !r->mean2) throw std::invalid_argument("gemm_nt: second BN reduction needs x2 and mean2");
      ep.part2 = reinterpret_cast<float*>(r->part2);
      ep.x2 = reinterpret_cast<const void*>(r->x2);
      ep.mean2 = reinterpret_cast<const float*>(r->mean2);
      *mode = EPI_BNRED2;
    }
  }
  return ep;
}

void gemm_nt(int dev, hipStream_t s, int64_t M, int N, int K, uintptr_t A, int64_t lda, uintptr_t B, int64_t ldb,
             uintptr_t C, int64_t ldc, uintptr_t stats, uintptr_t cin, uintptr_t cmask, const BnRed* red, bool f32,
             int64_t bps) {
  int mode;
  const EpiArgs ep = epi_args(stats, red, &mode);
  launch_nt(dev, s, M, N, K, A, lda, B, ldb, C, ldc, cin, cmask, nullptr, ep, mode, f32, 0, false, bps);
}

bool gemm_tn_supported(int64_t M, int N, int K) { return M > 0 && N % 64 == 0 && K % 64 == 0 && N > 0 && K > 0; }

// split-K plan: number of splits over M and rows per split, sized so the grid holds
// about as many blocks as can be resident (bf16 4-stage / fp32 2-stage ring: 64 KiB of
// LDS per 128x128 tile)
// MPIT_TN_OCC=1: one gemm_tn block per CU (its LDS request padded to kTnCapShm), so a CU
// running a backward-weight block of the side stream always has room for one block of the
// critical path's GEMMs (64 KiB) next to it; the split plan then targets one block per CU.
constexpr size_t kTnCapShm = 92 * 1024;
static bool tn_cap1() {
  static const bool on = [] {
    const char* e = std::getenv("MPIT_TN_OCC");
    return e && std::string(e) == "1";
  }();
  return on;
}

static int tn_plan(int dev, int64_t M, int N, int K, int64_t* rows_per_split, int* tbn, int* tbk, int cin = 0) {
  *tbn = N % 128 == 0 ? 128 : 64;
  // conv: a column tile never straddles two taps — except the row-tap stem (cin = kStemTap),
  // whose lanes locate their tap per 16-B chunk: there 128-wide tiles read dY half as often
  *tbk = (cin && cin != kStemTap ? cin : K) % 128 == 0 ? 128 : 64;
  const int64_t ntiles = int64_t(N / *tbn) * (K / *tbk);
  const int per_cu = tn_cap1() ? 1 : 2 * (128 / *tbn) * (128 / *tbk);
  // MPIT_TN_SPLIT_MUL=k: k times the splits (shorter blocks that free their CU sooner for
  // the critical path's kernels, at k times the partial-sum traffic) — A/B knob
  // (MPIT_TN_SPLIT_DIV=k: 1/k of them — longer blocks, less partial-sum traffic)
  static const int split_mul = [] {
    const char* e = std::getenv("MPIT_TN_SPLIT_MUL");
    return e ? std::max(1, std::min(8, std::atoi(e))) : 1;
  }();
  static const int split_div = [] {
    const char* e = std::getenv("MPIT_TN_SPLIT_DIV");
    return e ? std::max(1, std::min(8, std::atoi(e))) : 1;
  }();
  const int64_t target = std::max<int64_t>(1, int64_t(per_cu) * cu_count(dev) * split_mul / split_div);
  // floor: one more block than there are slots would run as a whole second round
  int64_t ns = std::max<int64_t>(1, target / ntiles);
  // keep >= 8 staged steps per block; MPIT_TN_MIN_ROWS=r raises the floor (fewer, longer splits
  // where M is deep and the output small — less partial-sum traffic; A/B knob)
  static const int64_t min_rows_env = [] {
    const char* e = std::getenv("MPIT_TN_MIN_ROWS");
    return e ? std::max<int64_t>(8 * kRows, std::atoll(e)) : int64_t(8 * kRows);
  }();
  const int64_t min_rows = min_rows_env;
  ns = std::min<int64_t>(ns, std::max<int64_t>(1, M / min_rows));
  ns = std::min<int64_t>(ns, int64_t(kReduceGroup) * kReduceGroup);  // two reduce levels at most
  int64_t rps = (M + ns - 1) / ns;
  rps = (rps + kRows - 1) / kRows * kRows;
  ns = (M + rps - 1) / rps;
  *rows_per_split = rps;
  return int(ns);
}

static int64_t tn_groups(int ns) { return ns > kReduceGroup ? (ns + kReduceGroup - 1) / kReduceGroup : 0; }

int64_t gemm_tn_ws_floats(int dev, int64_t M, int N, int K) {
  int64_t rps;
  int tbn, tbk;
  const int ns = tn_plan(dev, M, N, K, &rps, &tbn, &tbk);
  return ns > 1 ? (int64_t(ns) + tn_groups(ns)) * N * K : 0;
}

template <typename T>
static void launch_tn_t(int dev, hipStream_t s, int64_t M, int N, int K, uintptr_t Y, int64_t ldy, uintptr_t X,
                        int64_t ldx, uintptr_t out, uintptr_t ws, float beta, const ConvGeo* geo, uintptr_t amax_y,
                        uintptr_t amax_x, int64_t yps = 0, int64_t xps = 0) {
  constexpr bool F32 = sizeof(T) == 4;
  constexpr int EPC = epc<T>();
  if (!gemm_tn_supported(M, N, K))
    throw std::invalid_argument("gemm_tn: need N % 64 == 0 and K % 64 == 0");
  check_ptr(Y, "Y");
  check_ptr(X, "X");
  check_ptr(out, "out");
  if (ldy % EPC || ldx % EPC || ldy < N || (!geo && ldx < K))
    throw std::invalid_argument("gemm_tn: bad leading dimensions");
  hip_check(hipSetDevice(dev), "hipSetDevice");
  int64_t rps;
  int tbn, tbk;
  const int ns = tn_plan(dev, M, N, K, &rps, &tbn, &tbk, geo ? geo->C : 0);
  if (gemm_log())
    std::fprintf(stderr, "MPIT_GEMM tn %lld %d %d conv=%d splits=%d f32=%d\n", (long long)M, N, K, geo ? 1 : 0, ns,
                 F32 ? 1 : 0);
  if (geo && kTnBuf) {  // buffer-descriptor staging: a split's images span < 2^31 bytes
    const int64_t hw = int64_t(geo->Ho) * geo->Wo;
    const int64_t imgs = std::min<int64_t>((M + hw - 1) / hw, (rps + hw - 1) / hw + 1);
    if (imgs * geo->H * geo->W * int64_t(geo->pitch ? geo->pitch : geo->C) * int64_t(sizeof(T)) >= (int64_t(1) << 31))
      throw std::invalid_argument("gemm_tn: the images of one split span >= 2 GiB");
  }
  const int ntk = K / tbk;
  const int ntiles = (N / tbn) * ntk;
  const bool direct = ns == 1 && beta == 0.f;
  if (!direct && ws == 0) throw std::invalid_argument("gemm_tn: workspace required");
  if (!direct) check_ptr(ws, "ws");
  float* part = reinterpret_cast<float*>(direct ? out : ws);
  const auto* y = reinterpret_cast<const T*>(Y);
  const auto* x = reinterpret_cast<const T*>(X);
  const ConvGeo g = geo ? *geo : ConvGeo{};
  const dim3 grid(unsigned(int64_t(ntiles) * ns));
  // MPIT_TN_FUSED=1: the split reduction runs inside the GEMM (last block per tile / group).
  // Bitwise equal to the split_reduce launches but slower on ResNet-50's wgrads (the tail sum
  // of a tile is left to one block: profiles/tn_fused_reduction_ab_r02.md), so opt-in.
  static const bool fused_env = [] {
    const char* e = std::getenv("MPIT_TN_FUSED");
    return e && std::string(e) == "1";
  }();
  TnRed red{};
  // fp32 with both operand bounds: fp16x3 (FM 11), else bf16x6 (FM 1)
  if ((amax_y != 0) != (amax_x != 0)) throw std::invalid_argument("gemm_tn: fp16x3 needs both operand bounds");
  // fp16x3 wgrad: FM 12 (split once per element into fp16 planes in LDS, transposed fragment
  // reads) unless MPIT_TN_F16S=0 (FM 11: split per use after column reads)
  static const bool f16s = [] {
    const char* e = std::getenv("MPIT_TN_F16S");
    return !(e && std::string(e) == "0");
  }();
  const int tfm = !F32 || f32_mode() != 1 ? 0 : (amax_y ? (f16s ? 12 : 11) : 1);
  red.amax_y = reinterpret_cast<const float*>(amax_y);
  red.amax_x = reinterpret_cast<const float*>(amax_x);
  red.yps = yps;
  red.xps = xps;
  const bool p13 = !F32 && yps > 0;  // fp32 operands as fp16 planes (launch_tn)
  if (p13 && (!amax_y || !amax_x || xps <= 0 || !kTnBuf || (geo && geo->pitch)))
    throw std::invalid_argument("gemm_tn: fp16 planes need both bounds and plane strides");
  const int ngr = ns > kReduceGroup ? int(tn_groups(ns)) : 1;
  const bool fused = !direct && fused_env && int64_t(ntiles) * (ngr + 1) <= kTnMaxTickets;
  if (fused) {
    static std::atomic<uint32_t> launches{0};
    uint32_t* base = nullptr;
    hip_check(hipGetSymbolAddress(reinterpret_cast<void**>(&base), HIP_SYMBOL(g_tn_tickets)), "tn ticket symbol");
    red.tick = base + size_t(launches.fetch_add(1) % kTnTicketSlots) * kTnMaxTickets;
    red.out = reinterpret_cast<float*>(out);
    red.mid = part + int64_t(ns) * N * K;
    red.beta = beta;
    red.ns = ns;
    red.groups = ngr;
  }
  // MPIT_GEMM_TN_STAGES: ring depth (A/B measurements; bf16 4 by default). fp32 stages
  // twice the bytes per row and computes 16x longer per staged step: 2 stages.
  static const int tn_stages = [] {
    const char* e = std::getenv("MPIT_GEMM_TN_STAGES");
    return e && std::atoi(e) <= 2 ? 2 : 4;
  }();
  const int stages = F32 || p13 ? 2 : tn_stages;
  // fp32 128 x 128 tiles, MPIT_TN_F32S=1: the split-once kernel (experiment; bitwise equal,
  // slower so far: profiles/wgrad_split_once_r03.md)
  static const bool f32s = [] {
    const char* e = std::getenv("MPIT_TN_F32S");
    return e && std::string(e) == "1";
  }();
  if (F32 && tfm == 1 && f32s && !fused && tbn == 128 && tbk == 128 && (!geo || (!geo->pitch && geo->C % 128 == 0))) {
    const size_t shm = size_t(2) * 3 * 256 * kTsR * 2;
    const auto* yf = reinterpret_cast<const float*>(Y);
    const auto* xf = reinterpret_cast<const float*>(X);
    if (geo)
      hipLaunchKernelGGL(gemm_tn_f32s_kernel<true>, grid, dim3(256), shm, s, yf, ldy, xf, ldx, part, M, N, K, rps, ntk,
                         ntiles, g);
    else
      hipLaunchKernelGGL(gemm_tn_f32s_kernel<false>, grid, dim3(256), shm, s, yf, ldy, xf, ldx, part, M, N, K, rps,
                         ntk, ntiles, g);
  } else {
#define MPIT_TN_OPT_IN(A, B, ST, CV, FMV)                                                                          \
  do {                                                                                                             \
    static const bool opted = (hip_check(hipFuncSetAttribute(reinterpret_cast<const void*>(                       \
                                                             &gemm_tn_kernel<T, A, B, ST, CV, FMV>),              \
                                                         hipFuncAttributeMaxDynamicSharedMemorySize, int(shm)),    \
                                     "hipFuncSetAttribute"),                                                       \
                               true);                                                                              \
    (void)opted;                                                                                                   \
  } while (0)
#define MPIT_TN_LAUNCH1(A, B, ST)                                                                                  \
  do {                                                                                                             \
    size_t shm = size_t(ST) * kRows * (tbn + tbk) * sizeof(T);                                                   \
    if (tn_cap1()) {                                                                                               \
      shm = std::max(shm, kTnCapShm);                                                                              \
      if (geo && F32 && tfm == 12) MPIT_TN_OPT_IN(A, B, ST, true, F32 ? 12 : 0);                                   \
      else if (F32 && tfm == 12) MPIT_TN_OPT_IN(A, B, ST, false, F32 ? 12 : 0);                                    \
      else if (geo && F32 && tfm == 11) MPIT_TN_OPT_IN(A, B, ST, true, F32 ? 11 : 0);                              \
      else if (F32 && tfm == 11) MPIT_TN_OPT_IN(A, B, ST, false, F32 ? 11 : 0);                                    \
      else if (geo && F32 && f32_mode() == 1) MPIT_TN_OPT_IN(A, B, ST, true, F32 ? 1 : 0);                         \
      else if (F32 && f32_mode() == 1) MPIT_TN_OPT_IN(A, B, ST, false, F32 ? 1 : 0);                               \
      else if (geo) MPIT_TN_OPT_IN(A, B, ST, true, 0);                                                             \
      else MPIT_TN_OPT_IN(A, B, ST, false, 0);                                                                     \
    }                                                                                                              \
    if (geo && F32 && tfm == 12)                                                                                   \
      hipLaunchKernelGGL((gemm_tn_kernel<T, A, B, ST, true, F32 ? 12 : 0>), grid, dim3(256), shm, s, y, ldy, x,    \
                         ldx, part, M, N, K, rps, ntk, ntiles, g, red);                                            \
    else if (F32 && tfm == 12)                                                                                     \
      hipLaunchKernelGGL((gemm_tn_kernel<T, A, B, ST, false, F32 ? 12 : 0>), grid, dim3(256), shm, s, y, ldy, x,   \
                         ldx, part, M, N, K, rps, ntk, ntiles, g, red);                                            \
    else if (geo && F32 && tfm == 11)                                                                              \
      hipLaunchKernelGGL((gemm_tn_kernel<T, A, B, ST, true, F32 ? 11 : 0>), grid, dim3(256), shm, s, y, ldy, x,    \
                         ldx, part, M, N, K, rps, ntk, ntiles, g, red);                                            \
    else if (F32 && tfm == 11)                                                                                     \
      hipLaunchKernelGGL((gemm_tn_kernel<T, A, B, ST, false, F32 ? 11 : 0>), grid, dim3(256), shm, s, y, ldy, x,   \
                         ldx, part, M, N, K, rps, ntk, ntiles, g, red);                                            \
    else if (geo && F32 && f32_mode() == 1)                                                                        \
      hipLaunchKernelGGL((gemm_tn_kernel<T, A, B, ST, true, F32 ? 1 : 0>), grid, dim3(256), shm, s, y, ldy, x,     \
                         ldx, part, M, N, K, rps, ntk, ntiles, g, red);                                            \
    else if (F32 && f32_mode() == 1)                                                                               \
      hipLaunchKernelGGL((gemm_tn_kernel<T, A, B, ST, false, F32 ? 1 : 0>), grid, dim3(256), shm, s, y, ldy, x,    \
                         ldx, part, M, N, K, rps, ntk, ntiles, g, red);                                            \
    else if (geo)                                                                                                  \
      hipLaunchKernelGGL((gemm_tn_kernel<T, A, B, ST, true>), grid, dim3(256), shm, s, y, ldy, x, ldx, part, M, N, \
                         K, rps, ntk, ntiles, g, red);                                                             \
    else                                                                                                           \
      hipLaunchKernelGGL((gemm_tn_kernel<T, A, B, ST, false>), grid, dim3(256), shm, s, y, ldy, x, ldx, part, M,   \
                         N, K, rps, ntk, ntiles, g, red);                                                          \
  } while (0)
#define MPIT_TN_LAUNCH(A, B)               \
  do {                                     \
    if (stages == 2) MPIT_TN_LAUNCH1(A, B, 2); \
    else MPIT_TN_LAUNCH1(A, B, 4);         \
  } while (0)
  // bf16: 64-row staged steps on a 2-deep ring (MPIT_TN_KR_STAGES=3: 3-deep) — the LDS of a
  // 4 x 32-row ring, half its barriers per row. Default since r05o: VGG-16 bf16 5,557 vs 5,480
  // img/s, ResNet-50 bf16 11,674 vs 11,596 (r05d). MPIT_TN_KROWS=32: the 4 x 32-row ring
  static const int kr64_stages = [] {
    const char* e = std::getenv("MPIT_TN_KROWS");
    if (e && std::atoi(e) == 32) return 0;
    const char* st = std::getenv("MPIT_TN_KR_STAGES");
    return st && std::atoi(st) == 3 ? 3 : 2;
  }();
  bool done64 = false;
  if constexpr (!F32) {
    if (p13) {  // fp16x3 planes: 32-row steps on a 2-deep ring (FM 12's LDS)
#define MPIT_TN_P13(A, B)                                                                                          \
  do {                                                                                                             \
    const size_t shm = size_t(2) * kRows * (tbn + tbk) * 2 * sizeof(T);                                             \
    if (geo) {                                                                                                     \
      if (shm > 65536) MPIT_TN_OPT_IN13(A, B, true);                                                               \
      hipLaunchKernelGGL((gemm_tn_kernel<T, A, B, 2, true, 13, kRows>), grid, dim3(256), shm, s, y, ldy, x, ldx,   \
                         part, M, N, K, rps, ntk, ntiles, g, red);                                                 \
    } else {                                                                                                       \
      if (shm > 65536) MPIT_TN_OPT_IN13(A, B, false);                                                              \
      hipLaunchKernelGGL((gemm_tn_kernel<T, A, B, 2, false, 13, kRows>), grid, dim3(256), shm, s, y, ldy, x, ldx,  \
                         part, M, N, K, rps, ntk, ntiles, g, red);                                                 \
    }                                                                                                              \
  } while (0)
#define MPIT_TN_OPT_IN13(A, B, CV)                                                                                 \
  do {                                                                                                             \
    static const bool opted = (hip_check(hipFuncSetAttribute(reinterpret_cast<const void*>(                       \
                                                             &gemm_tn_kernel<T, A, B, 2, CV, 13, kRows>),         \
                                                         hipFuncAttributeMaxDynamicSharedMemorySize, int(shm)),    \
                                     "hipFuncSetAttribute"),                                                       \
                               true);                                                                              \
    (void)opted;                                                                                                   \
  } while (0)
      if (tbn == 128 && tbk == 128) MPIT_TN_P13(128, 128);
      else if (tbn == 128) MPIT_TN_P13(128, 64);
      else if (tbk == 128) MPIT_TN_P13(64, 128);
      else MPIT_TN_P13(64, 64);
#undef MPIT_TN_P13
#undef MPIT_TN_OPT_IN13
      done64 = true;
    }
    if (!done64 && kr64_stages && !fused) {
#define MPIT_TN_K64(A, B, ST)                                                                                      \
  do {                                                                                                             \
    const size_t shm = size_t(ST) * 64 * (tbn + tbk) * sizeof(T);                                                  \
    if (geo) {                                                                                                     \
      if (shm > 65536) MPIT_TN_OPT_IN64(A, B, ST, true);                                                           \
      hipLaunchKernelGGL((gemm_tn_kernel<T, A, B, ST, true, 0, 64>), grid, dim3(256), shm, s, y, ldy, x, ldx, part, \
                         M, N, K, rps, ntk, ntiles, g, red);                                                       \
    } else {                                                                                                       \
      if (shm > 65536) MPIT_TN_OPT_IN64(A, B, ST, false);                                                          \
      hipLaunchKernelGGL((gemm_tn_kernel<T, A, B, ST, false, 0, 64>), grid, dim3(256), shm, s, y, ldy, x, ldx,    \
                         part, M, N, K, rps, ntk, ntiles, g, red);                                                 \
    }                                                                                                              \
  } while (0)
#define MPIT_TN_OPT_IN64(A, B, ST, CV)                                                                             \
  do {                                                                                                             \
    static const bool opted = (hip_check(hipFuncSetAttribute(reinterpret_cast<const void*>(                       \
                                                             &gemm_tn_kernel<T, A, B, ST, CV, 0, 64>),            \
                                                         hipFuncAttributeMaxDynamicSharedMemorySize, int(shm)),    \
                                     "hipFuncSetAttribute"),                                                       \
                               true);                                                                              \
    (void)opted;                                                                                                   \
  } while (0)
#define MPIT_TN_K64S(A, B)                  \
  do {                                      \
    if (kr64_stages == 3) MPIT_TN_K64(A, B, 3); \
    else MPIT_TN_K64(A, B, 2);              \
  } while (0)
      if (tbn == 128 && tbk == 128) MPIT_TN_K64S(128, 128);
      else if (tbn == 128) MPIT_TN_K64S(128, 64);
      else if (tbk == 128) MPIT_TN_K64S(64, 128);
      else MPIT_TN_K64S(64, 64);
#undef MPIT_TN_K64S
#undef MPIT_TN_K64
#undef MPIT_TN_OPT_IN64
      done64 = true;
    }
  }
  if (!done64) {
  if (tbn == 128 && tbk == 128) MPIT_TN_LAUNCH(128, 128);
  else if (tbn == 128) MPIT_TN_LAUNCH(128, 64);
  else if (tbk == 128) MPIT_TN_LAUNCH(64, 128);
  else MPIT_TN_LAUNCH(64, 64);
  }
  }
#undef MPIT_TN_LAUNCH
#undef MPIT_TN_LAUNCH1
#undef MPIT_TN_OPT_IN
  hip_check(hipGetLastError(), "gemm_tn launch");
  if (!direct && !fused) {
    const int64_t n4 = int64_t(N) * K / 4;
    const unsigned gx = unsigned((n4 + 255) / 256);
    const int64_t groups = tn_groups(ns);
    const float4* src = reinterpret_cast<const float4*>(part);
    int nsrc = ns;
    if (groups) {  // level 1: groups of kReduceGroup splits -> ws tail
      float4* mid = reinterpret_cast<float4*>(part + int64_t(ns) * N * K);
      hipLaunchKernelGGL(split_reduce_kernel, dim3(gx, unsigned(groups)), dim3(256), 0, s, src, ns, n4, mid, beta);
      hip_check(hipGetLastError(), "gemm_tn reduce launch");
      src = mid;
      nsrc = int(groups);
    }
    hipLaunchKernelGGL(split_reduce_kernel, dim3(gx, 1), dim3(256), 0, s, src, nsrc, n4,
                       reinterpret_cast<float4*>(out), beta);
    hip_check(hipGetLastError(), "gemm_tn reduce launch");
  }
}

static void launch_tn(int dev, hipStream_t s, int64_t M, int N, int K, uintptr_t Y, int64_t ldy, uintptr_t X,
                      int64_t ldx, uintptr_t out, uintptr_t ws, float beta, const ConvGeo* geo, bool f32,
                      uintptr_t amax_y = 0, uintptr_t amax_x = 0, int64_t yps = 0, int64_t xps = 0) {
  // fp32 operands given as fp16 planes (yps / xps > 0): the 16-bit kernel's FM 13
  if (f32 && (yps > 0 || xps > 0)) {
    if (yps <= 0 || xps <= 0) throw std::invalid_argument("gemm_tn: both operands must be planes (FM 13)");
    if (f32_mode() != 1) throw std::invalid_argument("gemm_tn: fp16 planes are the fp16x3 path");
    launch_tn_t<uint16_t>(dev, s, M, N, K, Y, ldy, X, ldx, out, ws, beta, geo, amax_y, amax_x, yps, xps);
    return;
  }
  if (f32) launch_tn_t<float>(dev, s, M, N, K, Y, ldy, X, ldx, out, ws, beta, geo, amax_y, amax_x);
  else if (amax_y || amax_x || yps || xps) throw std::invalid_argument("gemm_tn: operand bounds are for fp32 (fp16x3) calls");
  else launch_tn_t<uint16_t>(dev, s, M, N, K, Y, ldy, X, ldx, out, ws, beta, geo, 0, 0);
}

void gemm_tn(int dev, hipStream_t s, int64_t M, int N, int K, uintptr_t Y, int64_t ldy, uintptr_t X, int64_t ldx,
             uintptr_t out, uintptr_t ws, float beta, bool f32, uintptr_t amax_y, uintptr_t amax_x, int64_t yps,
             int64_t xps) {
  launch_tn(dev, s, M, N, K, Y, ldy, X, ldx, out, ws, beta, nullptr, f32, amax_y, amax_x, yps, xps);
}

// ------------------------------------------------------------------ convolutions
static ConvGeo conv_geo(int H, int W, int C, int R, int S, int stride, int pad, int* Ho, int* Wo) {
  if (H <= 0 || W <= 0 || C <= 0 || R <= 0 || S <= 0 || stride <= 0 || pad < 0)
    throw std::invalid_argument("conv: bad geometry");
  *Ho = (H + 2 * pad - R) / stride + 1;
  *Wo = (W + 2 * pad - S) / stride + 1;
  if (*Ho <= 0 || *Wo <= 0) throw std::invalid_argument("conv: empty output");
  return ConvGeo{H, W, C, *Ho, *Wo, S, stride, pad, pad, 1, 0, 0, *Ho, *Wo, 0};
}

bool conv_supported(int C, int Co) { return C % 32 == 0 && Co % 64 == 0; }

void conv_fwd(int dev, hipStream_t s, int Nb, int H, int W, int C, int Co, int R, int S, int stride, int pad,
              uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t stats, uintptr_t cin, uintptr_t bias, bool relu,
              const BnRed* red, bool f32, int64_t bps) {
  if (!conv_supported(C, Co)) throw std::invalid_argument("conv_fwd: need C % 32 == 0 and Co % 64 == 0");
  if (int64_t(Nb) * H * W * C >= (int64_t(1) << 31)) throw std::invalid_argument("conv_fwd: input too large");
  int Ho, Wo;
  const ConvGeo g = conv_geo(H, W, C, R, S, stride, pad, &Ho, &Wo);
  const int64_t M = int64_t(Nb) * Ho * Wo;
  int mode;
  const EpiArgs ep = epi_args(stats, red, &mode);
  launch_nt(dev, s, M, Co, R * S * C, x, C, w, int64_t(R) * S * C, y, Co, cin, 0, &g, ep, mode, f32, bias, relu, bps);
}

int64_t conv_wgrad_ws_floats(int dev, int Nb, int H, int W, int C, int Co, int R, int S, int stride, int pad) {
  int Ho, Wo;
  conv_geo(H, W, C, R, S, stride, pad, &Ho, &Wo);
  const int64_t M = int64_t(Nb) * Ho * Wo;
  const int K = R * S * C;
  int64_t rps;
  int tbn, tbk;
  const int ns = tn_plan(dev, M, Co, K, &rps, &tbn, &tbk, C);
  return ns > 1 ? (int64_t(ns) + tn_groups(ns)) * Co * K : 0;
}

void conv_wgrad(int dev, hipStream_t s, int Nb, int H, int W, int C, int Co, int R, int S, int stride, int pad,
                uintptr_t dy, uintptr_t x, uintptr_t dw, uintptr_t ws, float beta, bool f32, uintptr_t amax_y,
                uintptr_t amax_x, int64_t yps, int64_t xps) {
  if (C % 64 || Co % 64) throw std::invalid_argument("conv_wgrad: need C % 64 == 0 and Co % 64 == 0");
  if (int64_t(Nb) * H * W * C >= (int64_t(1) << 31)) throw std::invalid_argument("conv_wgrad: input too large");
  int Ho, Wo;
  const ConvGeo g = conv_geo(H, W, C, R, S, stride, pad, &Ho, &Wo);
  const int64_t M = int64_t(Nb) * Ho * Wo;
  launch_tn(dev, s, M, Co, R * S * C, dy, Co, x, C, dw, ws, beta, &g, f32, amax_y, amax_x, yps, xps);
}

// Row-tap stem convolution: x is a zero-padded NHWC4 image [Nb][Hp][Wp][4] (bf16 / fp32), the
// kernel has `rows` rows of 8 pixels x 4 channels (K = rows * 32; a 7x7x3 kernel zero-extended
// to 8 rows, a 3x3x3 one to 3), output pixel (ho, wo) reads rows ho*stride + r, pixels
// wo*stride .. +7 of each.
static ConvGeo stem_geo(int Nb, int Hp, int Wp, int Ho, int Wo, int stride, int rows) {
  if (rows < 1 || rows > 8) throw std::invalid_argument("conv_stem: 1 <= rows <= 8");
  if (Nb <= 0 || Ho <= 0 || Wo <= 0 || stride <= 0 || Hp < (Ho - 1) * stride + rows || Wp < (Wo - 1) * stride + 8)
    throw std::invalid_argument("conv_stem: padded image too small for the output");
  if (int64_t(Nb) * Hp * Wp * 4 >= (int64_t(1) << 31)) throw std::invalid_argument("conv_stem: input too large");
  return ConvGeo{Hp, Wp, kStemTap, Ho, Wo, 1, stride, 0, 0, 1, 0, 0, Ho, Wo, 0, 4};
}

int stem_wgrad_rows(int rows) { return rows + (rows & 1); }

void conv_stem_fwd(int dev, hipStream_t s, int Nb, int Hp, int Wp, int Co, int Ho, int Wo, int stride, uintptr_t x,
                   uintptr_t w, uintptr_t y, uintptr_t stats, bool f32, int64_t bps, uintptr_t amax_a,
                   uintptr_t amax_b, const BnRed* fold, int rows, uintptr_t bias, bool relu) {
  if (Co % 64) throw std::invalid_argument("conv_stem_fwd: need Co % 64 == 0");
  const ConvGeo g = stem_geo(Nb, Hp, Wp, Ho, Wo, stride, rows);
  int mode;
  BnRed r = fold ? *fold : BnRed{};
  r.amax_a = amax_a;
  r.amax_b = amax_b;
  const EpiArgs ep = epi_args(stats, &r, &mode);
  if (mode != EPI_NONE && (bias || relu)) throw std::invalid_argument("conv_stem_fwd: statistics and bias/ReLU are exclusive");
  const int K = rows * kStemTap;
  launch_nt(dev, s, int64_t(Nb) * Ho * Wo, Co, K, x, kStemTap, w, K, y, Co, 0, 0, &g, ep, mode, f32, bias, relu, bps);
}

int64_t conv_stem_wgrad_ws_floats(int dev, int Nb, int Ho, int Wo, int Co, int rows) {
  const int K = stem_wgrad_rows(rows) * kStemTap;
  int64_t rps;
  int tbn, tbk;
  const int ns = tn_plan(dev, int64_t(Nb) * Ho * Wo, Co, K, &rps, &tbn, &tbk, kStemTap);
  return ns > 1 ? (int64_t(ns) + tn_groups(ns)) * Co * K : 0;
}

void conv_stem_wgrad(int dev, hipStream_t s, int Nb, int Hp, int Wp, int Co, int Ho, int Wo, int stride, uintptr_t dy,
                     uintptr_t x, uintptr_t dw, uintptr_t ws, bool f32, uintptr_t amax_y, uintptr_t amax_x, int rows) {
  if (Co % 64) throw std::invalid_argument("conv_stem_wgrad: need Co % 64 == 0");
  const int rw = stem_wgrad_rows(rows);
  const ConvGeo g = stem_geo(Nb, Hp, Wp, Ho, Wo, stride, rw);
  launch_tn(dev, s, int64_t(Nb) * Ho * Wo, Co, rw * kStemTap, dy, Co, x, kStemTap, dw, ws, 0.f, &g, f32, amax_y,
            amax_x);
}

static void launch_cast(int dev, hipStream_t s, uintptr_t w, int R, int Cc, uintptr_t wb, uintptr_t wt, int taps,
                        const TapMap& map, bool f32) {
  if (taps < 1 || taps > kMaxTaps) throw std::invalid_argument("cast_transpose: 1 <= taps <= 49");
  hip_check(hipSetDevice(dev), "hipSetDevice");
  const dim3 grid((Cc + 31) / 32, (R + 31) / 32, taps);
  if (f32)
    hipLaunchKernelGGL(cast_transpose_kernel<float>, grid, dim3(256), 0, s, reinterpret_cast<const float*>(w), R, Cc,
                       taps, reinterpret_cast<float*>(wb), reinterpret_cast<float*>(wt), map);
  else
    hipLaunchKernelGGL(cast_transpose_kernel<uint16_t>, grid, dim3(256), 0, s, reinterpret_cast<const float*>(w), R,
                       Cc, taps, reinterpret_cast<uint16_t*>(wb), reinterpret_cast<uint16_t*>(wt), map);
  hip_check(hipGetLastError(), "cast_transpose launch");
}

void cast_transpose(int dev, hipStream_t s, uintptr_t w, int R, int Cc, uintptr_t wb, uintptr_t wt, int taps, bool f32) {
  TapMap map{};
  for (int t = 0; t < taps && t < kMaxTaps; ++t) {
    map.base[t] = 0;
    map.tc[t] = int16_t(taps);
    map.dt[t] = int16_t(taps - 1 - t);
  }
  launch_cast(dev, s, w, R, Cc, wb, wt, taps, map, f32);
}

// ---- backward-data of a strided conv as stride^2 parity classes ----------------------
// Output pixel h = st*i + ph receives taps r with (ph + pad - r) % st == 0 from dY row
// i + q(r), q(r) = (ph + pad - r) / st. Class (ph, pw) is a stride-1 implicit GEMM over dY
// with the kernel {r} x {s} ordered by ascending q (window start = min q -> padding -min q)
// whose epilogue writes pixel (st*i + ph, st*j + pw).
struct StridedPlan {
  int ncls = 0;
  struct Cls {
    int ph, pw, nr, ns, padh, padw, Hc, Wc;
    int64_t base;  // element offset of the class weight [C][nr][ns][Co] in the packed buffer
  } cls[16];
  int64_t wfloats = 0;  // total bf16 elements of the packed class weights
  bool any_empty = false;
  TapMap map{};
};

static StridedPlan strided_plan(int H, int W, int C, int Co, int R, int S, int st, int pad) {
  StridedPlan P;
  if (st < 2 || st > 4 || R * S > kMaxTaps) throw std::invalid_argument("conv_dgrad_strided: bad geometry");
  for (int ph = 0; ph < st; ++ph)
    for (int pw = 0; pw < st; ++pw) {
      int rl[16], sl[16], nr = 0, ns = 0;
      for (int r = R - 1; r >= 0; --r)  // descending r = ascending q
        if (((ph + pad - r) % st + st) % st == 0) rl[nr++] = r;
      for (int c = S - 1; c >= 0; --c)
        if (((pw + pad - c) % st + st) % st == 0) sl[ns++] = c;
      // a class with no pixels (tiny image) keeps its weights in the layout; it is skipped
      // at launch
      const int Hc = std::max(0, (H - ph + st - 1) / st), Wc = std::max(0, (W - pw + st - 1) / st);
      if (nr == 0 || ns == 0) {
        if (Hc > 0 && Wc > 0) P.any_empty = true;
        continue;
      }
      auto q = [&](int p, int r) { return (p + pad - r) / st; };  // exact: divisible
      StridedPlan::Cls& k = P.cls[P.ncls++];
      k = {ph, pw, nr, ns, -q(ph, rl[0]), -q(pw, sl[0]), Hc, Wc, P.wfloats};
      for (int a = 0; a < nr; ++a)
        for (int b = 0; b < ns; ++b) {
          const int t = rl[a] * S + sl[b];
          P.map.base[t] = k.base;
          P.map.tc[t] = int16_t(nr * ns);
          P.map.dt[t] = int16_t(a * ns + b);
        }
      P.wfloats += int64_t(C) * nr * ns * Co;
    }
  return P;
}

int64_t conv_dgrad_strided_wfloats(int C, int Co, int R, int S, int stride, int pad) {
  return strided_plan(2 * stride, 2 * stride, C, Co, R, S, stride, pad).wfloats;
}

void conv_dgrad_strided_weights(int dev, hipStream_t s, uintptr_t w, int Co, int C, int R, int S, int stride, int pad,
                                uintptr_t wb, uintptr_t wcls, bool f32) {
  const StridedPlan P = strided_plan(2 * stride, 2 * stride, C, Co, R, S, stride, pad);
  launch_cast(dev, s, w, Co, C, wb, wcls, R * S, P.map, f32);
}

int64_t conv_dgrad_strided_tiles(int Nb, int H, int W, int C, int Co, int R, int S, int stride, int pad) {
  const StridedPlan P = strided_plan(H, W, C, Co, R, S, stride, pad);
  int64_t t = 0;
  for (int k = 0; k < P.ncls; ++k)
    if (P.cls[k].Hc > 0 && P.cls[k].Wc > 0) t += gemm_nt_tiles(int64_t(Nb) * P.cls[k].Hc * P.cls[k].Wc);
  return t;
}

int64_t cast_job_bytes() { return int64_t(sizeof(CastJob)); }

int64_t cast_jobs_build(uintptr_t host_table, const std::vector<std::array<int64_t, 11>>& specs) {
  auto* jobs = reinterpret_cast<CastJob*>(host_table);
  int64_t blocks = 0;
  for (size_t k = 0; k < specs.size(); ++k) {
    const auto& q = specs[k];
    // q[0] = kind | f32 << 8 (fp32 outputs: transposes only, the plain copy is the master weight)
    //        | 512: wb as three pre-split bf16 planes (else none: the forward reads the master)
    //        | 1024: wt as three pre-split bf16 planes (else fp32)
    //        | 2048: the planes are fp16x3's two fp16 planes, scaled by the bound at q[10]
    //        | 4096: a classifier weight: its transpose only (bf16, or fp32 with f32; 64 x 64 tiles
    //          when they fit), rows of q[9] elements when q[9] > 0 (a padded output layer's
    //          wt[K][Np]: the Np - Co pad columns are never written, the caller zeroes them once)
    const int kind = int(q[0] & 0xff), Co = int(q[4]), C = int(q[5]), R = int(q[6]), S = int(q[7]);
    const int stride = int(q[8]), pad = int(q[9]);
    CastJob J{};
    J.w = reinterpret_cast<const float*>(q[1]);
    const bool pl_b = (q[0] >> 9) & 1, pl_t = (q[0] >> 10) & 1;
    J.f32 = pl_b || pl_t ? 2 : int((q[0] >> 8) & 1);
    J.f16 = int((q[0] >> 11) & 1);
    J.amax = reinterpret_cast<const float*>(q[10]);
    if (J.f16 && (J.f32 != 2 || !J.amax)) throw std::invalid_argument("cast_jobs_build: fp16 planes need planes and a bound");
    J.wb = (J.f32 == 1 || (J.f32 == 2 && !pl_b)) ? nullptr : reinterpret_cast<void*>(q[2]);
    if (J.f32 == 2) {
      J.pb = int64_t(Co) * R * S * C;
      J.pt = !pl_t ? 0 : kind == 1 ? conv_dgrad_strided_wfloats(C, Co, R, S, stride, pad) : int64_t(C) * R * S * Co;
    }
    J.wt = reinterpret_cast<void*>(q[3]);
    J.R = Co;
    J.Cc = C;
    J.T = R * S;
    J.ldt = ((q[0] >> 12) & 1) && pad > 0 ? pad : Co;
    if (J.ldt < Co) throw std::invalid_argument("cast_jobs_build: transpose rows shorter than the weight's");
    if (J.T < 1 || J.T > kMaxTaps) throw std::invalid_argument("cast_jobs_build: 1 <= taps <= 49");
    if (kind == 1) {  // strided backward-data: parity-class packed weights
      J.map = strided_plan(2 * stride, 2 * stride, C, Co, R, S, stride, pad).map;
    } else {  // tap-flipped transpose (a plain transpose for 1x1), or no transpose (kind 2)
      for (int t = 0; t < J.T; ++t) {
        J.map.base[t] = 0;
        J.map.tc[t] = int16_t(J.T);
        J.map.dt[t] = int16_t(J.T - 1 - t);
      }
      if (kind == 2) J.wt = nullptr;
    }
    J.big = ((q[0] >> 12) & 1) && J.f32 == 0 && kind == 0 && J.T == 1 && C % 64 == 0 && Co % 128 == 0 && !J.wb &&
            J.wt && q[1] % 16 == 0 && q[3] % 8 == 0 && J.ldt == Co;
    J.tcx = J.big ? C / 64 : (C + 31) / 32;
    J.tcy = J.big ? Co / 128 : (Co + 31) / 32;
    J.block0 = blocks;
    blocks += int64_t(J.tcx) * J.tcy * J.T;
    jobs[k] = J;
  }
  if (blocks > INT32_MAX) throw std::invalid_argument("cast_jobs_build: too many blocks");
  return blocks;
}

void cast_jobs_run(int dev, hipStream_t s, uintptr_t dev_table, int njobs, int64_t nblocks, uintptr_t amax) {
  if (njobs <= 0 || nblocks <= 0) return;
  hip_check(hipSetDevice(dev), "hipSetDevice");
  if (amax) {  // the fp16-plane jobs' bound (every such job points at this buffer)
    hip_check(hipMemsetAsync(reinterpret_cast<void*>(amax), 0, kBoundFloats * sizeof(float), s), "cast amax zero");
    hipLaunchKernelGGL(cast_amax_kernel, dim3(unsigned(nblocks)), dim3(256), 0, s,
                       reinterpret_cast<const CastJob*>(dev_table), njobs, nblocks);
  }
  hipLaunchKernelGGL(cast_batch_kernel, dim3(unsigned(nblocks)), dim3(256), 0, s,
                     reinterpret_cast<const CastJob*>(dev_table), njobs);
  hip_check(hipGetLastError(), "cast_batch launch");
}

void conv_dgrad_strided(int dev, hipStream_t s, int Nb, int H, int W, int C, int Co, int R, int S, int stride, int pad,
                        uintptr_t dy, uintptr_t wcls, uintptr_t dx, const BnRed* red, bool f32, int64_t bps) {
  if (C % 64 || Co % 32) throw std::invalid_argument("conv_dgrad_strided: need C % 64 == 0 and Co % 32 == 0");
  int Ho, Wo;
  conv_geo(H, W, C, R, S, stride, pad, &Ho, &Wo);
  if (int64_t(Nb) * Ho * Wo * Co >= (int64_t(1) << 31)) throw std::invalid_argument("conv_dgrad_strided: too large");
  const StridedPlan P = strided_plan(H, W, C, Co, R, S, stride, pad);
  // the only class with taps is (0,0) of a stride-2 conv: its epilogue zero-fills the rest
  const bool ozero = P.any_empty && stride == 2 && P.ncls == 1 && P.cls[0].ph == 0 && P.cls[0].pw == 0;
  if (P.any_empty && !ozero) {
    hip_check(hipSetDevice(dev), "hipSetDevice");
    hip_check(hipMemsetAsync(reinterpret_cast<void*>(dx), 0, size_t(Nb) * H * W * C * (f32 ? 4 : 2), s), "dgrad zero fill");
  }
  int64_t row0 = 0;
  for (int k = 0; k < P.ncls; ++k) {
    const auto& c = P.cls[k];
    if (c.Hc == 0 || c.Wc == 0) continue;
    ConvGeo g{Ho, Wo, Co, c.Hc, c.Wc, c.ns, 1, c.padh, c.padw, stride, c.ph, c.pw, H, W, ozero ? 1 : 0};
    const int64_t M = int64_t(Nb) * c.Hc * c.Wc;
    const int K = c.nr * c.ns * Co;
    // BN reduction: each class writes its own run of partial rows (zero-filled pixels
    // contribute nothing)
    int mode;
    EpiArgs ep = epi_args(0, red, &mode);
    ep.fcoef = nullptr;  // several launches write the partials: no folded finalize
    ep.row0 += row0;
    row0 += gemm_nt_tiles(M);
    // bps > 0: wcls holds three bf16 planes of bps elements each (class offsets in elements)
    launch_nt(dev, s, M, C, K, dy, Co, wcls + uintptr_t(c.base) * (f32 && !bps ? 4 : 2), K, dx, C, 0, 0, &g, ep, mode,
              f32, 0, false, bps);
  }
}

}  // namespace mpit

// Public C++ interface of the mpit HIP kernels (gfx950) and their host twins.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <array>
#include <vector>

namespace mpit {

// ---- fused elementwise update rules (updates.hip) --------------------------------
enum Rule : int {
  kApply = 0,        // K1   [p, g, (out)]                     sc: a
  kApplySum = 1,     // K1   [p, g0..g{NG-1}, (out)]           sc: a          variant |= NG << 8
  kRMSProp = 2,      // K2   [p, g, ga, gs, u, (out)]          sc: decay lr mom eps
  kAdam = 3,         // K3   [p, g, m, v, (out)]               sc: b1 b2 eps lr_t
  kAdamax = 4,       // K4   [p, g, m, u, (out)]               sc: b1 b2 eps lr_t
  kAdagrad = 5,      // K5   [p, g, var, (out)]                sc: eps clr
  kAdadelta = 6,     // K6   [p, g, var, acc, (out)]           sc: rho eps lr
  kNesterovPre = 7,  // K7   [vt, w]                           sc: mom
  kNesterovPost = 8, // K8   [w, g, vt, sug]                   sc: gscale l2wd clr
  kDownpour = 9,     // K9   [g, w, acc]                       sc: lr gscale l2wd  variant = mode
  kElastic = 10,     // K10  [w, c, sug]                       sc: mva
  kRegClip = 11,     // K11  [g, p]                            sc: gscale l1 l2 clip
  kScale = 12,       // K14  [x]                               sc: a
  kCopy = 13,        //      [dst, src]                        sc: a
  kFill = 14,        //      [dst]                             sc: v
  kAxpby = 15,       //      [y, x]                            sc: a b
};
enum Variant : int {
  kOut = 1 << 2,  // server rules: also write the new p to the last operand
  kAdd = 1 << 3,  // RMSProp: add u into p (global mode); otherwise produce u only (local)
  kVt = 1 << 4,   // Nesterov post: momentum buffer present
  kSug = 1 << 5,  // Nesterov post: fused EASGD "w -= sug"
};

// dev < 0 → host; else launch on `s` (device `dev`). bf = bitmask of bf16 operands.
void ew_update(int rule, int variant, int dev, hipStream_t s, int64_t n, const std::vector<uintptr_t>& ptrs,
               uint32_t bf, const std::vector<float>& sc);
// The same rule over several disjoint segments (ns[i] elements, operands ptrs[i]) in ONE
// launch (ew.h ew_multi_kernel); host, unaligned or > 16 segments: one pass per segment.
void ew_update_multi(int rule, int variant, int dev, hipStream_t s, const std::vector<int64_t>& ns,
                     const std::vector<std::vector<uintptr_t>>& ptrs, uint32_t bf, const std::vector<float>& sc);

// ---- reductions (reduce.hip) ------------------------------------------------------
// out[0] = Σ|x|, out[1] = Σx², out[2] = max|x|  (deterministic two-pass; `ws` holds
// kNormWsFloats floats of device scratch; ignored on host).
constexpr int kNormMaxBlocks = 1024;
constexpr int kNormWsFloats = 3 * kNormMaxBlocks;
void norms(int dev, hipStream_t s, const void* x, bool bf16, int64_t n, float* out, float* ws);
// out[0] = Σ x*y (fp32 accumulate), deterministic
void dot(int dev, hipStream_t s, const void* x, const void* y, bool bf16, int64_t n, float* out, float* ws);

// G[j] = clamp(G[j] + g[k][j] + l1*sign(p[j]) + l2*p[j], -c, c) for k = 0..n-1 in order
// (c <= 0: no clamp): the reference's per-example regularise + clamp of the accumulated
// gradient (BiCNN/bicnn.lua:398-409). g: n rows of stride ldg floats. fp32, dev < 0 = host.
void clamp_scan(int dev, hipStream_t s, float* G, const float* g, const float* p, int64_t P, int64_t ldg, int n,
                float l1, float l2, float c);

// ---- multi-tensor pack / unpack with cast (multi_copy.hip) ------------------------
struct CopyChunk {
  uint64_t src;    // byte address of the first element
  uint64_t dst;
  int64_t n;       // elements
  int32_t flags;   // bit0 src bf16, bit1 dst bf16
  int32_t pad;
};
// `table` = device (or host when dev < 0) array of `nchunks` CopyChunk. dst = scale*src.
void multi_copy(int dev, hipStream_t s, const CopyChunk* table, int64_t nchunks, float scale);

// ---- gradient gather + Downpour scale (gather.hip) ---------------------------------
// dst[off_t + i] = a*src_t[i] + b*aux[off_t + i]  (fp32; aux optional), one launch per
// kGatherMaxT tensors, table passed by value.
constexpr int kGatherMaxT = 128;
void gather_scale(int dev, hipStream_t s, const std::vector<uintptr_t>& srcs, const std::vector<int64_t>& offs,
                  const std::vector<int64_t>& ns, uintptr_t dst, uintptr_t aux, float a, float b);

// ---- fused BatchNorm (+residual) (+ReLU), NHWC, training (bn_act.hip) -------------
// x / res / y / dy / dx / dres: [M, C] row-major (channels_last), bf16 or fp32.
// mask: ReLU bit mask written by the forward (bn_mask_bytes: one byte per 8 channels, either
// dtype) and read by the backward. C % 8 == 0.
int64_t bn_workspace_floats(int C);
// fp16 planes output of an fp32 apply pass (the fp16x3 GEMMs then split nothing: gemm.hip
// FM 13). The pass writes h, l = the two fp16 planes of out * 2^e (h at element i, l at
// element i + numel of the 16-bit view of the output), e from a bound of |out| known BEFORE
// the pass: the maxima of its inputs (xmax / xmax2 / gmax: epoch slots a GEMM epilogue raised,
// gemm.hip EpiArgs::omax; rbound: the residual's bound) times its per-channel coefficients.
// obound (kBoundFloats) receives that bound in slot 0 (the other slots 0) for the consumers.
// rplanes: the residual arrives as planes (decoded with rbound's scale).
struct PlaneSpec {
  uintptr_t obound = 0;
  uintptr_t xmax = 0, xmax2 = 0, gmax = 0;
  uint32_t xep = 0, xep2 = 0, gep = 0;
  uintptr_t rbound = 0;
  int rplanes = 0;
};
int64_t bn_mask_bytes(bool bf16, int64_t M, int C);
// stats / nstat (optional): the statistics of x as per-128-row-tile (mean, M2) partials
// [nstat][2][C] emitted by the GEMM that produced x (EPI_STATS) — the statistics pass over
// x is skipped.
void bn_act_fwd(int dev, hipStream_t s, bool bf16, uintptr_t x, uintptr_t res, uintptr_t y, int64_t M, int C,
                uintptr_t gamma, uintptr_t beta, uintptr_t rmean, uintptr_t rvar, uintptr_t save_mean,
                uintptr_t save_rstd, uintptr_t ws, float momentum, float eps, bool relu, uintptr_t mask,
                uintptr_t stats = 0, int64_t nstat = 0, uintptr_t amax = 0, uintptr_t coef = 0,
                const PlaneSpec* planes = nullptr);
// amax (optional, fp32 [1]): max |y| over the tensor (bn_act_bwd: max |dx|), the scale bound of the
// fp16x3 GEMMs that read it: zeroed by this call's finalize, raised by its apply pass. With
// y / dx null (the coefficient-only calls of a bn_pair) amax is only zeroed, for the pair
// apply that follows. Given coefficients (bn_act_bwd coef), the GEMM that folded the finalize
// zeroed it (BnRed::fzero).
// y = act(x*coef[c] + coef[C+c] (+res))  — eval mode / precomputed coefficients
void bn_act_apply(int dev, hipStream_t s, bool bf16, uintptr_t x, uintptr_t res, uintptr_t y, int64_t M, int C,
                  uintptr_t coef, bool relu);
// part / npart (optional): (sum dz, sum dz*(x-mean)) partials [npart][2][C] already
// produced by the GEMM that wrote dy (EPI_BNRED) — the reduction pass is skipped.
void bn_act_bwd(int dev, hipStream_t s, bool bf16, uintptr_t dy, uintptr_t mask, uintptr_t x, uintptr_t dx,
                uintptr_t dres, int64_t M, int C, uintptr_t gamma, uintptr_t mean, uintptr_t rstd, uintptr_t dgamma,
                uintptr_t dbeta, uintptr_t ws, bool relu, uintptr_t part = 0, int64_t npart = 0,
                uintptr_t coef = 0, uintptr_t amax = 0, const PlaneSpec* planes = nullptr);
// coef (optional): the apply coefficients [3][C] already computed (the finalize folded into
// the GEMM that wrote dy, BnRed::fcoef; dgamma / dbeta written there too): apply pass only.

// bn_act_fwd with y == 0 / bn_act_bwd with dx == 0 only compute the coefficients into
// ws[0, 2C) (scale, shift) / ws[0, 3C) (A, C, B) and the running stats / dgamma, dbeta.
// A block's last BN and its downsample shortcut's BN as one op (bf16 or fp32, ReLU):
// y = relu(bn1(x1) + bn2(x2)) from the two forward coefficient sets, and the backward
// dx1 / dx2 from the two backward sets, one pass each.
void bn_pair_apply(int dev, hipStream_t s, uintptr_t x1, uintptr_t coef1, uintptr_t x2, uintptr_t coef2, uintptr_t y,
                   int64_t M, int C, uintptr_t mask, bool f32 = false, uintptr_t amax = 0, uintptr_t scratch = 0,
                   const PlaneSpec* planes = nullptr);
// amax / amax1 / amax2: raised by the pass (zeroed beforehand: the bn_act_fwd / bwd coefficient
// calls of the pair zero them); scratch: unused (kept for the call signature)
void bn_pair_bwd_apply(int dev, hipStream_t s, uintptr_t dy, uintptr_t mask, uintptr_t x1, uintptr_t coef1,
                       uintptr_t dx1, uintptr_t x2, uintptr_t coef2, uintptr_t dx2, int64_t M, int C, bool f32 = false,
                       uintptr_t amax1 = 0, uintptr_t amax2 = 0, uintptr_t scratch = 0,
                       const PlaneSpec* planes1 = nullptr, const PlaneSpec* planes2 = nullptr);

// ---- MFMA GEMMs for NHWC 1x1 convolutions (gemm.hip), fp32 accumulate -------------------
// Operands and outputs are bf16 (v_mfma_f32_32x32x16_bf16) or, with f32 = true, fp32
// (v_mfma_f32_32x32x2_f32: exact fp32 products). Everything said below of bf16 tensors holds
// for fp32 ones in an f32 call; ReLU bit masks are one byte per 8 channels either way.
// C[M,N] (bf16) = A[M,K] . B[N,K]^T; optional per-column (mean, M2) partials of C per
// 128-row tile into stats[ceil(M/128)][2][N] (gemm_nt_stats_floats); optional bf16 cin
// [M, ldc] added to the product before rounding (may alias C); optional cmask (with cin,
// ldc == N): the bn_act ReLU bit mask of cin (1 byte / 8 channels) — adds cin*mask.
// Optional red: C is the output gradient of a bn_act layer (x, mask, mean its forward
// input / ReLU mask / batch mean, [.., N] like C): the GEMM also writes that layer's
// backward reduction partials (sum dz, sum dz*(x-mean)), dz = C*mask, one row pair per
// 128-row tile at part[row0 + tile][2][N] — bn_act_bwd(part, npart) then skips its pass.
// x2 / mean2 / part2 (optional): a second BN fed by the same gradient (the downsample
// shortcut's BN of a bn_pair): its (sum dz, sum dz*(x2-mean2)) go to part2.
// Output bounds (fp16x3 operand scales): kBoundSlots fp32 maxima kBoundStride floats apart
// (one 128-B line each, so the producers' one-atomic-per-block maxima spread over 16 lines
// instead of serialising on one address); the bound is the max over the slots.
constexpr int kBoundSlots = 16, kBoundStride = 32, kBoundFloats = kBoundSlots * kBoundStride;
struct BnRed {
  uintptr_t part = 0, x = 0, mask = 0, mean = 0;
  int64_t row0 = 0;
  uintptr_t part2 = 0, x2 = 0, mean2 = 0;
  // fold the BN backward's finalize into the GEMM (single EPI_BNRED launch): coefficients
  // [3][N], dgamma / dbeta [N], from gamma (or 0) and rstd; lvl: gemm_nt_fold_lvl_floats(N)
  uintptr_t fcoef = 0, fgamma = 0, frstd = 0, fdgamma = 0, fdbeta = 0, flvl = 0;
  // fp32 fp16x3 GEMMs (gemm.hip FM 11): device fp32 upper bounds of |A| and of |B|; amax_b
  // marks B (bps > 0) as the two fp16 planes of the weight scaled by its bound's 2^e
  uintptr_t amax_a = 0, amax_b = 0;
  // with fcoef: an output bound the folded finalize sets to zero (the BN backward's apply pass
  // then raises it to max |dx|)
  uintptr_t fzero = 0;
  // with the forward statistics (stats != 0): fold the BN forward's finalize into the GEMM
  // (single launch): scale / shift [2][N], save mean / rstd [N], running mean / var (or 0)
  // updated with momentum, from gamma / beta (or 0) and eps; lvl: gemm_nt_fold_lvl_floats(N);
  // zero: the BN output's bound, set to zero (the BN apply pass raises it)
  uintptr_t scoef = 0, sgamma = 0, sbeta = 0, srmean = 0, srvar = 0, smean = 0, srstd = 0, slvl = 0, szero = 0;
  float seps = 1e-5f, smom = 0.1f;
  // relu_y: instead of a BN reduction, the epilogue applies the ReLU of the conv(+bias)(+ReLU)
  // layer whose output x is this GEMM's input-gradient target: C = A.B^T * (x > 0) is that
  // layer's dz, and part[tile][0][N] its per-tile column sums (its bias gradient, col_sums)
  int relu_y = 0;
  // ftag: the fold's partials are (value, epoch) pairs (2 x the floats of part) in a buffer
  // that held only pairs of earlier launches (zeroed once, never garbage): the tagged fold
  // protocol of gemm.hip, in which no block waits for its own output stores
  int ftag = 0;
  // aps > 0 (with amax_b): A is two fp16 planes h, l of A * 2^e (e from amax_a), the l plane
  // aps elements after the h plane (gemm.hip FM 13: nothing split in the kernel)
  int64_t aps = 0;
  // omax (fp32 GEMMs): the launch's max |C| as 64-bit (epoch oepoch, value) maxima in kBoundSlots
  // slots kBoundStride floats apart (planes.h epoch_max reads them)
  uintptr_t omax = 0;
  uint32_t oepoch = 0;
};
int64_t gemm_nt_fold_lvl_floats(int N);
bool gemm_nt_supported(int64_t M, int N, int K, bool f32 = false);
int64_t gemm_nt_tiles(int64_t M);
int64_t gemm_nt_stats_floats(int64_t M, int N);
// bps > 0 (fp32 only): B is three pre-split bf16 planes h, m, l (x = h + m + l exactly, see
// cast_jobs kind flag 512) of bps elements each — the kernel splits only A in registers
void gemm_nt(int dev, hipStream_t s, int64_t M, int N, int K, uintptr_t A, int64_t lda, uintptr_t B, int64_t ldb,
             uintptr_t C, int64_t ldc, uintptr_t stats, uintptr_t cin, uintptr_t cmask = 0,
             const BnRed* red = nullptr, bool f32 = false, int64_t bps = 0);
// out[N,K] (fp32) = beta*out + Y[M,N]^T . X[M,K]  (split over M; ws: gemm_tn_ws_floats)
bool gemm_tn_supported(int64_t M, int N, int K);
int64_t gemm_tn_ws_floats(int dev, int64_t M, int N, int K);
// compute units of device `dev`; a stream restricted to the CUs of `mask` (gemm.hip)
int device_cu_count(int dev);
uintptr_t stream_create_cu_masked(int dev, const std::vector<uint32_t>& mask);
// amax_y / amax_x (fp32, both or neither): device bounds of |Y|, |X| -> fp16x3 split products
void gemm_tn(int dev, hipStream_t s, int64_t M, int N, int K, uintptr_t Y, int64_t ldy, uintptr_t X, int64_t ldx,
             uintptr_t out, uintptr_t ws, float beta, bool f32 = false, uintptr_t amax_y = 0, uintptr_t amax_x = 0, int64_t yps = 0,
             int64_t xps = 0);
// fp32 w[R][T][Cc] -> bf16 wb[R][T][Cc] (optional) and bf16 tap-flipped transpose
// wt[Cc][T-1-t][R] (optional); T = 1 is the plain transpose
void cast_transpose(int dev, hipStream_t s, uintptr_t w, int R, int Cc, uintptr_t wb, uintptr_t wt, int taps = 1,
                    bool f32 = false);
// Many casts in one launch. Job spec: {kind, w, wb, wt, Co, C, R, S, stride, pad}, kind 0 =
// cast + tap-flipped transpose (conv_weights / cast_transpose), 1 = cast + strided
// parity-class weights (conv_dgrad_strided_weights), 2 = cast only. The table is built on the
// host (cast_job_bytes() per job) and uploaded once; cast_jobs_run launches it.
int64_t cast_job_bytes();
int64_t cast_jobs_build(uintptr_t host_table, const std::vector<std::array<int64_t, 11>>& specs);
void cast_jobs_run(int dev, hipStream_t s, uintptr_t dev_table, int njobs, int64_t nblocks, uintptr_t amax = 0);

// ---- NHWC RxS convolutions as implicit GEMMs on the same MFMA kernels ----------------
// x [Nb,H,W,C], w [Co,R,S,C] (bf16), y [Nb,Ho,Wo,Co] (bf16); stats / cin as gemm_nt.
// Backward-data of a stride-1 conv = conv_fwd(dy, wt, pad' = R-1-pad) with wt the
// tap-flipped transpose [C,R,S,Co] (cast_transpose taps = R*S).
bool conv_supported(int C, int Co);
// bias (fp32 [Co], optional) and ReLU are applied in the epilogue.
void conv_fwd(int dev, hipStream_t s, int Nb, int H, int W, int C, int Co, int R, int S, int stride, int pad,
              uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t stats, uintptr_t cin, uintptr_t bias = 0,
              bool relu = false, const BnRed* red = nullptr, bool f32 = false, int64_t bps = 0);
// ReLU + bias backward: dz = dy * (y > 0) (bf16 [M, C]), db[c] = sum_m dz (fp32, optional,
// deterministic); ws: relu_bias_bwd_ws_floats(C)
// Backward-data of a strided conv (stride 2..4) as stride^2 parity-class implicit GEMMs
// over dy; wcls = packed class weights (conv_dgrad_strided_wfloats bf16 elements) made by
// conv_dgrad_strided_weights from the fp32 master (also writes wb like cast_transpose).
int64_t conv_dgrad_strided_wfloats(int C, int Co, int R, int S, int stride, int pad);
void conv_dgrad_strided_weights(int dev, hipStream_t s, uintptr_t w, int Co, int C, int R, int S, int stride, int pad,
                                uintptr_t wb, uintptr_t wcls, bool f32 = false);
// partial rows a BN reduction over the strided backward-data writes (all classes)
int64_t conv_dgrad_strided_tiles(int Nb, int H, int W, int C, int Co, int R, int S, int stride, int pad);
void conv_dgrad_strided(int dev, hipStream_t s, int Nb, int H, int W, int C, int Co, int R, int S, int stride, int pad,
                        uintptr_t dy, uintptr_t wcls, uintptr_t dx, const BnRed* red = nullptr, bool f32 = false,
                        int64_t bps = 0);
// softmax cross-entropy over rows of logits x [rows][ldx] (bf16 or fp32; loss.hip): per-row
// loss (fp32 [rows]) and the logits' gradient d = (softmax - onehot) * scale (fp32 [rows][C])
void softmax_xent(int dev, hipStream_t s, int64_t rows, int C, uintptr_t x, int64_t ldx, bool bf16, uintptr_t tgt,
                  float scale, uintptr_t loss, uintptr_t d);
int64_t relu_bias_bwd_ws_floats(int C);
// out[c] = sum over rows k < nb of part[k * ld + c] (fp32, fixed order: deterministic); mid:
// col_sums_ws_floats(C) floats of workspace (needed when nb > 64)
int64_t col_sums_ws_floats(int C);
void col_sums(hipStream_t s, const float* part, int64_t nb, int64_t ld, int C, float* out, float* mid);
void col_sums(int dev, hipStream_t s, uintptr_t part, int64_t nb, int64_t ld, int C, uintptr_t out, uintptr_t mid);
void relu_bias_bwd(int dev, hipStream_t s, int64_t M, int C, uintptr_t dy, uintptr_t y, uintptr_t dz, uintptr_t db,
                   uintptr_t ws, bool f32 = false);
// dw [Co,R,S,C] (fp32) = beta*dw + dY^T . im2col(x)   (C % 64 == 0, Co % 64 == 0)
int64_t conv_wgrad_ws_floats(int dev, int Nb, int H, int W, int C, int Co, int R, int S, int stride, int pad);
void conv_wgrad(int dev, hipStream_t s, int Nb, int H, int W, int C, int Co, int R, int S, int stride, int pad,
                uintptr_t dy, uintptr_t x, uintptr_t dw, uintptr_t ws, float beta, bool f32 = false,
                uintptr_t amax_y = 0, uintptr_t amax_x = 0, int64_t yps = 0,
                int64_t xps = 0);

// Row-tap stem conv (7x7 / stride-2 / 3-channel ResNet stem on MFMA; VGG's 3x3 / 3-channel
// first layer with rows = 3): x = zero-padded NHWC4 image [Nb][Hp][Wp][4], w = [Co][rows][8][4]
// (bf16, zero-extended kernel), y = [Nb][Ho][Wo][Co]; dw = [Co][rows_w][8][4] fp32 with rows_w =
// rows rounded up to even (the weight-gradient GEMM's K = rows_w * 32 must be a multiple of 64;
// the image then needs Hp >= (Ho - 1) * stride + rows_w); stats: BN statistics of y as conv_fwd;
// bias / relu: the conv(+bias)(+ReLU) epilogue of conv_fwd
void conv_stem_fwd(int dev, hipStream_t s, int Nb, int Hp, int Wp, int Co, int Ho, int Wo, int stride, uintptr_t x,
                   uintptr_t w, uintptr_t y, uintptr_t stats, bool f32 = false, int64_t bps = 0, uintptr_t amax_a = 0,
                   uintptr_t amax_b = 0, const BnRed* fold = nullptr, int rows = 8, uintptr_t bias = 0,
                   bool relu = false);
// (fp32 fp16x3: w as two fp16 planes of plane stride bps with bound amax_b, the image's bound amax_a;
// the wgrad's amax_y / amax_x as gemm_tn)
int64_t conv_stem_wgrad_ws_floats(int dev, int Nb, int Ho, int Wo, int Co, int rows = 8);
void conv_stem_wgrad(int dev, hipStream_t s, int Nb, int Hp, int Wp, int Co, int Ho, int Wo, int stride, uintptr_t dy,
                     uintptr_t x, uintptr_t dw, uintptr_t ws, bool f32 = false, uintptr_t amax_y = 0,
                     uintptr_t amax_x = 0, int rows = 8);
int stem_wgrad_rows(int rows);

// ---- NHWC bf16 / fp32 max pooling with a uint8 argmax per output element (pool.hip) ---
// x [N,H,W,C] -> y, idx [N,Ho,Wo,C]; dx [N,H,W,C] gathered from dy + idx (no atomics).
// obound (fp32, with ibound: x's slotted bound): y as fp16 planes (planes.h) scaled by x's bound
void maxpool_fwd(int dev, hipStream_t s, int N, int H, int W, int C, int K, int stride, int pad, uintptr_t x,
                 uintptr_t y, uintptr_t idx, bool f32 = false, uintptr_t ibound = 0, uintptr_t obound = 0);
// ypool (optional): the pool's output, when its input is a ReLU'd conv(+bias) output: dx is
// then that conv's dz = dx * (y > 0), and db (optional, fp32 [C]) its bias gradient; ws:
// maxpool_bwd_ws_floats(C) floats. Needs 256 % (C / 8) == 0.
void maxpool_bwd(int dev, hipStream_t s, int N, int H, int W, int C, int K, int stride, int pad, uintptr_t dy,
                 uintptr_t idx, uintptr_t dx, bool f32 = false, uintptr_t ypool = 0, uintptr_t db = 0,
                 uintptr_t ws = 0);
int64_t maxpool_bwd_ws_floats(int C);
// global average pool backward over NHWC: dx[n][p][c] = dy[n][c] / HW (bf16 / fp32)
void avgpool_bwd(int dev, hipStream_t s, int N, int HW, int C, uintptr_t dy, uintptr_t dx, bool f32 = false);

}  // namespace mpit

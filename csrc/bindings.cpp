// Python bindings of the mpit native runtime + kernels (module mpit_amd._mpit).
// Tensors cross the boundary as (data_ptr, numel, flags); streams as hipStream_t values
// (torch.cuda.current_stream().cuda_stream). Every blocking call releases the GIL.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "core/engine.h"
#include "core/ps.h"
#include "core/window.h"
#include "kernels/kernels.h"
#include "kernels/stem_pack.h"

namespace py = pybind11;
using namespace mpit;

namespace {
hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }
py::tuple st_tuple(const Status& s) { return py::make_tuple(s.source, s.tag, s.error, s.count, s.cancelled); }
}  // namespace

// the BN forward-finalize fold of a stats GEMM (gemm.hip stats_fold): None, or the tuple
// (coef, gamma, beta, running_mean, running_var, save_mean, save_rstd, lvl, zero, eps, momentum)
static void apply_sfold(BnRed& r, const py::object& f) {
  if (f.is_none()) return;
  auto t = f.cast<py::tuple>();
  if (t.size() != 11 && t.size() != 12) throw std::invalid_argument("bn fold: 11 or 12 fields");
  r.scoef = t[0].cast<uintptr_t>();
  r.sgamma = t[1].cast<uintptr_t>();
  r.sbeta = t[2].cast<uintptr_t>();
  r.srmean = t[3].cast<uintptr_t>();
  r.srvar = t[4].cast<uintptr_t>();
  r.smean = t[5].cast<uintptr_t>();
  r.srstd = t[6].cast<uintptr_t>();
  r.slvl = t[7].cast<uintptr_t>();
  r.szero = t[8].cast<uintptr_t>();
  r.seps = t[9].cast<float>();
  r.smom = t[10].cast<float>();
  if (t.size() == 12) r.ftag = t[11].cast<int>();  // tagged partials (gemm.hip stats_fold)
}

// a PlaneSpec (kernels.h) from Python: None, or a dict of its fields (missing ones 0)
static bool plane_spec(const py::object& o, PlaneSpec& ps) {
  if (o.is_none()) return false;
  const py::dict d = o.cast<py::dict>();
  auto u = [&](const char* k) -> uintptr_t { return d.contains(k) ? d[k].cast<uintptr_t>() : 0; };
  ps.obound = u("obound");
  ps.xmax = u("xmax");
  ps.xmax2 = u("xmax2");
  ps.gmax = u("gmax");
  ps.xep = uint32_t(u("xep"));
  ps.xep2 = uint32_t(u("xep2"));
  ps.gep = uint32_t(u("gep"));
  ps.rbound = u("rbound");
  ps.rplanes = int(u("rplanes"));
  return true;
}

PYBIND11_MODULE(_mpit, m) {
  m.doc() = "mpit_amd native runtime: shm control plane, IPC windows, parameter server, CDNA4 kernels";
  m.attr("ANY_SOURCE") = kAnySource;
  m.attr("ANY_TAG") = kAnyTag;
  m.attr("NORM_WS_FLOATS") = kNormWsFloats;

  py::module_ k = m.def_submodule("rule");
  k.attr("APPLY") = int(kApply);
  k.attr("APPLY_SUM") = int(kApplySum);
  k.attr("RMSPROP") = int(kRMSProp);
  k.attr("ADAM") = int(kAdam);
  k.attr("ADAMAX") = int(kAdamax);
  k.attr("ADAGRAD") = int(kAdagrad);
  k.attr("ADADELTA") = int(kAdadelta);
  k.attr("NESTEROV_PRE") = int(kNesterovPre);
  k.attr("NESTEROV_POST") = int(kNesterovPost);
  k.attr("DOWNPOUR") = int(kDownpour);
  k.attr("ELASTIC") = int(kElastic);
  k.attr("REGCLIP") = int(kRegClip);
  k.attr("SCALE") = int(kScale);
  k.attr("COPY") = int(kCopy);
  k.attr("FILL") = int(kFill);
  k.attr("AXPBY") = int(kAxpby);
  k.attr("OUT") = int(kOut);
  k.attr("ADD") = int(kAdd);
  k.attr("VT") = int(kVt);
  k.attr("SUG") = int(kSug);

  m.def(
      "ew_update",
      [](int rule, int variant, int dev, uintptr_t stream, int64_t n, std::vector<uintptr_t> ptrs, uint32_t bf,
         std::vector<float> sc) { ew_update(rule, variant, dev, S(stream), n, ptrs, bf, sc); },
      py::arg("rule"), py::arg("variant"), py::arg("dev"), py::arg("stream"), py::arg("n"), py::arg("ptrs"),
      py::arg("bf"), py::arg("scalars"));
  m.def(
      "ew_update_multi",
      [](int rule, int variant, int dev, uintptr_t stream, std::vector<int64_t> ns,
         std::vector<std::vector<uintptr_t>> ptrs, uint32_t bf, std::vector<float> sc) {
        ew_update_multi(rule, variant, dev, S(stream), ns, ptrs, bf, sc);
      },
      py::arg("rule"), py::arg("variant"), py::arg("dev"), py::arg("stream"), py::arg("ns"), py::arg("ptrs"),
      py::arg("bf"), py::arg("scalars"));
  m.def("norms", [](int dev, uintptr_t stream, uintptr_t x, bool bf16, int64_t n, uintptr_t out, uintptr_t ws) {
    norms(dev, S(stream), reinterpret_cast<const void*>(x), bf16, n, reinterpret_cast<float*>(out),
          reinterpret_cast<float*>(ws));
  });
  m.def("dot", [](int dev, uintptr_t stream, uintptr_t x, uintptr_t y, bool bf16, int64_t n, uintptr_t out,
                  uintptr_t ws) {
    dot(dev, S(stream), reinterpret_cast<const void*>(x), reinterpret_cast<const void*>(y), bf16, n,
        reinterpret_cast<float*>(out), reinterpret_cast<float*>(ws));
  });
  m.def("clamp_scan", [](int dev, uintptr_t stream, uintptr_t G, uintptr_t g, uintptr_t p, int64_t P, int64_t ldg,
                         int n, float l1, float l2, float c) {
    clamp_scan(dev, S(stream), reinterpret_cast<float*>(G), reinterpret_cast<const float*>(g),
               reinterpret_cast<const float*>(p), P, ldg, n, l1, l2, c);
  });
  m.def("multi_copy", [](int dev, uintptr_t stream, uintptr_t table, int64_t nchunks, float scale) {
    multi_copy(dev, S(stream), reinterpret_cast<const CopyChunk*>(table), nchunks, scale);
  });
  m.attr("COPY_CHUNK_BYTES") = int(sizeof(CopyChunk));
  m.def("gather_scale", [](int dev, uintptr_t s, std::vector<uintptr_t> srcs, std::vector<int64_t> offs,
                           std::vector<int64_t> ns, uintptr_t dst, uintptr_t aux, float a,
                           float b) { gather_scale(dev, S(s), srcs, offs, ns, dst, aux, a, b); });
  m.def("bn_workspace_floats", &bn_workspace_floats);
  m.def("bn_mask_bytes", &bn_mask_bytes);
  m.def(
      "bn_act_fwd",
      [](int dev, uintptr_t s, bool bf16, uintptr_t x, uintptr_t res, uintptr_t y, int64_t M, int C, uintptr_t gamma,
         uintptr_t beta, uintptr_t rmean, uintptr_t rvar, uintptr_t save_mean, uintptr_t save_rstd, uintptr_t ws,
         float momentum, float eps, bool relu, uintptr_t mask, uintptr_t stats, int64_t nstat, uintptr_t amax,
         uintptr_t coef, py::object planes) {
        PlaneSpec ps;
        const bool pl = plane_spec(planes, ps);
        bn_act_fwd(dev, S(s), bf16, x, res, y, M, C, gamma, beta, rmean, rvar, save_mean, save_rstd, ws, momentum, eps,
                   relu, mask, stats, nstat, amax, coef, pl ? &ps : nullptr);
      },
      py::arg("dev"), py::arg("stream"), py::arg("bf16"), py::arg("x"), py::arg("res"), py::arg("y"), py::arg("M"),
      py::arg("C"), py::arg("gamma"), py::arg("beta"), py::arg("rmean"), py::arg("rvar"), py::arg("save_mean"),
      py::arg("save_rstd"), py::arg("ws"), py::arg("momentum"), py::arg("eps"), py::arg("relu"), py::arg("mask"),
      py::arg("stats") = 0, py::arg("nstat") = 0, py::arg("amax") = 0, py::arg("coef") = 0,
      py::arg("planes") = py::none());
  m.def("bn_act_apply", [](int dev, uintptr_t s, bool bf16, uintptr_t x, uintptr_t res, uintptr_t y, int64_t M, int C,
                           uintptr_t coef, bool relu) { bn_act_apply(dev, S(s), bf16, x, res, y, M, C, coef, relu); });
  m.def(
      "bn_act_bwd",
      [](int dev, uintptr_t s, bool bf16, uintptr_t dy, uintptr_t mask, uintptr_t x, uintptr_t dx, uintptr_t dres,
         int64_t M, int C, uintptr_t gamma, uintptr_t mean, uintptr_t rstd, uintptr_t dgamma, uintptr_t dbeta,
         uintptr_t ws, bool relu, uintptr_t part, int64_t npart, uintptr_t coef, uintptr_t amax, py::object planes) {
        PlaneSpec ps;
        const bool pl = plane_spec(planes, ps);
        bn_act_bwd(dev, S(s), bf16, dy, mask, x, dx, dres, M, C, gamma, mean, rstd, dgamma, dbeta, ws, relu, part, npart,
                   coef, amax, pl ? &ps : nullptr);
      },
      py::arg("dev"), py::arg("stream"), py::arg("bf16"), py::arg("dy"), py::arg("mask"), py::arg("x"), py::arg("dx"),
      py::arg("dres"), py::arg("M"), py::arg("C"), py::arg("gamma"), py::arg("mean"), py::arg("rstd"),
      py::arg("dgamma"), py::arg("dbeta"), py::arg("ws"), py::arg("relu"), py::arg("part") = 0, py::arg("npart") = 0,
      py::arg("coef") = 0, py::arg("amax") = 0, py::arg("planes") = py::none());
  m.def(
      "bn_pair_apply",
      [](int dev, uintptr_t s, uintptr_t x1, uintptr_t coef1, uintptr_t x2, uintptr_t coef2, uintptr_t y, int64_t M,
         int C, uintptr_t mask, bool f32, uintptr_t amax, uintptr_t scratch, py::object planes) {
        PlaneSpec ps;
        const bool pl = plane_spec(planes, ps);
        bn_pair_apply(dev, S(s), x1, coef1, x2, coef2, y, M, C, mask, f32, amax, scratch, pl ? &ps : nullptr);
      },
      py::arg("dev"), py::arg("stream"), py::arg("x1"), py::arg("coef1"), py::arg("x2"), py::arg("coef2"), py::arg("y"),
      py::arg("M"), py::arg("C"), py::arg("mask"), py::arg("f32") = false, py::arg("amax") = 0, py::arg("scratch") = 0,
      py::arg("planes") = py::none());
  m.def(
      "bn_pair_bwd_apply",
      [](int dev, uintptr_t s, uintptr_t dy, uintptr_t mask, uintptr_t x1, uintptr_t coef1, uintptr_t dx1, uintptr_t x2,
         uintptr_t coef2, uintptr_t dx2, int64_t M, int C, bool f32, uintptr_t amax1, uintptr_t amax2,
         uintptr_t scratch, py::object planes1, py::object planes2) {
        PlaneSpec p1, p2;
        const bool a = plane_spec(planes1, p1), b = plane_spec(planes2, p2);
        bn_pair_bwd_apply(dev, S(s), dy, mask, x1, coef1, dx1, x2, coef2, dx2, M, C, f32, amax1, amax2, scratch,
                          a ? &p1 : nullptr, b ? &p2 : nullptr);
      },
      py::arg("dev"), py::arg("stream"), py::arg("dy"), py::arg("mask"), py::arg("x1"), py::arg("coef1"),
      py::arg("dx1"), py::arg("x2"), py::arg("coef2"), py::arg("dx2"), py::arg("M"), py::arg("C"),
      py::arg("f32") = false, py::arg("amax1") = 0, py::arg("amax2") = 0, py::arg("scratch") = 0,
      py::arg("planes1") = py::none(), py::arg("planes2") = py::none());
  m.def("gemm_nt_supported", &gemm_nt_supported, py::arg("M"), py::arg("N"), py::arg("K"), py::arg("f32") = false);
  m.def("gemm_nt_stats_floats", &gemm_nt_stats_floats);
  m.def("gemm_nt_tiles", &gemm_nt_tiles);
  m.def(
      "gemm_nt",
      [](int dev, uintptr_t s, int64_t M, int N, int K, uintptr_t A, int64_t lda, uintptr_t B, int64_t ldb, uintptr_t C,
         int64_t ldc, uintptr_t stats, uintptr_t cin, uintptr_t cmask, uintptr_t red_part, uintptr_t red_x,
         uintptr_t red_mask, uintptr_t red_mean, int64_t red_row0, uintptr_t red_part2, uintptr_t red_x2,
         uintptr_t red_mean2, bool f32, uintptr_t fold_coef, uintptr_t fold_gamma, uintptr_t fold_rstd,
         uintptr_t fold_dgamma, uintptr_t fold_dbeta, uintptr_t fold_lvl, int64_t bps, uintptr_t amax_a,
         uintptr_t amax_b, uintptr_t fold_zero, py::object bn_fold, bool fold_tag, int64_t aps, uintptr_t omax,
         uint32_t oepoch) {
        BnRed r{red_part, red_x, red_mask, red_mean, red_row0, red_part2, red_x2, red_mean2};
        r.fcoef = fold_coef; r.fgamma = fold_gamma; r.frstd = fold_rstd;
        r.fdgamma = fold_dgamma; r.fdbeta = fold_dbeta; r.flvl = fold_lvl; r.fzero = fold_zero;
        r.amax_a = amax_a; r.amax_b = amax_b; r.aps = aps; r.omax = omax; r.oepoch = oepoch;
        r.ftag = fold_tag ? 1 : 0;
        apply_sfold(r, bn_fold);
        gemm_nt(dev, S(s), M, N, K, A, lda, B, ldb, C, ldc, stats, cin, cmask, &r, f32, bps);
      },
      py::arg("dev"), py::arg("stream"), py::arg("M"), py::arg("N"), py::arg("K"), py::arg("A"), py::arg("lda"),
      py::arg("B"), py::arg("ldb"), py::arg("C"), py::arg("ldc"), py::arg("stats") = 0, py::arg("cin") = 0,
      py::arg("cmask") = 0, py::arg("red_part") = 0, py::arg("red_x") = 0, py::arg("red_mask") = 0,
      py::arg("red_mean") = 0, py::arg("red_row0") = 0, py::arg("red_part2") = 0, py::arg("red_x2") = 0,
      py::arg("red_mean2") = 0, py::arg("f32") = false, py::arg("fold_coef") = 0, py::arg("fold_gamma") = 0,
      py::arg("fold_rstd") = 0, py::arg("fold_dgamma") = 0, py::arg("fold_dbeta") = 0, py::arg("fold_lvl") = 0,
      py::arg("bps") = 0, py::arg("amax_a") = 0, py::arg("amax_b") = 0, py::arg("fold_zero") = 0,
      py::arg("bn_fold") = py::none(), py::arg("fold_tag") = false, py::arg("aps") = 0, py::arg("omax") = 0,
      py::arg("oepoch") = 0);
  m.def("gemm_nt_fold_lvl_floats", &gemm_nt_fold_lvl_floats);
  m.def("bound_floats", [] { return kBoundFloats; });
  m.def("gemm_tn_supported", &gemm_tn_supported);
  m.def("gemm_tn_ws_floats", &gemm_tn_ws_floats);
  m.def("device_cu_count", &device_cu_count);
  m.def("stream_create_cu_masked", &stream_create_cu_masked);
  m.def(
      "gemm_tn",
      [](int dev, uintptr_t s, int64_t M, int N, int K, uintptr_t Y, int64_t ldy, uintptr_t X, int64_t ldx,
         uintptr_t out, uintptr_t ws, float beta, bool f32, uintptr_t amax_y, uintptr_t amax_x, int64_t yps,
         int64_t xps) {
        gemm_tn(dev, S(s), M, N, K, Y, ldy, X, ldx, out, ws, beta, f32, amax_y, amax_x, yps, xps);
      },
      py::arg("dev"), py::arg("stream"), py::arg("M"), py::arg("N"), py::arg("K"), py::arg("Y"), py::arg("ldy"),
      py::arg("X"), py::arg("ldx"), py::arg("out"), py::arg("ws"), py::arg("beta"), py::arg("f32") = false,
      py::arg("amax_y") = 0, py::arg("amax_x") = 0, py::arg("yps") = 0, py::arg("xps") = 0);
  m.def(
      "cast_transpose",
      [](int dev, uintptr_t s, uintptr_t w, int R, int Cc, uintptr_t wb, uintptr_t wt, int taps, bool f32) {
        cast_transpose(dev, S(s), w, R, Cc, wb, wt, taps, f32);
      },
      py::arg("dev"), py::arg("stream"), py::arg("w"), py::arg("R"), py::arg("Cc"), py::arg("wb"), py::arg("wt"),
      py::arg("taps") = 1, py::arg("f32") = false);
  m.def("cast_job_bytes", &cast_job_bytes);
  m.def("cast_jobs_build", [](uintptr_t table, std::vector<std::array<int64_t, 11>> specs) {
    return cast_jobs_build(table, specs);
  });
  m.def(
      "cast_jobs_run",
      [](int dev, uintptr_t s, uintptr_t table, int njobs, int64_t nblocks, uintptr_t amax) {
        cast_jobs_run(dev, S(s), table, njobs, nblocks, amax);
      },
      py::arg("dev"), py::arg("s"), py::arg("table"), py::arg("njobs"), py::arg("nblocks"), py::arg("amax") = 0);
  m.def(
      "maxpool_fwd",
      [](int dev, uintptr_t s, int N, int H, int W, int C, int K, int stride, int pad, uintptr_t x, uintptr_t y,
         uintptr_t idx, bool f32, uintptr_t ibound, uintptr_t obound) {
        maxpool_fwd(dev, S(s), N, H, W, C, K, stride, pad, x, y, idx, f32, ibound, obound);
      },
      py::arg("dev"), py::arg("stream"), py::arg("N"), py::arg("H"), py::arg("W"), py::arg("C"), py::arg("K"),
      py::arg("stride"), py::arg("pad"), py::arg("x"), py::arg("y"), py::arg("idx"), py::arg("f32") = false,
      py::arg("ibound") = 0, py::arg("obound") = 0);
  m.def(
      "maxpool_bwd",
      [](int dev, uintptr_t s, int N, int H, int W, int C, int K, int stride, int pad, uintptr_t dy, uintptr_t idx,
         uintptr_t dx, bool f32, uintptr_t ypool, uintptr_t db, uintptr_t ws) {
        maxpool_bwd(dev, S(s), N, H, W, C, K, stride, pad, dy, idx, dx, f32, ypool, db, ws);
      },
      py::arg("dev"), py::arg("stream"), py::arg("N"), py::arg("H"), py::arg("W"), py::arg("C"), py::arg("K"),
      py::arg("stride"), py::arg("pad"), py::arg("dy"), py::arg("idx"), py::arg("dx"), py::arg("f32") = false,
      py::arg("ypool") = 0, py::arg("db") = 0, py::arg("ws") = 0);
  m.def("maxpool_bwd_ws_floats", &maxpool_bwd_ws_floats);
  m.def(
      "avgpool_bwd",
      [](int dev, uintptr_t s, int N, int HW, int C, uintptr_t dy, uintptr_t dx, bool f32) {
        avgpool_bwd(dev, S(s), N, HW, C, dy, dx, f32);
      },
      py::arg("dev"), py::arg("stream"), py::arg("N"), py::arg("HW"), py::arg("C"), py::arg("dy"), py::arg("dx"),
      py::arg("f32") = false);
  m.def("col_sums_ws_floats", &col_sums_ws_floats);
  m.def(
      "col_sums",
      [](int dev, uintptr_t s, uintptr_t part, int64_t nb, int64_t ld, int C, uintptr_t out, uintptr_t mid) {
        col_sums(dev, S(s), part, nb, ld, C, out, mid);
      },
      py::arg("dev"), py::arg("stream"), py::arg("part"), py::arg("nb"), py::arg("ld"), py::arg("C"), py::arg("out"),
      py::arg("mid") = 0);
  m.def("conv_supported", &conv_supported);
  m.def(
      "conv_fwd",
      [](int dev, uintptr_t s, int Nb, int H, int W, int C, int Co, int R, int S_, int stride, int pad, uintptr_t x,
         uintptr_t w, uintptr_t y, uintptr_t stats, uintptr_t cin, uintptr_t bias, bool relu, uintptr_t red_part,
         uintptr_t red_x, uintptr_t red_mask, uintptr_t red_mean, int64_t red_row0, uintptr_t red_part2,
         uintptr_t red_x2, uintptr_t red_mean2, bool f32, uintptr_t fold_coef, uintptr_t fold_gamma,
         uintptr_t fold_rstd, uintptr_t fold_dgamma, uintptr_t fold_dbeta, uintptr_t fold_lvl, int64_t bps,
         uintptr_t amax_a, uintptr_t amax_b, uintptr_t fold_zero, py::object bn_fold, bool red_relu,
         bool fold_tag, int64_t aps, uintptr_t omax, uint32_t oepoch) {
        BnRed r{red_part, red_x, red_mask, red_mean, red_row0, red_part2, red_x2, red_mean2};
        r.fcoef = fold_coef; r.fgamma = fold_gamma; r.frstd = fold_rstd;
        r.fdgamma = fold_dgamma; r.fdbeta = fold_dbeta; r.flvl = fold_lvl; r.fzero = fold_zero;
        r.amax_a = amax_a; r.amax_b = amax_b; r.aps = aps; r.omax = omax; r.oepoch = oepoch;
        r.relu_y = red_relu ? 1 : 0;
        r.ftag = fold_tag ? 1 : 0;
        apply_sfold(r, bn_fold);
        conv_fwd(dev, S(s), Nb, H, W, C, Co, R, S_, stride, pad, x, w, y, stats, cin, bias, relu, &r, f32, bps);
      },
      py::arg("dev"), py::arg("stream"), py::arg("Nb"), py::arg("H"), py::arg("W"), py::arg("C"), py::arg("Co"),
      py::arg("R"), py::arg("S"), py::arg("stride"), py::arg("pad"), py::arg("x"), py::arg("w"), py::arg("y"),
      py::arg("stats") = 0, py::arg("cin") = 0, py::arg("bias") = 0, py::arg("relu") = false, py::arg("red_part") = 0,
      py::arg("red_x") = 0, py::arg("red_mask") = 0, py::arg("red_mean") = 0, py::arg("red_row0") = 0,
      py::arg("red_part2") = 0, py::arg("red_x2") = 0, py::arg("red_mean2") = 0, py::arg("f32") = false,
      py::arg("fold_coef") = 0, py::arg("fold_gamma") = 0, py::arg("fold_rstd") = 0, py::arg("fold_dgamma") = 0,
      py::arg("fold_dbeta") = 0, py::arg("fold_lvl") = 0, py::arg("bps") = 0, py::arg("amax_a") = 0,
      py::arg("amax_b") = 0, py::arg("fold_zero") = 0, py::arg("bn_fold") = py::none(), py::arg("red_relu") = false,
      py::arg("fold_tag") = false, py::arg("aps") = 0, py::arg("omax") = 0, py::arg("oepoch") = 0);
  m.def("conv_dgrad_strided_wfloats", &conv_dgrad_strided_wfloats);
  m.def(
      "conv_dgrad_strided_weights",
      [](int dev, uintptr_t s, uintptr_t w, int Co, int C, int R, int S_, int stride, int pad, uintptr_t wb,
         uintptr_t wcls, bool f32) { conv_dgrad_strided_weights(dev, S(s), w, Co, C, R, S_, stride, pad, wb, wcls, f32); },
      py::arg("dev"), py::arg("stream"), py::arg("w"), py::arg("Co"), py::arg("C"), py::arg("R"), py::arg("S"),
      py::arg("stride"), py::arg("pad"), py::arg("wb"), py::arg("wcls"), py::arg("f32") = false);
  m.def("conv_dgrad_strided_tiles", &conv_dgrad_strided_tiles);
  m.def(
      "conv_dgrad_strided",
      [](int dev, uintptr_t s, int Nb, int H, int W, int C, int Co, int R, int S_, int stride, int pad, uintptr_t dy,
         uintptr_t wcls, uintptr_t dx, uintptr_t red_part, uintptr_t red_x, uintptr_t red_mask, uintptr_t red_mean,
         uintptr_t red_part2, uintptr_t red_x2, uintptr_t red_mean2, bool f32, int64_t bps, uintptr_t amax_a,
         uintptr_t amax_b, int64_t aps, uintptr_t omax, uint32_t oepoch) {
        BnRed r{red_part, red_x, red_mask, red_mean, 0, red_part2, red_x2, red_mean2};
        r.amax_a = amax_a; r.amax_b = amax_b; r.aps = aps; r.omax = omax; r.oepoch = oepoch;
        conv_dgrad_strided(dev, S(s), Nb, H, W, C, Co, R, S_, stride, pad, dy, wcls, dx, &r, f32, bps);
      },
      py::arg("dev"), py::arg("stream"), py::arg("Nb"), py::arg("H"), py::arg("W"), py::arg("C"), py::arg("Co"),
      py::arg("R"), py::arg("S"), py::arg("stride"), py::arg("pad"), py::arg("dy"), py::arg("wcls"), py::arg("dx"),
      py::arg("red_part") = 0, py::arg("red_x") = 0, py::arg("red_mask") = 0, py::arg("red_mean") = 0,
      py::arg("red_part2") = 0, py::arg("red_x2") = 0, py::arg("red_mean2") = 0, py::arg("f32") = false,
      py::arg("bps") = 0, py::arg("amax_a") = 0, py::arg("amax_b") = 0, py::arg("aps") = 0, py::arg("omax") = 0,
      py::arg("oepoch") = 0);
  m.def(
      "softmax_xent",
      [](int dev, uintptr_t s, int64_t rows, int C, uintptr_t x, int64_t ldx, bool bf16, uintptr_t tgt, float scale,
         uintptr_t loss, uintptr_t d) { softmax_xent(dev, S(s), rows, C, x, ldx, bf16, tgt, scale, loss, d); },
      py::arg("dev"), py::arg("stream"), py::arg("rows"), py::arg("C"), py::arg("x"), py::arg("ldx"),
      py::arg("bf16"), py::arg("tgt"), py::arg("scale"), py::arg("loss"), py::arg("d"));
  m.def("relu_bias_bwd_ws_floats", &relu_bias_bwd_ws_floats);
  m.def(
      "relu_bias_bwd",
      [](int dev, uintptr_t s, int64_t M, int C, uintptr_t dy, uintptr_t y, uintptr_t dz, uintptr_t db, uintptr_t ws,
         bool f32) { relu_bias_bwd(dev, S(s), M, C, dy, y, dz, db, ws, f32); },
      py::arg("dev"), py::arg("stream"), py::arg("M"), py::arg("C"), py::arg("dy"), py::arg("y"), py::arg("dz"),
      py::arg("db"), py::arg("ws"), py::arg("f32") = false);
  m.def(
      "conv_stem_fwd",
      [](int dev, uintptr_t s, int Nb, int Hp, int Wp, int Co, int Ho, int Wo, int stride, uintptr_t x, uintptr_t w,
         uintptr_t y, uintptr_t stats, bool f32, int64_t bps, uintptr_t amax_a, uintptr_t amax_b, py::object bn_fold,
         int rows, uintptr_t bias, bool relu) {
        BnRed r{};
        apply_sfold(r, bn_fold);
        conv_stem_fwd(dev, S(s), Nb, Hp, Wp, Co, Ho, Wo, stride, x, w, y, stats, f32, bps, amax_a, amax_b, &r, rows,
                      bias, relu);
      },
      py::arg("dev"), py::arg("stream"), py::arg("Nb"), py::arg("Hp"), py::arg("Wp"), py::arg("Co"), py::arg("Ho"),
      py::arg("Wo"), py::arg("stride"), py::arg("x"), py::arg("w"), py::arg("y"), py::arg("stats"),
      py::arg("f32") = false, py::arg("bps") = 0, py::arg("amax_a") = 0, py::arg("amax_b") = 0,
      py::arg("bn_fold") = py::none(), py::arg("rows") = 8, py::arg("bias") = 0, py::arg("relu") = false);
  m.def(
      "stem_weight_planes",
      [](int dev, uintptr_t s, uintptr_t w, int Co, int C, int R, int Sk, uintptr_t planes, uintptr_t bound) {
        stem_weight_planes(dev, S(s), w, Co, C, R, Sk, planes, bound);
      },
      py::arg("dev"), py::arg("stream"), py::arg("w"), py::arg("Co"), py::arg("C"), py::arg("R"), py::arg("S"),
      py::arg("planes"), py::arg("bound"));
  m.def("conv_stem_wgrad_ws_floats", &conv_stem_wgrad_ws_floats, py::arg("dev"), py::arg("Nb"), py::arg("Ho"),
        py::arg("Wo"), py::arg("Co"), py::arg("rows") = 8);
  m.def("stem_wgrad_rows", &stem_wgrad_rows);
  m.def(
      "conv_stem_wgrad",
      [](int dev, uintptr_t s, int Nb, int Hp, int Wp, int Co, int Ho, int Wo, int stride, uintptr_t dy, uintptr_t x,
         uintptr_t dw, uintptr_t ws, bool f32, uintptr_t amax_y, uintptr_t amax_x, int rows) {
        conv_stem_wgrad(dev, S(s), Nb, Hp, Wp, Co, Ho, Wo, stride, dy, x, dw, ws, f32, amax_y, amax_x, rows);
      },
      py::arg("dev"), py::arg("stream"), py::arg("Nb"), py::arg("Hp"), py::arg("Wp"), py::arg("Co"), py::arg("Ho"),
      py::arg("Wo"), py::arg("stride"), py::arg("dy"), py::arg("x"), py::arg("dw"), py::arg("ws"),
      py::arg("f32") = false, py::arg("amax_y") = 0, py::arg("amax_x") = 0, py::arg("rows") = 8);
  m.def("conv_wgrad_ws_floats", &conv_wgrad_ws_floats);
  m.def(
      "conv_wgrad",
      [](int dev, uintptr_t s, int Nb, int H, int W, int C, int Co, int R, int S_, int stride, int pad, uintptr_t dy,
         uintptr_t x, uintptr_t dw, uintptr_t ws, float beta, bool f32, uintptr_t amax_y, uintptr_t amax_x,
         int64_t yps, int64_t xps) {
        conv_wgrad(dev, S(s), Nb, H, W, C, Co, R, S_, stride, pad, dy, x, dw, ws, beta, f32, amax_y, amax_x, yps, xps);
      },
      py::arg("dev"), py::arg("stream"), py::arg("Nb"), py::arg("H"), py::arg("W"), py::arg("C"), py::arg("Co"),
      py::arg("R"), py::arg("S"), py::arg("stride"), py::arg("pad"), py::arg("dy"), py::arg("x"), py::arg("dw"),
      py::arg("ws"), py::arg("beta"), py::arg("f32") = false, py::arg("amax_y") = 0, py::arg("amax_x") = 0,
      py::arg("yps") = 0, py::arg("xps") = 0);

  py::class_<Engine>(m, "Engine")
      .def(py::init<const std::string&, int, int, bool, int, int64_t>(), py::arg("name"), py::arg("world"),
           py::arg("rank"), py::arg("create"), py::arg("device"), py::arg("bulk_bytes"),
           py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("rank", &Engine::rank)
      .def_property_readonly("world", &Engine::world)
      .def_property_readonly("device", &Engine::device)
      .def("isend",
           [](Engine& e, uintptr_t buf, int64_t n, bool dev, int dst, int tag, int ctx, bool sync) {
             return e.isend(reinterpret_cast<const void*>(buf), n, dev, dst, tag, ctx, sync);
           })
      .def("irecv",
           [](Engine& e, uintptr_t buf, int64_t cap, bool dev, int src, int tag, int ctx) {
             return e.irecv(reinterpret_cast<void*>(buf), cap, dev, src, tag, ctx);
           })
      .def("test",
           [](Engine& e, int64_t id, bool keep) -> py::object {
             Status st;
             if (!e.test(id, &st, keep)) return py::none();
             return st_tuple(st);
           },
           py::arg("id"), py::arg("keep") = false)
      .def("wait",
           [](Engine& e, int64_t id) {
             Status st;
             {
               py::gil_scoped_release r;
               e.wait(id, &st);
             }
             return st_tuple(st);
           })
      .def("cancel", &Engine::cancel)
      .def("free_request", &Engine::free_request)
      .def("iprobe",
           [](Engine& e, int src, int tag, int ctx) -> py::object {
             Status st;
             if (!e.iprobe(src, tag, ctx, &st)) return py::none();
             return st_tuple(st);
           })
      .def("probe",
           [](Engine& e, int src, int tag, int ctx) {
             Status st;
             {
               py::gil_scoped_release r;
               e.probe(src, tag, ctx, &st);
             }
             return st_tuple(st);
           })
      .def("barrier", &Engine::barrier, py::call_guard<py::gil_scoped_release>())
      .def("allgather_small",
           [](Engine& e, py::bytes blob) {
             std::string s = blob;
             std::vector<std::string> out;
             {
               py::gil_scoped_release r;
               out = e.allgather_small(s);
             }
             py::list l;
             for (auto& x : out) l.append(py::bytes(x));
             return l;
           })
      .def("abort", &Engine::abort)
      .def("shutdown", &Engine::shutdown, py::call_guard<py::gil_scoped_release>())
      .def("unlink", [](Engine& e) { e.seg().unlink(); })
      .def("comm_stream", [](Engine& e) { return reinterpret_cast<uintptr_t>(e.comm_stream()); })
      .def("stats", [](Engine& e) {
        return py::dict(py::arg("bytes_sent") = e.bytes_sent(), py::arg("bytes_recv") = e.bytes_recv(),
                        py::arg("msgs_sent") = e.msgs_sent());
      });

  py::class_<Window>(m, "Window")
      .def(py::init([](Engine& e, int64_t id, uintptr_t local, int64_t bytes, bool device) {
             return new Window(e, id, local, bytes, device);
           }),
           py::keep_alive<1, 2>())
      .def("blob", [](Window& w) { return py::bytes(w.blob()); })
      .def("connect",
           [](Window& w, std::vector<py::bytes> blobs, std::vector<int> ranks, bool map_remote) {
             std::vector<std::string> b;
             for (auto& x : blobs) b.push_back(std::string(x));
             py::gil_scoped_release r;
             w.connect(b, ranks, map_remote);
           },
           py::arg("blobs"), py::arg("ranks"), py::arg("map_remote") = true)
      .def("unlink_names", &Window::unlink_names)
      .def_property_readonly("local_ptr", &Window::local_ptr)
      .def_property_readonly("bytes", &Window::bytes)
      .def_property_readonly("device", &Window::device)
      .def("remote_ptr", &Window::remote_ptr)
      .def("remote_bytes", &Window::remote_bytes)
      .def("remote_device", &Window::remote_device)
      .def("put", [](Window& w, int m, int64_t off, uintptr_t src, int64_t n, uintptr_t s) { w.put(m, off, src, n, S(s)); },
           py::call_guard<py::gil_scoped_release>())
      .def("get", [](Window& w, uintptr_t dst, int m, int64_t off, int64_t n, uintptr_t s) { w.get(dst, m, off, n, S(s)); },
           py::call_guard<py::gil_scoped_release>())
      .def("accumulate",
           [](Window& w, int m, int64_t off, uintptr_t src, bool src_dev, int64_t nelem, bool bf16, float a, float b,
              uintptr_t s) { w.accumulate(m, off, src, src_dev, nelem, bf16, a, b, S(s)); },
           py::call_guard<py::gil_scoped_release>())
      .def("lock", &Window::lock, py::call_guard<py::gil_scoped_release>())
      .def("try_lock", &Window::try_lock)
      .def("unlock", &Window::unlock)
      .def("flush", [](Window& w, uintptr_t s) { w.flush(S(s)); }, py::call_guard<py::gil_scoped_release>());

  py::class_<ServerRule>(m, "ServerRule")
      .def(py::init<>())
      .def_readwrite("kind", &ServerRule::kind)
      .def_readwrite("a", &ServerRule::a)
      .def_readwrite("lr", &ServerRule::lr)
      .def_readwrite("decay", &ServerRule::decay)
      .def_readwrite("mom", &ServerRule::mom)
      .def_readwrite("eps", &ServerRule::eps)
      .def_readwrite("b1", &ServerRule::b1)
      .def_readwrite("b2", &ServerRule::b2)
      .def_readwrite("rho", &ServerRule::rho)
      .def_readwrite("lrd", &ServerRule::lrd)
      .def_readwrite("step_div", &ServerRule::step_div);

  py::class_<PSServer>(m, "PSServer")
      .def(py::init<Engine&, int, Window&, Window&, std::vector<int>, std::vector<int>, int64_t, int64_t, bool, uintptr_t,
                    std::vector<uintptr_t>, uintptr_t, ServerRule, int, int64_t, bool, int>(),
           py::keep_alive<1, 2>(), py::keep_alive<1, 4>(), py::keep_alive<1, 5>())
      .def("start", &PSServer::start)
      .def("done", &PSServer::done)
      .def("wait_done", &PSServer::wait_done, py::call_guard<py::gil_scoped_release>())
      .def("version", &PSServer::version)
      .def("step", &PSServer::step)
      .def("set_counters", &PSServer::set_counters)
      .def("set_lr", &PSServer::set_lr)
      .def("sync", &PSServer::sync, py::call_guard<py::gil_scoped_release>())
      .def("set_link", &PSServer::set_link, py::keep_alive<1, 2>())
      .def("stats", [](PSServer& s) {
        auto st = s.stats();
        return py::dict(py::arg("grads") = st.grads, py::arg("pulls") = st.pulls,
                        py::arg("param_pushes") = st.param_pushes, py::arg("deferred") = st.deferred,
                        py::arg("batches") = st.batches, py::arg("multi") = st.multi);
      });

  py::class_<PSClient>(m, "PSClient")
      .def(py::init<Engine&, int, std::vector<int>, std::vector<int64_t>, std::vector<int64_t>>(), py::keep_alive<1, 2>())
      .def("start", &PSClient::start)
      .def("send_grad", [](PSClient& c, uintptr_t s, bool pull) { c.send_grad(S(s), pull); })
      .def("send_grad_to", [](PSClient& c, uintptr_t s, int k, bool pull) { c.send_grad_to(S(s), k, pull); })
      .def("recv_param", [](PSClient& c, uintptr_t s) { c.recv_param(S(s)); })
      .def("send_param", [](PSClient& c, uintptr_t s, bool from_rx) { c.send_param(S(s), from_rx); },
           py::arg("stream"), py::arg("from_rx") = false)
      .def("stop", &PSClient::stop, py::call_guard<py::gil_scoped_release>())
      .def("wait", &PSClient::wait, py::call_guard<py::gil_scoped_release>())
      .def("test", &PSClient::test)
      .def("take_deps", [](PSClient& c, uintptr_t s) { c.take_deps(S(s)); })
      .def("pending", &PSClient::pending)
      .def("replies", &PSClient::replies)
      .def("set_link", &PSClient::set_link, py::keep_alive<1, 2>());

  py::class_<PsLink>(m, "PsLink")
      .def(py::init<Engine&, int, std::vector<int>, bool>(), py::keep_alive<1, 2>())
      .def_property_readonly("device", &PsLink::device)
      .def_property_readonly("legacy", &PsLink::legacy)
      .def_property_readonly("sequencer", &PsLink::sequencer)
      .def("make_id", [](PsLink& l) { return py::bytes(l.make_id()); })
      .def("connect",
           [](PsLink& l, py::bytes id) {
             std::string v(id);
             py::gil_scoped_release r;
             l.connect(v);
           })
      .def("stats", [](PsLink& l) {
        return py::dict(py::arg("bytes_sent") = l.bytes_sent(), py::arg("bytes_recv") = l.bytes_recv(),
                        py::arg("ordered") = l.ordered(), py::arg("groups") = l.groups(),
                        py::arg("self_mode") = PsLink::self_mode());
      });
}

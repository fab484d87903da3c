"""Fused BatchNorm2d (+ residual add) (+ ReLU) for channels_last activations on MI355X.

Forward training = 2 HBM passes (statistics; normalise+add+ReLU), backward = 2 passes
(reductions; dx [+ residual grad]) — csrc/kernels/bn_act.hip. Replaces
BatchNorm -> add -> ReLU chains of 3 library/elementwise kernels each way.

Around the MFMA convolutions (ops/conv.py) one pass each way disappears:

* the convolution that produces the BN input emits its per-tile statistics from the GEMM
  accumulators (``conv.emit_stats``; the output tensor carries them as
  ``_mpit_tstats``), so the forward is a single normalise pass;
* the convolution that consumes the BN output computes, in its backward-data epilogue,
  the BN's backward reductions over the gradient it writes (the BN output carries a
  :class:`BNLink` as ``_mpit_bnlink``), so the backward is a single dx pass.

:class:`BatchNormAct2d` is an ``nn.BatchNorm2d`` (same parameters, buffers, state dict)
whose forward takes an optional residual and applies ReLU when ``act=True``. On CPU
tensors (tests, gloo plumbing) it computes the same function with PyTorch ops.
"""
from __future__ import annotations

import os

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .._ext import native
from . import conv as _conv
from .conv import amax_of, omax_buf, omax_of, planes_of, set_amax, set_planes


def _rows(x: torch.Tensor):
    n, c, h, w = x.shape
    return n * h * w, c


def _cl(x: torch.Tensor) -> torch.Tensor:
    return x if x.is_contiguous(memory_format=torch.channels_last) else x.contiguous(memory_format=torch.channels_last)


# how often each fused hand-over fired (tests assert the fused path ran)
COUNTERS = {"fwd_tile_stats": 0, "fwd_folded": 0, "bwd_linked": 0, "bwd_folded": 0, "fwd_planes": 0,
            "bwd_planes": 0}


class BNLink:
    """What a convolution consuming a BN layer's output needs to fold that layer's backward
    reduction into its backward-data GEMM, and where it leaves the result.

    Filled by the BN forward (its saved input ``x``, ReLU ``mask``, batch ``mean``); the
    consumer's backward writes ``part`` ([npart][2][C] partial sums) and records which
    gradient tensor they describe (``dy_ptr``, ``dy_ver``). The BN backward uses them only
    if it receives exactly that tensor, unmodified — when autograd summed gradients from
    several consumers it falls back to its own reduction pass."""

    __slots__ = ("x", "mask", "mean", "part", "npart", "dy_ptr", "dy_ver", "x2", "mean2", "part2", "w", "rstd",
                 "fold", "gbuf", "gep")

    def __init__(self):
        # gbuf: the epoch slots where the consumer's backward-data GEMM leaves max |dy| (gep: its
        # launch epoch) when this BN's backward writes fp16 planes (ops/conv.py _red_args)
        self.gbuf, self.gep = None, 0
        self.x = self.mask = self.mean = self.part = None
        self.x2 = self.mean2 = self.part2 = None  # the shortcut BN of a bn_pair
        self.w = self.rstd = None  # BN weight (fp32) and 1/std: the consumer may fold the finalize
        self.fold = None  # (coef [3C], dgamma, dbeta) written by the consumer's GEMM
        self.npart = 0
        self.dy_ptr = self.dy_ver = None

    def ready(self, x: torch.Tensor) -> bool:
        """True when ``x`` (a consumer's input) is this layer's output: same shape and dtype
        (bf16 or fp32 — the consumer's epilogue reads the BN input in its own dtype)."""
        return (self.x is not None and self.mean is not None and x.dtype == self.x.dtype
                and self.x.shape == x.shape)

    def publish(self, part: torch.Tensor, npart: int, dy: torch.Tensor, part2: torch.Tensor = None, fold=None):
        self.part, self.npart, self.part2, self.fold = part, int(npart), part2, fold
        self.dy_ptr, self.dy_ver = dy.data_ptr(), dy._version

    def take(self, dy: torch.Tensor, pair: bool = False):
        """(part, npart[, part2]) for a matching gradient, else empty; a folded finalize's
        buffers are left in ``self.fold`` for :meth:`take_fold`."""
        part, npart, part2 = self.part, self.npart, self.part2
        ok = part is not None and dy.data_ptr() == self.dy_ptr and dy._version == self.dy_ver
        ok = ok and (part2 is not None or not pair)
        self.part = self.x = self.mask = self.mean = self.x2 = self.mean2 = self.part2 = None
        self.w = self.rstd = None
        if not ok:
            self.fold = None
        if pair:
            return (part, npart, part2) if ok else (None, 0, None)
        return (part, npart) if ok else (None, 0)

    def take_fold(self):
        fold, self.fold = self.fold, None
        return fold


def tile_stats_of(x: torch.Tensor):
    """(partials, tiles, fold) a producing GEMM attached to ``x`` (see module docstring), or
    None; fold: a :class:`BNFold` when the GEMM also ran this BN's forward finalize."""
    ts = getattr(x, "_mpit_tstats", None)
    if ts is None or ts[2] != x.data_ptr():
        return None
    return ts[0], ts[1], ts[3]


# MPIT_BN_FOLD_FWD=1: the BN forward's finalize folded into the producing GEMM's epilogue
# (stats_fold, csrc/kernels/gemm.hip) instead of its own launch. Off by default: measured
# slower on two boxes (r05e/r05g, fp32 5380-5433 vs 5456-5517 img/s, bf16 11.5k vs 11.7-11.8k):
# every block of the statistics GEMMs waits for its own output stores before taking its ticket,
# +1.23 ms of GEMM time per fp32 step against the 0.53 ms of the 53 finalize launches it saves
# (profiles/bn_fold_fwd_ab_r05.md)
_FWD_FOLD = os.environ.get("MPIT_BN_FOLD_FWD", "0") == "1"


class BNFold:
    """A BN forward finalize run by the GEMM that produces the BN's input (gemm.hip
    stats_fold): that GEMM's last blocks turn the output's statistics into the BN's scale /
    shift (``coef``), ``mean`` / ``rstd`` and the running-statistics update, and zero the
    BN output's fp16x3 bound (``amax``) — the BN forward is then its apply pass alone.
    ``args``: the tuple the native GEMM calls take (bindings.cpp apply_sfold)."""

    __slots__ = ("coef", "mean", "rstd", "amax", "args", "tagged", "_buf")

    def __init__(self, bn: "BatchNormAct2d", C: int, want_amax: bool, device):
        m = native()
        nl = m.gemm_nt_fold_lvl_floats(C)
        nb = _conv.BOUND_FLOATS if want_amax else 0
        self._buf = buf = torch.empty(4 * C + nl + nb, dtype=torch.float32, device=device)
        self.coef, self.mean, self.rstd = buf[: 2 * C], buf[2 * C: 3 * C], buf[3 * C: 4 * C]
        lvl = buf[4 * C: 4 * C + nl]
        self.amax = buf[4 * C + nl:] if want_amax else None
        w = bn.weight if bn.affine else None
        b = bn.bias if bn.affine else None
        # tagged partials (gemm.hip stats_fold; ops/conv.py tagged_part), unless MPIT_FOLD_TAG=0
        self.tagged = _conv._FOLD_TAG
        self.args = (self.coef.data_ptr(), w.data_ptr() if w is not None else 0, b.data_ptr() if b is not None else 0,
                     bn.running_mean.data_ptr(), bn.running_var.data_ptr(), self.mean.data_ptr(), self.rstd.data_ptr(),
                     lvl.data_ptr(), self.amax.data_ptr() if want_amax else 0, float(bn.eps), float(bn.momentum),
                     int(self.tagged))


def bn_fold_for(bn, C: int, dt, device) -> Optional[BNFold]:
    """The fold of ``bn``'s forward finalize into the GEMM producing its [*, C] input of dtype
    ``dt``, when that BN's training forward can take it (fused kernels, running statistics
    with a fixed momentum, fp32 parameters); else None (the BN finalizes itself)."""
    if not (_FWD_FOLD and isinstance(bn, BatchNormAct2d) and bn.training and bn.track_running_stats
            and bn.momentum is not None and bn.num_features == C and C % 8 == 0
            and dt in (torch.bfloat16, torch.float32) and device.type == "cuda"):
        return None
    if bn.affine and (bn.weight.dtype != torch.float32 or not bn.weight.is_contiguous()
                      or bn.bias.dtype != torch.float32 or not bn.bias.is_contiguous()):
        return None
    return BNFold(bn, C, dt == torch.float32 and _conv._F32_SPLIT == "f16x3", device)


def _want_amax(x: torch.Tensor) -> bool:
    """fp32 outputs on the GPU carry max |out| for the fp16x3 GEMMs that read them (ops/conv.py)."""
    return x.is_cuda and x.dtype == torch.float32 and _conv._F32_SPLIT == "f16x3"


def _amax_buf(x: torch.Tensor):
    return torch.empty(_conv.BOUND_FLOATS, dtype=torch.float32, device=x.device) if _want_amax(x) else None


def _fwd_planes(bn, x: torch.Tensor, residual: Optional[torch.Tensor], out: bool):
    """(PlaneSpec dict for the native call or None, the output planes' bound or None) of an fp32
    forward: a residual given as fp16 planes is always decoded (its bound); the output is written
    as planes when ``out`` (the BN's consumers are GEMMs) and the input's max is known."""
    if not (x.is_cuda and x.dtype == torch.float32):
        return None, None
    spec, obound = {}, None
    if residual is not None:
        rp = planes_of(residual)
        if rp is not None:
            spec.update(rbound=rp.data_ptr(), rplanes=1)
        elif out:
            ra = amax_of(residual)
            if ra is None:
                out = False
            else:
                spec.update(rbound=ra.data_ptr())
    om = omax_of(x) if out else None
    if om is not None and _conv._F32_PLANES:
        obound = torch.empty(_conv.BOUND_FLOATS, dtype=torch.float32, device=x.device)
        spec.update(obound=obound.data_ptr(), xmax=om[0].data_ptr(), xep=om[1])
    elif spec.get("rplanes") != 1:
        return None, None
    else:
        spec.pop("obound", None)
    return spec, obound


class _BNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, residual, momentum, eps, relu, res_slot=None,
                tstats=None, link=None, amax=None, planes=None):
        x = _cl(x)
        if residual is not None and planes_of(residual) is None:
            residual = _cl(residual).to(x.dtype)
        M, C = _rows(x)
        m = native()
        dev = x.device.index
        stream = torch.cuda.current_stream(x.device).cuda_stream
        y = torch.empty_like(x, memory_format=torch.channels_last)
        mean = torch.empty(C, dtype=torch.float32, device=x.device)
        rstd = torch.empty(C, dtype=torch.float32, device=x.device)
        ws = torch.empty(m.bn_workspace_floats(C), dtype=torch.float32, device=x.device)
        w = weight.float().contiguous() if weight is not None else None
        b = bias.float().contiguous() if bias is not None else None
        bf16 = x.dtype == torch.bfloat16
        # ReLU: one mask bit per element replaces keeping / re-reading y in the backward
        mask = torch.empty(m.bn_mask_bytes(bf16, M, C), dtype=torch.uint8, device=x.device) if relu else None
        ts = tstats if (tstats is not None and tstats[1] == m.gemm_nt_tiles(M)) else None
        fold = ts[2] if ts is not None else None
        if ts is not None:
            COUNTERS["fwd_tile_stats"] += 1
        if fold is not None:  # the producing GEMM ran the finalize (stats_fold): apply pass only
            COUNTERS["fwd_folded"] += 1
            mean, rstd = fold.mean, fold.rstd
        m.bn_act_fwd(dev, stream, bf16, x.data_ptr(),
                     residual.data_ptr() if residual is not None else 0, y.data_ptr(), M, C,
                     w.data_ptr() if w is not None else 0, b.data_ptr() if b is not None else 0,
                     running_mean.data_ptr() if running_mean is not None else 0,
                     running_var.data_ptr() if running_var is not None else 0,
                     mean.data_ptr(), rstd.data_ptr(), ws.data_ptr(), float(momentum), float(eps), bool(relu),
                     mask.data_ptr() if mask is not None else 0,
                     stats=ts[0].data_ptr() if ts is not None else 0, nstat=ts[1] if ts is not None else 0,
                     amax=amax.data_ptr() if amax is not None else 0,
                     coef=fold.coef.data_ptr() if fold is not None else 0, planes=planes)
        ctx.save_for_backward(x, mask, w, mean, rstd)
        # fp16-planes backward (dx read only by GEMMs): max |x| of the forward for its bound
        ctx.xmax = omax_of(x) if (planes is not None or getattr(link, "gbuf", None) is not None) else None
        ctx.link = link
        if link is not None:
            link.x, link.mask, link.mean = x, mask, mean
            link.w, link.rstd = w, rstd
        ctx.relu = relu
        ctx.has_res = residual is not None
        ctx.res_slot = res_slot
        ctx.has_w = weight is not None
        ctx.has_b = bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mask, w, mean, rstd = ctx.saved_tensors
        dy = _cl(dy).to(x.dtype)
        M, C = _rows(x)
        m = native()
        dev = x.device.index
        stream = torch.cuda.current_stream(x.device).cuda_stream
        dx = torch.empty_like(x, memory_format=torch.channels_last)
        # residual gradient of act(bn(x) + res) = dy*mask: with a GradSlot consumer it is
        # handed over as (dy, mask) and never written
        park = ctx.has_res and ctx.res_slot is not None and ctx.relu and mask is not None
        dres = torch.empty_like(x, memory_format=torch.channels_last) if (ctx.has_res and not park) else None
        dgamma = torch.empty(C, dtype=torch.float32, device=x.device) if ctx.has_w else None
        dbeta = torch.empty(C, dtype=torch.float32, device=x.device) if ctx.has_b else None
        ws = torch.empty(m.bn_workspace_floats(C), dtype=torch.float32, device=x.device)
        # reductions folded into the consumer convolution's backward-data GEMM (BNLink); with
        # a folded finalize the GEMM also left the coefficients, dgamma and dbeta
        gm = (ctx.link.gbuf, ctx.link.gep) if ctx.link is not None else (None, 0)
        part, npart = ctx.link.take(dy) if ctx.link is not None else (None, 0)
        fold = ctx.link.take_fold() if part is not None else None
        # dx as fp16 planes: the consumer's GEMM wrote this very dy (linked) with its max, and the
        # forward's input max is known; not with a residual gradient to write
        pspec, pbound = None, None
        if (part is not None and gm[0] is not None and gm[1] and getattr(ctx, "xmax", None) is not None
                and dres is None and x.dtype == torch.float32):
            pbound = torch.empty(_conv.BOUND_FLOATS, dtype=torch.float32, device=x.device)
            pspec = dict(obound=pbound.data_ptr(), gmax=gm[0].data_ptr(), gep=gm[1], xmax=ctx.xmax[0].data_ptr(),
                         xep=ctx.xmax[1])
        coef = 0
        if part is not None:
            COUNTERS["bwd_linked"] += 1
        # the output bound of dx (fp16x3 GEMM operand): zeroed by the folded finalize, else by
        # this call's own finalize
        amax = _amax_buf(x)
        if fold is not None:
            COUNTERS["bwd_folded"] += 1
            coef = fold[0].data_ptr()
            dgamma = fold[1] if ctx.has_w else None
            dbeta = fold[2] if ctx.has_b else None
            part, npart = None, 0
            if amax is not None:
                amax = fold[3]
        m.bn_act_bwd(dev, stream, x.dtype == torch.bfloat16, dy.data_ptr(),
                     mask.data_ptr() if mask is not None else 0, x.data_ptr(), dx.data_ptr(),
                     dres.data_ptr() if dres is not None else 0, M, C, w.data_ptr() if w is not None else 0,
                     mean.data_ptr(), rstd.data_ptr(), dgamma.data_ptr() if dgamma is not None else 0,
                     dbeta.data_ptr() if dbeta is not None else 0, ws.data_ptr(), bool(ctx.relu),
                     part=part.data_ptr() if part is not None else 0, npart=npart, coef=coef,
                     amax=amax.data_ptr() if amax is not None else 0, planes=pspec)
        if pbound is not None:
            set_planes(dx, pbound)
            COUNTERS["bwd_planes"] += 1
        elif amax is not None:
            set_amax(dx, amax)
        if ctx.res_slot is not None:  # the shortcut's gradient is added by the block's first conv
            if park:
                if not ctx.res_slot.put(dy, mask):
                    raise RuntimeError("GradSlot consumer ran before the BN backward")
            elif not ctx.res_slot.put(dres):
                raise RuntimeError("GradSlot consumer ran before the BN backward")
            dres = None
        return dx, dgamma, dbeta, None, None, dres, None, None, None, None, None, None, None, None


def bn_act_eval(x, weight, bias, running_mean, running_var, eps, residual=None, relu=True):
    """Inference: coefficients from running statistics, one fused pass."""
    x = _cl(x)
    M, C = _rows(x)
    rstd = torch.rsqrt(running_var.float() + eps)
    sc = rstd * (weight.float() if weight is not None else 1.0)
    sh = (bias.float() if bias is not None else 0.0) - running_mean.float() * sc
    coef = torch.cat([sc.reshape(-1), sh.reshape(-1)]).contiguous()
    y = torch.empty_like(x, memory_format=torch.channels_last)
    if residual is not None:
        residual = _cl(residual).to(x.dtype)
    native().bn_act_apply(x.device.index, torch.cuda.current_stream(x.device).cuda_stream, x.dtype == torch.bfloat16,
                          x.data_ptr(), residual.data_ptr() if residual is not None else 0, y.data_ptr(), M, C,
                          coef.data_ptr(), bool(relu))
    return y


def _supported(x: torch.Tensor) -> bool:
    if not x.is_cuda or x.dim() != 4 or x.dtype not in (torch.bfloat16, torch.float32):
        return False
    return x.shape[1] % 8 == 0  # 8 channels per thread and per ReLU-mask byte, either dtype


class BatchNormAct2d(nn.BatchNorm2d):
    """``act(bn(x) + residual)`` with ReLU act; a drop-in ``nn.BatchNorm2d`` subclass."""

    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True, track_running_stats=True, act=True):
        super().__init__(num_features, eps, momentum, affine, track_running_stats)
        self.act = act
        # num_batches_tracked only matters to the math when momentum is None; otherwise the
        # count is kept on the host and folded into the buffer when the state is read
        # (one tiny "+= 1" kernel per BN per step otherwise: 53 launches in ResNet-50)
        self._nbt_pending = 0
        # fp32 steps: out_planes — the output is read only by fp16x3 GEMMs (and planes-aware
        # residual adds): written as fp16 planes (ops/conv.py _F32_PLANES); grad_planes — the
        # input gradient is read only by GEMMs: dx as planes. Set by the model that knows.
        self.out_planes = False
        self.grad_planes = False

    def sync_num_batches_tracked(self):
        if self._nbt_pending:
            with torch.no_grad():
                self.num_batches_tracked.add_(self._nbt_pending)
            self._nbt_pending = 0

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        self.sync_num_batches_tracked()
        super()._save_to_state_dict(destination, prefix, keep_vars)

    def _train_args(self):
        """(momentum, running_mean, running_var) of one training-mode forward (counts it)."""
        momentum = self.momentum
        if self.training and self.track_running_stats:
            if momentum is None:
                self.sync_num_batches_tracked()
                self.num_batches_tracked.add_(1)
                momentum = 1.0 / float(self.num_batches_tracked)
            else:
                self._nbt_pending += 1
        rm = self.running_mean if (self.training and self.track_running_stats) else None
        rv = self.running_var if (self.training and self.track_running_stats) else None
        return momentum or 0.0, rm, rv

    def fused(self, x: torch.Tensor) -> bool:
        """True when a training forward of ``x`` runs the fused kernels (honours res_slot)."""
        return _supported(x) and (self.training or not self.track_running_stats)

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None, res_slot=None) -> torch.Tensor:
        """``res_slot``: a :class:`mpit_amd.ops.conv.GradSlot` that receives the residual's
        gradient in the backward instead of autograd (fused path only)."""
        if res_slot is not None and not self.fused(x):
            raise RuntimeError("res_slot needs the fused training path (see BatchNormAct2d.fused)")
        if not _supported(x):
            y = super().forward(x)
            if residual is not None:
                y = y + residual
            return F.relu(y) if self.act else y
        if self.training or not self.track_running_stats:
            momentum, rm, rv = self._train_args()
            link = BNLink() if torch.is_grad_enabled() else None
            ts = tile_stats_of(x)
            fold = ts[2] if ts is not None else None
            # a folded finalize zeroed its own output bound (the apply pass raises it)
            amax = fold.amax if (fold is not None and _want_amax(x)) else _amax_buf(x)
            spec, obound = _fwd_planes(self, x, residual, self.out_planes)
            if obound is not None:
                amax = None
            if link is not None and self.grad_planes and _conv._F32_PLANES and x.dtype == torch.float32 \
                    and self.running_mean is not None:
                link.gbuf = omax_buf(self.running_mean, "g", x.device)
            y = _BNActFn.apply(x, self.weight, self.bias, rm, rv, residual, momentum, self.eps, self.act,
                               res_slot, ts, link, amax, spec)
            if link is not None:
                y._mpit_bnlink = link
            if obound is not None:
                set_planes(y, obound)
                COUNTERS["fwd_planes"] += 1
            elif amax is not None:
                set_amax(y, amax)
            return y
        return bn_act_eval(x, self.weight, self.bias, self.running_mean, self.running_var, self.eps, residual, self.act)


class _BNPairFn(torch.autograd.Function):
    """relu(bn1(x1) + bn2(x2)) for a ResNet block's last BN (bn1) and its downsample
    shortcut's BN (bn2): forward = the two coefficient sets (from the producing convs'
    tile statistics) and ONE pass writing y and the ReLU mask; backward = the two
    coefficient sets (from the consumer conv's paired epilogue reduction, BNLink.x2) and
    ONE pass writing dx1 and dx2. Replaces bn2's apply pass, its reduction pass and the
    residual-gradient tensor of the unpaired form."""

    @staticmethod
    def forward(ctx, x1, w1, b1, rm1, rv1, x2, w2, b2, rm2, rv2, mom1, eps1, mom2, eps2, ts1, ts2, link, amax=None,
                planes=None):
        x1, x2 = _cl(x1), _cl(x2).to(x1.dtype)
        M, C = _rows(x1)
        m = native()
        dev, stream = x1.device.index, torch.cuda.current_stream(x1.device).cuda_stream
        bf16 = x1.dtype == torch.bfloat16
        f32 = dict(dtype=torch.float32, device=x1.device)
        outs = []
        zeroed = False
        for x, w, b, rm, rv, mom, eps, ts in ((x1, w1, b1, rm1, rv1, mom1, eps1, ts1),
                                             (x2, w2, b2, rm2, rv2, mom2, eps2, ts2)):
            mean, rstd = torch.empty(C, **f32), torch.empty(C, **f32)
            ws = torch.empty(m.bn_workspace_floats(C), **f32)
            wf = w.float().contiguous() if w is not None else None
            bf = b.float().contiguous() if b is not None else None
            ts = ts if (ts is not None and ts[1] == m.gemm_nt_tiles(M)) else None
            if ts is not None:
                COUNTERS["fwd_tile_stats"] += 1
            fold = ts[2] if ts is not None else None
            if fold is not None:  # finalize run by the producing GEMM: its coefficients
                COUNTERS["fwd_folded"] += 1
                outs.append((wf, fold.mean, fold.rstd, fold.coef))
                continue
            # (the first finalize also zeroes the pair's output bound, raised by the pair apply)
            m.bn_act_fwd(dev, stream, bf16, x.data_ptr(), 0, 0, M, C, wf.data_ptr() if wf is not None else 0,
                         bf.data_ptr() if bf is not None else 0, rm.data_ptr() if rm is not None else 0,
                         rv.data_ptr() if rv is not None else 0, mean.data_ptr(), rstd.data_ptr(), ws.data_ptr(),
                         float(mom), float(eps), False, 0, stats=ts[0].data_ptr() if ts is not None else 0,
                         nstat=ts[1] if ts is not None else 0,
                         amax=amax.data_ptr() if (amax is not None and not zeroed) else 0)
            zeroed = True
            outs.append((wf, mean, rstd, ws))
        if amax is not None and not zeroed:  # both finalizes folded into their GEMMs
            amax.zero_()
        y = torch.empty_like(x1, memory_format=torch.channels_last)
        mask = torch.empty(m.bn_mask_bytes(bf16, M, C), dtype=torch.uint8, device=x1.device)
        # (scratch of the output bound: bn1's workspace past its coefficients)
        m.bn_pair_apply(dev, stream, x1.data_ptr(), outs[0][3].data_ptr(), x2.data_ptr(), outs[1][3].data_ptr(),
                        y.data_ptr(), M, C, mask.data_ptr(), f32=not bf16,
                        amax=amax.data_ptr() if amax is not None else 0, planes=planes)
        (wf1, mean1, rstd1, _), (wf2, mean2, rstd2, _) = outs
        ctx.save_for_backward(x1, x2, mask, wf1, mean1, rstd1, wf2, mean2, rstd2)
        ctx.has = (w1 is not None, b1 is not None, w2 is not None, b2 is not None)
        ctx.link = link
        if link is not None:
            link.x, link.mask, link.mean, link.x2, link.mean2 = x1, mask, mean1, x2, mean2
        ctx.xmax = (omax_of(x1), omax_of(x2)) if getattr(link, "gbuf", None) is not None else None
        return y

    @staticmethod
    def backward(ctx, dy):
        x1, x2, mask, wf1, mean1, rstd1, wf2, mean2, rstd2 = ctx.saved_tensors
        dy = _cl(dy).to(x1.dtype)
        M, C = _rows(x1)
        m = native()
        dev, stream = x1.device.index, torch.cuda.current_stream(x1.device).cuda_stream
        gm = (ctx.link.gbuf, ctx.link.gep) if ctx.link is not None else (None, 0)
        part, npart, part2 = ctx.link.take(dy, pair=True) if ctx.link is not None else (None, 0, None)
        xm = getattr(ctx, "xmax", None)
        planes = (part is not None and gm[0] is not None and gm[1] and xm is not None and xm[0] is not None
                  and xm[1] is not None and x1.dtype == torch.float32)
        if part is not None:
            COUNTERS["bwd_linked"] += 2
        f32 = dict(dtype=torch.float32, device=x1.device)
        grads, wss = [], []
        am1, am2 = _amax_buf(x1), _amax_buf(x1)  # bounds of dx1, dx2: zeroed by the two finalizes
        for x, wf, mean, rstd, p, hw, hb, am in ((x1, wf1, mean1, rstd1, part, ctx.has[0], ctx.has[1], am1),
                                                (x2, wf2, mean2, rstd2, part2, ctx.has[2], ctx.has[3], am2)):
            dg = torch.empty(C, **f32) if hw else None
            db = torch.empty(C, **f32) if hb else None
            ws = torch.empty(m.bn_workspace_floats(C), **f32)
            m.bn_act_bwd(dev, stream, x1.dtype == torch.bfloat16, dy.data_ptr(), mask.data_ptr(), x.data_ptr(), 0, 0, M, C,
                         wf.data_ptr() if wf is not None else 0, mean.data_ptr(), rstd.data_ptr(),
                         dg.data_ptr() if dg is not None else 0, db.data_ptr() if db is not None else 0, ws.data_ptr(),
                         True, part=p.data_ptr() if p is not None else 0, npart=npart if p is not None else 0,
                         amax=am.data_ptr() if am is not None else 0)
            grads.append((dg, db))
            wss.append(ws)
        dx1 = torch.empty_like(x1, memory_format=torch.channels_last)
        dx2 = torch.empty_like(x2, memory_format=torch.channels_last)
        p1 = p2 = None
        if planes:
            pb1 = torch.empty(_conv.BOUND_FLOATS, **f32)
            pb2 = torch.empty(_conv.BOUND_FLOATS, **f32)
            p1 = dict(obound=pb1.data_ptr(), gmax=gm[0].data_ptr(), gep=gm[1], xmax=xm[0][0].data_ptr(), xep=xm[0][1])
            p2 = dict(obound=pb2.data_ptr(), gmax=gm[0].data_ptr(), gep=gm[1], xmax=xm[1][0].data_ptr(), xep=xm[1][1])
        m.bn_pair_bwd_apply(dev, stream, dy.data_ptr(), mask.data_ptr(), x1.data_ptr(), wss[0].data_ptr(),
                            dx1.data_ptr(), x2.data_ptr(), wss[1].data_ptr(), dx2.data_ptr(), M, C,
                            f32=x1.dtype == torch.float32, amax1=am1.data_ptr() if am1 is not None else 0,
                            amax2=am2.data_ptr() if am2 is not None else 0, planes1=p1, planes2=p2)
        if planes:
            set_planes(dx1, pb1)
            set_planes(dx2, pb2)
            COUNTERS["bwd_planes"] += 2
        elif am1 is not None:
            set_amax(dx1, am1)
            set_amax(dx2, am2)
        (dg1, db1), (dg2, db2) = grads
        return (dx1, dg1, db1, None, None, dx2, dg2, db2, None, None, None, None, None, None, None, None, None, None,
                None)


def bn_pair(bn1: "BatchNormAct2d", x1: torch.Tensor, bn2: "BatchNormAct2d", x2: torch.Tensor) -> torch.Tensor:
    """``relu(bn1(x1) + bn2(x2))`` (bn1 with ReLU, bn2 without): one fused op on the GPU
    training path (:class:`_BNPairFn`), the two modules otherwise."""
    ok = (bn1.act and not bn2.act and bn1.training and bn2.training and bn1.track_running_stats
          and bn2.track_running_stats and _supported(x1) and x2.shape == x1.shape
          and x2.is_cuda and x2.dtype in (torch.bfloat16, torch.float32))
    if not ok:
        return bn1(x1, bn2(x2))
    mom1, rm1, rv1 = bn1._train_args()
    mom2, rm2, rv2 = bn2._train_args()
    link = BNLink() if torch.is_grad_enabled() else None
    amax = _amax_buf(x1)
    # fp16 planes: the output (both inputs' maxima known), the input gradients (bn1.grad_planes)
    spec = obound = None
    if bn1.out_planes and _conv._F32_PLANES and x1.dtype == torch.float32:
        o1, o2 = omax_of(x1), omax_of(x2)
        if o1 is not None and o2 is not None:
            obound = torch.empty(_conv.BOUND_FLOATS, dtype=torch.float32, device=x1.device)
            spec = dict(obound=obound.data_ptr(), xmax=o1[0].data_ptr(), xep=o1[1], xmax2=o2[0].data_ptr(), xep2=o2[1])
            amax = None
    if link is not None and bn1.grad_planes and _conv._F32_PLANES and x1.dtype == torch.float32 \
            and bn1.running_mean is not None and omax_of(x1) is not None and omax_of(x2) is not None:
        link.gbuf = omax_buf(bn1.running_mean, "g", x1.device)
    y = _BNPairFn.apply(x1, bn1.weight, bn1.bias, rm1, rv1, x2, bn2.weight, bn2.bias, rm2, rv2, mom1, bn1.eps, mom2,
                        bn2.eps, tile_stats_of(x1), tile_stats_of(x2), link, amax, spec)
    if link is not None:
        y._mpit_bnlink = link
    if obound is not None:
        set_planes(y, obound)
        COUNTERS["fwd_planes"] += 1
    elif amax is not None:
        set_amax(y, amax)
    return y

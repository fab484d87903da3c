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

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .._ext import native


def _rows(x: torch.Tensor):
    n, c, h, w = x.shape
    return n * h * w, c


def _cl(x: torch.Tensor) -> torch.Tensor:
    return x if x.is_contiguous(memory_format=torch.channels_last) else x.contiguous(memory_format=torch.channels_last)


# how often each fused hand-over fired (tests assert the fused path ran)
COUNTERS = {"fwd_tile_stats": 0, "bwd_linked": 0}


class BNLink:
    """What a convolution consuming a BN layer's output needs to fold that layer's backward
    reduction into its backward-data GEMM, and where it leaves the result.

    Filled by the BN forward (its saved input ``x``, ReLU ``mask``, batch ``mean``); the
    consumer's backward writes ``part`` ([npart][2][C] partial sums) and records which
    gradient tensor they describe (``dy_ptr``, ``dy_ver``). The BN backward uses them only
    if it receives exactly that tensor, unmodified — when autograd summed gradients from
    several consumers it falls back to its own reduction pass."""

    __slots__ = ("x", "mask", "mean", "part", "npart", "dy_ptr", "dy_ver")

    def __init__(self):
        self.x = self.mask = self.mean = self.part = None
        self.npart = 0
        self.dy_ptr = self.dy_ver = None

    def ready(self, x: torch.Tensor) -> bool:
        """True when ``x`` (a consumer's input) is this layer's output shape, bf16."""
        return (self.x is not None and self.mean is not None and x.dtype == torch.bfloat16
                and self.x.shape == x.shape)

    def publish(self, part: torch.Tensor, npart: int, dy: torch.Tensor):
        self.part, self.npart = part, int(npart)
        self.dy_ptr, self.dy_ver = dy.data_ptr(), dy._version

    def take(self, dy: torch.Tensor):
        part, npart = self.part, self.npart
        ok = part is not None and dy.data_ptr() == self.dy_ptr and dy._version == self.dy_ver
        self.part, self.x, self.mask, self.mean = None, None, None, None
        return (part, npart) if ok else (None, 0)


def tile_stats_of(x: torch.Tensor):
    """(partials, tiles) a producing GEMM attached to ``x`` (see module docstring), or None."""
    ts = getattr(x, "_mpit_tstats", None)
    if ts is None or ts[2] != x.data_ptr():
        return None
    return ts[0], ts[1]


class _BNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, residual, momentum, eps, relu, res_slot=None,
                tstats=None, link=None):
        x = _cl(x)
        if residual is not None:
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
        ts = tstats if (tstats is not None and bf16 and tstats[1] == m.gemm_nt_tiles(M)) else None
        if ts is not None:
            COUNTERS["fwd_tile_stats"] += 1
        m.bn_act_fwd(dev, stream, bf16, x.data_ptr(),
                     residual.data_ptr() if residual is not None else 0, y.data_ptr(), M, C,
                     w.data_ptr() if w is not None else 0, b.data_ptr() if b is not None else 0,
                     running_mean.data_ptr() if running_mean is not None else 0,
                     running_var.data_ptr() if running_var is not None else 0,
                     mean.data_ptr(), rstd.data_ptr(), ws.data_ptr(), float(momentum), float(eps), bool(relu),
                     mask.data_ptr() if mask is not None else 0,
                     stats=ts[0].data_ptr() if ts is not None else 0, nstat=ts[1] if ts is not None else 0)
        ctx.save_for_backward(x, mask, w, mean, rstd)
        ctx.link = link
        if link is not None and bf16:
            link.x, link.mask, link.mean = x, mask, mean
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
        park = ctx.has_res and ctx.res_slot is not None and ctx.relu and mask is not None and dy.dtype == torch.bfloat16
        dres = torch.empty_like(x, memory_format=torch.channels_last) if (ctx.has_res and not park) else None
        dgamma = torch.empty(C, dtype=torch.float32, device=x.device) if ctx.has_w else None
        dbeta = torch.empty(C, dtype=torch.float32, device=x.device) if ctx.has_b else None
        ws = torch.empty(m.bn_workspace_floats(C), dtype=torch.float32, device=x.device)
        # reductions folded into the consumer convolution's backward-data GEMM (BNLink)
        part, npart = ctx.link.take(dy) if ctx.link is not None else (None, 0)
        if part is not None:
            COUNTERS["bwd_linked"] += 1
        m.bn_act_bwd(dev, stream, x.dtype == torch.bfloat16, dy.data_ptr(),
                     mask.data_ptr() if mask is not None else 0, x.data_ptr(), dx.data_ptr(),
                     dres.data_ptr() if dres is not None else 0, M, C, w.data_ptr() if w is not None else 0,
                     mean.data_ptr(), rstd.data_ptr(), dgamma.data_ptr() if dgamma is not None else 0,
                     dbeta.data_ptr() if dbeta is not None else 0, ws.data_ptr(), bool(ctx.relu),
                     part=part.data_ptr() if part is not None else 0, npart=npart)
        if ctx.res_slot is not None:  # the shortcut's gradient is added by the block's first conv
            if park:
                if not ctx.res_slot.put(dy, mask):
                    raise RuntimeError("GradSlot consumer ran before the BN backward")
            elif not ctx.res_slot.put(dres):
                raise RuntimeError("GradSlot consumer ran before the BN backward")
            dres = None
        return dx, dgamma, dbeta, None, None, dres, None, None, None, None, None, None


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
    v = 8 if x.dtype == torch.bfloat16 else 4
    return x.shape[1] % v == 0


class BatchNormAct2d(nn.BatchNorm2d):
    """``act(bn(x) + residual)`` with ReLU act; a drop-in ``nn.BatchNorm2d`` subclass."""

    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True, track_running_stats=True, act=True):
        super().__init__(num_features, eps, momentum, affine, track_running_stats)
        self.act = act
        # num_batches_tracked only matters to the math when momentum is None; otherwise the
        # count is kept on the host and folded into the buffer when the state is read
        # (one tiny "+= 1" kernel per BN per step otherwise: 53 launches in ResNet-50)
        self._nbt_pending = 0

    def sync_num_batches_tracked(self):
        if self._nbt_pending:
            with torch.no_grad():
                self.num_batches_tracked.add_(self._nbt_pending)
            self._nbt_pending = 0

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        self.sync_num_batches_tracked()
        super()._save_to_state_dict(destination, prefix, keep_vars)

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
            link = BNLink() if (torch.is_grad_enabled() and x.dtype == torch.bfloat16) else None
            y = _BNActFn.apply(x, self.weight, self.bias, rm, rv, residual, momentum or 0.0, self.eps, self.act,
                               res_slot, tile_stats_of(x), link)
            if link is not None:
                y._mpit_bnlink = link
            return y
        return bn_act_eval(x, self.weight, self.bias, self.running_mean, self.running_var, self.eps, residual, self.act)

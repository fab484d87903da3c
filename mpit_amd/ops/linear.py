"""Fully connected layers (+ bias, + ReLU) of the VGG / AlexNet classifiers on the MFMA GEMM
kernels, bf16 steps (the reference's nn.Linear + nn.ReLU pairs: asyncsgd/models, the
Torch7 ``nn.Linear``).

Under autocast a plain ``nn.Linear`` costs, per step, a bf16 cast of its fp32 weight in the
forward, a hipBLASLt GEMM picked for a 64-row batch, and a bf16 -> fp32 cast of the weight
gradient in the backward. For VGG-16's first classifier layer (25088 x 4096, 411 MB of fp32
weight) the two casts alone move 1.2 GB per step. Here:

* the weight is cast ONCE per step by the model's :class:`ops.conv.WeightCastPlan` launch,
  as its transpose ``wt[K, N]`` only (rows padded to a multiple of 64 with zero columns for a
  1000-class layer; fp32 in an fp32 step): every GEMM below reads that one operand;
* forward ``y = x W^T`` runs as the split-K weight-gradient kernel ``gemm_tn`` over the
  K = in_features rows of ``wt`` and ``x^T``, a grid of (N / 128) x splits blocks instead of a
  64-row GEMM's N / 128 (which leaves most of the 256 CUs idle); bias + ReLU on its small
  [N, batch] fp32 output;
* backward: ``dz = dy * (y > 0)`` and the bias gradient in one pass (``relu_bias_bwd``),
  ``dx = dz W`` as ``gemm_nt`` against ``wt``, and the weight gradient ``dz^T x`` as
  ``gemm_tn`` written in fp32 straight into the gradient (no cast).

fp32 steps (and ResNet's fp32 classifier under bf16 autocast) run the same three GEMMs on fp32
operands (the kernels' bf16x6 split products: no operand bounds needed, fp32-class results),
so no library GEMM is left in those steps either.

Falls back to ``F.linear`` (+ ``F.relu``) off the MFMA path (CPU) or when the shapes do not
tile (in / out features % 64, batch % 64). MPIT_LINEAR_FUSE=0: always the fallback;
MPIT_LINEAR_F32=0: fp32 inputs take the fallback."""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from .._ext import native
from ..utils.flat import grad_out
from .conv import WeightCastPlan, mfma_dtype


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _np(n: int) -> int:
    return (n + 63) // 64 * 64


def _wt_of(mod, weight: torch.Tensor, dt=torch.bfloat16) -> torch.Tensor:
    """wt[K, Np] in ``dt`` of this step (Np = out_features rounded up to 64): the cast plan's,
    else cast here. A layer whose out_features is not a multiple of 64 (the 1000-class output
    layers) keeps a zero-padded transpose of its own and refreshes its first N columns."""
    n, k = weight.shape
    c = WeightCastPlan.cached(mod, dt)
    if c is not None:
        return c[1]
    if n % 64:
        buf = getattr(mod, "_mpit_wt_pad", None)
        if buf is None or buf.device != weight.device or buf.shape != (k, _np(n)) or buf.dtype != dt:
            buf = torch.zeros((k, _np(n)), dtype=dt, device=weight.device)
            mod._mpit_wt_pad = buf
        with torch.no_grad():
            buf[:, :n].copy_(weight.detach().t())
        return buf
    if dt == torch.float32:
        return weight.detach().t().contiguous()
    wt = torch.empty((k, n), dtype=torch.bfloat16, device=weight.device)
    w = weight.detach()
    if not w.is_contiguous():
        w = w.contiguous()
    native().cast_transpose(w.device.index, _stream(w), w.data_ptr(), n, k, 0, wt.data_ptr(), f32=False)
    return wt


class _LinearActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, act: bool, wt):
        m = native()
        dev = x.device.index
        st = _stream(x)
        dt = wt.dtype
        f32 = dt == torch.float32
        xb = x.to(dt)
        M, K = xb.shape
        N = weight.shape[0]
        Np = wt.shape[1]  # (N rounded up to 64: the padded columns of wt are zero)
        xt = xb.t().contiguous()  # [K, M]: the reduction runs over the rows of wt and x^T
        yt = torch.empty((Np, M), dtype=torch.float32, device=x.device)
        nws = m.gemm_tn_ws_floats(dev, K, Np, M)
        ws = torch.empty(nws, dtype=torch.float32, device=x.device) if nws else None
        m.gemm_tn(dev, st, K, Np, M, wt.data_ptr(), Np, xt.data_ptr(), M, yt.data_ptr(),
                  ws.data_ptr() if ws is not None else 0, 0.0, f32=f32)
        y = yt[:N].t().contiguous()  # [M, N] row-major (1 MB at VGG's shapes)
        if bias is not None:
            y.add_(bias)
        if act:
            y.relu_()
        y = y.to(dt)
        ctx.save_for_backward(xb, wt, y if act else None)
        ctx.flags = (act, bias is not None)
        ctx.wparam = weight
        ctx.n = N
        return y

    @staticmethod
    def backward(ctx, dy):
        xb, wt, y = ctx.saved_tensors
        act, has_bias = ctx.flags
        m = native()
        dev = xb.device.index
        st = _stream(xb)
        M, K = xb.shape
        N, Np = ctx.n, wt.shape[1]
        dt = wt.dtype
        f32 = dt == torch.float32
        dy = dy.to(dt).contiguous()
        want_db = has_bias and ctx.needs_input_grad[2]
        db = None
        if act:
            dz = torch.empty_like(dy)
            db = torch.empty(N, dtype=torch.float32, device=dy.device) if want_db else None
            rws = torch.empty(m.relu_bias_bwd_ws_floats(N), dtype=torch.float32, device=dy.device) if want_db else None
            m.relu_bias_bwd(dev, st, M, N, dy.data_ptr(), y.data_ptr(), dz.data_ptr(),
                            db.data_ptr() if db is not None else 0, rws.data_ptr() if rws is not None else 0,
                            f32=f32)
        else:
            dz = dy
            if want_db:
                db = dz.float().sum(0)
        dx = dw = None
        if Np != N:  # zero-padded columns (their products vanish against wt's zero columns)
            dzp = torch.zeros((M, Np), dtype=dt, device=dy.device)
            dzp[:, :N].copy_(dz)
            dz = dzp
        if ctx.needs_input_grad[0]:  # dx[M, K] = dz[M, N] . W[N, K] = dz . wt^T
            dx = torch.empty((M, K), dtype=dt, device=dy.device)
            m.gemm_nt(dev, st, M, K, Np, dz.data_ptr(), Np, wt.data_ptr(), Np, dx.data_ptr(), K, 0, f32=f32)
        if ctx.needs_input_grad[1]:  # dW[N, K] = dz^T . x, fp32 straight into the gradient
            full = grad_out(ctx.wparam, (N, K), dy.device) if Np == N else torch.empty(
                (Np, K), dtype=torch.float32, device=dy.device)
            nws = m.gemm_tn_ws_floats(dev, M, Np, K)
            ws = torch.empty(nws, dtype=torch.float32, device=dy.device) if nws else None
            m.gemm_tn(dev, st, M, Np, K, dz.data_ptr(), Np, xb.data_ptr(), K, full.data_ptr(),
                      ws.data_ptr() if ws is not None else 0, 0.0, f32=f32)
            dw = full[:N]
        return dx, dw, db, None, None


class LinearAct(nn.Linear):
    """``act(linear(x))`` with act = ReLU or identity; the bf16 MFMA path above when it
    applies (see module docstring), ``F.linear`` (+ ``F.relu``) otherwise."""

    _mpit_linear = True  # (ops.conv.WeightCastPlan: cast with the model's convolutions)
    enabled = os.environ.get("MPIT_LINEAR_FUSE", "1") != "0"
    f32_enabled = os.environ.get("MPIT_LINEAR_F32", "1") != "0"

    def __init__(self, in_features: int, out_features: int, bias: bool = True, act: bool = True,
                 pad_out: bool = False):
        super().__init__(in_features, out_features, bias=bias)
        self.act = act
        # out_features not a multiple of 64 (a 1000-class output layer): run the GEMMs on N
        # padded to 64 with zero columns (its transpose then is cast here, not by the plan)
        self.pad_out = pad_out

    def fused(self, x: torch.Tensor) -> bool:
        dt = mfma_dtype(x)
        return (LinearAct.enabled and x.is_cuda and x.dim() == 2
                and (dt == torch.bfloat16 or (dt == torch.float32 and LinearAct.f32_enabled))
                and self.in_features % 64 == 0 and (self.out_features % 64 == 0 or self.pad_out)
                and x.shape[0] % 64 == 0 and self.weight.dtype == torch.float32 and self.weight.is_contiguous())

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.fused(x):
            dt = mfma_dtype(x)  # (outside the autocast-off region: bf16 under bf16 autocast)
            with torch.autocast("cuda", enabled=False):
                return _LinearActFn.apply(x, self.weight, self.bias, self.act, _wt_of(self, self.weight, dt))
        y = F.linear(x, self.weight, self.bias)
        return F.relu(y) if self.act else y

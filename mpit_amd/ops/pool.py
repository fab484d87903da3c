"""NHWC max pooling on MI355X (csrc/kernels/pool.hip): the ResNet stem's 3x3/2 pool.

The forward keeps a one-byte argmax per output element; the backward gathers, for each
input pixel, the gradients of the windows that selected it (dx written once, no atomics,
no zero fill). :class:`MaxPool2dNHWC` is a drop-in ``nn.MaxPool2d`` that takes this path
for bf16 / fp32 channels_last CUDA tensors with C % 8 == 0 and falls back to PyTorch otherwise.
Below a conv(+bias)+ReLU (VGG, AlexNet: ``ops.conv.ReluLink`` on the input) the backward also
applies that ReLU (mask = pooled output > 0) and sums the conv's bias gradient.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .._ext import native
from . import conv as _conv
from .conv import ReluLink, amax_of, set_amax, set_planes


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k: int, stride: int, pad: int, obound=None):
        up = ReluLink.of(x)
        if up is not None and 256 % (x.shape[1] // 8):
            up = None
        if not x.is_contiguous(memory_format=torch.channels_last):
            x = x.contiguous(memory_format=torch.channels_last)
        n, c, h, w = x.shape
        ho, wo = (h + 2 * pad - k) // stride + 1, (w + 2 * pad - k) // stride + 1
        y = torch.empty((n, c, ho, wo), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
        idx = torch.empty((n, ho, wo, c), dtype=torch.uint8, device=x.device)
        ib = amax_of(x) if obound is not None else None
        if obound is not None and (ib is None or up is not None or x.dtype != torch.float32):
            raise RuntimeError("max pool planes output needs an fp32 input with its bound and no ReLU link")
        native().maxpool_fwd(x.device.index, _stream(x), n, h, w, c, k, stride, pad, x.data_ptr(), y.data_ptr(),
                             idx.data_ptr(), f32=x.dtype == torch.float32, ibound=ib.data_ptr() if ib is not None else 0,
                             obound=obound.data_ptr() if obound is not None else 0)
        ctx.dt = x.dtype
        ctx.up = up
        ctx.save_for_backward(idx, y if up is not None else None)
        ctx.geo = (n, c, h, w, k, stride, pad)
        return y

    @staticmethod
    def backward(ctx, dy):
        idx, yp = ctx.saved_tensors
        n, c, h, w, k, stride, pad = ctx.geo
        if dy.dtype != ctx.dt:
            dy = dy.to(ctx.dt)
        if not dy.is_contiguous(memory_format=torch.channels_last):
            dy = dy.contiguous(memory_format=torch.channels_last)
        dx = torch.empty((n, c, h, w), dtype=ctx.dt, device=dy.device, memory_format=torch.channels_last)
        m = native()
        kw, db, up = {}, None, ctx.up
        if up is not None:  # dx is the conv's dz (ReLU applied), db its bias gradient
            ws = torch.empty(m.maxpool_bwd_ws_floats(c), dtype=torch.float32, device=dy.device)
            db = torch.empty(c, dtype=torch.float32, device=dy.device) if up.has_bias else None
            kw = dict(ypool=yp.data_ptr(), db=db.data_ptr() if db is not None else 0, ws=ws.data_ptr())
        m.maxpool_bwd(dy.device.index, _stream(dy), n, h, w, c, k, stride, pad, dy.data_ptr(), idx.data_ptr(),
                      dx.data_ptr(), f32=ctx.dt == torch.float32, **kw)
        if up is not None:
            up.give(dx, db)
        return dx, None, None, None, None


def _int(v):
    return v[0] if isinstance(v, (tuple, list)) else v


class MaxPool2dNHWC(nn.MaxPool2d):
    """``nn.MaxPool2d(k, stride, padding)`` with the HIP path for bf16 / fp32 NHWC tensors."""

    def fused(self, x: torch.Tensor) -> bool:
        k, s, p = _int(self.kernel_size), _int(self.stride), _int(self.padding)
        return (x.is_cuda and x.dim() == 4 and x.dtype in (torch.bfloat16, torch.float32) and x.shape[1] % 8 == 0
                and _int(self.dilation) == 1 and not self.ceil_mode and not self.return_indices
                and 2 * p <= k <= 15 and self.kernel_size in (k, (k, k)) and self.stride in (s, (s, s))
                and self.padding in (p, (p, p)))

    # out_planes (fp32 steps): the output is read only by fp16x3 GEMMs (a ResNet stem pool feeds
    # the first block's convolutions and its residual add): written as fp16 planes scaled by the
    # input's bound (ops/conv.py _F32_PLANES). Set by the model.
    out_planes = False

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.fused(x):
            a = amax_of(x)
            pl = (self.out_planes and _conv._F32_PLANES and x.dtype == torch.float32 and a is not None
                  and ReluLink.of(x) is None and self.training)
            ob = torch.empty(_conv.BOUND_FLOATS, dtype=torch.float32, device=x.device) if pl else None
            y = _MaxPoolFn.apply(x, _int(self.kernel_size), _int(self.stride), _int(self.padding), ob)
            if ob is not None:
                set_planes(y, ob)
            elif a is not None:  # every output is one of the inputs: the input's bound holds
                set_amax(y, a)
            return y
        return super().forward(x)


class _GlobalAvgPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.geo = (x.shape, x.dtype)
        return F.adaptive_avg_pool2d(x, 1)

    @staticmethod
    def backward(ctx, dy):
        (n, c, h, w), dt = ctx.geo
        dy = dy.reshape(n, c).to(dt).contiguous()
        dx = torch.empty((n, c, h, w), dtype=dt, device=dy.device, memory_format=torch.channels_last)
        native().avgpool_bwd(dy.device.index, _stream(dy), n, h * w, c, dy.data_ptr(), dx.data_ptr(),
                             f32=dt == torch.float32)
        return dx


class GlobalAvgPoolNHWC(nn.AdaptiveAvgPool2d):
    """``nn.AdaptiveAvgPool2d(1)`` whose backward writes the channels_last input gradient in one
    HIP pass (csrc/kernels/pool.hip ``avgpool_bwd``: dy / HW broadcast over the pixels) instead
    of PyTorch's expand + copy (~1 TB/s; 80-100 us per ResNet-50 step). Forward unchanged."""

    def __init__(self):
        super().__init__(1)

    def fused(self, x: torch.Tensor) -> bool:
        return (x.is_cuda and x.dim() == 4 and x.dtype in (torch.bfloat16, torch.float32) and x.shape[1] % 8 == 0
                and x.is_contiguous(memory_format=torch.channels_last) and torch.is_grad_enabled())

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.fused(x):
            return _GlobalAvgPoolFn.apply(x)
        return super().forward(x)

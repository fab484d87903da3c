"""Softmax cross-entropy of the classifier's logits on one native kernel (csrc/kernels/loss.hip;
the reference's nn.CrossEntropyCriterion / ClassNLLCriterion over LogSoftMax,
asyncsgd/goot.lua).

The forward computes each row's loss AND the logits' gradient of the mean loss in one pass
over the logits (bf16 logits are read as they are: no fp32 copy); the backward is one multiply
by the incoming scalar gradient. PyTorch's path is log_softmax + nll_loss forward, their two
backward kernels and their fills (plus a cast for bf16 logits) — small launches at the turn
from forward to backward, where the host issues them one by one.

Falls back to ``F.cross_entropy`` on the CPU, for other dtypes, targets on another device or
given as probabilities. Class weights, ignore_index, label smoothing and other reductions are
not part of this API (call ``F.cross_entropy``). A target outside [0, C) gives a NaN loss (PyTorch
raises a device-side assert). MPIT_FUSED_XENT=0: always the fallback."""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from .._ext import native

_ENABLED = os.environ.get("MPIT_FUSED_XENT", "1") != "0"


class _SoftmaxXentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target):
        rows, C = logits.shape
        x = logits if logits.stride(1) == 1 else logits.contiguous()
        tgt = target if target.dtype == torch.int64 and target.is_contiguous() else target.long().contiguous()
        loss = torch.empty(rows, dtype=torch.float32, device=logits.device)
        d = torch.empty((rows, C), dtype=torch.float32, device=logits.device)
        native().softmax_xent(logits.device.index, torch.cuda.current_stream(logits.device).cuda_stream, rows, C,
                              x.data_ptr(), x.stride(0), x.dtype == torch.bfloat16, tgt.data_ptr(), 1.0 / rows,
                              loss.data_ptr(), d.data_ptr())
        ctx.save_for_backward(d)
        return loss.mean()

    @staticmethod
    def backward(ctx, g):
        (d,) = ctx.saved_tensors
        return d * g, None


def fused_ok(logits: torch.Tensor, target: torch.Tensor) -> bool:
    # (the kernel reads the targets on the logits' device: anything else takes PyTorch's path,
    # which also raises the usual errors for it)
    return (_ENABLED and logits.is_cuda and logits.dim() == 2 and logits.dtype in (torch.float32, torch.bfloat16)
            and target.dim() == 1 and target.shape[0] == logits.shape[0] and logits.shape[0] > 0
            and target.device == logits.device and not target.dtype.is_floating_point)


def cross_entropy(logits: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """Mean softmax cross-entropy (``F.cross_entropy(logits.float(), target)``), fp32 math."""
    if fused_ok(logits, target):
        return _SoftmaxXentFn.apply(logits, target)
    return F.cross_entropy(logits.float(), target)

"""Flat parameter / gradient storage for a module (the reference's ``getParameters``,
asyncsgd/goot.lua:41, BiCNN/bicnn.lua:255).

Every parameter becomes a view into one contiguous fp32 buffer (which can be a PS or
all-reduce window: the parameter server then writes pulled shards straight into the
model), and every ``.grad`` a view into one contiguous gradient buffer that autograd
accumulates into in place. 4-D conv weights may be laid out channels_last inside the
flat buffer (the view carries NHWC strides), so MIOpen's NHWC kernels read them directly.
Shared (tied) parameters are stored once, as ``getParameters`` does.
"""
from __future__ import annotations

import weakref
from typing import List, Optional

import torch

# id(parameter) -> (weakref to it, weakref to its stealing FlatParams, offset): see
# FlatParams.steal_grads / grad_out (a registry, not an attribute on the Parameter, which would
# follow it into pickles; keyed by id: tensors compare elementwise, so no WeakKeyDictionary)
_GSLOTS = {}


class FlatParams:
    def __init__(self, module: torch.nn.Module, param_buffer: Optional[torch.Tensor] = None,
                 grad_buffer: Optional[torch.Tensor] = None, channels_last: bool = False,
                 grad_dtype: torch.dtype = torch.float32, align: int = 64):
        params: List[torch.nn.Parameter] = []
        seen = set()
        for p in module.parameters():
            if id(p) in seen:
                continue
            seen.add(id(p))
            params.append(p)
        self.params = params
        self.channels_last = channels_last
        # offsets aligned to `align` elements so every view starts 16-B aligned
        offs, o = [], 0
        for p in params:
            offs.append(o)
            o += (p.numel() + align - 1) // align * align
        self.offsets = offs
        self.numel = o
        dev = params[0].device if params else torch.device("cpu")
        if param_buffer is None:
            param_buffer = torch.zeros(self.numel, dtype=torch.float32, device=dev)
        if param_buffer.numel() < self.numel:
            raise ValueError(f"param buffer too small: {param_buffer.numel()} < {self.numel}")
        self.flat = param_buffer.reshape(-1)
        if grad_buffer is None:
            grad_buffer = torch.zeros(self.numel, dtype=grad_dtype, device=self.flat.device)
        self.grad = grad_buffer.reshape(-1)
        with torch.no_grad():
            for p, off in zip(params, offs):
                pv = self._view(self.flat, p, off)
                pv.copy_(p.data.to(self.flat.device))
                p.data = pv
                p.grad = self._view(self.grad, p, off)

    def _view(self, buf: torch.Tensor, p: torch.Tensor, off: int) -> torch.Tensor:
        n = p.numel()
        seg = buf[off: off + n]
        if self.channels_last and p.dim() == 4:
            o, i, h, w = p.shape
            return seg.view(o, h, w, i).permute(0, 3, 1, 2)
        return seg.view(p.shape)

    # ------------------------------------------------------------------ steal mode
    def steal_grads(self):
        """Switch to "steal" mode: ``.grad`` is left unset so autograd hands over its
        own gradient tensors (no per-parameter ``grad += new`` kernels, no memset);
        :meth:`stolen` then gathers them in one fused kernel (ops.gather_scale_).

        A backward that knows its parameter can write the gradient straight into the flat
        gradient buffer instead (:func:`grad_out`: the MFMA convolutions' and classifier
        layers' weight-gradient GEMMs). Autograd then steals that view as ``.grad``, and
        :meth:`StolenGrads.materialize` skips it. VGG-16's 138 M gradients are otherwise
        copied once more per step. MPIT_GRAD_INPLACE=0 disables it."""
        import os

        for p, off in zip(self.params, self.offsets):
            p.grad = None
            _GSLOTS[id(p)] = (weakref.ref(p), weakref.ref(self), off)
        self._steal = True
        self.inplace = os.environ.get("MPIT_GRAD_INPLACE", "1") != "0"
        self._handed = set()  # parameters whose slot grad_out handed out since the last gather
        return self

    def grad_view(self, p: torch.Tensor, off: int) -> torch.Tensor:
        """A fresh view of ``p``'s slot in the flat gradient buffer (laid out like ``p``)."""
        return self._view(self.grad, p, off)

    def stolen(self) -> "StolenGrads":
        return StolenGrads(self)

    def rebind(self, param_buffer: torch.Tensor):
        """Move the parameters into another flat buffer (e.g. a host shm window)."""
        with torch.no_grad():
            param_buffer.reshape(-1)[: self.numel].copy_(self.flat[: self.numel])
            self.flat = param_buffer.reshape(-1)
            for p, off in zip(self.params, self.offsets):
                p.data = self._view(self.flat, p, off)

    def zero_grad(self):
        self.grad.zero_()

    def __len__(self):
        return self.numel


class StolenGrads:
    """The gradients autograd produced for a :class:`FlatParams` in steal mode.

    ``gather(dst, a, aux, b)`` writes ``dst[off] = a*g + b*aux[off]`` for every parameter in
    one launch (K12 bucketing fused with K9's scale); ``materialize()`` gathers into the
    flat gradient buffer for rules that need it. Either call releases the tensors."""

    def __init__(self, flat: FlatParams):
        self.flat = flat

    def _table(self, skip_inplace: bool = False):
        srcs, offs, ns = [], [], []
        self.missing = []
        gbase = self.flat.grad.data_ptr()
        es = self.flat.grad.element_size()
        for p, off in zip(self.flat.params, self.flat.offsets):
            g = p.grad
            if g is None:
                self.missing.append((p, off))
                continue
            if skip_inplace and g.data_ptr() == gbase + off * es and g.dtype == self.flat.grad.dtype:
                continue  # written in place by its backward (grad_out)
            if not g.is_contiguous(memory_format=torch.channels_last if g.dim() == 4 and self.flat.channels_last
                                   else torch.contiguous_format):
                g = g.contiguous(memory_format=torch.channels_last) if (g.dim() == 4 and self.flat.channels_last) \
                    else g.contiguous()
                p.grad = g
            srcs.append(g.data_ptr())
            offs.append(off)
            ns.append(g.numel())
        return srcs, offs, ns

    def gather(self, dst: torch.Tensor, a: float = 1.0, aux: torch.Tensor = None, b: float = 0.0):
        from ..ops.fused import gather_scale_

        inplace = dst.data_ptr() == self.flat.grad.data_ptr() and a == 1.0 and (aux is None or b == 0.0)
        srcs, offs, ns = self._table(skip_inplace=inplace)
        if self.missing:
            if inplace:  # (the in-place gradients already sit in dst: zero only the missing slots)
                for p, off in self.missing:
                    dst[off: off + p.numel()].zero_()
            else:
                dst.zero_()
            if aux is not None and b != 0.0:
                # parameters without a gradient this step still get the weight-decay term:
                # the reference adds l2wd*w to the whole dfdx (asyncsgd/optim-downpour.lua:24)
                for p, off in self.missing:
                    torch.mul(aux[off: off + p.numel()], b, out=dst[off: off + p.numel()])
        if srcs:
            gather_scale_(dst, srcs, offs, ns, a, aux, b)
        for p in self.flat.params:
            p.grad = None
        self.flat._handed = set()  # the next step's backwards may take the slots again
        return dst

    def materialize(self) -> torch.Tensor:
        return self.gather(self.flat.grad, 1.0)


def grad_out(param, shape, device, memory_format=torch.contiguous_format) -> torch.Tensor:
    """Where a backward should write ``param``'s fp32 gradient: its slot in the flat gradient
    buffer when the parameter belongs to a stealing :class:`FlatParams` (see
    ``steal_grads``), else a new tensor.

    The slot is handed out once per step: a parameter used twice in one forward (a module
    applied twice, tied weights) gets its slot for the first backward that runs and a fresh
    tensor for every later one, which autograd then adds into the slot (g1 + g2). Handing the
    slot out twice would let the second backward overwrite the first gradient and autograd
    sum two aliases of one buffer (2 g2)."""
    s = _GSLOTS.get(id(param)) if param is not None else None
    if s is not None and s[0]() is param:
        flat = s[1]()
        if flat is not None and getattr(flat, "inplace", False) and flat.grad.dtype == torch.float32:
            handed = flat.__dict__.setdefault("_handed", set())
            v = flat.grad_view(param, s[2])
            if (id(param) not in handed and tuple(v.shape) == tuple(shape)
                    and v.is_contiguous(memory_format=memory_format)):
                handed.add(id(param))
                return v
            if id(param) in handed:
                # a repeated use: autograd adds this tensor into the slot on the compute
                # stream, so its producer must not write it on the side stream (conv.py)
                g = torch.empty(shape, dtype=torch.float32, device=device, memory_format=memory_format)
                g._mpit_repeat = True
                return g
    return torch.empty(shape, dtype=torch.float32, device=device, memory_format=memory_format)

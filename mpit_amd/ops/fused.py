"""Fused update ops (SURVEY §2.7 K1–K14) over flat fp32 / bf16 tensors.

Every function runs ONE native pass: a HIP kernel (gfx950) on the tensor's current HIP
stream for device tensors, the identical C++ functor on the host for CPU tensors. The
math of each rule, with its reference citation, lives in csrc/kernels/update_rules.h;
the pure-PyTorch fp32 oracles used by the tests live in mpit_amd/ops/reference.py.

All operands of one call must have the same numel, be contiguous and live on the same
device. Dtypes: fp32 everywhere, bf16 allowed where noted (gradients, outputs, casts).
"""
from __future__ import annotations

import math
from typing import Optional, Sequence

import torch

from .._ext import native


def _check(ts: Sequence[Optional[torch.Tensor]]):
    ref = None
    for t in ts:
        if t is None:
            continue
        if not t.is_contiguous():
            raise ValueError("mpit ops need contiguous tensors")
        if t.dtype not in (torch.float32, torch.bfloat16):
            raise TypeError(f"mpit ops support float32/bfloat16, got {t.dtype}")
        if ref is None:
            ref = t
        else:
            if t.numel() != ref.numel():
                raise ValueError(f"operand size mismatch: {t.numel()} vs {ref.numel()}")
            if t.device != ref.device:
                raise ValueError("operands on different devices")
    return ref


def _launch(rule: int, variant: int, ts: Sequence[Optional[torch.Tensor]], scalars: Sequence[float], bf_ok=()):
    ref = _check(ts)
    n = ref.numel()
    m = native()
    if ref.is_cuda:
        dev = ref.device.index
        stream = torch.cuda.current_stream(ref.device).cuda_stream
    else:
        dev, stream = -1, 0
    ptrs, bf = [], 0
    for k, t in enumerate(ts):
        if t is None:
            ptrs.append(0)
            continue
        ptrs.append(t.data_ptr())
        if t.dtype == torch.bfloat16:
            if k not in bf_ok:
                raise TypeError(f"operand {k} of this rule must be float32")
            bf |= 1 << k
    m.ew_update(rule, variant, dev, stream, n, ptrs, bf, [float(s) for s in scalars])


def _R():
    return native().rule


# ---------------------------------------------------------------- server rules (K1–K6)

def apply_(p, g, a: float = 1.0, out=None):
    """K1: ``p += a*g`` (``out = p`` fused). asyncsgd/pserver.lua:91."""
    R = _R()
    ts = [p, g] + ([out] if out is not None else [])
    _launch(R.APPLY, R.OUT if out is not None else 0, ts, [a], bf_ok=(1, 2))
    return p


def apply_multi_(ps: Sequence[torch.Tensor], gs: Sequence[torch.Tensor], a: float = 1.0, outs=None):
    """K1 over several disjoint (p, g[, out]) segments in ONE launch (a server applying all
    the shard pieces that are due; ``csrc/kernels/ew.h`` ew_multi_kernel). Same result as
    one :func:`apply_` per segment, bit for bit."""
    R = _R()
    if len(ps) != len(gs) or (outs is not None and len(outs) != len(ps)):
        raise ValueError("apply_multi_: one gradient (and out) per parameter segment")
    if not ps:
        return ps
    segs, ns, bf = [], [], None
    for i, (p, g) in enumerate(zip(ps, gs)):
        ts = [p, g] + ([outs[i]] if outs is not None else [])
        ref = _check(ts)
        if ref.device != ps[0].device:
            raise ValueError("apply_multi_: segments on different devices")
        b = sum(1 << k for k, t in enumerate(ts) if t.dtype == torch.bfloat16)
        if b & 1:
            raise TypeError("operand 0 of this rule must be float32")
        if bf is not None and b != bf:
            raise TypeError("apply_multi_: every segment needs the same operand dtypes")
        bf = b
        segs.append([t.data_ptr() for t in ts])
        ns.append(ref.numel())
    if ps[0].is_cuda:
        dev, stream = ps[0].device.index, torch.cuda.current_stream(ps[0].device).cuda_stream
    else:
        dev, stream = -1, 0
    native().ew_update_multi(R.APPLY, R.OUT if outs is not None else 0, dev, stream, ns, segs, bf, [float(a)])
    return ps


def apply_sum_(p, grads: Sequence[torch.Tensor], a: float = 1.0, out=None):
    """K1 multi-inbox: ``p += a*Σ g_k`` in one pass (1..8 inboxes)."""
    R = _R()
    ng = len(grads)
    if not 1 <= ng <= 8:
        raise ValueError("apply_sum_ takes 1..8 gradients")
    ts = [p] + list(grads) + ([out] if out is not None else [])
    var = (ng << 8) | (R.OUT if out is not None else 0)
    _launch(R.APPLY_SUM, var, ts, [a], bf_ok=(1, ng + 1) if ng == 1 else (ng + 1,))
    return p


def rmsprop_(p, g, ga, gs, u, decay, lr, mom, eps, add: bool = True, out=None):
    """K2 centered RMSProp (BiCNN/pserver.lua:130-136). ``add=False`` = local mode:
    only the state and the update ``u`` are produced (BiCNN/optim-rmsprop.lua:49-54)."""
    R = _R()
    ts = [p if add else u, g, ga, gs, u] + ([out] if out is not None else [])
    var = (R.ADD if add else 0) | (R.OUT if out is not None else 0)
    _launch(R.RMSPROP, var, ts, [decay, lr, mom, eps], bf_ok=(1, 5))
    return p


def adam_(p, g, m, v, b1, b2, eps, lr_t, out=None):
    """K3 Adam with a host-computed step size ``lr_t`` (BiCNN/pserver.lua:147-154)."""
    R = _R()
    ts = [p, g, m, v] + ([out] if out is not None else [])
    _launch(R.ADAM, R.OUT if out is not None else 0, ts, [b1, b2, eps, lr_t], bf_ok=(1, 4))
    return p


def adam_lr_t(lr, b1, b2, t, step_div=1):
    """Step size of BiCNN's server Adam: bias correction on ``floor(t/stepDiv)+1``."""
    k = t // max(1, step_div) + 1
    return lr * math.sqrt(1 - b2 ** k) / (1 - b1 ** k)


def adamax_(p, g, m, u, b1, b2, eps, lr_t, out=None):
    """K4 Adamax (BiCNN/pserver.lua:163-170), ``lr_t = lr/(1-b1^t)``."""
    R = _R()
    ts = [p, g, m, u] + ([out] if out is not None else [])
    _launch(R.ADAMAX, R.OUT if out is not None else 0, ts, [b1, b2, eps, lr_t], bf_ok=(1, 4))
    return p


def adagrad_(p, g, var, eps, clr, out=None):
    """K5 Adagrad (BiCNN/pserver.lua:177-182), ``clr = lr/(1+t*lrd)``."""
    R = _R()
    ts = [p, g, var] + ([out] if out is not None else [])
    _launch(R.ADAGRAD, R.OUT if out is not None else 0, ts, [eps, clr], bf_ok=(1, 3))
    return p


def adadelta_(p, g, var, acc, rho, eps, lr, out=None):
    """K6 Adadelta (BiCNN/pserver.lua:189-193)."""
    R = _R()
    ts = [p, g, var, acc] + ([out] if out is not None else [])
    _launch(R.ADADELTA, R.OUT if out is not None else 0, ts, [rho, eps, lr], bf_ok=(1, 4))
    return p


# ---------------------------------------------------------------- worker rules (K7–K11, K14)

def nesterov_pre_(vt, w, mom):
    """K7: ``vt *= mom; w += vt`` (asyncsgd/optim-msgd.lua:27-28)."""
    _launch(_R().NESTEROV_PRE, 0, [vt, w], [mom])
    return w


def nesterov_post_(w, g, vt=None, sug=None, clr=0.0, gscale=1.0, l2wd=0.0):
    """K8 (+K14, +K10b): ``g' = gscale*g + l2wd*w; w -= clr*g' (+ sug); vt -= clr*g'``
    (asyncsgd/optim-msgd.lua:31-39, optim-eamsgd.lua:36-44,70)."""
    R = _R()
    var = (R.VT if vt is not None else 0) | (R.SUG if sug is not None else 0)
    _launch(R.NESTEROV_POST, var, [w, g, vt, sug], [gscale, l2wd, clr], bf_ok=(1, 3))
    return w


def downpour_(g, w, acc, lr, mode: int = 0, gscale=1.0, l2wd=0.0):
    """K9 (+K14): ``d = -lr*(gscale*g + l2wd*w)``; mode 0 ``acc = d``; 1 ``acc += d``;
    2 ``acc += d; w += d`` (asyncsgd/optim-downpour.lua:24-48)."""
    _launch(_R().DOWNPOUR, int(mode), [g, w, acc], [lr, gscale, l2wd], bf_ok=(0, 2) if mode == 0 else (0,))
    return acc


def elastic_(w, center, sug, mva):
    """K10a: ``sug = mva*(w - center)`` (asyncsgd/optim-eamsgd.lua:62-64)."""
    _launch(_R().ELASTIC, 0, [w, center, sug], [mva], bf_ok=(2,))
    return sug


def regclip_(g, p, gscale=1.0, l1=0.0, l2=0.0, clip=0.0):
    """K11: ``g = clamp(gscale*g + l1*sign(p) + l2*p, -clip, clip)`` (BiCNN/bicnn.lua:398-409)."""
    _launch(_R().REGCLIP, 0, [g, p], [gscale, l1, l2, clip], bf_ok=(0,))
    return g


def clamp_scan_(G: torch.Tensor, g: torch.Tensor, p: torch.Tensor, l1: float = 0.0, l2: float = 0.0,
                clip: float = 0.0) -> torch.Tensor:
    """K11 per example (BiCNN/bicnn.lua:398-409): for each row ``g[k]`` in order,
    ``G = clamp(G + g[k] + l1*sign(p) + l2*p, -clip, clip)`` (``clip <= 0``: no clamp) — the
    reference regularises and clamps the ACCUMULATED gradient after every violating example.
    G, p: [P] fp32; g: [n, ldg >= P] fp32 rows. One pass over g (HIP on the GPU)."""
    if G.dtype != torch.float32 or g.dtype != torch.float32 or p.dtype != torch.float32:
        raise TypeError("clamp_scan_ takes fp32 tensors")
    if g.dim() != 2 or g.stride(1) != 1 or not G.is_contiguous() or not p.is_contiguous():
        raise ValueError("clamp_scan_: G, p contiguous [P]; g [n, ldg] with unit column stride")
    P = G.numel()
    if p.numel() != P or g.shape[1] < P or g.device != G.device or p.device != G.device:
        raise ValueError("clamp_scan_: shape / device mismatch")
    if g.shape[0] == 0:
        return G
    dev = G.device.index if G.is_cuda else -1
    stream = torch.cuda.current_stream(G.device).cuda_stream if G.is_cuda else 0
    native().clamp_scan(dev, stream, G.data_ptr(), g.data_ptr(), p.data_ptr(), P, g.stride(0), g.shape[0],
                        float(l1), float(l2), float(clip))
    return G


def scale_(x, a):
    """K14: ``x *= a`` (asyncsgd/goot.lua:213)."""
    _launch(_R().SCALE, 0, [x], [a], bf_ok=(0,))
    return x


def copy_(dst, src, a: float = 1.0):
    """``dst = a*src`` with fp32<->bf16 cast."""
    _launch(_R().COPY, 0, [dst, src], [a], bf_ok=(0, 1))
    return dst


def fill_(x, v: float):
    _launch(_R().FILL, 0, [x], [v], bf_ok=(0,))
    return x


def axpby_(y, x, a: float, b: float):
    """``y = a*x + b*y``."""
    _launch(_R().AXPBY, 0, [y, x], [a, b], bf_ok=(0, 1))
    return y


# ---------------------------------------------------------------- reductions

_ws_cache = {}


def _ws(device):
    key = str(device)
    t = _ws_cache.get(key)
    if t is None:
        t = torch.empty(native().NORM_WS_FLOATS + 8, dtype=torch.float32, device=device)
        _ws_cache[key] = t
    return t


def norms(x: torch.Tensor) -> torch.Tensor:
    """``[Σ|x|, Σx², max|x|]`` as a 3-element fp32 tensor on x's device (deterministic)."""
    _check([x])
    out = torch.empty(3, dtype=torch.float32, device=x.device)
    m = native()
    if x.is_cuda:
        ws = _ws(x.device)
        m.norms(x.device.index, torch.cuda.current_stream(x.device).cuda_stream, x.data_ptr(),
                x.dtype == torch.bfloat16, x.numel(), out.data_ptr(), ws.data_ptr())
    else:
        m.norms(-1, 0, x.data_ptr(), x.dtype == torch.bfloat16, x.numel(), out.data_ptr(), 0)
    return out


def dot(x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    _check([x, y])
    if x.dtype != y.dtype:
        raise TypeError("dot operands must share a dtype")
    out = torch.empty(1, dtype=torch.float32, device=x.device)
    m = native()
    if x.is_cuda:
        ws = _ws(x.device)
        m.dot(x.device.index, torch.cuda.current_stream(x.device).cuda_stream, x.data_ptr(), y.data_ptr(),
              x.dtype == torch.bfloat16, x.numel(), out.data_ptr(), ws.data_ptr())
    else:
        m.dot(-1, 0, x.data_ptr(), y.data_ptr(), x.dtype == torch.bfloat16, x.numel(), out.data_ptr(), 0)
    return out


def gather_scale_(dst: torch.Tensor, srcs, offs, ns, a: float = 1.0, aux=None, b: float = 0.0):
    """K12+K9: ``dst[off_t:off_t+n_t] = a*src_t + b*aux[off_t:...]`` for raw fp32 tensor
    pointers ``srcs`` (one launch per 128 tensors)."""
    if dst.dtype != torch.float32 or (aux is not None and aux.dtype != torch.float32):
        raise TypeError("gather_scale_ works on float32")
    m = native()
    if dst.is_cuda:
        dev, stream = dst.device.index, torch.cuda.current_stream(dst.device).cuda_stream
    else:
        dev, stream = -1, 0
    m.gather_scale(dev, stream, list(srcs), list(offs), list(ns), dst.data_ptr(),
                   aux.data_ptr() if aux is not None else 0, float(a), float(b))
    return dst

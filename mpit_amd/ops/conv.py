"""Convolutions on the hand-written MFMA GEMMs (csrc/kernels/gemm.hip).

Two compute dtypes, chosen per call from the input and the autocast state (:func:`mfma_dtype`):

* bf16 (bf16 autocast / bf16 tensors): ``v_mfma_f32_32x32x16_bf16``, fp32 accumulate, bf16
  activations; the fp32 master weights are cast once per step (:class:`WeightCastPlan`);
* fp32 (fp32 tensors, no autocast — the reference's training precision,
  asyncsgd/glaunch.lua:11, BiCNN/plaunch.lua:200): fp32 operands split in registers into
  three bf16 planes and multiplied as six ``v_mfma_f32_32x32x16_bf16`` partial products
  (exact to fp32 accuracy, ``tests/test_fp32_path.py``; ``MPIT_F32_MFMA=native`` selects the
  fp32-input ``v_mfma_f32_32x32x2_f32`` instead), fp32 activations; the forward reads the
  fp32 master weight itself, the backward-data its fp32 (tap-flipped) transpose.

A stride-1 1x1 convolution over a channels_last activation is a GEMM over its [N*H*W, C]
row-major view. Measured on MI355X (benchmarks/conv_vs_gemm.py, ResNet-50 at batch 256)
MIOpen runs these at 100-450 TFLOP/s, and every backward-weight call also costs a zero
fill + an fp32->bf16 cast of MIOpen's own. Here:

* forward: ``Y = X . W^T`` (``gemm_nt``, bf16 out), optionally emitting the per-channel
  batch-norm statistics of ``Y`` from the accumulators;
* backward-data: ``dX = dY . W`` (``gemm_nt`` with a transposed bf16 copy of ``W`` made in
  the forward by ``cast_transpose``);
* backward-weight: ``dW = dY^T . X`` in fp32 straight from the accumulators (``gemm_tn``,
  split over M, deterministic reduce) — the fp32 master weight gets an fp32 gradient with
  no bf16 rounding and no cast kernel.

:class:`Conv1x1` is a drop-in ``nn.Conv2d`` that takes this path on the GPU for bf16
(autocast) channels_last inputs whose channel counts are multiples of 64, and falls
back to ``F.conv2d`` otherwise (CPU tests, odd shapes, strides).

:class:`ConvNHWC` does the same for RxS convolutions (ResNet's 3x3s, VGG, AlexNet) as
implicit GEMMs: forward and stride-1 backward-data gather the im2col rows straight from
the NHWC activation inside the kernel (padding taps read a zero line), backward-weight
reduces into the fp32 master gradient directly. Only the backward-data of a strided conv
stays on MIOpen.
"""
from __future__ import annotations

import os

import weakref

import torch
import torch.nn as nn
import torch.nn.functional as F

from .._ext import native
from ..utils.flat import grad_out


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


# MPIT_DEBUG_SIDE_DELAY=cycles (diagnostics only): a spin kernel ahead of every weight-gradient
# GEMM on the side stream, so a consumer that misses the join reads an unwritten gradient
_SIDE_DELAY = int(os.environ.get("MPIT_DEBUG_SIDE_DELAY", "0"))


class WgradStream:
    """Weight-gradient GEMMs on a second HIP stream.

    In a convolution's backward the input gradient is on the critical path (the next
    layer's BN backward needs it) while the weight gradient is only read by the optimizer
    step, so the backward-weight GEMM (compute-bound, ~18 % of a ResNet-50 step) is queued
    on a side stream and overlaps the memory-bound BN / ReLU kernels of the layers below.
    Both wait on the gradient of the convolution's output; the side stream joins back into
    the compute stream at :meth:`join`, which every consumer of the weight gradients calls
    first (the trainer after ``backward()``, the shard pusher before a gather). Only
    enabled by a trainer whose gradients are stolen (no autograd kernel reads them before
    that join); tensors the side stream touches are held until that join (``_used_on``) so
    the caching allocator does not recycle them early. MPIT_WGRAD_STREAM=0 disables it.
    """

    enabled = False
    _side = {}
    _pending = set()
    # tensors the side stream uses, per device, released at join (see _used_on)
    hold = os.environ.get("MPIT_SIDE_HOLD", "1") != "0"
    _held = {}
    _ev = {}
    # MPIT_WGRAD_AFTER=1: the side stream starts a convolution's weight gradient after its
    # input-gradient GEMM (so it overlaps the memory-bound BN backward that follows instead
    # of sharing the CUs with that compute-bound GEMM); default: before it
    after = os.environ.get("MPIT_WGRAD_AFTER", "0") == "1"
    # MPIT_WGRAD_SIDE: which weight gradients go to the side stream. all (default) | deep (RxS
    # convolutions only: their wgrad is compute-bound) | fp32 (fp32 calls only) | deep16 (RxS
    # convolutions, and every fp32 call). Concurrent memory-bound bf16 pairs run slower than
    # back to back (profiles/epi_roofline_r05.md); the others stay on the compute stream.
    policy = os.environ.get("MPIT_WGRAD_SIDE", "all")

    @classmethod
    def wants(cls, f32: bool, deep: bool) -> bool:
        p = cls.policy
        return (p == "all" or (p == "deep" and deep) or (p == "fp32" and f32)
                or (p == "deep16" and (deep or f32)))

    @classmethod
    def enable(cls, on: bool = True):
        if cls.enabled and not on and torch.cuda.is_available():
            cls.join()  # release what is held for the current stream(s) before switching off
        cls.enabled = bool(on) and os.environ.get("MPIT_WGRAD_STREAM", "1") != "0"

    @staticmethod
    def forced() -> bool:
        """MPIT_WGRAD_STREAM=force: enable even where ranks share a GPU (correctness runs)."""
        return os.environ.get("MPIT_WGRAD_STREAM", "1") == "force"

    @classmethod
    def begin(cls, dev: torch.device):
        """The side stream, ordered after everything queued so far on the current stream
        (issue before the input-gradient kernel so the side stream does not wait for it)."""
        if not cls.enabled:
            return None
        st = cls.side(dev)
        # one reused event per device (Stream.wait_stream creates a new HIP event per call: ~53
        # per ResNet-50 step); re-recording is safe, the wait below was queued with this record
        ev = cls._ev.get(dev.index)
        if ev is None:
            ev = cls._ev[dev.index] = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dev))
        st.wait_event(ev)
        if _SIDE_DELAY:  # race diagnostics: every weight gradient lands late
            with torch.cuda.stream(st):
                torch.cuda._sleep(_SIDE_DELAY)
        cls._pending.add(dev.index)
        return st

    @classmethod
    def side(cls, dev: torch.device):
        """The side stream of ``dev`` when enabled (created on first use), else None."""
        if not cls.enabled:
            return None
        st = cls._side.get(dev.index)
        if st is None:
            st = cls._side[dev.index] = cls._make_side(dev)
        return st

    @staticmethod
    def cu_mask(ncu: int, reserve: int) -> list:
        """CU mask (32-bit words, bit i = CU i) of the side stream: every CU except
        ``reserve`` kept for the critical path, picked on the diagonal of (i % 8, i // 8) so
        they spread evenly whether consecutive CU ids walk the XCDs or fill one XCD first."""
        period = max(1, ncu // max(1, reserve))
        words = [0] * ((ncu + 31) // 32)
        for i in range(ncu):
            if ((i % 8) + (i // 8)) % period != 0:
                words[i // 32] |= 1 << (i % 32)
        return words

    @classmethod
    def _make_side(cls, dev: torch.device):
        # MPIT_SIDE_CU_RESERVE=R: the side stream may not use R of the device's CUs, so the
        # critical path's small kernels always find a free CU (default 0 = all CUs)
        reserve = int(os.environ.get("MPIT_SIDE_CU_RESERVE", "0"))
        if reserve <= 0:
            return torch.cuda.Stream(dev)
        m = native()
        handle = m.stream_create_cu_masked(dev.index, cls.cu_mask(m.device_cu_count(dev.index), reserve))
        return torch.cuda.ExternalStream(handle, device=dev)

    @classmethod
    def join(cls):
        """Order the current stream after every weight gradient issued so far."""
        for idx in set(cls._pending) | {i for i, _ in cls._held}:
            cur = torch.cuda.current_stream(idx)
            cur.wait_stream(cls._side[idx])
            # this stream now runs behind every side-stream use of the tensors held for it: their
            # blocks may go back to the allocator, which hands them out on this stream only. A
            # join on another stream (a gradient hook runs on its AccumulateGrad node's stream)
            # releases nothing of the compute stream's.
            cls._held.pop((idx, cur.cuda_stream), None)
        cls._pending.clear()


def _cl(x: torch.Tensor) -> torch.Tensor:
    return x if x.is_contiguous(memory_format=torch.channels_last) else x.contiguous(memory_format=torch.channels_last)


def mfma_dtype(x: torch.Tensor):
    """Compute dtype of the MFMA path for input ``x``: bf16 under bf16 autocast or for bf16
    tensors, fp32 for fp32 tensors outside autocast, else None (no MFMA path)."""
    if torch.is_autocast_enabled("cuda"):
        return torch.bfloat16 if torch.get_autocast_dtype("cuda") == torch.bfloat16 else None
    return x.dtype if x.dtype in (torch.bfloat16, torch.float32) else None


# MPIT_F32_BSPLIT=0: fp32 steps split the weight operand in the GEMM's registers like the
# activation (round-2 kernels); default: the per-step weight plan writes it pre-split into
# three bf16 planes and the GEMM splits only the activation (csrc/kernels/gemm.hip FM 4)
_F32_BSPLIT = os.environ.get("MPIT_F32_BSPLIT", "1") != "0"
# column width from which a weight operand is pre-split (bf16x6: MPIT_F32_PLANES_N=64 also
# plane the N = 64 GEMMs on 128x64 tiles, 2 blocks per CU instead of 3; the fp16x3 planes are
# smaller and take every width)
_F32_PLANES_N = int(os.environ.get("MPIT_F32_PLANES_N",
                                   "64" if os.environ.get("MPIT_F32_SPLIT", "f16x3") == "f16x3" else "128"))


# MPIT_F32_SPLIT: how an fp32 step's GEMMs use the 16-bit matrix cores (csrc/kernels/gemm.hip):
#   f16x3 (default): operands scaled by a power of two from a device-side bound of |x| and split
#     into two fp16 terms, 3 fp16 MFMAs per product (FM 11) — the weight plan writes the two
#     fp16 planes of each weight, the activation / gradient operand is split in registers with
#     the bound its producer (the BN apply pass) wrote;
#   bf16x6: three bf16 terms, 6 bf16 MFMAs per product (FM 9 / FM 3, rounds 2-3).
_F32_SPLIT = os.environ.get("MPIT_F32_SPLIT", "f16x3")
if _F32_SPLIT not in ("f16x3", "bf16x6"):
    raise ValueError(f"MPIT_F32_SPLIT={_F32_SPLIT!r}: expected f16x3 or bf16x6")
# MPIT_WPLAN_TORCH_BOUND=1 (A/B): the weight plan's fp16-plane bound by torch launches
# (foreach_norm + amax into slot 0) instead of gemm.hip cast_amax_kernel
_WPLAN_TORCH_BOUND = os.environ.get("MPIT_WPLAN_TORCH_BOUND", "0") == "1"


def _bps(w: torch.Tensor, f32: bool) -> int:
    """Plane stride of a pre-split weight operand of an fp32 GEMM ([3, ...] bf16 planes h, m, l
    or [2, ...] fp16 planes h, l), else 0 (the operand is fp32 / the call is bf16)."""
    return w[0].numel() if (f32 and w is not None and w.dtype in (torch.bfloat16, torch.float16)) else 0


def _bamax(w: torch.Tensor) -> int:
    """Device pointer of the bound of |w| that scales fp16 weight planes (0: not fp16 planes)."""
    if w is None or w.dtype != torch.float16:
        return 0
    return w._mpit_wamax.data_ptr()


def _f16_exp(amax: torch.Tensor) -> torch.Tensor:
    """gemm.hip fp16_exp on the host side (tensor ops, no sync): e with amax * 2^e in [2^13, 2^14)."""
    e = (14 - torch.frexp(amax.float())[1]).clamp(-126, 116)
    ok = (amax > 0) & torch.isfinite(amax)
    return torch.where(ok, e, torch.zeros_like(e))


def _exp2i(e: torch.Tensor) -> torch.Tensor:
    """2^e (integer e in [-126, 127]) as an exact fp32 tensor (gemm.hip exp2i: the exponent field;
    torch.ldexp goes through pow and need not be exact)."""
    return ((e.to(torch.int32) + 127) << 23).view(torch.float32)


def _unsplit(w: torch.Tensor) -> torch.Tensor:
    """fp32 weight back from its planes (exact: w == h + m + l, or (h + l / 2^11) / 2^e)."""
    if w.dtype == torch.float16:
        return (w[0].float() + w[1].float() / 2048.0) * _exp2i(-_f16_exp(bound_value(w._mpit_wamax)))
    return (w[0].float() + w[1].float()) + w[2].float()


def f16_planes(w: torch.Tensor, amax: torch.Tensor) -> torch.Tensor:
    """[2, *w.shape] fp16 planes (h, l) of ``w * 2^e`` for the fp16x3 GEMMs, with e from the bound
    ``amax`` >= max |w| (gemm.hip split1h's arithmetic on PyTorch ops: the same bits as the
    weight plan's). ``(h + l / 2^11) / 2^e`` carries w to 2^-22 relative wherever |w| >= 2^-27
    ``amax``, to 2^-48 ``amax`` absolute below that."""
    e = _f16_exp(bound_value(amax) if amax.numel() > 1 else amax)
    wf = w.float()
    h = (wf * _exp2i(e)).half()
    lo = (wf * _exp2i(e + 11) - h.float() * 2048.0).half()
    p = torch.stack([h, lo])
    p._mpit_wamax = amax
    return p


# an output bound on the device: 16 fp32 slots 32 floats apart (csrc/kernels/kernels.h
# kBoundSlots); producers raise one slot per block, consumers take the max over the slots
BOUND_SLOTS, BOUND_STRIDE = 16, 32
BOUND_FLOATS = BOUND_SLOTS * BOUND_STRIDE


def bound_value(amax: torch.Tensor) -> torch.Tensor:
    """The bound a slotted buffer holds ([1] tensor)."""
    return amax[:BOUND_FLOATS].view(BOUND_SLOTS, BOUND_STRIDE)[:, 0].amax().reshape(1)


def bound_of_value(v: torch.Tensor) -> torch.Tensor:
    """A slotted bound buffer holding the [1] tensor ``v``."""
    b = torch.zeros(BOUND_FLOATS, dtype=torch.float32, device=v.device)
    b[:1].copy_(v.reshape(1))
    return b


def set_amax(t: torch.Tensor, amax: torch.Tensor) -> torch.Tensor:
    """Attach the device bound ``amax`` ([1] fp32, >= max |t|) to ``t`` (the fp16x3 GEMM operand
    scale); valid for this storage and version only."""
    t._mpit_amax = (amax, t.data_ptr(), t._version)
    return t


def amax_of(t: torch.Tensor):
    """The bound attached to ``t`` by its producer (:func:`set_amax`), or None."""
    a = getattr(t, "_mpit_amax", None)
    if a is None or a[1] != t.data_ptr() or a[2] != t._version:
        return None
    return a[0]


# fp32 steps (fp16x3): activations and gradients that only GEMMs read are written by their
# producers (BN apply passes, the stem's max pool) as the two fp16 planes h, l of x * 2^e
# (csrc/kernels/planes.h), with e from a bound known before the pass; the GEMMs then split
# nothing (gemm.hip FM 13: A planes in gemm_nt, both operands in gemm_tn). Same 4 bytes per
# element as fp32, so the tensor keeps its fp32 dtype and shape; the tag below says its memory
# holds planes. MPIT_F32_PLANES=0: fp32 activations (the GEMMs split them, FM 11 / 12).
_F32_PLANES = os.environ.get("MPIT_F32_PLANES", "1") != "0" and _F32_SPLIT == "f16x3"


def set_planes(t: torch.Tensor, bound: torch.Tensor) -> torch.Tensor:
    """Mark ``t``'s memory as fp16 planes scaled by the slotted ``bound`` (valid for this
    storage and version only)."""
    t._mpit_planes = (bound, t.data_ptr(), t._version)
    return t


def planes_of(t: torch.Tensor):
    """The bound of ``t``'s fp16 planes when its memory holds planes, else None."""
    a = getattr(t, "_mpit_planes", None)
    if a is None or a[1] != t.data_ptr() or a[2] != t._version:
        return None
    return a[0]


def unplanes(t: torch.Tensor) -> torch.Tensor:
    """A planes tensor as plain fp32 values (PyTorch ops; for the rare consumer without a
    planes path): (h + l / 2^11) / 2^e, exact."""
    b = planes_of(t)
    if b is None:
        return t
    if t.dim() == 4:
        n, c, h, w = t.shape
        flat = t.permute(0, 2, 3, 1).reshape(-1).view(torch.float16)
    else:
        flat = t.reshape(-1).view(torch.float16)
    ne = t.numel()
    v = (flat[:ne].float() + flat[ne:].float() / 2048.0) * _exp2i(-_f16_exp(bound_value(b)))
    COUNTERS["unplanes"] += 1
    if t.dim() == 4:
        return v.view(n, h, w, c).permute(0, 3, 1, 2)
    return v.view(t.shape)


_OEPOCH = [0]


def next_epoch() -> int:
    """A fresh launch epoch for the (epoch, max) slots of gemm.hip EpiArgs::omax (never 0)."""
    _OEPOCH[0] = _OEPOCH[0] % 0xFFFFFFF0 + 1
    return _OEPOCH[0]


def omax_buf(key: torch.Tensor, site: str, device) -> torch.Tensor:
    """The persistent epoch-slot buffer of a (key, site) GEMM output maximum (zeroed once; its
    slots only ever hold pairs of earlier launches, so a stale slot is never taken for ours)."""
    return tagged_part(key, "omax_" + site, BOUND_FLOATS, device)


def omax_of(t: torch.Tensor):
    """(slot buffer, epoch) of max |t| left by the GEMM that wrote ``t``, or None."""
    a = getattr(t, "_mpit_omax", None)
    if a is None or a[2] != t.data_ptr():
        return None
    return a[0], a[1]


def _amax_arg(t: torch.Tensor, keep: list) -> int:
    """Device pointer of a bound of |t| for an fp16x3 GEMM: the producer's, else one reduction
    (the tensor is kept alive in ``keep`` until the launch is queued)."""
    a = amax_of(t)
    if a is None:
        if planes_of(t) is not None:
            raise RuntimeError("an fp16-planes tensor reached an fp32 operand path")
        a = bound_of_value(torch.linalg.vector_norm(t, float("inf")))
        COUNTERS["amax_fallback"] += 1
    keep.append(a)
    return a.data_ptr()


def _split_kw(a: torch.Tensor, w: torch.Tensor, f32: bool, keep: list) -> dict:
    """GEMM keyword arguments of the weight operand ``w`` (planes) and the operand ``a`` (fp32,
    or fp16 planes: FM 13)."""
    bps = _bps(w, f32)
    kw = dict(bps=bps)
    bam = _bamax(w) if bps else 0
    pb = planes_of(a) if f32 else None
    if pb is not None:
        if not bam:
            raise RuntimeError("an fp16-planes operand needs the weight as fp16 planes (fp16x3)")
        keep.append(pb)
        COUNTERS["nt_planes"] += 1
        kw.update(amax_a=pb.data_ptr(), amax_b=bam, aps=a.numel())
    elif bam:
        kw.update(amax_a=_amax_arg(a, keep), amax_b=bam)
    return kw


def _as_operand(a: torch.Tensor, w: torch.Tensor, f32: bool) -> torch.Tensor:
    """``a`` as the A operand of an fp32 GEMM against ``w``: fp16 planes need the weight as fp16
    planes too (the step's weight plan, WeightCastPlan); a call without the plan decodes them
    (counted in COUNTERS["unplanes"])."""
    if f32 and w is not None and planes_of(a) is not None and not _bamax(w):
        v = _cl(unplanes(a))
        return set_amax(v, bound_of_value(torch.linalg.vector_norm(v, float("inf"))))
    return a


def _wgrad_kw(dy: torch.Tensor, xamax, f32: bool, side, keep: list, x: torch.Tensor = None, xplanes=False) -> dict:
    """fp16x3 operand bounds of a backward-weight GEMM (both producers' bounds, else the bf16x6
    path: a fallback reduction on the compute stream would not be ordered before the side
    stream's GEMM); the bound tensors are kept alive for the side stream. Operands given as
    fp16 planes (both: FM 13; :func:`_wgrad_operands` settles a mixed pair first) add their
    plane strides."""
    ya = planes_of(dy) if f32 else None
    if ya is not None or xplanes:
        if ya is None or not xplanes or xamax is None:
            raise RuntimeError("backward-weight GEMM: one operand is fp16 planes, the other fp32")
        keep += [ya, xamax]
        _used_on(side, ya, xamax)
        COUNTERS["wgrad_planes"] += 1
        return dict(amax_y=ya.data_ptr(), amax_x=xamax.data_ptr(), yps=dy.numel(), xps=x.numel())
    ya = amax_of(dy)
    if not f32 or _F32_SPLIT != "f16x3" or ya is None or xamax is None:
        return {}
    keep += [ya, xamax]
    _used_on(side, ya, xamax)
    COUNTERS["wgrad_f16x3"] += 1
    return dict(amax_y=ya.data_ptr(), amax_x=xamax.data_ptr())


def _wgrad_operands(dy: torch.Tensor, x: torch.Tensor, xamax, xplanes: bool):
    """(dy, x, xamax, xplanes, mixed) for a backward-weight GEMM: when exactly one operand is
    fp16 planes (a gradient that came through autograd's sum instead of a planes-writing BN),
    the planes one is decoded to fp32 (on the compute stream: the caller then keeps the GEMM
    there) — counted, never silent."""
    yp = planes_of(dy) is not None
    if yp == bool(xplanes):
        return dy, x, xamax, xplanes, False
    COUNTERS["wgrad_mixed"] += 1
    if yp:
        dyf = _cl(unplanes(dy))
        return set_amax(dyf, bound_of_value(torch.linalg.vector_norm(dyf, float("inf")))), x, xamax, xplanes, True
    xf = _cl(unplanes(x))
    return dy, xf, bound_of_value(torch.linalg.vector_norm(xf, float("inf"))), False, True


COUNTERS = {"amax_fallback": 0, "wgrad_f16x3": 0, "nt_planes": 0, "wgrad_planes": 0, "wgrad_mixed": 0,
            "unplanes": 0}


def _to(x: torch.Tensor, dt) -> torch.Tensor:
    x = _cl(x)
    return x if x.dtype == dt else x.to(dt)


def tile_stats_to_sums(part: torch.Tensor, M: int, N: int) -> torch.Tensor:
    """Per-128-row-tile (mean, M2) partials ([tiles][2][N]) -> [2, N] (sum, sum of squares)."""
    p = part.view(-1, 2, N).double()
    n = (M - 128 * torch.arange(p.shape[0], device=p.device, dtype=torch.float64)).clamp(max=128)[:, None]
    mean, m2 = p[:, 0], p[:, 1]
    return torch.stack([(n * mean).sum(0), (m2 + n * mean * mean).sum(0)]).float()


def gemm_nt(a: torch.Tensor, b: torch.Tensor, stats: bool = False, f16x3: bool = False):
    """``a[M,K] . b[N,K]^T`` in bf16 or fp32 (fp32 accumulate; result in the operands'
    dtype). With ``stats`` also returns the per-column ``[sum, sum of squares]`` of the
    result as a [2, N] fp32 tensor (from the epilogue's per-tile (mean, M2) partials).
    ``f16x3`` (fp32): the fp16x3 split products (b as fp16 planes, bounds from reductions)
    instead of the bf16x6 in-register split."""
    if a.dtype not in (torch.bfloat16, torch.float32) or b.dtype != a.dtype:
        raise TypeError("gemm_nt takes two bf16 or two fp32 operands")
    if a.dim() != 2 or b.dim() != 2 or a.shape[1] != b.shape[1] or a.stride(1) != 1 or b.stride(1) != 1:
        raise ValueError("gemm_nt: a[M,K], b[N,K] with unit column stride")
    M, K = a.shape
    N = b.shape[0]
    c = torch.empty((M, N), dtype=a.dtype, device=a.device)
    m = native()
    st = torch.empty(m.gemm_nt_stats_floats(M, N), dtype=torch.float32, device=a.device) if stats else None
    kw, keep = {}, []
    if f16x3:
        if a.dtype != torch.float32:
            raise TypeError("gemm_nt: f16x3 is an fp32 GEMM")
        b = f16_planes(b.contiguous(), bound_of_value(torch.linalg.vector_norm(b, float("inf"))))
        kw = _split_kw(a, b, True, keep)
    m.gemm_nt(a.device.index, _stream(a), M, N, K, a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(-2), c.data_ptr(),
              N, st.data_ptr() if st is not None else 0, f32=a.dtype == torch.float32, **kw)
    if stats:
        return c, tile_stats_to_sums(st, M, N)
    return c


def gemm_tn(y: torch.Tensor, x: torch.Tensor, out: torch.Tensor = None, beta: float = 0.0,
            f16x3: bool = False) -> torch.Tensor:
    """``out[N,K] = beta*out + y[M,N]^T . x[M,K]`` in fp32 from bf16 or fp32 operands
    (``f16x3``: fp32 operands on the fp16x3 split products, bounds from reductions)."""
    if y.dtype not in (torch.bfloat16, torch.float32) or x.dtype != y.dtype:
        raise TypeError("gemm_tn takes two bf16 or two fp32 operands")
    M, N = y.shape
    K = x.shape[1]
    if x.shape[0] != M or y.stride(1) != 1 or x.stride(1) != 1:
        raise ValueError("gemm_tn: y[M,N], x[M,K] with unit column stride")
    if out is None:
        out = torch.empty((N, K), dtype=torch.float32, device=y.device)
        beta = 0.0
    m = native()
    dev = y.device.index
    # split partials; with a single split and beta != 0 the one partial goes through the reduce
    nws = m.gemm_tn_ws_floats(dev, M, N, K) or (N * K if beta != 0.0 else 0)
    ws = torch.empty(nws, dtype=torch.float32, device=y.device) if nws else None
    kw, keep = {}, []
    if f16x3:
        if y.dtype != torch.float32:
            raise TypeError("gemm_tn: f16x3 is an fp32 GEMM")
        keep = [bound_of_value(torch.linalg.vector_norm(t, float("inf"))) for t in (y, x)]
        kw = dict(amax_y=keep[0].data_ptr(), amax_x=keep[1].data_ptr())
    m.gemm_tn(dev, _stream(y), M, N, K, y.data_ptr(), y.stride(0), x.data_ptr(), x.stride(0), out.data_ptr(),
              ws.data_ptr() if ws is not None else 0, float(beta), f32=y.dtype == torch.float32, **kw)
    return out


def cast_transpose(w: torch.Tensor, dtype=torch.bfloat16):
    """fp32 ``w[R, C]`` -> (copy [R, C], transpose [C, R]) in ``dtype``, one launch. For fp32
    the copy is ``w`` itself (2-D view) and only the transpose is written."""
    w2 = w.reshape(w.shape[0], -1)
    if w2.dtype != torch.float32 or not w2.is_contiguous():
        w2 = w2.float().contiguous()
    R, C = w2.shape
    f32 = dtype == torch.float32
    wb = w2 if f32 else torch.empty((R, C), dtype=torch.bfloat16, device=w.device)
    wt = torch.empty((C, R), dtype=dtype, device=w.device)
    native().cast_transpose(w.device.index, _stream(w), w2.data_ptr(), R, C, 0 if f32 else wb.data_ptr(),
                            wt.data_ptr(), f32=f32)
    return wb, wt


# MPIT_BN_FOLD=0: the BN backward's finalize as its own launch instead of in the GEMM
_BN_FOLD = os.environ.get("MPIT_BN_FOLD", "1") != "0"
# MPIT_FOLD_TAG=0: the folds' first protocol (every block drains its own output stores before
# its ticket) instead of tagged (value, epoch) partials (gemm.hip stats_fold)
_FOLD_TAG = os.environ.get("MPIT_FOLD_TAG", "1") != "0"
# id(key tensor) -> (weakref to it, buffer): the tagged partials of one fold site, kept across
# steps. Zeroed once, then only ever holding (value, epoch) pairs of earlier launches, so a
# reader can never take stale memory for a fresh pair (torch.empty memory could hold anything)
_TAG_PARTS = {}


def tagged_part(key: torch.Tensor, site: str, nfloats: int, device) -> torch.Tensor:
    """The persistent tagged-partials buffer of fold site (``key``, ``site``)."""
    k = (id(key), site)
    e = _TAG_PARTS.get(k)
    if e is not None and e[0]() is key and e[1].numel() >= nfloats and e[1].device == device:
        return e[1]
    buf = torch.zeros(nfloats, dtype=torch.float32, device=device)
    _TAG_PARTS[k] = (weakref.ref(key), buf)
    return buf


def _red_args(link, c: int, ntiles: int, device, fold: bool = False):
    """(kernel keyword arguments, partials, second partials or None, fold buffers or None)
    of a BN backward reduction folded into a backward-data GEMM (see ops/bn.py BNLink; a
    bn_pair link also reduces for its shortcut BN). ``fold`` (single-launch GEMMs, single
    BN): the GEMM's last blocks also run the BN backward's finalize and write its apply
    coefficients, dgamma and dbeta — the separate finalize launch (which in the backward
    waits for CU slots behind the side stream's GEMMs) disappears."""
    folding = fold and _BN_FOLD and link.rstd is not None and link.x2 is None
    if folding and _FOLD_TAG and link.w is not None:  # (value, epoch) pairs: twice the floats
        part = tagged_part(link.w, "bwd", ntiles * 4 * c, device)
    else:
        part = torch.empty(ntiles * 2 * c, dtype=torch.float32, device=device)
    kw = dict(red_part=part.data_ptr(), red_x=link.x.data_ptr(),
              red_mask=link.mask.data_ptr() if link.mask is not None else 0, red_mean=link.mean.data_ptr())
    if getattr(link, "gbuf", None) is not None:  # the BN backward writes fp16 planes: max |dy| first
        link.gep = next_epoch()
        kw.update(omax=link.gbuf.data_ptr(), oepoch=link.gep)
    part2 = fb = None
    if link.x2 is not None:
        part2 = torch.empty(ntiles * 2 * c, dtype=torch.float32, device=device)
        kw.update(red_part2=part2.data_ptr(), red_x2=link.x2.data_ptr(), red_mean2=link.mean2.data_ptr())
    elif fold and _BN_FOLD and link.rstd is not None:
        nl = native().gemm_nt_fold_lvl_floats(c)
        buf = torch.empty(5 * c + nl + BOUND_FLOATS, dtype=torch.float32, device=device)
        coef, dgamma, dbeta, lvl = buf[: 3 * c], buf[3 * c: 4 * c], buf[4 * c: 5 * c], buf[5 * c: 5 * c + nl]
        amax = buf[5 * c + nl:]  # the BN backward's output bound: zeroed by the fold, raised by its apply
        kw.update(fold_coef=coef.data_ptr(), fold_gamma=link.w.data_ptr() if link.w is not None else 0,
                  fold_rstd=link.rstd.data_ptr(), fold_dgamma=dgamma.data_ptr(), fold_dbeta=dbeta.data_ptr(),
                  fold_lvl=lvl.data_ptr(), fold_zero=amax.data_ptr(),
                  fold_tag=bool(_FOLD_TAG and link.w is not None))
        fb = (coef, dgamma, dbeta, amax)
    return kw, part, part2, fb


def _link_of(x: torch.Tensor, dt, pair_ok: bool = True):
    """The BNLink of the BN layer that produced ``x`` when the consumer computes in ``dt`` (the
    BN's dtype); a bn_pair link only for consumers whose backward-data GEMM can run the
    paired reduction (``pair_ok``: the 1x1 GEMMs)."""
    link = getattr(x, "_mpit_bnlink", None)
    if link is None or not link.ready(x) or x.dtype != dt or (link.x2 is not None and not pair_ok):
        return None
    return link


class _Hold(list):
    """Receives (partials, tiles, fold) from a statistics GEMM. ``bn``: the BatchNormAct2d the
    output feeds, whose forward finalize the GEMM then runs in its last blocks (ops/bn.py
    bn_fold_for, gemm.hip stats_fold) — the BN forward is left with its apply pass. ``omax``:
    (slot buffer, epoch) of the output's max |C| (a planes-writing BN's input bound)."""

    def __init__(self, bn=None):
        super().__init__()
        self.bn = bn
        self.omax = None


# conv -> weak reference of the BN its output feeds (kept outside the modules: no submodule,
# and a deep copy of a model does not inherit the original's BN — it finalizes separately)
_FOLD_TARGET = weakref.WeakKeyDictionary()


def _hold_for(conv) -> "_Hold":
    """The statistics hold of a convolution's forward (None: no statistics wanted)."""
    if not (conv.emit_stats and conv.training):
        return None
    ref = _FOLD_TARGET.get(conv)
    return _Hold(ref() if ref is not None else None)


def feeds_bn(conv, bn) -> None:
    """Mark ``conv`` as producing the input of ``bn``: it emits the BN's statistics and runs
    its forward finalize."""
    conv.emit_stats = True
    _FOLD_TARGET[conv] = weakref.ref(bn)


def _tile_stats(co: int, M: int, device, hold=None, dt=None):
    """(partials, tiles, fold): the statistics buffer of a GEMM emitting its output's BN
    statistics, and the fold of the fed BN's finalize when that BN can take it."""
    nt = native().gemm_nt_tiles(M)
    fold = None
    if hold is not None and getattr(hold, "bn", None) is not None:
        from .bn import bn_fold_for

        fold = bn_fold_for(hold.bn, co, dt, device)
    if fold is not None and fold.tagged:  # (value, epoch) pairs, read by the fold only
        return tagged_part(hold.bn.running_mean, "fwd", nt * 4 * co, device), nt, fold
    return torch.empty(nt * 2 * co, dtype=torch.float32, device=device), nt, fold


def _fold_arg(fold):
    return fold.args if fold is not None else None


def _omax_kw(hold, device, dt) -> dict:
    """fp32 statistics GEMM feeding a BN that writes fp16 planes: the launch's max |C| in epoch
    slots (the BN's output bound needs it before its pass), recorded on the hold."""
    bn = getattr(hold, "bn", None) if hold is not None else None
    if not (_F32_PLANES and dt == torch.float32 and bn is not None
            and (getattr(bn, "out_planes", False) or getattr(bn, "grad_planes", False))
            and getattr(bn, "running_mean", None) is not None):
        return {}
    buf, ep = omax_buf(bn.running_mean, "x", device), next_epoch()
    hold.omax = (buf, ep)
    return dict(omax=buf.data_ptr(), oepoch=ep)


def _attach_stats(y: torch.Tensor, hold: list) -> torch.Tensor:
    if hold:
        part, nt, fold = hold[0]
        y._mpit_tstats = (part, nt, y.data_ptr(), fold)
        om = getattr(hold, "omax", None)
        if om is not None:
            y._mpit_omax = (om[0], om[1], y.data_ptr())
    return y


class GradSlot:
    """Hands a gradient from one backward to a later one outside autograd's accumulation.

    A ResNet identity shortcut makes the block input feed both the first 1x1 convolution
    and the last BN's residual add, so autograd would sum the two input gradients with a
    separate add kernel (read 2, write 1 over the block input). Instead the BN backward
    parks its residual gradient here — as the pair (dy, ReLU bit mask), since the
    residual gradient of act(bn(y) + res) is just dy*mask — and the convolution's
    backward-data GEMM adds ``dy*mask`` in its epilogue (``C = dY.W + dy*mask``): the
    residual gradient is never written. The BN backward always runs first: the
    convolution's output feeds, through the block, the BN's input.

    A downsample block parks the shortcut convolution's input gradient the same way
    (:class:`ParkGrad`), as a plain tensor. If the consumer's backward ran before the
    producer's, the slot is closed and the producer returns its gradient to autograd."""

    __slots__ = ("grad", "mask", "closed")

    def __init__(self):
        self.grad = None
        self.mask = None
        self.closed = False

    def put(self, grad, mask=None) -> bool:
        """Park ``grad`` (times ``mask`` when given); False if the consumer already ran."""
        if self.closed:
            return False
        self.grad, self.mask = grad, mask
        return True

    def take(self):
        g, m = self.grad, self.mask
        self.grad = self.mask = None
        self.closed = True
        return g, m


class _ParkGradFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, slot):
        ctx.slot = slot
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        if ctx.slot.put(g):
            return None, None
        return g, None


def park_grad(x: torch.Tensor, slot: GradSlot) -> torch.Tensor:
    """Identity whose backward parks the incoming gradient in ``slot`` for a later
    GEMM epilogue to add (see :class:`GradSlot`). The view keeps x's output bound."""
    v = _ParkGradFn.apply(x, slot)
    a = amax_of(x)
    if a is not None:
        set_amax(v, a)
    p = planes_of(x)
    if p is not None:
        set_planes(v, p)
    return v


class ReluLink:
    """Hands the ReLU (+ bias) backward of a conv(+bias)+ReLU layer (VGG, AlexNet) to the
    kernel that produces its output gradient, so the separate pass over (dy, y) of
    ``relu_bias_bwd`` disappears:

    * a stride-1 convolution consuming the output computes its input gradient with the
      ``red_relu`` GEMM epilogue (csrc/kernels/gemm.hip ``EPI_RELUB``): C = dY.W * (y > 0) is
      the layer's dz, and the per-tile column sums its bias gradient (``col_sums``);
    * a max pool consuming it masks with its pooled output (csrc/kernels/pool.hip: at a
      window's argmax y is the pooled value) and sums the bias gradient as it writes.

    The producer attaches the link to its output (``y._mpit_relu``); a consumer that finds it
    on its input ``give``s (dz, db); the layer's backward ``take``s them when the gradient it
    receives IS that dz (same storage) and otherwise runs the ReLU backward itself — a
    gradient autograd summed from several consumers is a new tensor and takes that path, which
    stays exact (dz is already masked, and masking is idempotent). MPIT_RELU_FUSE=0 disables."""

    enabled = os.environ.get("MPIT_RELU_FUSE", "1") != "0"
    hits = 0  # backwards that took a handed dz (tests)
    __slots__ = ("dz", "db", "has_bias", "__weakref__")

    def __init__(self, has_bias: bool):
        self.dz = self.db = None
        self.has_bias = bool(has_bias)

    @staticmethod
    def of(x: torch.Tensor):
        link = getattr(x, "_mpit_relu", None) if ReluLink.enabled else None
        return link

    def give(self, dz: torch.Tensor, db):
        self.dz, self.db = dz, db

    def take(self, dy: torch.Tensor):
        """(True, db) when ``dy`` is the handed dz, else (False, None)."""
        dz, db = self.dz, self.db
        self.dz = self.db = None
        if dz is not None and dy.data_ptr() == dz.data_ptr() and dy.shape == dz.shape and dy.dtype == dz.dtype:
            ReluLink.hits += 1
            return True, db
        return False, None


def relu_dgrad_args(y: torch.Tensor, c: int, M: int, keep: list) -> dict:
    """conv_fwd kwargs of the ``red_relu`` epilogue: the masking layer's output ``y`` (NHWC,
    laid out like the input gradient) and per-tile column partials of dz."""
    nt = native().gemm_nt_tiles(M)
    part = torch.empty(nt * 2 * c, dtype=torch.float32, device=y.device)
    keep.append((part, nt))
    return dict(red_part=part.data_ptr(), red_x=y.data_ptr(), red_relu=True)


def relu_bias_from_parts(up: "ReluLink", dz: torch.Tensor, keep: list, c: int, stream: int):
    part, nt = keep[-1]
    db = None
    if up.has_bias:
        m = native()
        db = torch.empty(c, dtype=torch.float32, device=dz.device)
        mid = torch.empty(m.col_sums_ws_floats(c), dtype=torch.float32, device=dz.device)
        m.col_sums(dz.device.index, stream, part.data_ptr(), nt, 2 * c, c, db.data_ptr(), mid.data_ptr())
    up.give(dz, db)


class _Conv1x1Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, slot=None, hold=None, link=None, wcast=None, dt=torch.bfloat16):
        x = _to(x, dt)
        f32 = dt == torch.float32
        n, ci, h, w = x.shape
        co = weight.shape[0]
        M = n * h * w
        wb, wt = wcast if wcast is not None else cast_transpose(weight, dt)
        x = _as_operand(x, wb, f32)
        y = torch.empty((n, co, h, w), dtype=dt, device=x.device, memory_format=torch.channels_last)
        m = native()
        st = None
        fold = None
        if hold is not None:  # batch-norm statistics of y from the accumulators
            st, nt, fold = _tile_stats(co, M, x.device, hold, dt)
            hold.append((st, nt, fold))
        keep = []
        m.gemm_nt(x.device.index, _stream(x), M, co, ci, x.data_ptr(), ci, wb.data_ptr(), ci, y.data_ptr(), co,
                  st.data_ptr() if st is not None else 0, f32=f32, bn_fold=_fold_arg(fold),
                  **_split_kw(x, wb, f32, keep), **(_omax_kw(hold, x.device, dt) if st is not None else {}))
        ctx.save_for_backward(x, wt)
        xp = planes_of(x) if f32 else None
        ctx.xplanes = xp is not None
        ctx.xamax = xp if xp is not None else (amax_of(x) if f32 else None)
        ctx.wshape = weight.shape
        ctx.wparam = weight
        ctx.slot = slot
        ctx.link = link
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wt = ctx.saved_tensors
        dt = x.dtype
        f32 = dt == torch.float32
        dy = _to(dy, dt)
        n, ci, h, w = x.shape
        co = dy.shape[1]
        M = n * h * w
        m = native()
        dev, s = x.device.index, _stream(x)
        dx = dw = None
        use_side = ctx.needs_input_grad[1] and WgradStream.wants(f32, False)
        side = WgradStream.begin(x.device) if use_side and not WgradStream.after else None
        extra, emask = ctx.slot.take() if ctx.slot is not None else (None, None)
        if ctx.needs_input_grad[0]:
            dy = _as_operand(dy, wt, f32)
            dx = torch.empty_like(x, memory_format=torch.channels_last)
            kw, part, part2 = {}, None, None
            if ctx.link is not None:  # the producing BN's backward reduction, in the epilogue
                nt = m.gemm_nt_tiles(M)
                kw, part, part2, fb = _red_args(ctx.link, ci, nt, x.device, fold=True)
            keep = []
            kw.update(_split_kw(dy, wt, f32, keep))
            if extra is not None:  # gradient parked by the block (GradSlot): added in the epilogue
                extra = _to(extra, dt)
                if extra.shape != x.shape:
                    raise RuntimeError("GradSlot gradient does not match the convolution input")
                m.gemm_nt(dev, s, M, ci, co, dy.data_ptr(), co, wt.data_ptr(), co, dx.data_ptr(), ci, 0,
                          extra.data_ptr(), emask.data_ptr() if emask is not None else 0, f32=f32, **kw)
            else:
                m.gemm_nt(dev, s, M, ci, co, dy.data_ptr(), co, wt.data_ptr(), co, dx.data_ptr(), ci, 0, f32=f32,
                          **kw)
            if part is not None:
                ctx.link.publish(part, nt, dx, part2, fb)
        if ctx.needs_input_grad[1]:
            if WgradStream.after and use_side:
                side = WgradStream.begin(x.device)
            dw = grad_out(ctx.wparam, ctx.wshape, x.device)
            if getattr(dw, "_mpit_repeat", False):
                side = None  # a weight used twice: autograd sums the gradients on this stream
            wy, wx, xam, xpl, mixed = _wgrad_operands(dy, x, ctx.xamax, ctx.xplanes)
            if mixed:
                side = None  # the decoded operand was made on this stream
            nws = m.gemm_tn_ws_floats(dev, M, co, ci)
            ws = torch.empty(nws, dtype=torch.float32, device=x.device) if nws else None
            keep = []
            m.gemm_tn(dev, side.cuda_stream if side is not None else s, M, co, ci, wy.data_ptr(), co, wx.data_ptr(),
                      ci, dw.data_ptr(), ws.data_ptr() if ws is not None else 0, 0.0, f32=f32,
                      **_wgrad_kw(wy, xam, f32, side, keep, wx, xpl))
            _used_on(side, wy, wx, ws, out=dw)
        return dx, dw, None, None, None, None, None


def conv1x1_supported(x: torch.Tensor, weight: torch.Tensor) -> bool:
    if not x.is_cuda or x.dim() != 4 or mfma_dtype(x) is None:
        return False
    co, ci = weight.shape[0], weight.shape[1]
    return ci % 64 == 0 and co % 64 == 0 and x.shape[1] == ci


def conv1x1(x: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """Stride-1, unpadded, bias-free 1x1 convolution (MFMA GEMM path when supported)."""
    if conv1x1_supported(x, weight):
        return _Conv1x1Fn.apply(x, weight, None, None, None, None, mfma_dtype(x))
    return F.conv2d(x, weight)


class Conv1x1(nn.Conv2d):
    """``nn.Conv2d(i, o, 1, bias=False)`` whose stride-1 forward/backward run on the MFMA
    GEMMs on MI355X (see module docstring)."""

    def __init__(self, in_channels: int, out_channels: int, stride: int = 1):
        super().__init__(in_channels, out_channels, 1, stride=stride, bias=False)
        self.emit_stats = False  # output feeds a training BatchNormAct2d: emit its statistics

    def fused(self, x: torch.Tensor) -> bool:
        """True when ``forward(x)`` takes the MFMA path (and so honours a GradSlot)."""
        return self.stride == (1, 1) and conv1x1_supported(x, self.weight)

    def forward(self, x: torch.Tensor, slot: "GradSlot" = None) -> torch.Tensor:
        if self.fused(x):
            hold = _hold_for(self)
            dt = mfma_dtype(x)
            y = _Conv1x1Fn.apply(x, self.weight, slot, hold, _link_of(x, dt) if torch.is_grad_enabled() else None,
                                 WeightCastPlan.cached(self, dt), dt)
            return _attach_stats(y, hold)
        if slot is not None:
            raise RuntimeError("GradSlot needs the MFMA path (see Conv1x1.fused)")
        return super().forward(x)


# ------------------------------------------------------------------ RxS convolutions

def _weight_nhwc(weight: torch.Tensor) -> torch.Tensor:
    """fp32 [Co, C, R, S] weight whose memory is [Co][R][S][C] (channels_last)."""
    w = weight if weight.dtype == torch.float32 else weight.float()
    return w if w.is_contiguous(memory_format=torch.channels_last) else w.contiguous(memory_format=torch.channels_last)


def _as_rsc(w: torch.Tensor) -> torch.Tensor:
    """[Co, C, R, S] channels_last fp32 weight as its [Co, R, S, C] memory view (no copy)."""
    return w.permute(0, 2, 3, 1)


def conv_weights(weight: torch.Tensor, dgrad: bool, dtype=torch.bfloat16):
    """(forward weight [Co][R][S][C], tap-flipped transpose [C][R][S][Co] or None) in
    ``dtype``, one launch. fp32: the forward weight is the master itself."""
    co, c, r, s = weight.shape
    w = _weight_nhwc(weight)
    f32 = dtype == torch.float32
    wb = _as_rsc(w) if f32 else torch.empty((co, r, s, c), dtype=torch.bfloat16, device=w.device)
    wt = torch.empty((c, r, s, co), dtype=dtype, device=w.device) if dgrad else None
    if wt is not None or not f32:
        native().cast_transpose(w.device.index, _stream(w), w.data_ptr(), co, c, 0 if f32 else wb.data_ptr(),
                                wt.data_ptr() if wt is not None else 0, r * s, f32=f32)
    return wb, wt


_HOLD_MAX = 4096  # tensors held for one stream before _used_on joins by itself


def _used_on(side, *ts, out=None):
    """Keep tensors the side stream reads or writes from being recycled before it is done:
    held until the next :meth:`WgradStream.join` (default), or ``record_stream`` (MPIT_SIDE_HOLD=0).
    record_stream leaves one event per tensor that the caching allocator queries on its next
    allocation once the GPU has passed it — ~200 queries per ResNet-50 step, paid by the first
    allocation of the next step (~0.3 ms of host time while the GPU idles at the step start,
    profiles/boundary_r04/README.md). Holding needs no event: after the join every later use of
    the freed blocks on the compute stream is ordered behind the side stream.
    ``out``: the weight gradient the side stream writes. Never held: autograd steals a gradient
    only while nothing else references it, and would otherwise copy it on a stream that is not
    ordered after the side stream; it lives until the gather that follows the join anyway."""
    if side is None:
        return
    if WgradStream.hold:
        # keyed by the stream the tensors belong to (the compute stream issuing this backward):
        # only a join ON that stream may release them
        key = (side.device.index, torch.cuda.current_stream(side.device).cuda_stream)
        held = WgradStream._held.setdefault(key, [])
        held.extend(t for t in ts if t is not None)
        if len(held) > _HOLD_MAX:  # a caller that never joins: bound the memory, keep it correct
            WgradStream.join()
        return
    for t in ts + (out,):
        if t is not None:
            t.record_stream(side)


def _conv_backward(ctx, x, wb, wt, dz, stride: int, pad: int, link=None, up=None):
    """(dx, dw) of an NHWC implicit-GEMM conv from the gradient ``dz`` of its output; with a
    BNLink the backward-data GEMM also produces the producing BN's backward reduction, with a
    ReluLink (``up``) the producing conv's ReLU / bias backward."""
    nb, c, h, w = x.shape
    f32 = x.dtype == torch.float32
    co, r, s, _ = wb.shape[-4:]  # (pre-split planes carry a leading dim of 3)
    ho, wo = dz.shape[2], dz.shape[3]
    m = native()
    dev, st = x.device.index, _stream(x)
    dx = dw = None
    use_side = ctx.needs_input_grad[1] and WgradStream.wants(f32, r * s > 1)
    side = WgradStream.begin(x.device) if use_side and not WgradStream.after else None
    if ctx.needs_input_grad[0]:
        dz = _as_operand(dz, wt, f32)
        if stride == 1 and wt is not None:
            # backward-data = forward conv of dz with the flipped, transposed weight
            dx = torch.empty_like(x, memory_format=torch.channels_last)
            kw, part, nt = {}, None, 0
            rkeep = []
            if link is not None:
                nt = m.gemm_nt_tiles(nb * h * w)
                kw, part, _, fb = _red_args(link, c, nt, x.device, fold=True)
            elif up is not None and x.is_contiguous(memory_format=torch.channels_last):
                kw = relu_dgrad_args(x, c, nb * h * w, rkeep)
            keep = []
            m.conv_fwd(dev, st, nb, ho, wo, co, c, r, s, 1, r - 1 - pad, dz.data_ptr(), wt.data_ptr(),
                       dx.data_ptr(), f32=f32, **_split_kw(dz, wt, f32, keep), **kw)
            if part is not None:
                link.publish(part, nt, dx, None, fb)
            elif rkeep:
                relu_bias_from_parts(up, dx, rkeep, c, st)
        elif wt is not None:
            # strided: stride^2 parity classes, each a stride-1 implicit GEMM over dz whose
            # epilogue writes its pixels of dx (wt = the packed class weights)
            dx = torch.empty_like(x, memory_format=torch.channels_last)
            kw, part, nt = {}, None, 0
            if link is not None:
                nt = m.conv_dgrad_strided_tiles(nb, h, w, c, co, r, s, stride, pad)
                kw, part, _, _ = _red_args(link, c, nt, x.device)
            keep = []
            m.conv_dgrad_strided(dev, st, nb, h, w, c, co, r, s, stride, pad, dz.data_ptr(), wt.data_ptr(),
                                 dx.data_ptr(), f32=f32, **_split_kw(dz, wt, f32, keep), **kw)
            if part is not None:
                link.publish(part, nt, dx)
        else:  # MIOpen's NHWC backward-data
            dz, x = unplanes(dz), unplanes(x)
            wf = _unsplit(wb) if _bps(wb, f32) else wb
            wv = wf.permute(0, 3, 1, 2).to(x.dtype)  # [Co, C, R, S] view with channels_last strides
            dx = torch.ops.aten.convolution_backward(dz, x, wv, None, [stride, stride], [pad, pad], [1, 1], False,
                                                     [0, 0], 1, [True, False, False])[0]
    if ctx.needs_input_grad[1]:
        if WgradStream.after and use_side:
            side = WgradStream.begin(x.device)
        dw = grad_out(getattr(ctx, "wparam", None), (co, c, r, s), x.device, torch.channels_last)
        if getattr(dw, "_mpit_repeat", False):
            side = None  # a weight used twice: autograd sums the gradients on this stream
        wy, wx, xam, xpl, mixed = _wgrad_operands(dz, x, getattr(ctx, "xamax", None), getattr(ctx, "xplanes", False))
        if mixed:
            side = None  # the decoded operand was made on this stream
        nws = m.conv_wgrad_ws_floats(dev, nb, h, w, c, co, r, s, stride, pad)
        ws = torch.empty(nws, dtype=torch.float32, device=x.device) if nws else None
        keep = []
        m.conv_wgrad(dev, side.cuda_stream if side is not None else st, nb, h, w, c, co, r, s, stride, pad,
                     wy.data_ptr(), wx.data_ptr(), dw.data_ptr(), ws.data_ptr() if ws is not None else 0, 0.0, f32=f32,
                     **_wgrad_kw(wy, xam, f32, side, keep, wx, xpl))
        _used_on(side, wy, wx, ws, out=dw)
    return dx, dw


def _bf16_cl(t: torch.Tensor) -> torch.Tensor:
    return _to(t, torch.bfloat16)


def strided_dgrad_supported(c: int, co: int, stride: int) -> bool:
    return 2 <= stride <= 4 and c % 64 == 0 and co % 32 == 0


def strided_dgrad_weights(weight: torch.Tensor, stride: int, pad: int, dtype=torch.bfloat16):
    """(forward weight [Co][R][S][C], packed parity-class backward-data weights) in ``dtype``,
    one launch (fp32: the forward weight is the master itself)."""
    co, c, r, s = weight.shape
    w = _weight_nhwc(weight)
    m = native()
    f32 = dtype == torch.float32
    wb = _as_rsc(w) if f32 else torch.empty((co, r, s, c), dtype=torch.bfloat16, device=w.device)
    wc = torch.empty(m.conv_dgrad_strided_wfloats(c, co, r, s, stride, pad), dtype=dtype, device=w.device)
    m.conv_dgrad_strided_weights(w.device.index, _stream(w), w.data_ptr(), co, c, r, s, stride, pad,
                                 0 if f32 else wb.data_ptr(), wc.data_ptr(), f32=f32)
    return wb, wc


class _ConvFn(torch.autograd.Function):
    """conv (+ bias) (+ ReLU): the bias and the ReLU run in the GEMM epilogue; the backward
    of the ReLU / bias is one pass over (dy, y) (csrc/kernels/act.hip)."""

    @staticmethod
    def forward(ctx, x, weight, stride: int, pad: int, bias=None, relu: bool = False, hold=None, link=None,
                wcast=None, dt=torch.bfloat16, rlink=None):
        up = ReluLink.of(x)  # x is a ReLU'd conv output: its ReLU / bias backward rides on our dgrad
        x = _to(x, dt)
        f32 = dt == torch.float32
        nb, c, h, w = x.shape
        co, _, r, s = weight.shape
        ho, wo = (h + 2 * pad - r) // stride + 1, (w + 2 * pad - s) // stride + 1
        need_dx = ctx.needs_input_grad[0]
        if wcast is not None:  # cast for this step by the model's WeightCastPlan
            wb, wt = wcast
        elif need_dx and stride > 1 and strided_dgrad_supported(c, co, stride):
            wb, wt = strided_dgrad_weights(weight, stride, pad, dt)
        else:
            wb, wt = conv_weights(weight, need_dx and stride == 1, dt)
        x = _as_operand(x, wb, f32)
        y = torch.empty((nb, co, ho, wo), dtype=dt, device=x.device, memory_format=torch.channels_last)
        b = None
        if bias is not None:
            b = bias if (bias.dtype == torch.float32 and bias.is_contiguous()) else bias.float().contiguous()
        st = None
        fold = None
        if hold is not None and not relu and b is None:  # batch-norm statistics of y
            st, nt, fold = _tile_stats(co, nb * ho * wo, x.device, hold, dt)
            hold.append((st, nt, fold))
        keep = []
        native().conv_fwd(x.device.index, _stream(x), nb, h, w, c, co, r, s, stride, pad, x.data_ptr(), wb.data_ptr(),
                          y.data_ptr(), stats=st.data_ptr() if st is not None else 0,
                          bias=b.data_ptr() if b is not None else 0, relu=bool(relu), f32=f32,
                          bn_fold=_fold_arg(fold), **_split_kw(x, wb, f32, keep),
                          **(_omax_kw(hold, x.device, dt) if st is not None else {}))
        ctx.save_for_backward(x, wb, wt, y if relu else None)
        xp = planes_of(x) if f32 else None
        ctx.xplanes = xp is not None
        ctx.xamax = xp if xp is not None else (amax_of(x) if f32 else None)
        ctx.geo = (stride, pad, bias is not None, bool(relu))
        ctx.wparam = weight
        ctx.link = link
        ctx.up = up if (up is not None and need_dx and stride == 1 and link is None) else None
        ctx.rlink = rlink
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wb, wt, y = ctx.saved_tensors
        stride, pad, has_bias, relu = ctx.geo
        dt = x.dtype
        dy = _to(dy, dt)
        db = None
        fused, fdb = ctx.rlink.take(dy) if ctx.rlink is not None else (False, None)
        if fused:  # the consumer's kernel already applied the ReLU (and summed the bias gradient)
            dz = dy
            if has_bias and ctx.needs_input_grad[4]:
                db = fdb
        elif relu:
            nb_, co, ho, wo = dy.shape
            M = nb_ * ho * wo
            dz = torch.empty_like(dy, memory_format=torch.channels_last)
            m = native()
            want_db = has_bias and ctx.needs_input_grad[4]
            db = torch.empty(co, dtype=torch.float32, device=dy.device) if want_db else None
            ws = torch.empty(m.relu_bias_bwd_ws_floats(co), dtype=torch.float32, device=dy.device) if want_db else None
            m.relu_bias_bwd(dy.device.index, _stream(dy), M, co, dy.data_ptr(), y.data_ptr(), dz.data_ptr(),
                            db.data_ptr() if db is not None else 0, ws.data_ptr() if ws is not None else 0,
                            f32=dt == torch.float32)
        else:
            dz = dy
            if has_bias and ctx.needs_input_grad[4]:
                db = dy.float().sum(dim=(0, 2, 3))
        dx, dw = _conv_backward(ctx, x, wb, wt, dz, stride, pad, ctx.link, ctx.up)
        return dx, dw, None, None, db, None, None, None, None, None, None


def conv_supported(x: torch.Tensor, weight: torch.Tensor) -> bool:
    """The MFMA implicit-GEMM path takes bf16 (autocast) or fp32 NHWC-able inputs with
    channel counts that are multiples of 64 (wgrad tiles are 64 wide)."""
    if not x.is_cuda or x.dim() != 4 or weight.dim() != 4 or mfma_dtype(x) is None:
        return False
    co, ci = weight.shape[0], weight.shape[1]
    return ci % 64 == 0 and co % 64 == 0 and x.shape[1] == ci


class ConvAct2d(nn.Conv2d):
    """``act(conv2d(x) + bias)`` with act = ReLU or identity (square kernel / stride /
    padding, groups = dilation = 1): on the MFMA implicit-GEMM path the bias and the ReLU
    are applied in the GEMM epilogue; otherwise ``nn.Conv2d`` followed by ``F.relu``."""

    def __init__(self, in_channels: int, out_channels: int, kernel_size: int, stride: int = 1, padding: int = 0,
                 bias: bool = True, act: bool = True):
        super().__init__(in_channels, out_channels, kernel_size, stride=stride, padding=padding, bias=bias)
        self.act = act

    def fused(self, x: torch.Tensor) -> bool:
        return conv_supported(x, self.weight)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        rl = ReluLink(self.bias is not None) if (self.act and ReluLink.enabled and torch.is_grad_enabled()) else None
        if self.fused(x):
            dt = mfma_dtype(x)
            y = _ConvFn.apply(x, self.weight, self.stride[0], self.padding[0], self.bias, self.act, None, None,
                              WeightCastPlan.cached(self, dt), dt, rl)
        elif stem_supported(x, self) and self.kernel_size[0] <= 4:  # VGG's 3-channel first layer
            y = _StemConvFn.apply(x, self.weight, self.stride[0], self.padding[0], None, mfma_dtype(x), self.bias,
                                  self.act, rl)
        else:
            y = super().forward(x)
            return F.relu(y) if self.act else y
        if rl is not None:
            y._mpit_relu = rl
        return y


class ConvNHWC(nn.Conv2d):
    """``nn.Conv2d(i, o, k, stride, padding, bias=False)`` (square kernel / stride /
    padding, groups = dilation = 1) whose training forward/backward run as MFMA implicit
    GEMMs on MI355X (see module docstring); falls back to ``nn.Conv2d`` otherwise."""

    def __init__(self, in_channels: int, out_channels: int, kernel_size: int, stride: int = 1, padding: int = 0):
        super().__init__(in_channels, out_channels, kernel_size, stride=stride, padding=padding, bias=False)
        self.emit_stats = False  # output feeds a training BatchNormAct2d: emit its statistics

    def fused(self, x: torch.Tensor) -> bool:
        return conv_supported(x, self.weight)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.fused(x):
            hold = _hold_for(self)
            dt = mfma_dtype(x)
            y = _ConvFn.apply(x, self.weight, self.stride[0], self.padding[0], None, False, hold,
                              _link_of(x, dt, pair_ok=False) if torch.is_grad_enabled() else None,
                              WeightCastPlan.cached(self, dt), dt)
            return _attach_stats(y, hold)
        return super().forward(x)


class WeightCastPlan:
    """The per-step weight operands of every MFMA convolution of a model, made in ONE launch
    per step (csrc/kernels/gemm.hip ``cast_batch_kernel``) instead of one kernel per conv.

    bf16 plan (``dtype=torch.bfloat16``): ``run()`` casts the current fp32 master weights
    into persistent bf16 buffers (plain + tap-flipped transposes, or the strided parity-class
    weights). fp32 plan: the forward reads the master weight itself and ``run()`` writes only
    the fp32 transposes the backward-data GEMMs read (a snapshot taken before the forward, so
    a shard pulled into the model during the backward does not change this step's gradient).
    Until ``invalidate()`` the convolutions use them. The trainer brackets its
    forward/backward with the two calls, so a weight update in between (PS pull, optimizer)
    is never missed; forwards outside that window cast per call as before."""

    def __init__(self, model: nn.Module, dtype=torch.bfloat16):
        self.model = model
        self.dtype = dtype
        self.valid = False
        self._build()

    def _build(self):
        specs, self.mods = [], []
        m = native()
        f32 = self.dtype == torch.float32
        planes = f32 and _F32_BSPLIT
        # fp16x3: two fp16 planes per weight operand, scaled by the bound of |w| over the plan
        # (self.amax, refreshed by run() before the cast launch)
        f16p = planes and _F32_SPLIT == "f16x3"
        npl, pdt = (2, torch.float16) if f16p else (3, torch.bfloat16)
        self.wlist = []
        self.amax = None
        for mod in self.model.modules():
            kind = None
            if getattr(mod, "_mpit_linear", False):  # ops/linear.py LinearAct: its transpose wt[K, Np] only
                w = mod.weight
                if not w.is_cuda or w.dtype != torch.float32 or not w.is_contiguous():
                    continue
                co, c = w.shape
                # out_features not a multiple of 64 (a 1000-class output layer): rows of Np, the
                # pad columns zeroed here once and never written by the cast (bf16 or fp32)
                np_ = (co + 63) // 64 * 64
                wt = (torch.zeros if np_ != co else torch.empty)((c, np_), dtype=self.dtype, device=w.device)
                specs.append([4096 | (256 if f32 else 0), w.data_ptr(), 0, wt.data_ptr(), co, c, 1, 1, 1,
                              np_ if np_ != co else 0, 0])
                self.mods.append((mod, w.data_ptr(), (None, wt)))
                continue
            if isinstance(mod, Conv1x1) and mod.stride == (1, 1):
                kind = 0
            elif isinstance(mod, (ConvNHWC, ConvAct2d)):
                st = mod.stride[0]
                co, c = mod.weight.shape[0], mod.weight.shape[1]
                if c % 64 or co % 64:  # never on the MFMA path (conv_supported): no plan entry
                    continue
                kind = 0 if st == 1 else (1 if strided_dgrad_supported(c, co, st) else 2)
            if kind is None:
                continue
            w = mod.weight
            if not w.is_cuda or w.dtype != torch.float32 or not w.is_contiguous(memory_format=torch.channels_last):
                continue
            co, c, r, sw = w.shape
            # pre-split planes h, m, l (bf16, a leading dim of 3) for an fp32 step, per operand:
            # only where the GEMM reading it runs 128-wide column tiles (N = co forward, c
            # backward-data) — the 128x64 tiles of N = 64 keep 3 blocks per CU only with the
            # smaller fp32 image, and split that operand in registers
            pl_b = planes and co % _F32_PLANES_N == 0
            pl_t = planes and c % _F32_PLANES_N == 0 and kind != 2
            # a detached view: the plan outlives every step, and a view WITH autograd history
            # would keep the weight's AccumulateGrad node (made at build time, on the stream
            # current then) alive into every step — autograd then warns that the node's stream
            # differs from the step's and inserts a cross-stream wait per weight
            if f16p and (pl_b or pl_t) and self.amax is None:
                self.amax = torch.zeros(BOUND_FLOATS, dtype=torch.float32, device=w.device)  # slotted bound
            if f32 and not pl_b:
                wb = _as_rsc(w.detach())
            else:
                wb = torch.empty(((npl,) if pl_b else ()) + (co, r, sw, c), dtype=pdt if pl_b else torch.bfloat16,
                                 device=w.device)
            lt = (npl,) if pl_t else ()
            odt = pdt if pl_t else self.dtype
            if kind == 0:
                wt = torch.empty(lt + (c, r, sw, co), dtype=odt, device=w.device)
            elif kind == 1:
                wt = torch.empty(lt + (m.conv_dgrad_strided_wfloats(c, co, r, sw, mod.stride[0], mod.padding[0]),),
                                 dtype=odt, device=w.device)
            else:
                wt = None
            if isinstance(mod, Conv1x1):  # the 1x1 path takes 2-D [co, ci] / [ci, co] views
                wb, wt = wb.reshape(((npl,) if pl_b else ()) + (co, c)), wt.view(lt + (c, co))
            if f32 and not (pl_b or pl_t) and wt is None:
                self.mods.append((mod, w.data_ptr(), (wb, wt)))  # nothing to write
                continue
            if f16p and (pl_b or pl_t):
                self.wlist.append(w.detach())
                for t in (wb, wt):
                    if t is not None and t.dtype == torch.float16:
                        t._mpit_wamax = self.amax
            flags = (kind | (256 if f32 else 0) | (512 if pl_b else 0) | (1024 if pl_t else 0)
                     | (2048 if f16p and (pl_b or pl_t) else 0))
            specs.append([flags, w.data_ptr(), wb.data_ptr() if (pl_b or not f32) else 0,
                          wt.data_ptr() if wt is not None else 0, co, c, r, sw, mod.stride[0], mod.padding[0],
                          self.amax.data_ptr() if (f16p and (pl_b or pl_t)) else 0])
            self.mods.append((mod, w.data_ptr(), (wb, wt)))
        self.njobs = len(specs)
        self.table = None
        if specs:
            host = torch.empty(self.njobs * m.cast_job_bytes(), dtype=torch.uint8)
            self.nblocks = m.cast_jobs_build(host.data_ptr(), specs)
            self.table = host.to(self.mods[0][0].weight.device)
        # bind once per build (nn.Module.__setattr__ per conv per step costs ~0.1 ms of host
        # time at the start of every forward, while the GPU idles); run() only flips valid
        for mod, _, pair in self.mods:
            mod._mpit_wcast = (self, pair)

    def run(self):
        # (parameters dict lookups: Module.__getattr__ per conv per step is measurable host time)
        if any(mod._parameters["weight"].data_ptr() != ptr for mod, ptr, _ in self.mods):
            self._build()  # parameters moved (FlatParams.rebind)
        if self.table is not None:
            dev = self.table.device
            native_bound = bool(self.wlist) and not _WPLAN_TORCH_BOUND
            if self.wlist and _WPLAN_TORCH_BOUND:  # A/B: the bound by torch launches, slot 0 only
                with torch.no_grad():
                    self.amax.zero_()
                    torch.amax(torch.stack(torch._foreach_norm(self.wlist, float("inf"))), 0, keepdim=True,
                               out=self.amax[:1])
            # fp16 planes: the same launch sequence first writes their scale's bound, max |w| over
            # the plan's fp16-plane weights, into self.amax (gemm.hip cast_amax_kernel)
            native().cast_jobs_run(dev.index, torch.cuda.current_stream(dev).cuda_stream, self.table.data_ptr(),
                                   self.njobs, self.nblocks, self.amax.data_ptr() if native_bound else 0)
        self.valid = True

    def invalidate(self):
        self.valid = False

    @staticmethod
    def cached(mod, dtype=torch.bfloat16):
        """The (wb, wt) operands for ``mod`` by a valid plan of ``dtype``, else None."""
        c = getattr(mod, "_mpit_wcast", None)
        if c is None or not c[0].valid or c[0].dtype != dtype:
            return None
        return c[1]


# ------------------------------------------------------------------ the 7x7 stem

class _StemPackBuf:
    """The zero-padded NHWC4 stem input, kept across steps: the zero border and the fourth
    channel are written once, each step copies only the image into the interior (one copy
    kernel instead of a full-size fill + copy, and no per-step allocation of the buffer).
    A buffer still saved for a pending backward (``busy``) is never reused: the next
    forward then takes a fresh one. Every use (the forward's copy + GEMM, the backward's
    weight-gradient GEMM) records the entry's event on its stream; a later use on another
    stream waits on it first, so a refill never overtakes a pending reader whatever the
    streams. MPIT_STEM_PACK_REUSE=0: pad anew every call."""

    enabled = os.environ.get("MPIT_STEM_PACK_REUSE", "1") != "0"
    bufs = {}

    class Entry:
        __slots__ = ("buf", "busy", "event", "stream")

        def __init__(self, buf):
            self.buf, self.busy, self.event, self.stream = buf, False, None, None

        def order_after_last_use(self, dev):
            cur = torch.cuda.current_stream(dev)
            if self.event is not None and self.stream != cur.cuda_stream:
                cur.wait_event(self.event)

        def used(self, dev):
            """Record the last use (queued on the current stream)."""
            cur = torch.cuda.current_stream(dev)
            if self.event is None:
                self.event = torch.cuda.Event()
            self.event.record(cur)
            self.stream = cur.cuda_stream

    @classmethod
    def get(cls, x: torch.Tensor, pad: int, hp: int, wp: int, dt):
        v = _to(x, dt).permute(0, 2, 3, 1)  # NHWC view of the channels_last tensor
        n, h, w, c = v.shape
        if not cls.enabled:
            return F.pad(v, (0, 4 - c, pad, wp - w - pad, pad, hp - h - pad)), None
        key = (x.device, dt, n, h, w, c, pad, hp, wp)
        ent = cls.bufs.get(key)
        if ent is None or ent.busy:
            ent = cls.Entry(torch.zeros((n, hp, wp, 4), dtype=dt, device=x.device))
            cls.bufs[key] = ent
        ent.order_after_last_use(x.device)
        ent.busy = True  # until the backward that reads it has been issued
        ent.buf[:, pad:pad + h, pad:pad + w, :c].copy_(v)
        return ent.buf, ent


def _stem_pack_input(x: torch.Tensor, pad: int, hp: int, wp: int, dt=torch.bfloat16) -> torch.Tensor:
    """[N, 3, H, W] -> zero-padded NHWC4 [N, hp, wp, 4] in ``dt`` (one pad kernel)."""
    v = _to(x, dt).permute(0, 2, 3, 1)  # NHWC view of the channels_last tensor
    n, h, w, c = v.shape
    return F.pad(v, (0, 4 - c, pad, wp - w - pad, pad, hp - h - pad))


_STEM_WBUF = {}


def _stem_pack_weight(weight: torch.Tensor, dt=torch.bfloat16, rows: int = 8) -> torch.Tensor:
    """[Co, C<=4, R<=rows, S<=8] -> [Co, rows, 8, 4] in ``dt``, zero-extended. With
    ``_StemPackBuf.enabled`` the zero-extended buffer is kept per (device, stream, shape):
    it is only read by this step's forward GEMM, queued on the same stream before the next
    step's refill, so only the weight itself is copied in each step."""
    co, c, r, s = weight.shape
    wp = None
    if _StemPackBuf.enabled and weight.is_cuda:
        key = (weight.device, dt, co, c, r, s, rows, _stream(weight))
        wp = _STEM_WBUF.get(key)
        if wp is None:
            wp = _STEM_WBUF[key] = torch.zeros((co, rows, 8, 4), dtype=dt, device=weight.device)
    if wp is None:
        wp = torch.zeros((co, rows, 8, 4), dtype=dt, device=weight.device)
    with torch.no_grad():  # a cached buffer must not carry an autograd edge to the weight
        wp[:, :r, :s, :c] = weight.permute(0, 2, 3, 1)
    return wp


_STEM_PBUF = {}
# MPIT_STEM_NATIVE_PLANES=0: the stem's fp16x3 weight planes from PyTorch ops (A/B knob)
_STEM_NATIVE_PLANES = os.environ.get("MPIT_STEM_NATIVE_PLANES", "1") != "0"


def stem_weight_planes(weight: torch.Tensor):
    """The stem weight's zero-extended [Co, 8, 8, 4] image as fp16x3 planes ([2, Co, 8, 8, 4] fp16:
    ``f16_planes`` of the image under the bound max |w|) and that slotted bound, from ONE native
    launch (csrc/kernels/stem_pack.hip). Kept per (device, stream, shape) like the bf16 image
    (``_stem_pack_weight``): only this step's forward GEMM, queued on the same stream before the
    next rewrite, reads them."""
    co, c, r, s = weight.shape
    w = weight.detach()
    if not w.is_contiguous(memory_format=torch.channels_last):
        w = w.contiguous(memory_format=torch.channels_last)
    key = (weight.device, co, c, r, s, _stream(weight))
    buf = _STEM_PBUF.get(key) if _StemPackBuf.enabled else None
    if buf is None:
        buf = (torch.empty((2, co, 8, 8, 4), dtype=torch.float16, device=weight.device),
               torch.empty(BOUND_FLOATS, dtype=torch.float32, device=weight.device))
        if _StemPackBuf.enabled:
            _STEM_PBUF[key] = buf
    planes, bound = buf
    native().stem_weight_planes(weight.device.index, _stream(weight), w.data_ptr(), co, c, r, s, planes.data_ptr(),
                                bound.data_ptr())
    return planes, bound


class _StemConvFn(torch.autograd.Function):
    """<= 8x8, <= 4-channel convolution (the ResNet 7x7/2 stem, VGG's 3x3 first layer) as a
    row-tap implicit GEMM on the MFMA kernels (csrc/kernels/gemm.hip ``conv_stem_*``): each
    kernel row is one 32-element tap = 8 pixels x 4 channels of a zero-padded NHWC4 copy of
    the image, so the 3-channel input needs no im2col and no per-channel gather; a kernel of
    R rows is an R-tap GEMM (K = 32 R). Forward emits the BN statistics of its output, or
    runs a bias (+ ReLU) epilogue (VGG); backward computes the weight (and bias) gradient only
    (the image needs none)."""

    @staticmethod
    def forward(ctx, x, weight, stride: int, pad: int, hold=None, dt=torch.bfloat16, bias=None, relu=False,
                rlink=None):
        nb, _, h, w = x.shape
        co, _, r, s = weight.shape
        f32 = dt == torch.float32
        m = native()
        rows = 8 if r > 4 else r  # (the ResNet stem keeps its 8-row layout and weight planes)
        rw = m.stem_wgrad_rows(rows)
        ho, wo = (h + 2 * pad - r) // stride + 1, (w + 2 * pad - s) // stride + 1
        hp, wp = max(h + 2 * pad, (ho - 1) * stride + rw), max(w + 2 * pad, (wo - 1) * stride + 8)
        xp, ent = _StemPackBuf.get(x, pad, hp, wp, dt)
        f16s = f32 and _F32_SPLIT == "f16x3"
        native_planes = _STEM_NATIVE_PLANES and rows == 8
        wb = None if f16s and native_planes else _stem_pack_weight(weight, dt, rows)
        y = torch.empty((nb, co, ho, wo), dtype=dt, device=x.device, memory_format=torch.channels_last)
        st = None
        fold = None
        if hold is not None:
            st, nt, fold = _tile_stats(co, nb * ho * wo, x.device, hold, dt)
            hold.append((st, nt, fold))
        kw, ctx.xbound = {}, None
        if f16s:
            # fp16x3: the image's bound (the padded copy only adds zeros) and the packed weight as
            # two fp16 planes; the row-tap GEMM then runs 32-deep tiles, one kernel row each
            ctx.xbound = amax_of(x)  # kept on the input while it is unchanged (a reused batch)
            if ctx.xbound is None:
                ctx.xbound = bound_of_value(torch.linalg.vector_norm(x, float("inf")))
                set_amax(x, ctx.xbound)
            if native_planes:
                wb, wam = stem_weight_planes(weight)
            else:  # the PyTorch-op planes (A/B; the 3x3 layout)
                wam = bound_of_value(torch.linalg.vector_norm(weight.detach(), float("inf")))
                wb = f16_planes(wb.reshape(co, -1), wam)
            kw = dict(bps=wb[0].numel(), amax_a=ctx.xbound.data_ptr(), amax_b=wam.data_ptr())
        b = None
        if bias is not None:
            b = bias if (bias.dtype == torch.float32 and bias.is_contiguous()) else bias.float().contiguous()
            kw["bias"] = b.data_ptr()
        if relu:
            kw["relu"] = True
        m.conv_stem_fwd(x.device.index, _stream(x), nb, hp, wp, co, ho, wo, stride, xp.data_ptr(), wb.data_ptr(),
                        y.data_ptr(), st.data_ptr() if st is not None else 0, f32=f32, bn_fold=_fold_arg(fold),
                        rows=rows, **kw)
        ctx.save_for_backward(xp, y if relu else None)
        ctx.geo = (nb, hp, wp, co, ho, wo, stride, tuple(weight.shape), rows, bias is not None, bool(relu))
        ctx.rlink = rlink
        ctx.pack = ent
        if ent is not None:
            ent.used(x.device)
            if not ctx.needs_input_grad[1]:
                ent.busy = False  # no backward will read it
        return y

    @staticmethod
    def backward(ctx, dy):
        xp, y = ctx.saved_tensors
        nb, hp, wp, co, ho, wo, stride, wshape, rows, has_bias, relu = ctx.geo
        dw = db = None
        dt = xp.dtype
        dy = _to(dy, dt)
        m = native()
        dev = xp.device.index
        fused, fdb = ctx.rlink.take(dy) if ctx.rlink is not None else (False, None)
        if fused:  # the consumer's kernel applied the ReLU and summed the bias gradient
            db = fdb if (has_bias and ctx.needs_input_grad[6]) else None
        elif relu:  # dz = dy * (y > 0) and the bias gradient in one pass (csrc/kernels/act.hip)
            dz = torch.empty_like(dy, memory_format=torch.channels_last)
            want_db = has_bias and ctx.needs_input_grad[6]
            db = torch.empty(co, dtype=torch.float32, device=dy.device) if want_db else None
            ws = torch.empty(m.relu_bias_bwd_ws_floats(co), dtype=torch.float32, device=dy.device) if want_db else None
            m.relu_bias_bwd(dev, _stream(dy), nb * ho * wo, co, dy.data_ptr(), y.data_ptr(), dz.data_ptr(),
                            db.data_ptr() if db is not None else 0, ws.data_ptr() if ws is not None else 0,
                            f32=dt == torch.float32)
            dy = dz
        elif has_bias and ctx.needs_input_grad[6]:
            db = dy.float().sum(dim=(0, 2, 3))
        if ctx.needs_input_grad[1]:
            rw = m.stem_wgrad_rows(rows)
            dwp = torch.empty((co, rw, 8, 4), dtype=torch.float32, device=xp.device)
            nws = m.conv_stem_wgrad_ws_floats(dev, nb, ho, wo, co, rows)
            ws = torch.empty(nws, dtype=torch.float32, device=xp.device) if nws else None
            ya = amax_of(dy)
            kw = dict(amax_y=ya.data_ptr(), amax_x=ctx.xbound.data_ptr()) if (
                ya is not None and ctx.xbound is not None) else {}
            m.conv_stem_wgrad(dev, _stream(xp), nb, hp, wp, co, ho, wo, stride, dy.data_ptr(), xp.data_ptr(),
                              dwp.data_ptr(), ws.data_ptr() if ws is not None else 0, f32=dt == torch.float32,
                              rows=rows, **kw)
            _, c, r, s = wshape
            dw = dwp[:, :r, :s, :c].permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
        if ctx.pack is not None:
            # the wgrad reading the buffer is queued: the next refill is ordered after it
            ctx.pack.used(xp.device)
            ctx.pack.busy = False
        return None, dw, None, None, None, None, db, None, None


def stem_supported(x: torch.Tensor, conv: nn.Conv2d) -> bool:
    """The row-tap MFMA path: a CUDA bf16 / fp32 image that needs no gradient, <= 4 channels,
    a square-strided / square-padded <= 8x8 kernel, Co % 64 == 0 (MPIT_MFMA_STEM=0: off)."""
    co, c, r, s = conv.weight.shape
    return (x.is_cuda and mfma_dtype(x) is not None and x.dim() == 4 and not x.requires_grad and c <= 4
            and r <= 8 and s <= 8 and co % 64 == 0 and conv.dilation == (1, 1) and conv.groups == 1
            and conv.stride[0] == conv.stride[1] and conv.padding[0] == conv.padding[1]
            and os.environ.get("MPIT_MFMA_STEM", "1") != "0")


class StemConv(nn.Conv2d):
    """``nn.Conv2d(c <= 4, co, k <= 8, stride, pad, bias=False)`` — the ResNet stem — on the
    MFMA row-tap kernels on MI355X when the input needs no gradient (see _StemConvFn);
    nn.Conv2d (MIOpen / CPU) otherwise. ``emit_stats`` as Conv1x1."""

    def __init__(self, in_channels: int, out_channels: int, kernel_size: int, stride: int, padding: int):
        super().__init__(in_channels, out_channels, kernel_size, stride=stride, padding=padding, bias=False)
        self.emit_stats = False

    def fused(self, x: torch.Tensor) -> bool:
        return stem_supported(x, self)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.fused(x):
            hold = _hold_for(self)
            y = _StemConvFn.apply(x, self.weight, self.stride[0], self.padding[0], hold, mfma_dtype(x))
            return _attach_stats(y, hold)
        return super().forward(x)

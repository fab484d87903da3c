"""Synchronous data parallelism: bucketed gradient all-reduce overlapped with backward.

The reference only exposes Allreduce / Iallreduce as primitives (mpifuncs.c:83,1357;
test/testreduceall.lua) and has no synchronous trainer; BASELINE.json
config 3 asks for one ("ResNet-50 sync all-reduce DP=8 over xGMI").

Design for MI355X: the model's gradients are views into ONE flat fp32 buffer
(:class:`~mpit_amd.utils.flat.FlatParams`), so a bucket is just a contiguous slice of it —
no pack/unpack copies. Buckets are formed in reverse parameter order (the order backward
produces gradients). Sizing for xGMI: an 8-GPU ring all-reduce moves 2·(N-1)/N of a bucket
over each of the 7 point-to-point links at ~153 GB/s, so a 25 MB bucket costs ~0.3 ms of
link time and ~10 µs of launch latency — large enough to stay bandwidth-bound, small
enough that ResNet-50's 102 MB of gradients makes 4-5 buckets which overlap the backward.
The first bucket (the last layers, complete first) is capped at ``first_bucket_mb`` so the
first all-reduce starts after a few layers of backward instead of a quarter of it. A
post-accumulate-grad hook counts finished parameters per bucket and launches the bucket's
non-blocking all-reduce (RCCL on its own stream) as soon as it is complete. ``finish()``
waits for the outstanding buckets; the 1/N averaging is fused into the optimizer kernel
(``gscale``).

``steal=True`` (the trainer's GPU path, as the parameter-server steps run it): gradients are
stolen (utils/flat.py ``steal_grads``). The MFMA layers' weight-gradient GEMMs write straight
into their flat slots on the side stream (ops/conv.py WgradStream), and autograd hands over
the other gradients as its own tensors. A complete bucket then joins the side stream, gathers
the handed-over gradients into its slice in one launch (ops.gather_scale_), zeroes the slots
of parameters without a gradient, and launches its all-reduce. No ``grad += new`` kernel per
parameter, no memset of the flat gradient per step.

``wire="bf16"``: each bucket is cast into a bf16 mirror of the flat gradient and reduced in
bf16 (half the bytes on every xGMI link), then cast back into the fp32 gradient at
``finish()``; the sum of the N gradients is rounded to bf16 once per ring step.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch

from ..comm import COMM_WORLD, SUM, Comm, Request
from ..utils.flat import FlatParams


class BucketedAllreduce:
    def __init__(self, model: torch.nn.Module, flat: FlatParams, bucket_mb: float = 25.0, comm: Optional[Comm] = None,
                 first_bucket_mb: float = 4.0, wire: str = "fp32", steal: bool = False):
        if wire not in ("fp32", "bf16"):
            raise ValueError(f"BucketedAllreduce: wire must be fp32 or bf16, not {wire!r}")
        self.comm = comm or COMM_WORLD()
        self.flat = flat
        self.steal = steal
        self.members: List[List[int]] = []  # parameter indices per bucket (steal mode)
        self.wire = wire
        self.wbuf = torch.empty(flat.numel, dtype=torch.bfloat16, device=flat.grad.device) if wire == "bf16" else None
        es = flat.grad.element_size()
        cap = int(bucket_mb * (1 << 20)) // es
        first = min(cap, int(first_bucket_mb * (1 << 20)) // es) if first_bucket_mb > 0 else cap
        order = list(range(len(flat.params)))[::-1]  # backward order
        self.buckets: List[tuple] = []  # (lo, hi) element range in the flat buffer
        self.bucket_of: Dict[int, int] = {}
        starts, n = [], 0  # first flat offset of each bucket, walking backward order
        for i in order:
            n += flat.params[i].numel()
            if n >= (first if not starts else cap):
                starts.append(flat.offsets[i])
                n = 0
        if not starts or starts[-1] != 0:
            starts.append(0)
        # contiguous [lo, hi) ranges covering the whole flat buffer (alignment padding
        # included), ascending
        starts = sorted(set(starts))
        self.buckets = [(lo, starts[k + 1] if k + 1 < len(starts) else flat.numel) for k, lo in enumerate(starts)]
        self.sizes = [0] * len(self.buckets)
        for i in range(len(flat.params)):
            off = flat.offsets[i]
            b = next(k for k, (lo, hi) in enumerate(self.buckets) if lo <= off < hi)
            self.bucket_of[i] = b
            self.sizes[b] += 1
        self.members = [[i for i in range(len(flat.params)) if self.bucket_of[i] == b] for b in range(len(self.buckets))]
        self.pending = list(self.sizes)
        self.reqs: List[Optional[Request]] = [None] * len(self.buckets)
        self._hooks = []
        for i, p in enumerate(flat.params):
            self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(i)))

    def _make_hook(self, i):
        def hook(p):
            b = self.bucket_of[i]
            self.pending[b] -= 1
            if self.pending[b] == 0:
                self._launch(b)

        return hook

    def _gather(self, b):
        """Steal mode: bucket b's gradients into its slice of the flat gradient."""
        from ..ops.conv import WgradStream
        from ..ops.fused import gather_scale_

        WgradStream.join()  # in-place weight gradients may still be in flight on the side stream
        fl = self.flat
        gbase, es = fl.grad.data_ptr(), fl.grad.element_size()
        srcs, offs, ns = [], [], []
        for i in self.members[b]:
            p, off = fl.params[i], fl.offsets[i]
            g = p.grad
            if g is None:  # no gradient this step: its slot holds the last step's
                fl.grad[off:off + p.numel()].zero_()
                continue
            if g.data_ptr() == gbase + off * es and g.dtype == fl.grad.dtype:
                p.grad = None  # written in place by its backward (grad_out)
                continue
            if g.dim() == 4 and fl.channels_last:
                g = g.contiguous(memory_format=torch.channels_last)
            else:
                g = g.contiguous()
            srcs.append(g.data_ptr())
            offs.append(off)
            ns.append(g.numel())
            p.grad = g  # alive until the gather is queued
        if srcs:
            gather_scale_(fl.grad, srcs, offs, ns, 1.0, None, 0.0)
        handed = fl.__dict__.get("_handed")
        for i in self.members[b]:
            fl.params[i].grad = None  # (the caching allocator orders any reuse on the stream)
            if handed:  # consumed: the next backward takes its flat slot again (grad_out)
                handed.discard(id(fl.params[i]))

    def _launch(self, b):
        if self.steal:
            self._gather(b)
        lo, hi = self.buckets[b]
        seg = self.flat.grad[lo:hi]
        if self.wbuf is not None:
            seg16 = self.wbuf[lo:hi]
            seg16.copy_(seg)  # cast on the compute stream, ordered before the collective
            seg = seg16
        self.reqs[b] = self.comm.Iallreduce(seg, seg, SUM)

    def finish(self):
        """Launch buckets whose parameters got no gradient, then wait for all."""
        for b in range(len(self.buckets)):
            if self.reqs[b] is None:
                self._launch(b)
        for b, r in enumerate(self.reqs):
            r.Wait()
            if self.wbuf is not None:
                lo, hi = self.buckets[b]
                self.flat.grad[lo:hi].copy_(self.wbuf[lo:hi])
        self.reqs = [None] * len(self.buckets)
        self.pending = list(self.sizes)

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []

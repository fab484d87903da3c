"""Downpour pushes overlapped with the backward pass, shard by shard.

The reference pushes the whole gradient after the backward and waits for the pulls
(asyncsgd/optim-downpour.lua:48-53). Here the flat parameter vector is split into the
servers' contiguous shards (asyncsgd/pclient.lua:116-128) and the backward produces
gradients last layer first, so the shards holding the last layers are complete long
before the backward ends. :class:`ShardPusher` watches the parameters with
post-accumulate-grad hooks; when every parameter overlapping shard k has its gradient it
gathers them into the push window with the Downpour scale (K12+K9, one launch) and sends
that shard with a fused pull, gated on an event of the compute stream. The servers apply
the update and write the refreshed shard back while the backward of the earlier layers
is still running, so only the last shard's round trip is left to wait for.

Safe because a shard is pushed only after every kernel that reads its parameters in
this step has been queued ahead of the gate: the convolutions' backward-data GEMMs read
the per-step weight copies made before the forward (bf16 casts, or the fp32 transposes of
an fp32 step — ops/conv.py WeightCastPlan), a layer's other parameter reads (the
classifier's grad_input, a BN layer's gamma) are issued by the same autograd node that
emits their gradients, i.e. before the shard can complete. tests/test_overlap.py checks
the overlapped parameters against the non-overlapped ones bit for bit on the GPU.
"""
from __future__ import annotations

import os
from typing import List

import torch

from ..ops.conv import WgradStream
from ..ops.fused import gather_scale_
from ..utils import trace as _trace


# MPIT_PUSH_ON_SIDE=1: gather + push gate on the side stream instead of joining it. Measured
# at N=1 (one shard, fired at the end of the backward): 11.1k vs 11.65k img/s, so off.
_PUSH_ON_SIDE = os.environ.get("MPIT_PUSH_ON_SIDE", "0") == "1"
# MPIT_DEBUG_GATE_DELAY=cycles (diagnostics only): a spin kernel on the compute stream right
# after each shard's gate, so the shard's pull lands before the rest of the backward runs and
# any later reader of its parameters sees the pulled values
_GATE_DELAY = int(os.environ.get("MPIT_DEBUG_GATE_DELAY", "0"))


class ShardPusher:
    def __init__(self, flat, pclient):
        self.flat, self.pc = flat, pclient
        ranges = [(o, n) for (_, o, n) in pclient.entries]  # (offset, length) per pushed shard
        self.nshards = len(ranges)
        self.params = list(flat.params)
        self.spans = []  # shards each parameter overlaps
        self.members: List[List[int]] = [[] for _ in ranges]
        for i, (p, off) in enumerate(zip(self.params, flat.offsets)):
            lo, hi = off, off + p.numel()
            ks = [k for k, (so, sl) in enumerate(ranges) if lo < so + sl and so < hi]
            self.spans.append(ks)
            for k in ks:
                self.members[k].append(i)
        self.index = {id(p): i for i, p in enumerate(self.params)}
        # per-step state, reset in place by arm(): a fresh list there was the first Python
        # allocation after the PS wait and paid for re-mapping the object arenas the previous
        # step had emptied (~0.2 ms of host time at the step start, GPU idle)
        self.left = [0] * self.nshards
        self.gathered = [False] * len(self.params)
        self.fired = [False] * self.nshards
        self._nots = [False] * len(self.params)
        self._reset = False
        self.armed = False
        self.handles = [p.register_post_accumulate_grad_hook(self._hook) for p in self.params]

    def close(self):
        for h in self.handles:
            h.remove()
        self.handles = []

    def arm(self, a: float, aux=None, b: float = 0.0):
        """Before the backward: gradients will be pushed as ``a*g + b*aux``."""
        self.a, self.aux, self.b = a, aux, b
        if not self._reset:
            self.reset()
        self._reset = False
        self.armed = True

    def reset(self):
        """The per-step counters back to a fresh step. The optimizer calls it once the step's
        last shard has fired and before it blocks on the PS (optim/distributed.py downpour),
        so this host work overlaps the wait instead of following it."""
        for k, m in enumerate(self.members):
            self.left[k] = len(m)
            self.fired[k] = False
        self.gathered[:] = self._nots
        self._reset = True

    def _hook(self, p):
        if not self.armed:
            return
        i = self.index[id(p)]
        for k in self.spans[i]:
            self.left[k] -= 1
            if self.left[k] == 0:
                self._fire(k)

    def _fire(self, k: int):
        # With backward-weight GEMMs on the side stream (ops/conv.py WgradStream) either the
        # compute stream joins it before the gather (default) or, MPIT_PUSH_ON_SIDE=1, the
        # gather and the push gate go on the side stream behind the compute stream's work so
        # far (the BN gradients), so the compute stream never waits for a shard
        side = WgradStream.side(self.pc.tx.device) if (self.pc.tx.is_cuda and _PUSH_ON_SIDE) else None
        if side is None:
            WgradStream.join()  # weight gradients may still be in flight on the side stream
            self._fire_on(k, None)
            return
        side.wait_stream(torch.cuda.current_stream(self.pc.tx.device))
        with torch.cuda.stream(side):
            self._fire_on(k, side)

    def _fire_on(self, k: int, side):
        srcs, offs, ns = [], [], []
        for i in self.members[k]:
            if self.gathered[i]:
                continue
            p = self.params[i]
            g = p.grad
            if g is None:  # unused this step: no gradient, but weight decay still applies
                sl = slice(self.flat.offsets[i], self.flat.offsets[i] + p.numel())
                if self.aux is not None and self.b != 0.0:  # a*0 + b*aux (optim-downpour.lua:24)
                    torch.mul(self.aux[sl], self.b, out=self.pc.tx[sl])
                else:
                    self.pc.tx[sl].zero_()
            else:
                if g.dim() == 4 and self.flat.channels_last:
                    g = g.contiguous(memory_format=torch.channels_last)
                else:
                    g = g.contiguous()
                srcs.append(g.data_ptr())
                offs.append(self.flat.offsets[i])
                ns.append(g.numel())
                p.grad = g  # keeps the source alive until the gather is queued
                if side is not None:  # produced on the compute stream, read on the side one
                    g.record_stream(side)
            self.gathered[i] = True
        if srcs:
            with _trace.range(f"gather_shard{k}"):
                gather_scale_(self.pc.tx, srcs, offs, ns, self.a, self.aux, self.b)
        handed = self.flat.__dict__.get("_handed")
        for i in self.members[k]:
            self.params[i].grad = None  # the caching allocator orders reuse on the stream
            if handed:  # consumed: the next step's backward takes its flat slot again (grad_out)
                handed.discard(id(self.params[i]))
        self.pc.async_send_grad_shard(k, pull=True)
        if _GATE_DELAY and self.pc.tx.is_cuda:  # race diagnostics: the pull lands before the rest
            torch.cuda._sleep(_GATE_DELAY)     # of this backward runs
        self.fired[k] = True

    def abort(self):
        """The backward failed: push nothing more (shards already pushed were complete)."""
        self.armed = False

    def finish(self):
        """After the backward: push the shards whose parameters never all got a gradient."""
        for k in range(self.nshards):
            if not self.fired[k]:
                self._fire(k)
        self.armed = False

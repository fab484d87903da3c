"""Data-parallel training driver shared by bench.py, the launchers and the tests.

Roles (mirroring asyncsgd/mlaunch.lua and BiCNN/plaunch.lua, re-designed for one process
per MI355X):
* ``colocated`` (default): every rank is a worker AND the server of one shard — N shards
  over N GPUs, each worker's push/pull fans out over all 7 xGMI links at once;
* ``dedicated``: the first ``servers`` ranks only serve (the reference's server ranks,
  BASELINE config "1 pserver + 7 workers"), the rest train;
* ``allreduce``: synchronous DP, gradients all-reduced with RCCL in buckets overlapped
  with backward (BASELINE config 3), no parameter server.

Optimizers: ``downpour`` (async SGD), ``eamsgd`` / ``easgd`` (elastic averaging),
``msgd`` (local Nesterov), plus the adaptive server rules via ``server_rule``.
"""
from __future__ import annotations

import os
import sys

import time
from dataclasses import dataclass, field
from typing import Optional

import torch
import torch.nn.functional as F

from . import ops
from . import runtime as _rt
from .comm import COMM_WORLD, MAX
from .models import get_model
from .models.cnn import INPUT_SHAPES
from .ops.loss import cross_entropy as xent
from .optim import distributed as dopt
from .parallel.ps import PClient, PServer, ServerOpt
from .utils import trace as _trace
from .utils.flat import FlatParams


@dataclass
class TrainConfig:
    model: str = "resnet50"
    batch: int = 256  # per worker
    num_classes: int = 1000
    optimizer: str = "downpour"  # downpour | eamsgd | easgd | msgd | allreduce
    topology: str = "colocated"  # colocated | dedicated
    servers: int = 1  # dedicated topology: ranks [0, servers) serve
    lr: float = 0.05
    su: int = 1
    mva: float = 0.0
    mom: float = 0.0
    l2wd: float = 0.0
    amp: bool = True  # bf16 autocast on GPU
    channels_last: bool = True
    datapath: int = 2  # 0 fused remote kernel, 1 serial SDMA, 2 per-client link streams, 3 RCCL send/recv
    staleness: int = -1  # bounded staleness (SSP) for the PS; -1 = fully asynchronous
    wire_dtype: str = "fp32"  # "bf16": EASGD elastic differences / all-reduce buckets cross xGMI in bf16
    server_rule: Optional[ServerOpt] = None
    seed: int = 1234
    bucket_mb: float = 25.0  # allreduce bucket size (parallel/ddp.py sizing note)
    extra: dict = field(default_factory=dict)


class Trainer:
    def __init__(self, cfg: TrainConfig):
        if not _rt.Initialized():
            _rt.Init()
        self.cfg = cfg
        st = _rt.state()
        self.rank, self.world = st.rank, st.world
        self.device = st.device if st.device is not None else torch.device("cpu")
        self.on_gpu = self.device.type == "cuda"
        if self.on_gpu and os.environ.get("MPIT_BLAS") == "rocblas":
            # the classifier's GEMMs (the only library GEMMs left) on rocBLAS instead of
            # hipBLASLt (A/B knob: host-side cost per call, GPU bubble around the fc layer)
            torch.backends.cuda.preferred_blas_library("cublas")
        # The step's critical path (forward, input gradients, BN, pushes) runs on a
        # high-priority stream; the backward-weight GEMMs of the side stream (lowest priority)
        # then only take the CUs the critical path leaves free, instead of delaying its small
        # kernels (BN finalize, apply) behind big split-K GEMMs. MPIT_HP_STREAM=0: off.
        self.hp_stream = None
        self._hp_ev = None  # reused step-boundary events (step)
        if self.on_gpu and os.environ.get("MPIT_HP_STREAM", "1") != "0" and not st.shared_devices:
            lo, hi = torch.cuda.Stream.priority_range()
            self.hp_stream = torch.cuda.Stream(self.device, priority=min(lo, hi))
        # MPIT_HP_INIT=1: build everything (model, flat buffers, PS, hooks) on the stream the
        # steps run on (AccumulateGrad stream diagnostic, benchmarks/diag_accgrad.py)
        if self.hp_stream is not None and os.environ.get("MPIT_HP_INIT", "0") == "1":
            cur = torch.cuda.current_stream(self.device)
            self.hp_stream.wait_stream(cur)
            with torch.cuda.stream(self.hp_stream):
                self._build(cfg, st)
            cur.wait_stream(self.hp_stream)
        else:
            self._build(cfg, st)

    def _build(self, cfg, st):
        # identical initial weights on every rank (per-rank seeds for data only)
        torch.manual_seed(cfg.seed)
        model = get_model(cfg.model, num_classes=cfg.num_classes)
        if self.on_gpu and cfg.channels_last:
            model = model.to(memory_format=torch.channels_last)
        model = model.to(self.device)
        self.model = model
        self.flat = FlatParams(model, channels_last=self.on_gpu and cfg.channels_last)
        self.plong = self.flat.numel
        torch.manual_seed(cfg.seed + 7919 * self.rank)
        self._roles()
        self._data()
        self.state = {}
        self.ps_server = None
        self.pc = None
        self.ddp = None
        if cfg.optimizer == "allreduce":
            from .parallel.ddp import BucketedAllreduce

            # the PS path's step machinery (gradients stolen, weight gradients on the side
            # stream written into their flat slots, next step's weight casts queued early)
            # unless MPIT_AR_STEAL=0; one rank has nothing to overlap: one bucket
            self.ar_steal = self.on_gpu and os.environ.get("MPIT_AR_STEAL", "1") != "0" and \
                cfg.extra.get("steal_grads", True)
            bmb = cfg.bucket_mb if self.world > 1 else float(1 << 20)
            self.ddp = BucketedAllreduce(self.model, self.flat, bucket_mb=bmb, wire=cfg.wire_dtype,
                                         first_bucket_mb=4.0 if self.world > 1 else 0.0, steal=self.ar_steal)
        else:
            self._start_ps()
        # Downpour su=1 on the GPU: let autograd hand over its gradient tensors and gather
        # them into the push window in one fused kernel (utils/flat.py StolenGrads)
        # The other GPU optimizers (EASGD / MSGD / Downpour su > 1) steal too: one gather into
        # the flat gradient replaces its memset plus one "grad += new" kernel per parameter.
        self.push_steal = (self.on_gpu and cfg.optimizer == "downpour" and cfg.su <= 1 and self.pc is not None
                           and cfg.extra.get("steal_grads", True))
        self.steal = self.push_steal or getattr(self, "ar_steal", False) or (
            self.on_gpu and cfg.optimizer != "allreduce" and cfg.extra.get("steal_grads", True))
        if self.steal:
            self.flat.steal_grads()
            # nothing reads a weight gradient before the join points (ops/conv.py WgradStream)
            from .ops.conv import WgradStream

            # not when several ranks share one GPU (1-GPU rehearsals): their extra queues
            # time-slice the card (4 ranks: 8136 -> 1809 img/s)
            WgradStream.enable(self.on_gpu and (not st.shared_devices or WgradStream.forced())
                               and cfg.extra.get("wgrad_stream", True))
        elif self.on_gpu:
            from .ops.conv import WgradStream

            WgradStream.enable(False)  # autograd accumulates the weight gradients: no side stream
        if self.push_steal:
            # push each shard during the backward as soon as its gradients are complete
            if cfg.extra.get("overlap_push", True):
                from .parallel.overlap import ShardPusher

                self.opt_config["pusher"] = ShardPusher(self.flat, self.pc)
                # defer the wait for the last shards' replies to the next read of w (cfg.extra
                # "defer_ps_wait": bench.py; MPIT_DEFER_PS_WAIT=0/1 overrides): step() then
                # returns with pulls in flight — read w only after sync() / the next step
                dw = os.environ.get("MPIT_DEFER_PS_WAIT")
                self.opt_config["defer_wait"] = (dw == "1") if dw is not None else bool(cfg.extra.get("defer_ps_wait", False))
        # bf16 casts of every MFMA conv weight in one launch per step (ops/conv.py)
        self.wcast = None
        if self.on_gpu and cfg.extra.get("batched_weight_casts", True):
            from .ops.conv import WeightCastPlan

            plan = WeightCastPlan(self.model, torch.bfloat16 if cfg.amp else torch.float32)
            self.wcast = plan if plan.njobs else None
        # Downpour su = 1 with pushed gradients and a waited pull: the weights change only by
        # the pulls, which have landed when step() returns, so the next step's weight casts
        # are queued right then (the GPU runs them while the host does the step boundary's
        # bookkeeping) instead of at the next forward. Anything else that writes the weights
        # between steps calls invalidate_precast() (load_checkpoint, set_amp). MPIT_PRECAST=0: off.
        # (sync all-reduce: the optimizer kernel at the end of step() is the weights' last
        # writer, so the casts queued after it see this step's update)
        self._precast_ok = (self.wcast is not None and (self.push_steal or getattr(self, "ar_steal", False))
                            and not getattr(self, "opt_config", {}).get("defer_wait", False)
                            and os.environ.get("MPIT_PRECAST", "1") != "0") if self.on_gpu else False
        self._precast = False
        self.steps = 0

    # ------------------------------------------------------------------ setup
    def _roles(self):
        c = self.cfg
        if c.optimizer in ("allreduce",) or self.world == 1 and c.topology == "dedicated":
            self.sranks, self.cranks = [], list(range(self.world))
        elif c.topology == "colocated":
            self.sranks = list(range(self.world))
            self.cranks = list(range(self.world))
        elif c.topology == "dedicated":
            ns = max(1, min(c.servers, self.world - 1))
            self.sranks = list(range(ns))
            self.cranks = list(range(ns, self.world))
        else:
            raise ValueError(f"unknown topology {c.topology!r}")
        self.is_server = self.rank in self.sranks
        self.is_worker = self.rank in self.cranks

    def _data(self):
        shape = INPUT_SHAPES.get(self.cfg.model, (3, 224, 224))
        dt = torch.bfloat16 if (self.on_gpu and self.cfg.amp) else torch.float32
        x = torch.randn((self.cfg.batch,) + tuple(shape), device=self.device, dtype=dt)
        if self.on_gpu and self.cfg.channels_last and len(shape) == 3:
            x = x.contiguous(memory_format=torch.channels_last)
        self.x = x
        self.y = torch.randint(0, self.cfg.num_classes, (self.cfg.batch,), device=self.device)

    def _start_ps(self):
        c = self.cfg
        rule = c.server_rule or ServerOpt("sum", a=1.0)
        # EASGD can ship the elastic difference in bf16 (half the xGMI bytes); gradients
        # pushed by Downpour stay fp32 (they are summed into the fp32 master shard)
        wire = torch.bfloat16 if (c.wire_dtype == "bf16" and c.optimizer in ("eamsgd", "easgd")) else torch.float32
        conf = dict(rank=self.rank, sranks=self.sranks, cranks=self.cranks, plong=self.plong, opt=rule,
                    datapath=c.datapath, staleness=c.staleness, grad_dtype=wire, ps_id=int(c.extra.get("ps_id", 0)),
                    shards_per_server=int(c.extra.get("shards_per_server", 1)))
        if self.is_server:
            self.ps_server = PServer(conf)
            self.ps_server.start(block=False)
        if self.is_worker:
            self.pc = PClient(conf)
            if c.optimizer in ("eamsgd", "easgd"):
                self.suw = torch.zeros(self.plong, device=self.device)
                self.sug = torch.zeros(self.plong, device=self.device, dtype=wire)
                self.pc.start(self.suw, self.sug, init=self.flat.flat)
            else:
                tx = torch.zeros(self.plong, device=self.device)
                self.pc.start(self.flat.flat, tx)
                if self.pc.rx.data_ptr() != self.flat.flat.data_ptr():  # host shm window
                    self.flat.rebind(self.pc.rx)
            self.opt_config = dict(lr=c.lr, su=c.su, mva=c.mva, mom=c.mom, l2wd=c.l2wd, pclient=self.pc)
            if c.optimizer == "downpour" and c.su == 0:
                self.opt_config["su"] = 1
        elif self.is_server and self.world > 1:
            pass  # dedicated server rank: serve until the workers stop (see run_server)

    # ------------------------------------------------------------------ step
    def _retire_deferred(self):
        """Wait for the pulls a deferred Downpour step left in flight (optim/distributed.py)."""
        st = getattr(self, "state", None)
        if st is not None and st.get("wait_pending"):
            t0 = time.perf_counter()
            self.pc.wait()
            st["dusync"] = st.get("dusync", 0.0) + time.perf_counter() - t0
            st["wait_pending"] = False

    def _feval(self, w):
        self._retire_deferred()  # the previous step's pulls land in w before anything reads it
        if not getattr(self, "steal", False):
            self.flat.zero_grad()
        if self.wcast is not None and not self._precast:  # the weights as they are now, for this step only
            with _trace.range("wcast"):
                self.wcast.run()
        self._precast = False
        try:
            with _trace.range("fwd"):
                if self.on_gpu and self.cfg.amp:
                    with torch.autocast("cuda", dtype=torch.bfloat16):
                        out = self.model(self.x)
                    loss = xent(out, self.y)  # (fp32 math on the bf16 logits)
                else:
                    out = self.model(self.x)
                    loss = (F.nll_loss(out, self.y) if self.cfg.model in ("cnn7", "lenet")
                            else xent(out, self.y))
            with _trace.range("bwd"):
                loss.backward()
        finally:
            if self.wcast is not None:
                self.wcast.invalidate()
            if self.steal:
                from .ops.conv import WgradStream

                WgradStream.join()
        if getattr(self, "push_steal", False):
            return loss.detach(), self.flat.stolen()  # gathered straight into the push window
        if getattr(self, "ar_steal", False):
            return loss.detach(), self.flat.grad  # gathered per bucket by the all-reduce (ddp.finish)
        if getattr(self, "steal", False):
            return loss.detach(), self.flat.stolen().materialize()
        return loss.detach(), self.flat.grad

    def step(self):
        """One training step of this worker; returns the loss tensor (not synced)."""
        with _trace.range("step"):
            if self.hp_stream is None:
                fx = self._step()
                self._precast_next()
                return fx
            cur = torch.cuda.current_stream(self.device)
            if self._hp_ev is None:
                # two reused events: Stream.wait_stream creates (and later destroys) a new HIP
                # event per call, tens of us of host time at the step boundary while the GPU idles
                self._hp_ev = (torch.cuda.Event(), torch.cuda.Event())
            with _trace.range("hp_wait"):
                self._hp_ev[0].record(cur)
                self.hp_stream.wait_event(self._hp_ev[0])
            with torch.cuda.stream(self.hp_stream):
                fx = self._step()
                self._precast_next()
            self._hp_ev[1].record(self.hp_stream)
            cur.wait_event(self._hp_ev[1])
            return fx

    def _precast_next(self):
        """Queue the next step's weight casts now (see __init__, ``_precast_ok``)."""
        if self._precast_ok and self.wcast is not None:
            with _trace.range("wcast"):
                self.wcast.run()
            self._precast = True

    def invalidate_precast(self):
        """The weights were written outside a step: the next step casts them anew."""
        if self._precast and self.wcast is not None:
            self.wcast.invalidate()
        self._precast = False

    def _step(self):
        c = self.cfg
        w = self.flat.flat
        if c.optimizer == "allreduce":
            loss, g = self._feval(w)
            self.ddp.finish()
            ops.nesterov_post_(w, g, None, None, clr=c.lr, gscale=1.0 / self.world, l2wd=c.l2wd)
            fx = loss
        elif c.optimizer == "downpour":
            _, (fx,) = dopt.downpour(self._feval, w, self.opt_config, self.state)
        elif c.optimizer in ("eamsgd", "easgd"):
            _, (fx,) = dopt.eamsgd(self._feval, w, self.opt_config, self.state)
        elif c.optimizer == "msgd":
            _, (fx,) = dopt.msgd(self._feval, w, dict(lr=c.lr, mom=c.mom, l2wd=c.l2wd), self.state)
        else:
            raise ValueError(f"unknown optimizer {c.optimizer!r}")
        self.steps += 1
        return fx

    # ------------------------------------------------------------------ checkpoint / resume
    def save_checkpoint(self, directory: str) -> str:
        """Collective: every rank writes its part of the job's state at a quiescent point
        (every worker first retires its in-flight push — EAMSGD leaves one outstanding —
        so after the barrier every push of every worker has been applied and acked): workers
        their flat parameters, model buffers, local optimizer state and RNG states;
        server ranks their shard, server optimizer state and rule counters
        (utils/checkpoint.py). The reference saves only worker models / the tester's
        parameters (asyncsgd/goot.lua:246-254, BiCNN/bicnn.lua:590-594)."""
        from .utils import checkpoint

        self.retire_pushes()
        self.sync()
        self.barrier()
        for m in self.model.modules():
            if hasattr(m, "sync_num_batches_tracked"):
                m.sync_num_batches_tracked()
        extra = {"steps": self.steps, "rng_cpu": torch.get_rng_state(),
                 "buffers": {n: b.detach().cpu() for n, b in self.model.named_buffers()}}
        if self.on_gpu:
            extra["rng_cuda"] = torch.cuda.get_rng_state(self.device)
        path = checkpoint.save(directory, self.steps, self.rank, self.flat if self.is_worker else None,
                               self.state if self.is_worker else None, self.ps_server, extra)
        self.barrier()
        return path

    def load_checkpoint(self, directory: str, path: Optional[str] = None) -> dict:
        """Collective: restore what :meth:`save_checkpoint` wrote (this rank's latest file in
        ``directory`` unless ``path``). Call right after construction: the barrier first
        lets the servers finish the first client's initial parameter push, which the
        restored shards then replace."""
        from .utils import checkpoint

        self.sync()
        self.barrier()
        self.invalidate_precast()  # the flat weights are about to be replaced
        path = path or checkpoint.latest(directory, self.rank)
        if path is None:
            raise FileNotFoundError(f"no checkpoint of rank {self.rank} in {directory}")
        obj = checkpoint.load(path, flat=self.flat if self.is_worker else None,
                              opt_state=self.state if self.is_worker else None, server=self.ps_server)
        ex = obj.get("extra", {})
        bufs = dict(self.model.named_buffers())
        with torch.no_grad():
            for n, v in ex.get("buffers", {}).items():
                if n in bufs:
                    bufs[n].copy_(v.to(bufs[n].device))
        if "rng_cpu" in ex:
            torch.set_rng_state(ex["rng_cpu"])
        if self.on_gpu and "rng_cuda" in ex:
            torch.cuda.set_rng_state(ex["rng_cuda"], self.device)
        self.steps = int(ex.get("steps", obj.get("step", 0)))
        self.sync()
        self.barrier()
        return obj

    def set_amp(self, amp: bool):
        """Switch the compute precision between steps: bf16 autocast (``amp``) or fp32. The
        parameters, the PS and the optimizer state are untouched; the synthetic batch and
        the per-step weight plan follow the new dtype."""
        if amp == self.cfg.amp:
            return
        self.invalidate_precast()
        self.cfg.amp = amp
        if self.on_gpu:
            self.x = self.x.to(torch.bfloat16 if amp else torch.float32)
            if self.wcast is not None:
                from .ops.conv import WeightCastPlan

                plan = WeightCastPlan(self.model, torch.bfloat16 if amp else torch.float32)
                self.wcast = plan if plan.njobs else None

    def verify_ps(self) -> dict:
        """Post-run consistency check of the parameter server (bench.py at N > 1).

        Every worker pulls every shard once more after all pushes are done (barrier), then
        each shard's bits are summed exactly (int64 sum of the fp32 words) on the worker's
        pulled copy and on the server that owns it; the sums must be identical on every
        rank. Returns {"ok", "shards", "workers", "mismatches"} on every rank."""
        from .parallel.ps import shard_ranges

        W = COMM_WORLD()
        self.retire_pushes()
        self.sync()
        self.barrier()
        if self.pc is not None:
            self.pc.async_recv_param()
            self.pc.wait()
        self.sync()
        self.barrier()

        def bits(t):
            return int(t.detach().reshape(-1).view(torch.int32).to(torch.int64).sum().item())

        mine = {"rank": self.rank, "worker": None, "server": None}
        if self.pc is not None and self.sranks:
            rx = self.pc.rx
            mine["worker"] = [bits(rx[o:o + n]) for (o, n) in shard_ranges(self.plong, len(self.sranks))]
        if self.ps_server is not None:
            self.ps_server.native.sync()
            mine["server"] = bits(self.ps_server.p)
        self.invalidate_precast()  # the pull above rewrote the weights
        allv = W.allgather_obj(mine)
        srv = {v["rank"]: v["server"] for v in allv if v["server"] is not None}
        bad = []
        for v in allv:
            if v["worker"] is None:
                continue
            for k, s in enumerate(self.sranks):
                if v["worker"][k] != srv.get(s):
                    bad.append((v["rank"], s))
        return {"ok": not bad and len(srv) == len(self.sranks), "shards": len(self.sranks),
                "workers": sum(v["worker"] is not None for v in allv), "mismatches": bad[:8]}

    def preflight(self) -> dict:
        """Collective check of every (worker, server) data path BEFORE a timed run (bench.py),
        the job's version of the reference's per-rank-GPU ping-pong (asyncsgd/ptest.lua:40-65):

        * ``devices``: each rank's GPU, and ``no_peer``: the (worker, server) pairs on distinct
          devices without peer access (a server's kernels read the worker's gradient window
          and write its parameter window directly); the windows themselves were mapped when
          the PS started — a mapping failure has already raised naming its pair
          (csrc/core/window.cpp);
        * the pull check of :meth:`verify_ps`: every worker pulls every shard once and the
          exact bit-sums must equal the owning server's; ``mismatches`` names the failing
          (worker, server) pairs.

        Returns the report on every rank; ``ok`` is False when any pair failed."""
        W = COMM_WORLD()
        dev = self.device.index if self.on_gpu else None
        devs = W.allgather_obj(dev)
        no_peer = []
        # MPIT_PREFLIGHT_NO_PEER="w:s,...": report these (worker, server) pairs as lacking peer
        # access (tests of the fallback on CPU ranks, which have no devices to ask)
        fake = {tuple(int(v) for v in p.split(":")) for p in os.environ.get("MPIT_PREFLIGHT_NO_PEER", "").split(",") if p}
        if self.pc is not None:
            for s in self.sranks:
                d = devs[s]
                if (self.rank, s) in fake or (self.on_gpu and d is not None and d != dev
                                              and not torch.cuda.can_device_access_peer(d, dev)):
                    no_peer.append((self.rank, s))
        no_peer = sorted({tuple(p) for lst in W.allgather_obj(no_peer) for p in lst})
        chk = self.verify_ps() if (self.pc is not None or self.ps_server is not None) else {"ok": True, "mismatches": []}
        bad = [tuple(p) for p in chk.get("mismatches", [])]
        # datapath 3 never maps a peer's memory: pairs without peer access are reported, but
        # only the exchanged bits decide there
        peer_ok = not no_peer or self.cfg.datapath == 3
        return {"ok": bool(chk["ok"]) and peer_ok, "devices": devs, "no_peer": [list(p) for p in no_peer],
                "mismatches": [list(p) for p in bad], "shards": chk.get("shards"), "workers": chk.get("workers"),
                "datapath": self.cfg.datapath}

    def retire_pushes(self):
        """Wait until every push / pull this worker issued has been acknowledged (EAMSGD
        deliberately leaves its last elastic push in flight, asyncsgd/optim-eamsgd.lua:65-67)."""
        if self.pc is not None:
            self.pc.wait()
            if getattr(self, "state", None) is not None:
                self.state["wait_pending"] = False

    def run_server(self):
        """Block a dedicated server rank until all workers sent stop."""
        if self.ps_server is not None and not self.is_worker:
            self.ps_server.wait_done()

    def stop(self):
        if self.pc is not None:
            self.pc.stop()
        if self.ps_server is not None:
            self.ps_server.wait_done()

    def sync(self):
        self._retire_deferred()
        if self.on_gpu:
            torch.cuda.synchronize()

    def barrier(self):
        COMM_WORLD().Barrier()

    def max_over_ranks(self, v: float) -> float:
        t = torch.tensor([v], dtype=torch.float64)
        out = torch.zeros(1, dtype=torch.float64)
        COMM_WORLD().Allreduce(t, out, MAX)
        return float(out.item())


def gc_settle() -> bool:
    """After setup / warmup: collect once, then move every surviving object (model, optimizer
    and PS state, CUDA caches) to Python's permanent generation (``gc.freeze``) so the
    cyclic collector's periodic full passes no longer walk them in the middle of a step —
    a host stall of a few hundred us that the GPU sees as idle time at the step boundary.
    Returns True when it froze; the caller unfreezes after its timed region (frozen
    objects are never collected, and trainers hold reference cycles).
    MPIT_GC_FREEZE=0 leaves the collector alone."""
    frozen = False
    if os.environ.get("MPIT_GC_FREEZE", "1") != "0":
        import gc

        gc.collect()
        gc.freeze()
        frozen = True
    if os.environ.get("MPIT_THREAD_DUMP") == "1":  # diagnostics: Python threads at the timed region
        import threading

        print("mpit threads:", [(t.name, t.daemon) for t in threading.enumerate()], file=sys.stderr, flush=True)
    sw = os.environ.get("MPIT_SWITCH_US")
    if sw:  # A/B knob: the interpreter's GIL switch interval (default 5000 us)
        sys.setswitchinterval(float(sw) * 1e-6)
    return frozen


def timed_steps(tr: Trainer, steps: int, warmup: int):
    """Warm up, then time exactly `steps` steps bracketed by barrier + device sync on both
    sides. Returns (max seconds over ranks, last loss)."""
    loss = None
    if tr.is_worker:
        for _ in range(warmup):
            loss = tr.step()
    tr.sync()
    tr.barrier()
    frozen = gc_settle()
    t0 = time.perf_counter()
    if tr.is_worker:
        for _ in range(steps):
            loss = tr.step()
    tr.sync()
    tr.barrier()
    dt = time.perf_counter() - t0
    if frozen:
        import gc

        gc.unfreeze()
    return tr.max_over_ranks(dt), loss

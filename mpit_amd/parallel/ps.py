"""Parameter server (pServer / pClient) on the native runtime.

Reference parity (asyncsgd/init.lua:3-10, asyncsgd/pserver.lua, asyncsgd/pclient.lua,
BiCNN/pserver.lua, BiCNN/pclient.lua):

* the eight PS tags (:data:`TAGS`);
* contiguous even sharding of the flat parameter vector over the servers, remainder on
  the last shard (:func:`shard_ranges`, 0-based; reference 1-based at
  asyncsgd/pclient.lua:116-128);
* the first client initialises every shard with its parameters
  (asyncsgd/pclient.lua:130-133; servers hold gradients / pulls back until then);
* ``async_send_grad`` / ``async_recv_param`` / ``async_send_param`` / ``ping`` / ``wait`` /
  ``reset`` / ``stop`` (asyncsgd/pclient.lua:97-190) and ``pServer.start``;
* server-side rules: plain ``p += g`` (Downpour / EASGD), global RMSProp, Adam with
  ``stepDivAdam``, Adamax, Adagrad, Adadelta (BiCNN/pserver.lua:115-205).

MI355X design (see csrc/core/ps.h): clients expose their flat parameter / gradient
tensors as IPC windows in HBM; the server of a shard reads the gradient shard straight
out of the client's HBM and writes the refreshed shard straight into the client's
parameters from ONE fused kernel on a high-priority stream; messages are 128-byte
control records. Servers may be co-located with workers on every GPU (the default of
:mod:`mpit_amd.launch`), dedicated ranks, or CPU processes (host windows in shm).
"""
from __future__ import annotations

import gc
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import torch

from .. import runtime as _rt
from .._ext import native
from ..comm import Comm
from ..utils import trace as _trace
from ..window import host_view

# MPIT_DEBUG_SYNC_GATE=1 (diagnostics only): a device synchronize ahead of every gated PS
# operation, taking the GPU-event gate out of the picture
_SYNC_GATE = __import__("os").environ.get("MPIT_DEBUG_SYNC_GATE", "0") == "1"
# MPIT_DEBUG_NO_SHARD_SYNC=1 (diagnostics only): the round-3 behaviour, shard fills not ordered
# before the server stream (tests/test_ps_gpu.py shows it fails then)
_NO_SHARD_SYNC = __import__("os").environ.get("MPIT_DEBUG_NO_SHARD_SYNC", "0") == "1"
# MPIT_GC_AT_WAIT=0: leave Python's young-generation collections where they fall (see PClient.wait)
_GC_AT_WAIT = __import__("os").environ.get("MPIT_GC_AT_WAIT", "1") != "0"

TAGS = dict(recv_init=1, recv_grad=2, send_param=3, recv_param=4, recv_header=5, recv_stop=6,
            recv_param_tail=7, recv_grad_tail=8)
tag_ps_recv_init = 1
tag_ps_recv_grad = 2
tag_ps_send_param = 3
tag_ps_recv_param = 4
tag_ps_recv_header = 5
tag_ps_recv_stop = 6
tag_ps_recv_param_tail = 7
tag_ps_recv_grad_tail = 8


def shard_ranges(plong: int, nservers: int) -> List[tuple]:
    """[(offset, size)] per server: floor(P/S) each, remainder on the last shard."""
    if nservers <= 0:
        raise ValueError("need at least one server")
    size = plong // nservers
    out, off = [], 0
    for i in range(nservers):
        n = plong - off if i == nservers - 1 else size
        out.append((off, n))
        off += n
    return out


@dataclass
class ServerOpt:
    """Server-side update rule. ``rule``: 'sum' (p += a*g: Downpour, EASGD, every
    'local'-mode optimizer), 'rmsprop', 'adam', 'adamax', 'adagrad', 'adadelta'."""

    rule: str = "sum"
    a: float = 1.0
    lr: float = 1e-3
    decay: float = 0.95
    momentum: float = 0.0
    eps: float = 1e-8
    beta1: float = 0.9
    beta2: float = 0.999
    rho: float = 0.95
    lr_decay: float = 0.0
    step_div: int = 1

    _KINDS = {"sum": 0, "rmsprop": 1, "adam": 2, "adamax": 3, "adagrad": 4, "adadelta": 5}
    _NSTATE = {0: 0, 1: 3, 2: 2, 3: 2, 4: 1, 5: 2}

    def native(self):
        r = native().ServerRule()
        r.kind = self._KINDS[self.rule]
        r.a, r.lr, r.decay, r.mom, r.eps = self.a, self.lr, self.decay, self.momentum, self.eps
        r.b1, r.b2, r.rho, r.lrd, r.step_div = self.beta1, self.beta2, self.rho, self.lr_decay, int(self.step_div)
        return r

    @property
    def nstate(self) -> int:
        return self._NSTATE[self._KINDS[self.rule]]

    @classmethod
    def from_bicnn_opt(cls, opt: dict) -> "ServerOpt":
        """Map BiCNN's plaunch flags (BiCNN/plaunch.lua:7-70) to a server rule."""
        o = opt.get("optimization", "sgd")
        if o == "rmsprop" and opt.get("modeRMSProp", "global") == "global":
            return cls("rmsprop", lr=opt.get("lrRMSProp", 1e-3), decay=opt.get("decayRMSProp", 0.95),
                       momentum=opt.get("momentumRMSProp", 0.9), eps=opt.get("epsilonRMSProp", 1e-4))
        if o in ("adam", "adamax") and opt.get("modeAdam", "global") == "global":
            return cls(o, lr=opt.get("lrAdam", 1e-3), beta1=opt.get("beta1Adam", 0.9), beta2=opt.get("beta2Adam", 0.999),
                       eps=opt.get("epsilonAdam", 1e-8), step_div=opt.get("stepDivAdam", 72) if o == "adam" else 1)
        if o == "adagrad" and opt.get("modeAdagrad", "global") == "global":
            return cls("adagrad", lr=opt.get("lrAdagrad", 1e-2), lr_decay=opt.get("lrDecayAdagrad", 0.0),
                       eps=opt.get("epsilonAdagrad", 1e-10))
        # reference quirk fixed: adadelta is gated on its own mode (BiCNN/pserver.lua:185)
        if o == "adadelta" and opt.get("modeAdadelta", opt.get("modeAdagrad", "global")) == "global":
            return cls("adadelta", lr=opt.get("lrAdadelta", 1.0), rho=opt.get("rhoAdadelta", 0.95),
                       eps=opt.get("epsilonAdadelta", 1e-6))
        return cls("sum")


# ------------------------------------------------------------------ shared group state

class PSMapError(RuntimeError):
    """A member could not map another member's device window (raised on every member)."""


class _Group:
    """Windows shared by all members (servers ∪ clients) of one PS instance."""

    def __init__(self, ps_id: int, servers: Sequence[int], clients: Sequence[int], plong: int,
                 rx: Optional[torch.Tensor], tx: Optional[torch.Tensor], grad_dtype=torch.float32, datapath: int = 2):
        st = _rt.state()
        self.ps_id = ps_id
        self.servers, self.clients = list(servers), list(clients)
        self.members = sorted(set(self.servers) | set(self.clients))
        self.plong = plong
        self.comm = Comm(self.members, (1 << 24) + 4 * ps_id, f"ps{ps_id}")
        self.device = st.device is not None and (rx is None or rx.is_cuda)
        eng = st.engine
        me_client = st.rank in self.clients
        # windows: clients expose rx (params, fp32) and tx (grads, fp32|bf16)
        self.rx_t = rx if me_client else None
        self.tx_t = tx if me_client else None
        self.wins = []
        for k, t in enumerate((self.rx_t, self.tx_t)):
            if t is not None:
                if not t.is_contiguous():
                    raise ValueError("pClient buffers must be contiguous")
                dev = t.is_cuda
                nbytes = t.numel() * t.element_size()
                w = native().Window(eng, (1 << 28) + 4 * ps_id + k, t.data_ptr(), nbytes, dev)
            else:
                w = native().Window(eng, (1 << 28) + 4 * ps_id + k, 0, 0, st.device is not None)
            self.wins.append(w)
        # datapath 3 moves the shards as two-sided messages (csrc/core/link.h): no rank maps
        # another's device window
        self.datapath = datapath
        err = None
        for w in self.wins:
            blobs = self.comm.allgather_obj(bytes(w.blob()))
            try:
                w.connect(blobs, self.members, datapath != 3)
            except RuntimeError as e:  # a peer mapping failed (the message names the pair)
                err = str(e)
        # agree before going on: every member raises the same error, none waits in a barrier
        # for a member that gave up (bench.py then retries on datapath 3)
        errs = [e for e in self.comm.allgather_obj(err) if e]
        if errs:
            raise PSMapError("; ".join(errs))
        if self.device and me_client:
            # the windows' contents as queued so far on our stream (rx / tx fills) are complete
            # before any server touches them from its own, unordered streams
            torch.cuda.current_stream(rx.device).synchronize()
        self.link = None
        if datapath == 3 and self.device and st.shared_devices:
            # RCCL refuses two ranks of one communicator on one GPU ("Duplicate GPU")
            raise ValueError("PS datapath 3 (RCCL send/recv) needs one GPU per rank; these ranks share a GPU")
        if datapath == 3:
            # one communicator over the members, one link stream per rank, every transfer in
            # the sequencer's (lowest member's) global order: csrc/core/link.h
            self.link = native().PsLink(eng, ps_id, self.members, self.device)
            ids = [bytes(i) for i in self.comm.allgather_obj(bytes(self.link.make_id())) if i]
            self.link.connect(ids[0] if ids else b"")
        self.comm.Barrier()
        for w in self.wins:
            w.unlink_names()
        # host windows live in shm: hand the client views of its own shm memory
        if me_client and not self.rx_t.is_cuda:
            self.rx_t = host_view(self.wins[0].local_ptr, self.wins[0].bytes, rx.dtype)
            self.tx_t = host_view(self.wins[1].local_ptr, self.wins[1].bytes, tx.dtype)
        self.server = None
        self.client = None


_groups: Dict[int, _Group] = {}
_pending_servers: Dict[int, "PServer"] = {}


def _conf_get(conf, k, default=None):
    if isinstance(conf, dict):
        return conf.get(k, default)
    return getattr(conf, k, default)


# ------------------------------------------------------------------ server

class PServer:
    """pServer(conf):start() — asyncsgd/pserver.lua:12-168, BiCNN/pserver.lua.

    conf: rank, sranks, cranks, plong, opt (ServerOpt | BiCNN opt dict), ps_id (0),
    datapath (0 fused remote kernel | 1 SDMA copies | 2 per-client link streams (default) |
    3 two-sided messages: RCCL send / recv between GPUs, csrc/core/link.h), staleness (-1 off),
    grad_dtype (float32 | bfloat16)."""

    def __init__(self, conf, state=None):
        st = _rt.state()
        self.conf = conf
        self.rank = _conf_get(conf, "rank", st.rank)
        self.sranks = list(_conf_get(conf, "sranks"))
        self.cranks = list(_conf_get(conf, "cranks"))
        self.plong = int(_conf_get(conf, "plong", 0))
        self.ps_id = int(_conf_get(conf, "ps_id", 0))
        opt = _conf_get(conf, "opt", None)
        if isinstance(opt, dict):
            opt = ServerOpt.from_bicnn_opt(opt)
        self.opt: ServerOpt = opt or ServerOpt()
        self.datapath = int(_conf_get(conf, "datapath", 2))
        self.staleness = int(_conf_get(conf, "staleness", -1))
        self.grad_dtype = _conf_get(conf, "grad_dtype", torch.float32)
        self.state = state or {}
        idx = self.sranks.index(self.rank)
        self.offset, self.size = shard_ranges(self.plong, len(self.sranks))[idx]
        self.native = None
        self.p = None
        self.opt_state: List[torch.Tensor] = []

    def _launch(self, grp: _Group):
        st = _rt.state()
        dev = st.device if (grp.device and st.device is not None) else torch.device("cpu")
        self.p = torch.zeros(self.size, dtype=torch.float32, device=dev)
        self.opt_state = [torch.zeros(self.size, dtype=torch.float32, device=dev) for _ in range(self.opt.nstate)]
        inbox = torch.empty(self.size, dtype=self.grad_dtype, device=dev) if (self.datapath == 1 and dev.type == "cuda") else None
        self._inbox = inbox
        if dev.type == "cuda" and not _NO_SHARD_SYNC:
            # the zero fills above are queued on the current (PyTorch) stream, but the server
            # updates these buffers from its own non-blocking stream (csrc/core/ps.cpp stream_),
            # which is not ordered after it: without this the fill of a recycled block could land
            # AFTER the first client's initial parameter push and zero part of the shard (seen as
            # the fp32 overlap test's 1.0 divergence in round 3: tests/test_ps_gpu.py)
            torch.cuda.current_stream(dev).synchronize()
        self.native = native().PSServer(
            st.engine, self.ps_id, grp.wins[0], grp.wins[1], grp.members, self.cranks, self.offset, self.size,
            dev.type == "cuda", self.p.data_ptr(), [t.data_ptr() for t in self.opt_state],
            inbox.data_ptr() if inbox is not None else 0, self.opt.native(), self.datapath, self.staleness,
            self.grad_dtype == torch.bfloat16, self.cranks[0])
        if grp.link is not None:
            self.native.set_link(grp.link)
        self.native.start()
        grp.server = self

    def start(self, block: Optional[bool] = None):
        """Serve this shard. Dedicated server ranks block until every client stopped
        (like the reference); a rank that is also a client returns immediately and the
        shard is served by the native progress thread."""
        st = _rt.state()
        colocated = st.rank in self.cranks
        if block is None:
            block = not colocated
        if colocated:
            if self.ps_id in _groups:
                self._launch(_groups[self.ps_id])
            else:
                _pending_servers[self.ps_id] = self  # launched by pClient.start
        else:
            grp = _Group(self.ps_id, self.sranks, self.cranks, self.plong, None, None, self.grad_dtype, self.datapath)
            _groups[self.ps_id] = grp
            self._launch(grp)
        if block:
            self.wait_done()
        return self

    def wait_done(self):
        self.native.wait_done()
        self.native.sync()

    def done(self) -> bool:
        return self.native is not None and self.native.done()

    def stats(self) -> dict:
        s = self.native.stats()
        s["version"] = self.native.version()
        return s

    def state_dict(self) -> dict:
        """Shard + optimizer state (the reference never checkpoints servers)."""
        self.native.sync()
        return {"offset": self.offset, "size": self.size, "p": self.p.detach().cpu(),
                "state": [t.detach().cpu() for t in self.opt_state], "version": self.native.version(),
                "step": self.native.step(), "rule": self.opt.rule}

    def load_state_dict(self, sd: dict):
        """Restore a quiescent server (no client message in flight): shard, rule state and
        the rule's step counter (Adam's bias correction) / update version."""
        self.native.sync()
        assert sd["offset"] == self.offset and sd["size"] == self.size, "checkpoint shard mismatch"
        self.p.copy_(sd["p"])
        for t, s in zip(self.opt_state, sd["state"]):
            t.copy_(s)
        self.native.set_counters(int(sd.get("step", 0)), int(sd.get("version", 0)))
        if self.p.is_cuda:
            torch.cuda.synchronize(self.p.device)


# ------------------------------------------------------------------ client

class PClient:
    """pClient(conf) — asyncsgd/pclient.lua:7-190.

    ``start(p, g)`` exposes p (parameters, fp32) and g (push buffer) as windows: the
    servers write pulled shards into p and read pushed shards out of g — no staging.
    ``reset(p, g)`` rebinds to other tensors (then one local copy per transfer)."""

    def __init__(self, conf, state=None):
        st = _rt.state()
        self.conf = conf
        self.rank = _conf_get(conf, "rank", st.rank)
        self.sranks = list(_conf_get(conf, "sranks"))
        self.cranks = list(_conf_get(conf, "cranks"))
        self.plong = int(_conf_get(conf, "plong", 0))
        self.ps_id = int(_conf_get(conf, "ps_id", 0))
        self.grad_dtype = _conf_get(conf, "grad_dtype", torch.float32)
        self.datapath = int(_conf_get(conf, "datapath", 2))
        self.state = state or {}
        # K > 1 splits every server's shard into K entries, each pushed / pulled as its own
        # shard (bench.py --emulate-shards: the N=K shard traffic of one worker on one GPU)
        self.shards_per_server = max(1, int(_conf_get(conf, "shards_per_server", 1)))
        self._set_layout()
        self.native = None
        self.rx = self.tx = None
        self._user_p = self._user_g = None
        self._pull_pending = False
        self.on = False

    def _set_layout(self):
        self.sinfo = {s: r for s, r in zip(self.sranks, shard_ranges(self.plong, len(self.sranks)))}
        self.entries = []  # (server rank, offset, length) per pushed / pulled shard
        for s in self.sranks:
            off, n = self.sinfo[s]
            for o, m in shard_ranges(n, self.shards_per_server) if n >= self.shards_per_server else [(0, n)]:
                self.entries.append((s, off + o, m))

    def _stream(self) -> int:
        if self.rx is not None and self.rx.is_cuda:
            if _SYNC_GATE:  # race diagnostics: everything queued so far is done before the gate
                torch.cuda.synchronize(self.rx.device)
            return torch.cuda.current_stream(self.rx.device).cuda_stream
        return 0

    def start(self, p: torch.Tensor, g: Optional[torch.Tensor] = None, init: Optional[torch.Tensor] = None):
        """Expose p / g and join the PS. ``init`` = the parameters the first client
        pushes to initialise the shards (default: p). EASGD passes its model weights here
        while p / g are the center / elastic-difference buffers."""
        if p.numel() != self.plong:
            if self.plong == 0:
                self.plong = p.numel()
                self._set_layout()
            else:
                raise ValueError(f"param size {p.numel()} != plong {self.plong}")
        if g is None:
            g = torch.zeros(self.plong, dtype=self.grad_dtype, device=p.device)
        if p.dtype != torch.float32:
            raise TypeError("pClient parameters must be float32")
        p, g = p.reshape(-1), g.reshape(-1)
        grp = _Group(self.ps_id, self.sranks, self.cranks, self.plong, p, g, self.grad_dtype, self.datapath)
        _groups[self.ps_id] = grp
        grp.client = self
        if self.ps_id in _pending_servers:
            _pending_servers.pop(self.ps_id)._launch(grp)
        self.rx, self.tx = grp.rx_t, grp.tx_t
        self._user_p, self._user_g = self.rx, self.tx
        self.native = native().PSClient(_rt.engine(), self.ps_id, [e[0] for e in self.entries],
                                        [e[1] for e in self.entries], [e[2] for e in self.entries])
        self.link = grp.link  # datapath 3's PsLink (its stats(): bytes, RCCL groups), else None
        if grp.link is not None:  # datapath 3: the shards' data from / into these very buffers
            self.native.set_link(grp.link, self.rx.data_ptr(), self.tx.data_ptr(), self.tx.element_size())
        self.native.start()
        self.on = True
        # the first client initialises every shard with its parameters
        if self.rank == self.cranks[0]:
            self.async_send_param(init)
            self.wait()
        return self

    # ------------------------------------------------------------ async ops
    def _stage_out(self, src: Optional[torch.Tensor]):
        if src is not None and src.data_ptr() != self.tx.data_ptr():
            self.tx.copy_(src.reshape(-1))

    def async_send_grad(self, pull: bool = False):
        """Push the gradient buffer to every server; ``pull=True`` also asks each server
        to write its refreshed shard back (fused push+pull, one kernel per shard)."""
        self._stage_out(self._user_g)
        _trace.mark("ps_push+pull" if pull else "ps_push")
        self.native.send_grad(self._stream(), bool(pull))
        if pull:
            self._pull_pending = True

    def async_send_grad_shard(self, k: int, pull: bool = False):
        """Push shard ``k`` (index into ``entries``; one per server unless
        ``shards_per_server`` > 1) of the gradient buffer only, gated on the work queued so
        far on the current stream (see parallel/overlap.py)."""
        _trace.mark(f"ps_push_shard{k}")
        self.native.send_grad_to(self._stream(), int(k), bool(pull))
        if pull:
            self._pull_pending = True

    def async_recv_param(self):
        _trace.mark("ps_pull")
        self.native.recv_param(self._stream())
        self._pull_pending = True

    def async_send_param(self, src: Optional[torch.Tensor] = None):
        """Push parameters (``src``, default the bound parameter tensor) to the servers,
        which overwrite their shards (tag 4, acked with tag 7). With a bf16 push window the
        parameters travel through the fp32 rx window instead (staged there when ``src`` is
        another tensor), so the shards get the exact fp32 values (BiCNN/pserver.lua:272-278)."""
        src = self._user_p if src is None else src
        if self.grad_dtype == torch.bfloat16:
            if src is not None and src.data_ptr() != self.rx.data_ptr():
                self.rx.copy_(src.reshape(-1))
            self.native.send_param(self._stream(), True)
            return
        self._stage_out(src)
        self.native.send_param(self._stream())

    def ping(self, nb: Optional[int] = None):
        """Kept for API parity (asyncsgd/pclient.lua:139-144): progress is driven by the
        native progress thread, so there is nothing to advance by hand."""
        return self.native.pending()

    def wait(self):
        if _GC_AT_WAIT and self.native.pending() and gc.isenabled():
            # the young generation's collection (~50 us, about once per training step) runs
            # here, where the host would block anyway, instead of wherever the allocation count
            # next crosses the threshold — which was the start of the next step, while the
            # GPU waits for its first kernels (profiles/boundary_r04/README.md)
            gc.collect(0)
        with _trace.range("ps_wait"):
            self.native.wait()
        self._take_deps()
        if self._pull_pending:
            self._pull_pending = False
            if self._user_p is not None and self._user_p.data_ptr() != self.rx.data_ptr():
                self._user_p.reshape(-1).copy_(self.rx)

    def _take_deps(self):
        """A co-located server replies once its update is QUEUED (csrc/core/ps.h
        PSClient::take_deps): the current stream waits on those updates before anything that
        follows reads the shard or rewrites the push window."""
        if self.rx is not None and self.rx.is_cuda:
            self.native.take_deps(torch.cuda.current_stream(self.rx.device).cuda_stream)

    def test(self) -> bool:
        done = self.native.test()
        if done:
            self._take_deps()
        return done

    def reset(self, p: Optional[torch.Tensor] = None, g: Optional[torch.Tensor] = None):
        """Rebind the client's parameter / gradient tensors (asyncsgd/pclient.lua:146-155)."""
        if p is not None:
            if p.numel() != self.plong:
                raise ValueError("reset: parameter size mismatch")
            self._user_p = p
        if g is not None:
            if g.numel() != self.plong:
                raise ValueError("reset: gradient size mismatch")
            self._user_g = g

    def stop(self):
        if self.native is not None and self.on:
            self.native.stop()
            self._take_deps()
            self.on = False

    def replies(self) -> int:
        return self.native.replies()


# reference-style names
pServer = PServer
pClient = PClient


def reset_groups():
    """Forget PS groups (tests)."""
    _groups.clear()
    _pending_servers.clear()

"""Communicators, requests, point-to-point and collective operations.

The reference exposes ~260 raw MPI calls taking ``(storage, count, datatype, ...)``
(mpifuncs.c, Appendix A of SURVEY.md). Here the buffer is a torch tensor (host or HBM)
and the element count / datatype are implied by it (an explicit ``count`` may shorten
it; a derived :class:`~mpit_amd.datatypes.Datatype` packs/unpacks it).

Transport is chosen by the tensor's device inside one native core:
* point-to-point: host tensors stream through the node's shm rings, HBM tensors use a
  rendezvous in which the receiver pulls the sender's buffer through HIP IPC (xGMI);
* collectives on HBM tensors go to RCCL through ``torch.distributed`` whenever every
  member owns a distinct GPU; otherwise (host tensors, or several ranks rehearsing on one
  GPU) they run as tree / ring algorithms over the point-to-point layer above.
"""
from __future__ import annotations

import os
import threading
from typing import Callable, List, Optional, Sequence

import torch

from . import runtime as _rt
from ._ext import native

ANY_SOURCE = -1
ANY_TAG = -1
PROC_NULL = -2
ROOT = -3
UNDEFINED = -32766
IDENT, CONGRUENT, SIMILAR, UNEQUAL = 0, 1, 2, 3
SUCCESS = 0
ERR_TRUNCATE = 15

_COLL_OFFSET = 1 << 20  # collective traffic of a communicator uses ctx + this
_coll_lock = threading.Lock()


# ============================================================================ Status / Request

class Status:
    """MPI_Status: source, tag, error, byte count, cancelled flag."""

    __slots__ = ("source", "tag", "error", "count", "cancelled", "_itemsize")

    def __init__(self, source=-1, tag=-1, error=0, count=0, cancelled=False, itemsize=1):
        self.source, self.tag, self.error, self.count, self.cancelled = source, tag, error, count, cancelled
        self._itemsize = itemsize

    @classmethod
    def _from(cls, t, itemsize=1, comm=None):
        src, tag, err, cnt, canc = t
        if comm is not None and src >= 0:
            src = comm._from_world(src)
        return cls(src, tag, err, cnt, canc, itemsize)

    def _fill(self, other: "Status"):
        for k in ("source", "tag", "error", "count", "cancelled", "_itemsize"):
            setattr(self, k, getattr(other, k))

    def Get_source(self):
        return self.source

    def Get_tag(self):
        return self.tag

    def Get_error(self):
        return self.error

    def Get_count(self, datatype=None) -> int:
        """Number of elements (bytes / element size of `datatype` or of the buffer)."""
        sz = datatype.Get_size() if datatype is not None else self._itemsize
        return self.count // max(1, sz)

    Get_elements = Get_count

    def Is_cancelled(self) -> bool:
        return self.cancelled

    def Set_cancelled(self, flag: bool):
        self.cancelled = bool(flag)

    def Set_elements(self, datatype, count: int):
        self.count = int(count) * (datatype.Get_size() if datatype is not None else self._itemsize)

    def __repr__(self):
        return f"Status(source={self.source}, tag={self.tag}, error={self.error}, count={self.count}, cancelled={self.cancelled})"


class Request:
    """A non-blocking operation. Keeps its buffers alive until completion."""

    def __init__(self, comm=None, rid: Optional[int] = None, keep=(), itemsize=1, on_done: Optional[Callable] = None,
                 work=None, thread=None, result=None):
        self.comm = comm
        self._rid = rid
        self._keep = keep
        self._itemsize = itemsize
        self._on_done = on_done
        self._work = work  # torch.distributed Work
        self._thread = thread  # background collective
        self._status: Optional[Status] = None
        self._result = result
        self._err = None
        self.persistent = None  # (callable) for *_init requests

    # -- completion
    def _complete(self, st: Status):
        self._status = st
        if self._on_done is not None:
            cb, self._on_done = self._on_done, None
            cb()
        self._keep = ()

    def Test(self, status: Optional[Status] = None) -> bool:
        if self._status is not None:
            if status is not None:
                status._fill(self._status)
            return True
        if self._rid is not None:
            t = _rt.engine().test(self._rid)
            if t is None:
                return False
            self._rid = None
            self._complete(Status._from(t, self._itemsize, self.comm))
        elif self._work is not None:
            if not self._work.is_completed():
                return False
            self._work.wait()
            self._work = None
            self._complete(Status(0, 0, 0, 0))
        elif self._thread is not None:
            if self._thread.is_alive():
                return False
            self._thread.join()
            self._thread = None
            if self._err is not None:
                raise self._err
            self._complete(Status(0, 0, 0, 0))
        else:
            self._complete(Status())
        if status is not None:
            status._fill(self._status)
        return True

    def Wait(self, status: Optional[Status] = None) -> Status:
        if self._status is None:
            if self._rid is not None:
                t = _rt.engine().wait(self._rid)
                self._rid = None
                self._complete(Status._from(t, self._itemsize, self.comm))
            elif self._work is not None:
                self._work.wait()
                self._work = None
                self._complete(Status(0, 0, 0, 0))
            elif self._thread is not None:
                self._thread.join()
                self._thread = None
                if self._err is not None:
                    raise self._err
                self._complete(Status(0, 0, 0, 0))
            else:
                self._complete(Status())
        if status is not None:
            status._fill(self._status)
        return self._status

    def Cancel(self) -> bool:
        if self._rid is not None and self._status is None:
            return bool(_rt.engine().cancel(self._rid))
        return False

    def Free(self):
        if self._rid is not None:
            try:
                _rt.engine().free_request(self._rid)
            except Exception:
                pass
            self._rid = None
        self._keep = ()

    def Get_status(self, status: Optional[Status] = None) -> bool:
        """MPI_Request_get_status: like Test but does not free the request."""
        if self._status is not None:
            if status is not None:
                status._fill(self._status)
            return True
        if self._rid is not None:
            t = _rt.engine().test(self._rid, keep=True)
            if t is None:
                return False
            if status is not None:
                status._fill(Status._from(t, self._itemsize, self.comm))
            return True
        return self.Test(status)

    def Start(self):
        """Start a persistent request (Send_init / Recv_init / ...)."""
        if self.persistent is None:
            raise RuntimeError("Start on a non-persistent request")
        r = self.persistent()
        self._rid, self._keep, self._status = r._rid, r._keep, None
        self._work, self._thread, self._on_done = r._work, r._thread, r._on_done
        r._rid = None
        return self

    @property
    def result(self):
        return self._result

    # -- multiple completion (MPI_Waitall etc.)
    @staticmethod
    def Waitall(reqs: Sequence["Request"], statuses: Optional[List[Status]] = None) -> List[Status]:
        out = [r.Wait() for r in reqs]
        if statuses is not None:
            statuses[:] = out
        return out

    @staticmethod
    def Testall(reqs: Sequence["Request"], statuses: Optional[List[Status]] = None) -> bool:
        if all(r.Test() for r in reqs):
            if statuses is not None:
                statuses[:] = [r._status for r in reqs]
            return True
        return False

    @staticmethod
    def Waitany(reqs: Sequence["Request"], status: Optional[Status] = None) -> int:
        import time

        if not reqs:
            return UNDEFINED
        while True:
            for i, r in enumerate(reqs):
                if r.Test(status):
                    return i
            time.sleep(0)

    @staticmethod
    def Testany(reqs: Sequence["Request"], status: Optional[Status] = None):
        for i, r in enumerate(reqs):
            if r.Test(status):
                return i, True
        return UNDEFINED, False

    @staticmethod
    def Waitsome(reqs: Sequence["Request"], statuses=None) -> List[int]:
        import time

        while True:
            done = Request.Testsome(reqs, statuses)
            if done:
                return done
            time.sleep(0)

    @staticmethod
    def Testsome(reqs: Sequence["Request"], statuses=None) -> List[int]:
        done = [i for i, r in enumerate(reqs) if r.Test()]
        if statuses is not None:
            statuses[:] = [reqs[i]._status for i in done]
        return done


class Grequest(Request):
    """Generalised request (MPI_Grequest_start / Grequest_complete)."""

    def __init__(self, query_fn=None, free_fn=None, cancel_fn=None, extra_state=None):
        super().__init__()
        self._done = threading.Event()
        self.query_fn, self.free_fn, self.cancel_fn, self.extra_state = query_fn, free_fn, cancel_fn, extra_state

    def Complete(self):
        self._done.set()

    def Test(self, status=None):
        if not self._done.is_set():
            return False
        st = Status(0, 0, 0, 0)
        if self.query_fn is not None:
            self.query_fn(self.extra_state, st)
        self._status = st
        if status is not None:
            status._fill(st)
        return True

    def Wait(self, status=None):
        self._done.wait()
        self.Test(status)
        return self._status

    def Cancel(self):
        if self.cancel_fn is not None:
            self.cancel_fn(self.extra_state, self._done.is_set())
        return False

    def Free(self):
        if self.free_fn is not None:
            self.free_fn(self.extra_state)


def Grequest_start(query_fn=None, free_fn=None, cancel_fn=None, extra_state=None) -> Grequest:
    return Grequest(query_fn, free_fn, cancel_fn, extra_state)


def Grequest_complete(req: Grequest):
    req.Complete()


# ============================================================================ reduction ops

class Op:
    """MPI_Op: a binary reduction on tensors (host or device)."""

    def __init__(self, fn: Callable[[torch.Tensor, torch.Tensor], torch.Tensor], commute: bool = True, name="user"):
        self.fn, self.commute, self.name = fn, commute, name

    def __call__(self, a, b):
        return self.fn(a, b)

    def Is_commutative(self) -> bool:
        return self.commute

    def Free(self):
        pass

    def __repr__(self):
        return f"Op({self.name})"


def _loc(better):
    def f(a, b):
        # (value, index) pairs in the last dimension; ties keep the smaller index
        va, ia, vb, ib = a[..., 0], a[..., 1], b[..., 0], b[..., 1]
        take_b = better(vb, va) | ((vb == va) & (ib < ia))
        return torch.stack([torch.where(take_b, vb, va), torch.where(take_b, ib, ia)], dim=-1)

    return f


# built-in ops that act element by element (safe to apply to any chunk of a buffer)
_ELEMENTWISE_OPS = {"SUM", "PROD", "MAX", "MIN", "LAND", "BAND", "LOR", "BOR", "LXOR", "BXOR"}
SUM = Op(lambda a, b: a + b, name="SUM")
PROD = Op(lambda a, b: a * b, name="PROD")
MAX = Op(torch.maximum, name="MAX")
MIN = Op(torch.minimum, name="MIN")
LAND = Op(lambda a, b: (a.bool() & b.bool()).to(a.dtype), name="LAND")
LOR = Op(lambda a, b: (a.bool() | b.bool()).to(a.dtype), name="LOR")
LXOR = Op(lambda a, b: (a.bool() ^ b.bool()).to(a.dtype), name="LXOR")
BAND = Op(lambda a, b: a & b, name="BAND")
BOR = Op(lambda a, b: a | b, name="BOR")
BXOR = Op(lambda a, b: a ^ b, name="BXOR")
MAXLOC = Op(_loc(lambda x, y: x > y), name="MAXLOC")
MINLOC = Op(_loc(lambda x, y: x < y), name="MINLOC")
REPLACE = Op(lambda a, b: b, commute=False, name="REPLACE")
NO_OP = Op(lambda a, b: a, commute=False, name="NO_OP")
OP_NULL = None


def Op_create(fn: Callable, commute: bool = True) -> Op:
    """User reduction ``fn(invec, inoutvec) -> result`` (returning the combined tensor)."""
    return Op(fn, commute)


def Reduce_local(inbuf: torch.Tensor, inoutbuf: torch.Tensor, op: Op = SUM):
    """MPI_Reduce_local (skipped by the reference's generator, readspec.py:73-75)."""
    inoutbuf.copy_(op(inbuf, inoutbuf))
    return inoutbuf


def _rccl_op(op: Op):
    import torch.distributed as dist

    return {SUM: dist.ReduceOp.SUM, PROD: dist.ReduceOp.PRODUCT, MAX: dist.ReduceOp.MAX, MIN: dist.ReduceOp.MIN,
            BAND: dist.ReduceOp.BAND, BOR: dist.ReduceOp.BOR, BXOR: dist.ReduceOp.BXOR}.get(op)


# ============================================================================ helpers

def _flat(buf: torch.Tensor, count: Optional[int] = None) -> torch.Tensor:
    if not isinstance(buf, torch.Tensor):
        raise TypeError("buffers are torch tensors")
    if not buf.is_contiguous():
        raise ValueError("communication buffers must be contiguous")
    v = buf.reshape(-1)
    if count is not None:
        v = v[:count]
    return v


def _nbytes(t: torch.Tensor) -> int:
    return t.numel() * t.element_size()


# ============================================================================ communicator

class Comm:
    """An MPI-style communicator over a subset of the world ranks."""

    def __init__(self, ranks: Sequence[int], ctx: int, name: str = ""):
        self._ranks = list(ranks)
        self._ctx = int(ctx)
        self._name = name
        self._attrs = {}
        self._errhandler = None
        self._pg = None
        self._pg_tried = False
        me = _rt.state().rank if _rt.Initialized() else 0
        self._rank = self._ranks.index(me) if me in self._ranks else UNDEFINED
        self._w2c = {w: i for i, w in enumerate(self._ranks)}
        self.topology = None  # set by Cart_create / Graph_create

    # ---------------------------------------------------------------- basics
    def Get_rank(self) -> int:
        return self._rank

    def Get_size(self) -> int:
        return len(self._ranks)

    rank = property(Get_rank)
    size = property(Get_size)

    def Get_group(self):
        from .group import Group

        return Group(self._ranks)

    def Get_name(self) -> str:
        return self._name

    def Set_name(self, name: str):
        self._name = name

    def Is_inter(self) -> bool:
        return False

    def Get_remote_size(self) -> int:
        raise RuntimeError("not an inter-communicator")

    def _to_world(self, r: int) -> int:
        if r in (ANY_SOURCE, PROC_NULL):
            return r
        return self._ranks[r]

    def _from_world(self, w: int) -> int:
        return self._w2c.get(w, w)

    @property
    def world_ranks(self) -> List[int]:
        return list(self._ranks)

    # ---------------------------------------------------------------- attributes / errhandlers
    def Set_attr(self, keyval: int, value):
        self._attrs[keyval] = value

    def Get_attr(self, keyval: int):
        return self._attrs.get(keyval)

    def Delete_attr(self, keyval: int):
        self._attrs.pop(keyval, None)

    def Set_errhandler(self, eh):
        self._errhandler = eh

    def Get_errhandler(self):
        return self._errhandler

    def Call_errhandler(self, errorcode: int):
        if self._errhandler is not None:
            self._errhandler(self, errorcode)

    # ---------------------------------------------------------------- point-to-point
    def _isend(self, buf, dest, tag, ctx, sync=False, count=None, datatype=None) -> Request:
        if dest == PROC_NULL:
            return Request(self)
        if datatype is not None and not datatype.is_contiguous_basic():
            buf = datatype.pack(buf, count)
            count = None
        t = _flat(buf, count)
        if t.is_cuda:  # the receiver pulls the bytes: what the stream is still producing must land first
            torch.cuda.current_stream(t.device).synchronize()
        rid = _rt.engine().isend(t.data_ptr(), _nbytes(t), t.is_cuda, self._to_world(dest), int(tag), ctx, sync)
        return Request(self, rid, keep=(t,), itemsize=t.element_size())

    def _irecv(self, buf, source, tag, ctx, count=None, datatype=None) -> Request:
        if source == PROC_NULL:
            r = Request(self)
            r._status = Status(PROC_NULL, ANY_TAG, 0, 0)
            return r
        if datatype is not None and not datatype.is_contiguous_basic():
            stage = datatype.staging(buf, count)
            rid = _rt.engine().irecv(stage.data_ptr(), _nbytes(stage), stage.is_cuda, self._to_world(source), int(tag), ctx)
            return Request(self, rid, keep=(stage, buf), itemsize=datatype.Get_size(),
                           on_done=lambda: datatype.unpack(stage, buf, count))
        t = _flat(buf, count)
        rid = _rt.engine().irecv(t.data_ptr(), _nbytes(t), t.is_cuda, self._to_world(source), int(tag), ctx)
        return Request(self, rid, keep=(t,), itemsize=t.element_size())

    def Isend(self, buf, dest: int, tag: int = 0, count=None, datatype=None) -> Request:
        return self._isend(buf, dest, tag, self._ctx, False, count, datatype)

    def Issend(self, buf, dest: int, tag: int = 0, count=None, datatype=None) -> Request:
        return self._isend(buf, dest, tag, self._ctx, True, count, datatype)

    # MPI's buffered / ready modes: the engine never needs the user's attached buffer (eager
    # messages are copied into the shm ring, large ones wait for the receiver) and a ready
    # send is a correct standard send, so both are the standard mode
    Ibsend = Isend
    Irsend = Isend

    def Send(self, buf, dest: int, tag: int = 0, count=None, datatype=None):
        self.Isend(buf, dest, tag, count, datatype).Wait()

    Bsend = Send
    Rsend = Send

    def Ssend(self, buf, dest: int, tag: int = 0, count=None, datatype=None):
        self.Issend(buf, dest, tag, count, datatype).Wait()

    def Irecv(self, buf, source: int = ANY_SOURCE, tag: int = ANY_TAG, count=None, datatype=None) -> Request:
        return self._irecv(buf, source, tag, self._ctx, count, datatype)

    def Recv(self, buf, source: int = ANY_SOURCE, tag: int = ANY_TAG, status: Optional[Status] = None,
             count=None, datatype=None) -> Status:
        return self.Irecv(buf, source, tag, count, datatype).Wait(status)

    def Sendrecv(self, sendbuf, dest, sendtag, recvbuf, source=ANY_SOURCE, recvtag=ANY_TAG, status=None,
                 sendcount=None, sendtype=None, recvcount=None, recvtype=None) -> Status:
        rr = self.Irecv(recvbuf, source, recvtag, recvcount, recvtype)
        sr = self.Isend(sendbuf, dest, sendtag, sendcount, sendtype)
        sr.Wait()
        return rr.Wait(status)

    def Sendrecv_replace(self, buf, dest, sendtag, source=ANY_SOURCE, recvtag=ANY_TAG, status=None,
                         count=None, datatype=None) -> Status:
        tmp = buf.clone()
        return self.Sendrecv(tmp, dest, sendtag, buf, source, recvtag, status, count, datatype, count, datatype)

    def Iprobe(self, source: int = ANY_SOURCE, tag: int = ANY_TAG, status: Optional[Status] = None) -> bool:
        src = self._to_world(source) if source >= 0 else source
        t = _rt.engine().iprobe(src, int(tag), self._ctx)
        if t is None:
            return False
        if status is not None:
            status._fill(Status._from(t, 1, self))
        return True

    def Probe(self, source: int = ANY_SOURCE, tag: int = ANY_TAG, status: Optional[Status] = None) -> Status:
        src = self._to_world(source) if source >= 0 else source
        st = Status._from(_rt.engine().probe(src, int(tag), self._ctx), 1, self)
        if status is not None:
            status._fill(st)
        return st

    # persistent requests
    def Send_init(self, buf, dest, tag=0, count=None, datatype=None) -> Request:
        r = Request(self)
        r._status = Status()
        r.persistent = lambda: self.Isend(buf, dest, tag, count, datatype)
        return r

    Bsend_init = Send_init
    Rsend_init = Send_init

    def Ssend_init(self, buf, dest, tag=0, count=None, datatype=None) -> Request:
        r = Request(self)
        r._status = Status()
        r.persistent = lambda: self.Issend(buf, dest, tag, count, datatype)
        return r

    def Recv_init(self, buf, source=ANY_SOURCE, tag=ANY_TAG, count=None, datatype=None) -> Request:
        r = Request(self)
        r._status = Status()
        r.persistent = lambda: self.Irecv(buf, source, tag, count, datatype)
        return r

    # object convenience (mpiT.serialize / deserialize, init.lua:111-132)
    def send_obj(self, obj, dest: int, tag: int = 0):
        from .utils.serialize import serialize

        payload = serialize(obj)
        n = torch.tensor([payload.numel()], dtype=torch.int64)
        self.Send(n, dest, tag)
        self.Send(payload, dest, tag)

    def recv_obj(self, source: int = ANY_SOURCE, tag: int = ANY_TAG):
        from .utils.serialize import deserialize

        n = torch.zeros(1, dtype=torch.int64)
        st = self.Recv(n, source, tag)
        payload = torch.empty(int(n.item()), dtype=torch.uint8)
        self.Recv(payload, st.source, st.tag)
        return deserialize(payload)

    # ---------------------------------------------------------------- collective plumbing
    def _cctx(self) -> int:
        return self._ctx + _COLL_OFFSET

    def _csend(self, buf, dest, tag=0) -> Request:
        return self._isend(buf, dest, tag, self._cctx())

    def _crecv(self, buf, source, tag=0) -> Request:
        return self._irecv(buf, source, tag, self._cctx())

    def _use_rccl(self, t: torch.Tensor) -> bool:
        """Run this collective through torch.distributed: RCCL for HBM tensors when every
        rank owns its GPU; gloo for host tensors only when MPIT_DIST_HOST=1 (the shm
        point-to-point algorithms below are the default host path; the switch exists so
        CPU tests exercise the torch.distributed branch and its Request(work=...))."""
        if self.Get_size() == 1:
            return False
        st = _rt.state()
        if t.is_cuda:
            if st.shared_devices:
                return False
        elif os.environ.get("MPIT_DIST_HOST") != "1":
            return False
        import torch.distributed as dist

        if not dist.is_initialized():
            return False
        if self._pg is None and not self._pg_tried:
            self._pg_tried = True
            # torch.distributed only for communicators over every rank in world order (WORLD,
            # its Dup, an all-ranks Split keyed by rank): the torch group's rank order is
            # then the communicator's. Sub-communicators run on the native point-to-point
            # engine (IPC peer copies over xGMI for HBM tensors): torch's locally
            # synchronised sub-groups deadlock when two of them overlap in a rank
            # (reproduced with gloo: [0,2] then [1,2]), and communicator creation is not
            # collective over WORLD, so world-synchronised groups cannot be made either.
            if list(self._ranks) == list(range(st.world)):
                self._pg = dist.group.WORLD
        return self._pg is not None

    # ---------------------------------------------------------------- collectives
    def Barrier(self):
        if self.Get_size() == 1:
            return
        if len(self._ranks) == _rt.state().world:
            _rt.engine().barrier()
            return
        # dissemination barrier over zero-byte messages
        n, r = self.Get_size(), self.Get_rank()
        z = torch.zeros(0, dtype=torch.uint8)
        k = 1
        while k < n:
            rr = self._crecv(torch.zeros(0, dtype=torch.uint8), (r - k) % n, 7)
            self._csend(z, (r + k) % n, 7).Wait()
            rr.Wait()
            k <<= 1

    def Bcast(self, buf: torch.Tensor, root: int = 0):
        n = self.Get_size()
        if n == 1:
            return buf
        t = _flat(buf)
        if self._use_rccl(t):
            import torch.distributed as dist

            dist.broadcast(t, src=self._ranks[root], group=self._pg)
            return buf
        r = (self.Get_rank() - root) % n  # relative rank, binomial tree
        mask = 1
        while mask < n:
            if r & mask:
                self._crecv(t, (r - mask + root) % n, 1).Wait()
                break
            mask <<= 1
        mask >>= 1
        while mask > 0:
            if r + mask < n:
                self._csend(t, (r + mask + root) % n, 1).Wait()
            mask >>= 1
        return buf

    def Reduce(self, sendbuf, recvbuf, op: Op = SUM, root: int = 0):
        n = self.Get_size()
        src = _flat(sendbuf)
        if n == 1:
            if recvbuf is not None and recvbuf is not sendbuf:
                _flat(recvbuf).copy_(src)
            return recvbuf
        if self._use_rccl(src) and _rccl_op(op) is not None:
            import torch.distributed as dist

            acc = src.clone()
            dist.reduce(acc, dst=self._ranks[root], op=_rccl_op(op), group=self._pg)
            if self.Get_rank() == root:
                _flat(recvbuf).copy_(acc)
            return recvbuf
        me = self.Get_rank()
        if not op.commute:
            # ordered linear reduction at the root: ((b0 op b1) op b2) ...
            if me == root:
                parts = []
                for q in range(n):
                    if q == me:
                        parts.append(src.clone())
                    else:
                        tmp = torch.empty_like(src)
                        self._crecv(tmp, q, 2).Wait()
                        parts.append(tmp)
                acc = parts[0]
                for q in range(1, n):
                    acc = op(acc, parts[q])
                _flat(recvbuf).copy_(acc)
            else:
                self._csend(src, root, 2).Wait()
            return recvbuf
        acc = src.clone()
        tmp = torch.empty_like(src)
        r = (me - root) % n
        mask = 1
        while mask < n:
            if r & mask:
                self._csend(acc, (r - mask + root) % n, 2).Wait()
                break
            if r + mask < n:
                self._crecv(tmp, (r + mask + root) % n, 2).Wait()
                acc = op(acc, tmp)
            mask <<= 1
        if me == root:
            _flat(recvbuf).copy_(acc)
        return recvbuf

    def Allreduce(self, sendbuf, recvbuf=None, op: Op = SUM):
        """MPI_Allreduce (mpifuncs.c:83). ``sendbuf is recvbuf`` (IN_PLACE) allowed."""
        if recvbuf is None:
            recvbuf = sendbuf
        n = self.Get_size()
        src = _flat(sendbuf)
        dst = _flat(recvbuf)
        if n == 1:
            if dst.data_ptr() != src.data_ptr():
                dst.copy_(src)
            return recvbuf
        if self._use_rccl(src) and _rccl_op(op) is not None:
            import torch.distributed as dist

            if dst.data_ptr() != src.data_ptr():
                dst.copy_(src)
            dist.all_reduce(dst, op=_rccl_op(op), group=self._pg)
            return recvbuf
        if op.name in _ELEMENTWISE_OPS and n > 2 and src.numel() >= 64 * n:
            if dst.data_ptr() != src.data_ptr():
                dst.copy_(src)
            self._ring_allreduce(dst, op)
            return recvbuf
        tmp = torch.empty_like(src)
        self.Reduce(src, tmp, op, 0)
        if self.Get_rank() == 0:
            dst.copy_(tmp)
        self.Bcast(dst, 0)
        return recvbuf

    def _ring_allreduce(self, buf: torch.Tensor, op: Op):
        """Ring reduce-scatter + all-gather over the point-to-point layer (commutative
        ops): every rank sends and receives 2(n-1)/n of the buffer, with both of its
        neighbour links busy every step, instead of a binomial reduce + broadcast that
        moves the whole buffer log2(n) times through the root."""
        n, r = self.Get_size(), self.Get_rank()
        m = buf.numel()
        bounds = [m * k // n for k in range(n + 1)]
        chunk = [buf[bounds[k]: bounds[k + 1]] for k in range(n)]
        # two receive buffers: step s's op kernel (queued on the compute stream) may still
        # read tmp[s % 2] while step s + 1's receive lands — the engine pulls on its own
        # stream. Step s + 2 reuses it only after step s + 1's send synchronised the stream.
        cap = max(bounds[k + 1] - bounds[k] for k in range(n))
        tmps = [torch.empty(cap, dtype=buf.dtype, device=buf.device) for _ in range(2)]
        right, left = (r + 1) % n, (r - 1) % n
        for s in range(n - 1):  # reduce-scatter: rank r ends owning chunk (r + 1) % n
            si, ri = (r - s) % n, (r - s - 1) % n
            t = tmps[s % 2][: chunk[ri].numel()]
            rq = self._crecv(t, left, 10)
            sq = self._csend(chunk[si], right, 10)
            rq.Wait()
            chunk[ri].copy_(op(chunk[ri], t))
            sq.Wait()
        for s in range(n - 1):  # all-gather of the reduced chunks
            si, ri = (r + 1 - s) % n, (r - s) % n
            rq = self._crecv(chunk[ri], left, 11)
            sq = self._csend(chunk[si], right, 11)
            rq.Wait()
            sq.Wait()

    def Iallreduce(self, sendbuf, recvbuf=None, op: Op = SUM) -> Request:
        """Non-blocking all-reduce (mpifuncs.c:1357). RCCL work handle on HBM tensors,
        a background progress thread otherwise."""
        if recvbuf is None:
            recvbuf = sendbuf
        src = _flat(sendbuf)
        if self.Get_size() == 1:
            # one rank: the reduction is the rank's own data — a stream-ordered copy (or
            # nothing, in place), complete at once; no background thread per call
            dst = _flat(recvbuf)
            if dst.data_ptr() != src.data_ptr():
                dst.copy_(src)
            return Request(self, keep=(sendbuf, recvbuf))
        if self._use_rccl(src) and _rccl_op(op) is not None:
            import torch.distributed as dist

            dst = _flat(recvbuf)
            if dst.data_ptr() != src.data_ptr():
                dst.copy_(src)
            w = dist.all_reduce(dst, op=_rccl_op(op), group=self._pg, async_op=True)
            return Request(self, work=w, keep=(sendbuf, recvbuf))
        return self._bg(lambda: self.Allreduce(sendbuf, recvbuf, op), keep=(sendbuf, recvbuf))

    def _bg(self, fn, keep=()) -> Request:
        req = Request(self, keep=keep)

        def run():
            try:
                with _coll_lock:
                    fn()
            except BaseException as e:  # surfaced by Wait/Test
                req._err = e

        th = threading.Thread(target=run, daemon=True)
        req._thread = th
        th.start()
        return req

    def Ibarrier(self) -> Request:
        return self._bg(self.Barrier)

    def Ibcast(self, buf, root=0) -> Request:
        return self._bg(lambda: self.Bcast(buf, root), keep=(buf,))

    def Ireduce(self, sendbuf, recvbuf, op=SUM, root=0) -> Request:
        return self._bg(lambda: self.Reduce(sendbuf, recvbuf, op, root), keep=(sendbuf, recvbuf))

    def Iallgather(self, sendbuf, recvbuf) -> Request:
        return self._bg(lambda: self.Allgather(sendbuf, recvbuf), keep=(sendbuf, recvbuf))

    def Ialltoall(self, sendbuf, recvbuf) -> Request:
        return self._bg(lambda: self.Alltoall(sendbuf, recvbuf), keep=(sendbuf, recvbuf))

    def Ireduce_scatter(self, sendbuf, recvbuf, recvcounts=None, op=SUM) -> Request:
        return self._bg(lambda: self.Reduce_scatter(sendbuf, recvbuf, recvcounts, op), keep=(sendbuf, recvbuf))

    def Gatherv(self, sendbuf, recvbuf, counts: Optional[Sequence[int]] = None, displs=None, root: int = 0):
        n, me = self.Get_size(), self.Get_rank()
        src = _flat(sendbuf)
        if me != root:
            self._csend(src, root, 3).Wait()
            return recvbuf
        dst = _flat(recvbuf)
        if counts is None:
            counts = [src.numel()] * n
        if displs is None:
            displs = [sum(counts[:i]) for i in range(n)]
        reqs = []
        for q in range(n):
            seg = dst[displs[q]: displs[q] + counts[q]]
            if q == me:
                seg.copy_(src[: counts[q]])
            else:
                reqs.append(self._crecv(seg, q, 3))
        Request.Waitall(reqs)
        return recvbuf

    def Gather(self, sendbuf, recvbuf, root: int = 0):
        return self.Gatherv(sendbuf, recvbuf, None, None, root)

    def Scatterv(self, sendbuf, recvbuf, counts: Optional[Sequence[int]] = None, displs=None, root: int = 0):
        n, me = self.Get_size(), self.Get_rank()
        dst = _flat(recvbuf)
        if me != root:
            self._crecv(dst, root, 4).Wait()
            return recvbuf
        src = _flat(sendbuf)
        if counts is None:
            counts = [dst.numel()] * n
        if displs is None:
            displs = [sum(counts[:i]) for i in range(n)]
        reqs = []
        for q in range(n):
            seg = src[displs[q]: displs[q] + counts[q]]
            if q == me:
                dst[: counts[q]].copy_(seg)
            else:
                reqs.append(self._csend(seg.contiguous(), q, 4))
        Request.Waitall(reqs)
        return recvbuf

    def Scatter(self, sendbuf, recvbuf, root: int = 0):
        return self.Scatterv(sendbuf, recvbuf, None, None, root)

    def Allgatherv(self, sendbuf, recvbuf, counts: Optional[Sequence[int]] = None, displs=None):
        n = self.Get_size()
        src = _flat(sendbuf)
        dst = _flat(recvbuf)
        if counts is None and self._use_rccl(src):
            import torch.distributed as dist

            dist.all_gather_into_tensor(dst, src, group=self._pg)
            return recvbuf
        if counts is None:
            counts = [src.numel()] * n
        if displs is None:
            displs = [sum(counts[:i]) for i in range(n)]
        self.Gatherv(src, dst, counts, displs, 0)
        self.Bcast(dst, 0)
        return recvbuf

    def Allgather(self, sendbuf, recvbuf):
        return self.Allgatherv(sendbuf, recvbuf, None, None)

    def Alltoallv(self, sendbuf, sendcounts, sdispls, recvbuf, recvcounts, rdispls):
        n, me = self.Get_size(), self.Get_rank()
        src, dst = _flat(sendbuf), _flat(recvbuf)
        reqs = []
        for q in range(n):
            rseg = dst[rdispls[q]: rdispls[q] + recvcounts[q]]
            sseg = src[sdispls[q]: sdispls[q] + sendcounts[q]]
            if q == me:
                rseg.copy_(sseg)
            else:
                reqs.append(self._crecv(rseg, q, 5))
                reqs.append(self._csend(sseg.contiguous(), q, 5))
        Request.Waitall(reqs)
        return recvbuf

    def Alltoall(self, sendbuf, recvbuf):
        n = self.Get_size()
        src, dst = _flat(sendbuf), _flat(recvbuf)
        if self._use_rccl(src):
            import torch.distributed as dist

            dist.all_to_all_single(dst, src, group=self._pg)
            return recvbuf
        c = src.numel() // n
        d = [i * c for i in range(n)]
        return self.Alltoallv(src, [c] * n, d, dst, [c] * n, d)

    def Alltoallw(self, sendbufs: Sequence[torch.Tensor], recvbufs: Sequence[torch.Tensor]):
        """Per-peer tensors of arbitrary dtype/shape (MPI_Alltoallw's per-peer types)."""
        n, me = self.Get_size(), self.Get_rank()
        reqs = []
        for q in range(n):
            if q == me:
                recvbufs[q].copy_(sendbufs[q])
            else:
                reqs.append(self._crecv(recvbufs[q], q, 6))
                reqs.append(self._csend(sendbufs[q].contiguous(), q, 6))
        Request.Waitall(reqs)
        return recvbufs

    def Reduce_scatter(self, sendbuf, recvbuf, recvcounts: Optional[Sequence[int]] = None, op: Op = SUM):
        n = self.Get_size()
        src, dst = _flat(sendbuf), _flat(recvbuf)
        if recvcounts is None:
            recvcounts = [src.numel() // n] * n
        if self._use_rccl(src) and _rccl_op(op) is not None and len(set(recvcounts)) == 1:
            import torch.distributed as dist

            dist.reduce_scatter_tensor(dst[: recvcounts[0]], src[: recvcounts[0] * n].contiguous(),
                                       op=_rccl_op(op), group=self._pg)
            return recvbuf
        tmp = torch.empty_like(src) if self.Get_rank() == 0 else None
        self.Reduce(src, tmp if tmp is not None else src, op, 0)
        displs = [sum(recvcounts[:i]) for i in range(n)]
        self.Scatterv(tmp, dst, recvcounts, displs, 0)
        return recvbuf

    def Reduce_scatter_block(self, sendbuf, recvbuf, op: Op = SUM):
        return self.Reduce_scatter(sendbuf, recvbuf, None, op)

    def Scan(self, sendbuf, recvbuf, op: Op = SUM):
        """Inclusive prefix reduction (linear chain, order-preserving)."""
        n, me = self.Get_size(), self.Get_rank()
        src, dst = _flat(sendbuf), _flat(recvbuf)
        acc = src.clone()
        if me > 0:
            prev = torch.empty_like(src)
            self._crecv(prev, me - 1, 8).Wait()
            acc = op(prev, acc)
        if me < n - 1:
            self._csend(acc, me + 1, 8).Wait()
        dst.copy_(acc)
        return recvbuf

    def Exscan(self, sendbuf, recvbuf, op: Op = SUM):
        """Exclusive prefix reduction; rank 0's recvbuf is left untouched (MPI)."""
        n, me = self.Get_size(), self.Get_rank()
        src, dst = _flat(sendbuf), _flat(recvbuf)
        if me > 0:
            prev = torch.empty_like(src)
            self._crecv(prev, me - 1, 9).Wait()
            out = prev.clone()
            acc = op(prev, src)
        else:
            out = None
            acc = src.clone()
        if me < n - 1:
            self._csend(acc, me + 1, 9).Wait()
        if out is not None:
            dst.copy_(out)
        return recvbuf

    # object collectives (host, small)
    def allgather_obj(self, obj) -> list:
        import pickle

        data = torch.frombuffer(bytearray(pickle.dumps(obj)), dtype=torch.uint8)
        n = torch.tensor([data.numel()], dtype=torch.int64)
        sizes = torch.zeros(self.Get_size(), dtype=torch.int64)
        self.Allgather(n, sizes)
        buf = torch.zeros(int(sizes.sum()), dtype=torch.uint8)
        self.Allgatherv(data, buf, sizes.tolist())
        out, o = [], 0
        for s in sizes.tolist():
            out.append(pickle.loads(buf[o: o + s].numpy().tobytes()))
            o += s
        return out

    def bcast_obj(self, obj, root=0):
        return self.allgather_obj(obj if self.Get_rank() == root else None)[root]

    # ---------------------------------------------------------------- constructors
    def _agree_ctx(self) -> int:
        """Collectively agree on a fresh context id (max of the members' counters)."""
        st = _rt.state()
        mine = torch.tensor([st.next_ctx], dtype=torch.int64)
        out = torch.zeros(1, dtype=torch.int64)
        self.Allreduce(mine, out, MAX)
        ctx = int(out.item())
        st.next_ctx = ctx + 1
        return ctx * 2  # even: user p2p; ctx + 2^20: collectives

    def Dup(self) -> "Comm":
        c = Comm(self._ranks, self._agree_ctx(), self._name + "_dup")
        c._attrs = dict(self._attrs)
        return c

    Idup = Dup

    def Create(self, group) -> Optional["Comm"]:
        ctx = self._agree_ctx()
        if _rt.state().rank not in group.world_ranks:
            return None
        return Comm(group.world_ranks, ctx)

    def Split(self, color: int, key: int = 0) -> Optional["Comm"]:
        ctx = self._agree_ctx()
        entries = self.allgather_obj((color, key, _rt.state().rank))
        if color == UNDEFINED:
            return None
        mine = sorted([(k, w) for (c, k, w) in entries if c == color])
        colors = sorted({c for (c, _, _) in entries if c != UNDEFINED})
        return Comm([w for (_, w) in mine], ctx + 2 * _COLL_OFFSET * (1 + colors.index(color)))

    def Compare(self, other: "Comm") -> int:
        if other is self:
            return IDENT
        if self._ranks == other._ranks:
            return CONGRUENT
        if sorted(self._ranks) == sorted(other._ranks):
            return SIMILAR
        return UNEQUAL

    def Free(self):
        self._pg = None

    def Disconnect(self):
        self.Barrier()
        self.Free()

    def Abort(self, code: int = 1):
        _rt.Abort(code)

    def __repr__(self):
        return f"Comm(name={self._name!r}, rank={self.Get_rank()}, size={self.Get_size()})"


COMM_NULL = None
_world: Optional[Comm] = None
_self: Optional[Comm] = None


def COMM_WORLD() -> Comm:
    global _world
    st = _rt.state()
    if _world is None or _world._ranks != list(range(st.world)):
        _world = Comm(list(range(st.world)), 0, "MPI_COMM_WORLD")
    return _world


def COMM_SELF() -> Comm:
    global _self
    st = _rt.state()
    if _self is None or _self._ranks != [st.rank]:
        _self = Comm([st.rank], 2, "MPI_COMM_SELF")
    return _self


def _reset_singletons():
    global _world, _self
    _world = None
    _self = None

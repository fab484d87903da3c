"""One-sided communication: MPI_Win_* over HIP IPC (device) or shm (host).

``Win.Create(tensor, comm)`` exposes a tensor of every member; afterwards any member can
``Put`` / ``Get`` / ``Accumulate`` into any other member's tensor without the target's
participation. On HBM the data moves as one peer copy over xGMI (hipMemcpyAsync between
IPC-mapped allocations) and Accumulate is a fused read-modify-write kernel on the remote
memory; host windows are POSIX shm objects mapped by every member.
Synchronisation: ``Fence`` (active target, collective), ``Lock``/``Unlock`` (passive target,
shm reader/writer lock per target), ``Post``/``Start``/``Complete``/``Wait`` (PSCW), ``Flush``.
Reference: the generated Win_* / Put / Get / Accumulate wrappers (mpifuncs.c:9,1131,1656,
2322-2493); the reference never uses them, SURVEY §7.1 lists them as Tier 2.
"""
from __future__ import annotations

import ctypes
import weakref
from typing import Optional

import torch

from . import runtime as _rt
from ._ext import native

LOCK_EXCLUSIVE, LOCK_SHARED = 234, 235
MODE_NOCHECK = 1024

_open = weakref.WeakSet()
_next_id = [1 << 30]


def _close_all():
    for w in list(_open):
        try:
            w.Free()
        except Exception:
            pass


def host_view(ptr: int, nbytes: int, dtype: torch.dtype) -> torch.Tensor:
    """A tensor aliasing host memory at ``ptr`` (no copy)."""
    if nbytes == 0:
        return torch.empty(0, dtype=dtype)
    buf = (ctypes.c_uint8 * nbytes).from_address(ptr)
    return torch.frombuffer(buf, dtype=dtype)


class Win:
    def __init__(self, native_win, comm, tensor: torch.Tensor, disp_unit: int, info=None):
        self._w = native_win
        self.comm = comm
        self.tensor = tensor  # the local exposed memory (a shm view for host windows)
        self.disp_unit = disp_unit
        self.info = info or {}
        self._attrs = {}
        self._name = ""
        self._epoch_targets = []
        self._errhandler = None
        _open.add(self)

    # ------------------------------------------------------------ creation
    @classmethod
    def _make(cls, tensor: Optional[torch.Tensor], nbytes: int, device: bool, comm, disp_unit: int, dtype, info=None,
              win_id: Optional[int] = None):
        eng = _rt.engine()
        if win_id is None:
            win_id = comm._agree_ctx() + (1 << 29)
        local = tensor.data_ptr() if tensor is not None and nbytes > 0 else 0
        w = native().Window(eng, int(win_id), local, int(nbytes), bool(device))
        blobs = comm.allgather_obj(bytes(w.blob()))
        w.connect(blobs, comm.world_ranks)
        if device:
            # window creation is collective: what this rank queued into the exposed memory (the
            # Allocate zero fill, the caller's writes) completes before any peer may access it
            # from its own streams, which are not ordered after ours
            torch.cuda.current_stream().synchronize()
        comm.Barrier()
        w.unlink_names()
        if device:
            exposed = tensor if tensor is not None else torch.empty(0, dtype=dtype, device=_rt.device())
        else:
            exposed = host_view(w.local_ptr, nbytes, dtype)
        return cls(w, comm, exposed, disp_unit, info)

    @classmethod
    def Create(cls, tensor: torch.Tensor, comm=None, disp_unit: Optional[int] = None, info=None) -> "Win":
        """Expose ``tensor`` (HBM: zero-copy; host: the window is a shm copy, use ``win.tensor``)."""
        from .comm import COMM_WORLD

        comm = comm or COMM_WORLD()
        if not tensor.is_contiguous():
            raise ValueError("window memory must be contiguous")
        du = disp_unit or tensor.element_size()
        return cls._make(tensor, tensor.numel() * tensor.element_size(), tensor.is_cuda, comm, du, tensor.dtype, info)

    @classmethod
    def Allocate(cls, numel: int, dtype=torch.float32, comm=None, device: Optional[bool] = None, info=None) -> "Win":
        from .comm import COMM_WORLD

        comm = comm or COMM_WORLD()
        if device is None:
            device = _rt.device() is not None
        if device:
            t = torch.zeros(numel, dtype=dtype, device=_rt.device())
            return cls._make(t, t.numel() * t.element_size(), True, comm, t.element_size(), dtype, info)
        es = torch.empty(0, dtype=dtype).element_size()
        return cls._make(None, numel * es, False, comm, es, dtype, info)

    Allocate_shared = Allocate

    # ------------------------------------------------------------ data movement
    def _stream(self):
        if _rt.device() is not None:
            return torch.cuda.current_stream().cuda_stream
        return 0

    def Put(self, origin: torch.Tensor, target_rank: int, target_disp: int = 0):
        o = origin.contiguous().reshape(-1)
        self._w.put(target_rank, target_disp * self.disp_unit, o.data_ptr(), o.numel() * o.element_size(), self._stream())
        self._keep = o

    def Get(self, origin: torch.Tensor, target_rank: int, target_disp: int = 0):
        if not origin.is_contiguous():
            raise ValueError("Get needs a contiguous origin buffer")
        self._w.get(origin.data_ptr(), target_rank, target_disp * self.disp_unit,
                    origin.numel() * origin.element_size(), self._stream())

    def Accumulate(self, origin: torch.Tensor, target_rank: int, target_disp: int = 0, op=None):
        """target += origin (SUM) or target = origin (REPLACE); fp32/bf16. Atomic with
        respect to other Accumulates on the same target (exclusive target lock)."""
        from .comm import REPLACE, SUM

        op = op or SUM
        o = origin.contiguous().reshape(-1)
        if o.dtype not in (torch.float32, torch.bfloat16):
            raise TypeError("Accumulate supports float32 / bfloat16")
        if op is SUM:
            a, b = 1.0, 1.0
        elif op is REPLACE:
            a, b = 1.0, 0.0
        else:
            raise ValueError("Accumulate supports SUM and REPLACE")
        self._w.accumulate(target_rank, target_disp * self.disp_unit, o.data_ptr(), o.is_cuda, o.numel(),
                           o.dtype == torch.bfloat16, a, b, self._stream())

    # byte-addressed forms (the datatype-faithful Put / Get / Accumulate of mpiT.py): one
    # copy / accumulate per contiguous run of the target datatype
    def _put_bytes(self, data: torch.Tensor, target_rank: int, byte_disp: int):
        self._w.put(target_rank, int(byte_disp), data.data_ptr(), data.numel(), self._stream())
        self._keep_all = getattr(self, "_keep_all", [])
        self._keep_all.append(data)

    def _get_bytes(self, out: torch.Tensor, target_rank: int, byte_disp: int):
        self._w.get(out.data_ptr(), target_rank, int(byte_disp), out.numel() * out.element_size(), self._stream())

    def _acc_elems(self, data: torch.Tensor, target_rank: int, byte_disp: int, a: float, b: float):
        self._w.accumulate(target_rank, int(byte_disp), data.data_ptr(), data.is_cuda, data.numel(),
                           data.dtype == torch.bfloat16, a, b, self._stream())
        self._keep_all = getattr(self, "_keep_all", [])
        self._keep_all.append(data)

    def Raccumulate(self, *a, **k):
        from .comm import Request

        self.Accumulate(*a, **k)
        return Request(self.comm)

    def Rput(self, *a, **k):
        from .comm import Request

        self.Put(*a, **k)
        return Request(self.comm)

    def Rget(self, *a, **k):
        from .comm import Request

        self.Get(*a, **k)
        return Request(self.comm)

    # ------------------------------------------------------------ synchronisation
    def _flush(self):
        # every epoch-closing synchronisation completes the origin reads of the queued copies:
        # the origin buffers held for them (_put_bytes / _acc_elems) are released here, so a
        # Fence- or Unlock-synchronised Put loop keeps only the current epoch's origins alive
        self._w.flush(self._stream())
        self._keep_all = []

    def Flush(self, rank: Optional[int] = None):
        self._flush()

    Flush_all = Flush
    Flush_local = Flush
    Flush_local_all = Flush
    Sync = Flush

    def Fence(self, assertion: int = 0):
        self._flush()
        self.comm.Barrier()

    def Lock(self, rank: int, lock_type: int = LOCK_EXCLUSIVE, assertion: int = 0):
        self._w.lock(rank, lock_type == LOCK_EXCLUSIVE)

    def Unlock(self, rank: int):
        self._flush()
        self._w.unlock(rank)

    def Lock_all(self, assertion: int = 0):
        for r in range(self.comm.Get_size()):
            self._w.lock(r, False)

    def Unlock_all(self):
        self._flush()
        for r in range(self.comm.Get_size()):
            self._w.unlock(r)

    # PSCW: exposure epoch (Post/Wait) on the target, access epoch (Start/Complete) on the origin
    def Post(self, group, assertion: int = 0):
        z = torch.zeros(1, dtype=torch.uint8)
        self._posted = [self.comm._csend(z, self.comm._from_world(w), 31) for w in group.world_ranks]
        self._post_group = group

    def Start(self, group, assertion: int = 0):
        z = torch.zeros(1, dtype=torch.uint8)
        for w in group.world_ranks:
            self.comm._crecv(z, self.comm._from_world(w), 31).Wait()
        self._epoch_targets = list(group.world_ranks)

    def Complete(self):
        self._flush()
        z = torch.zeros(1, dtype=torch.uint8)
        for w in self._epoch_targets:
            self.comm._csend(z, self.comm._from_world(w), 32).Wait()
        self._epoch_targets = []

    def Wait(self):
        z = torch.zeros(1, dtype=torch.uint8)
        for r in getattr(self, "_posted", []):
            r.Wait()
        for w in self._post_group.world_ranks:
            self.comm._crecv(z, self.comm._from_world(w), 32).Wait()

    def Test(self) -> bool:
        self.Wait()
        return True

    # ------------------------------------------------------------ misc
    def Get_group(self):
        return self.comm.Get_group()

    def Get_attr(self, k):
        return self._attrs.get(k)

    def Set_attr(self, k, v):
        self._attrs[k] = v

    def Delete_attr(self, k):
        self._attrs.pop(k, None)

    def Get_name(self):
        return self._name

    def Set_name(self, n):
        self._name = n

    def Set_errhandler(self, eh):
        self._errhandler = eh

    def Get_errhandler(self):
        return self._errhandler

    def Call_errhandler(self, code):
        if self._errhandler:
            self._errhandler(self, code)

    def remote_ptr(self, rank: int) -> int:
        return self._w.remote_ptr(rank)

    def Free(self):
        if self._w is not None:
            try:
                self._w.flush(self._stream())
            except Exception:
                pass
            self._w = None
            self.tensor = None

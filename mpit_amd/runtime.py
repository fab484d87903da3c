"""Process-level runtime state: Init / Finalize, the native engine, device binding.

Replaces ``mpiT.Init`` / ``Init_MTF/MTS/MTM`` / ``Finalize`` (lua-mpi.h:80-121,
mpifuncs.c:1081) for the one-process-per-GPU MI355X node:

* ranks come from the launcher's environment (``RANK``/``WORLD_SIZE``/``LOCAL_RANK``, as
  set by ``torch.distributed.run`` or :mod:`mpit_amd.launch`); a bare ``python x.py`` is a
  world of one;
* rank r binds HIP device ``LOCAL_RANK % device_count``;
* ``torch.distributed`` is initialised with ``cpu:gloo,cuda:nccl`` (RCCL on ROCm) for the
  collectives on HBM tensors, and is also used once to agree on the name of the node's
  shared-memory segment;
* the native :class:`Engine` (csrc/core/engine.cpp) owns that segment and a progress
  thread; every point-to-point, window and parameter-server operation goes through it.
"""
from __future__ import annotations

import atexit
import os
import socket
import threading
import time
import uuid
from dataclasses import dataclass, field
from typing import Optional

import torch

from ._ext import native

THREAD_SINGLE, THREAD_FUNNELED, THREAD_SERIALIZED, THREAD_MULTIPLE = 0, 1, 2, 3


@dataclass
class _State:
    initialized: bool = False
    finalized: bool = False
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: Optional[torch.device] = None
    engine: object = None
    thread_level: int = THREAD_MULTIPLE
    main_thread: int = 0
    dist_owner: bool = False
    shared_devices: bool = False  # some ranks share one GPU (1-GPU rehearsal of N ranks)
    device_map: list = field(default_factory=list)
    next_ctx: int = 16
    windows: int = 0
    t0: float = 0.0


_S = _State()
_lock = threading.Lock()


def _env_int(*names, default=None):
    for n in names:
        v = os.environ.get(n)
        if v not in (None, ""):
            return int(v)
    return default


def state() -> _State:
    if not _S.initialized:
        raise RuntimeError("mpit is not initialised: call mpit_amd.Init() first")
    return _S


def engine():
    return state().engine


def Init(thread_level: int = THREAD_MULTIPLE, device: Optional[object] = "auto", bulk_bytes: int = 4 << 20,
         dist_backend: Optional[str] = "auto") -> int:
    """Join the job. Returns the provided thread level (always THREAD_MULTIPLE: the
    engine is internally synchronised, so the MTF/MTS/MTM variants of the reference
    — lua-mpi.h:87-121 — all succeed)."""
    with _lock:
        if _S.initialized:
            return _S.thread_level
        rank = _env_int("RANK", "OMPI_COMM_WORLD_RANK", "PMI_RANK", default=0)
        world = _env_int("WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE", default=1)
        local_rank = _env_int("LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", default=rank)
        dev = None
        if device == "auto":
            if os.environ.get("MPIT_CPU_ONLY") != "1" and torch.cuda.is_available():
                dev = torch.device("cuda", local_rank % torch.cuda.device_count())
        elif device is not None and device is not False:
            dev = torch.device(device)
        if dev is not None and dev.type == "cuda":
            torch.cuda.set_device(dev)
        # bootstrap: agree on the segment name
        import torch.distributed as dist

        name = f"/mpit_{os.getpid()}_{uuid.uuid4().hex[:10]}"
        if world > 1:
            if not dist.is_initialized():
                backend = dist_backend
                if backend == "auto":
                    backend = "cpu:gloo,cuda:nccl" if dev is not None else "gloo"
                os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
                dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                        device_id=None)
                _S.dist_owner = True
            obj = [name]
            dist.broadcast_object_list(obj, src=0)
            name = obj[0]
        eng = native().Engine(name, world, rank, rank == 0, dev.index if dev is not None else -1, int(bulk_bytes))
        # every rank attached -> the name can go (no /dev/shm leak even if a rank dies)
        eng.barrier()
        if rank == 0:
            eng.unlink()
        host = socket.gethostname()
        import pickle

        infos = [pickle.loads(b) for b in eng.allgather_small(pickle.dumps((host, dev.index if dev is not None else -1)))]
        _S.device_map = infos
        devs = [i for i in infos if i[1] >= 0]
        _S.shared_devices = len(set(devs)) != len(devs)
        _S.rank, _S.world, _S.local_rank = rank, world, local_rank
        _S.device, _S.engine = dev, eng
        _S.thread_level = thread_level
        _S.main_thread = threading.get_ident()
        _S.initialized, _S.finalized = True, False
        _S.t0 = time.perf_counter()
        atexit.register(_atexit)
        return THREAD_MULTIPLE


def Init_thread(required: int = THREAD_MULTIPLE, **kw) -> int:
    return Init(thread_level=required, **kw)


def Initialized() -> bool:
    return _S.initialized


def Finalized() -> bool:
    return _S.finalized


def Finalize():
    """Leave the job: drain, barrier, stop the progress thread."""
    with _lock:
        if not _S.initialized or _S.finalized:
            return
        eng = _S.engine
        try:
            eng.barrier()
        finally:
            from . import window as _w

            _w._close_all()
            eng.shutdown()
            import torch.distributed as dist

            if _S.dist_owner and dist.is_initialized():
                try:
                    dist.destroy_process_group()
                except Exception:
                    pass
            _S.finalized = True
            _S.initialized = False
            _S.engine = None


def _atexit():
    if _S.initialized and not _S.finalized:
        try:
            _S.engine.shutdown()
        except Exception:
            pass


def Abort(code: int = 1):
    """Terminate every rank of the job (shm abort flag seen by all progress threads)."""
    if _S.initialized:
        _S.engine.abort(int(code))
    os._exit(int(code) or 1)


def Wtime() -> float:
    return time.perf_counter()


def Wtick() -> float:
    return time.get_clock_info("perf_counter").resolution


def Get_processor_name() -> str:
    return socket.gethostname()


def Get_version():
    """(major, minor) of the MPI standard subset mirrored (MPI-3.1 semantics)."""
    return (3, 1)


def Query_thread() -> int:
    return state().thread_level


def Is_thread_main() -> bool:
    return threading.get_ident() == state().main_thread


def device() -> Optional[torch.device]:
    return _S.device


def alloc_ctx(n: int = 1) -> int:
    """Reserve local context ids (made collective by the communicator constructors)."""
    c = _S.next_ctx
    _S.next_ctx += n
    return c

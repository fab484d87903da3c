"""mpit_amd — an MI355X-native framework with the capabilities of mpiT (MPI for Torch).

MPI-style API (``Init``, ``COMM_WORLD()``, ``Isend``/``Irecv``/``Iprobe``/``Test``/``Cancel``,
collectives, groups, windows) over a native C++ runtime (node shm control plane + HIP IPC
over xGMI + RCCL), a sharded asynchronous parameter server (pServer / pClient), the
Downpour / EASGD / EAMSGD / adaptive distributed optimizers, and fused CDNA4 HIP kernels
for every update rule. See README.md and SURVEY.md.
"""
from . import comm as _comm
from .comm import (
    ANY_SOURCE,
    ANY_TAG,
    BAND,
    BOR,
    BXOR,
    CONGRUENT,
    IDENT,
    LAND,
    LOR,
    LXOR,
    MAX,
    MAXLOC,
    MIN,
    MINLOC,
    NO_OP,
    PROC_NULL,
    PROD,
    REPLACE,
    ROOT,
    SIMILAR,
    SUCCESS,
    SUM,
    UNDEFINED,
    UNEQUAL,
    Comm,
    Grequest_complete,
    Grequest_start,
    Op,
    Op_create,
    Reduce_local,
    Request,
    Status,
)
from .group import GROUP_EMPTY, Group
from .runtime import (
    THREAD_FUNNELED,
    THREAD_MULTIPLE,
    THREAD_SERIALIZED,
    THREAD_SINGLE,
    Abort,
    Finalize,
    Finalized,
    Get_processor_name,
    Get_version,
    Init,
    Init_thread,
    Initialized,
    Is_thread_main,
    Query_thread,
    Wtick,
    Wtime,
)
from .window import LOCK_EXCLUSIVE, LOCK_SHARED, Win

from . import datatypes, misc, ops, optim, parallel, topology  # noqa: E402

__version__ = "0.1.0"


def COMM_WORLD() -> Comm:
    return _comm.COMM_WORLD()


def COMM_SELF() -> Comm:
    return _comm.COMM_SELF()


def get_rank(comm=None) -> int:
    """mpiT.get_rank (init.lua:28-32)."""
    return (comm or COMM_WORLD()).Get_rank()


def get_size(comm=None) -> int:
    """mpiT.get_size (init.lua:34-38)."""
    return (comm or COMM_WORLD()).Get_size()


def Init_MTF():
    return Init_thread(THREAD_FUNNELED)


def Init_MTS():
    return Init_thread(THREAD_SERIALIZED)


def Init_MTM():
    return Init_thread(THREAD_MULTIPLE)


def Waitall(reqs, statuses=None):
    return Request.Waitall(reqs, statuses)


def Waitany(reqs, status=None):
    return Request.Waitany(reqs, status)


def Waitsome(reqs, statuses=None):
    return Request.Waitsome(reqs, statuses)


def Testall(reqs, statuses=None):
    return Request.Testall(reqs, statuses)


def Testany(reqs, status=None):
    return Request.Testany(reqs, status)


def Testsome(reqs, statuses=None):
    return Request.Testsome(reqs, statuses)


def Startall(reqs):
    for r in reqs:
        r.Start()
    return reqs

"""Info objects, error classes / handlers, attribute key values, memory allocation,
buffered-send buffers, profiling control.

Reference: lua-mpi.h:210-230 (21 error classes), mpifuncs.c Info_* (9), Add_error_* /
Error_* / *_errhandler (environmental management), *_keyval / *_attr (caching),
Alloc_mem / Free_mem, Buffer_attach / Buffer_detach, and MPI_Pcontrol (skipped by the
reference's generator, readspec.py:73 — here it toggles roctx tracing).
"""
from __future__ import annotations

import itertools
from collections import OrderedDict
from typing import Callable, Optional

import torch

# ------------------------------------------------------------------ error classes
SUCCESS = 0
ERR_BUFFER, ERR_COUNT, ERR_TYPE, ERR_TAG, ERR_COMM, ERR_RANK, ERR_ROOT, ERR_GROUP = 1, 2, 3, 4, 5, 6, 7, 8
ERR_OP, ERR_TOPOLOGY, ERR_DIMS, ERR_ARG, ERR_UNKNOWN, ERR_TRUNCATE, ERR_OTHER, ERR_INTERN = 9, 10, 11, 12, 13, 15, 16, 17
ERR_IN_STATUS, ERR_PENDING, ERR_REQUEST = 18, 19, 20
ERR_LASTCODE = 92

_ERR_STRINGS = {
    SUCCESS: "MPI_SUCCESS: no errors", ERR_BUFFER: "MPI_ERR_BUFFER: invalid buffer pointer",
    ERR_COUNT: "MPI_ERR_COUNT: invalid count argument", ERR_TYPE: "MPI_ERR_TYPE: invalid datatype",
    ERR_TAG: "MPI_ERR_TAG: invalid tag", ERR_COMM: "MPI_ERR_COMM: invalid communicator",
    ERR_RANK: "MPI_ERR_RANK: invalid rank", ERR_ROOT: "MPI_ERR_ROOT: invalid root",
    ERR_GROUP: "MPI_ERR_GROUP: invalid group", ERR_OP: "MPI_ERR_OP: invalid reduce operation",
    ERR_TOPOLOGY: "MPI_ERR_TOPOLOGY: invalid communicator topology", ERR_DIMS: "MPI_ERR_DIMS: invalid dimension argument",
    ERR_ARG: "MPI_ERR_ARG: invalid argument of some other kind", ERR_UNKNOWN: "MPI_ERR_UNKNOWN: unknown error",
    ERR_TRUNCATE: "MPI_ERR_TRUNCATE: message truncated", ERR_OTHER: "MPI_ERR_OTHER: known error not in this list",
    ERR_INTERN: "MPI_ERR_INTERN: internal error", ERR_IN_STATUS: "MPI_ERR_IN_STATUS: error code is in status",
    ERR_PENDING: "MPI_ERR_PENDING: pending request", ERR_REQUEST: "MPI_ERR_REQUEST: invalid request",
}
_err_class_of = {}
_next_class = itertools.count(ERR_LASTCODE + 1)
_next_code = itertools.count(1000)


class MPIError(RuntimeError):
    def __init__(self, code: int, msg: str = ""):
        super().__init__(msg or Error_string(code))
        self.code = code

    def Get_error_class(self):
        return Error_class(self.code)

    def Get_error_code(self):
        return self.code


def Error_string(code: int) -> str:
    return _ERR_STRINGS.get(code, f"MPI error code {code}")


def Error_class(code: int) -> int:
    return _err_class_of.get(code, code if code in _ERR_STRINGS else ERR_UNKNOWN)


def Add_error_class() -> int:
    c = next(_next_class)
    _ERR_STRINGS[c] = f"user error class {c}"
    return c


def Add_error_code(errorclass: int) -> int:
    c = next(_next_code)
    _err_class_of[c] = errorclass
    return c


def Add_error_string(code: int, string: str):
    _ERR_STRINGS[code] = string


class Errhandler:
    def __init__(self, fn: Optional[Callable] = None, name: str = "user"):
        self.fn, self.name = fn, name

    def __call__(self, obj, code):
        if self.fn is not None:
            self.fn(obj, code)

    def Free(self):
        pass


def _fatal(obj, code):
    raise MPIError(code)


ERRORS_ARE_FATAL = Errhandler(_fatal, "ERRORS_ARE_FATAL")
ERRORS_RETURN = Errhandler(None, "ERRORS_RETURN")
ERRHANDLER_NULL = None


def Comm_create_errhandler(fn) -> Errhandler:
    return Errhandler(fn)


Win_create_errhandler = File_create_errhandler = Comm_create_errhandler


def Errhandler_free(eh: Errhandler):
    eh.Free()


def Comm_set_errhandler(comm, eh):
    comm.Set_errhandler(eh)


def Comm_get_errhandler(comm):
    return comm.Get_errhandler()


def Comm_call_errhandler(comm, code):
    comm.Call_errhandler(code)


# ------------------------------------------------------------------ Info
class Info:
    def __init__(self, items=None):
        self._d = OrderedDict(items or {})

    def Set(self, key: str, value: str):
        self._d[str(key)] = str(value)

    def Get(self, key: str, valuelen: Optional[int] = None):
        v = self._d.get(key)
        if v is not None and valuelen is not None:
            v = v[:valuelen]
        return v

    def Delete(self, key: str):
        if key not in self._d:
            raise MPIError(ERR_ARG, f"Info key {key!r} not set")
        del self._d[key]

    def Get_nkeys(self) -> int:
        return len(self._d)

    def Get_nthkey(self, n: int) -> str:
        return list(self._d)[n]

    def Get_valuelen(self, key: str):
        v = self._d.get(key)
        return (len(v), True) if v is not None else (0, False)

    def Dup(self) -> "Info":
        return Info(self._d)

    def Free(self):
        self._d.clear()

    def items(self):
        return self._d.items()


INFO_NULL = None


def Info_create() -> Info:
    return Info()


# ------------------------------------------------------------------ attribute caching
KEYVAL_INVALID = -1
TAG_UB, HOST, IO, WTIME_IS_GLOBAL = 0, 1, 2, 3  # predefined attribute keys
_keyvals = {}
_next_key = itertools.count(100)


def _create_keyval(copy_fn=None, delete_fn=None, extra_state=None) -> int:
    k = next(_next_key)
    _keyvals[k] = (copy_fn, delete_fn, extra_state)
    return k


Comm_create_keyval = Type_create_keyval = Win_create_keyval = _create_keyval


def _free_keyval(k: int) -> int:
    _keyvals.pop(k, None)
    return KEYVAL_INVALID


Comm_free_keyval = Type_free_keyval = Win_free_keyval = _free_keyval


def Comm_set_attr(obj, k, v):
    obj.Set_attr(k, v)


def Comm_get_attr(obj, k):
    return obj.Get_attr(k)


def Comm_delete_attr(obj, k):
    cb = _keyvals.get(k, (None, None, None))[1]
    if cb is not None:
        cb(obj, k, obj.Get_attr(k), _keyvals[k][2])
    obj.Delete_attr(k)


Type_set_attr = Win_set_attr = Comm_set_attr
Type_get_attr = Win_get_attr = Comm_get_attr
Type_delete_attr = Win_delete_attr = Comm_delete_attr


# ------------------------------------------------------------------ memory
def Alloc_mem(nbytes: int, info: Optional[Info] = None, device: Optional[bool] = None) -> torch.Tensor:
    """Page-locked host memory (fast DMA to HBM) or, with device=True, HBM."""
    if device:
        from . import runtime as _rt

        return torch.empty(nbytes, dtype=torch.uint8, device=_rt.device())
    t = torch.empty(nbytes, dtype=torch.uint8)
    if torch.cuda.is_available():
        t = t.pin_memory()
    return t


def Free_mem(t: torch.Tensor):
    del t


_attached = [None]


def Buffer_attach(buf: torch.Tensor):
    """Bsend buffer: accepted for API parity — sends complete into the shm rings, so no
    user buffer space is consumed."""
    _attached[0] = buf


def Buffer_detach():
    b, _attached[0] = _attached[0], None
    return b


# ------------------------------------------------------------------ profiling control
_pcontrol = [1]


def Pcontrol(level: int):
    """0 disables, >=1 enables the framework's roctx ranges / timers (utils.trace)."""
    _pcontrol[0] = int(level)
    from .utils import trace

    trace.enable(level > 0)


def pcontrol_level() -> int:
    return _pcontrol[0]

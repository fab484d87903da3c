"""mpiT-style functional API: the reference's function names with MPI-C argument order.

The reference binds 262 MPI functions (mpifuncs.c:2514-2777) as
``mpiT.<Name>(storage, count, datatype, ...)`` plus Lua helpers (init.lua). This module
offers the same names over the mpit_amd runtime so reference code ports line by line:

* buffers are torch tensors (host or HBM), ``count`` elements of ``datatype`` are used
  (derived datatypes are packed / unpacked);
* output arguments are *returned* (requests, statuses, ranks, new communicators ...)
  instead of written into pre-allocated Lua userdata;
* errors raise :class:`~mpit_amd.misc.MPIError` (the reference returned codes and every
  caller ignored them); calls that succeed return ``SUCCESS`` where MPI returns only a code.

Lua-level helpers of init.lua are here too: ``get_rank``/``get_size``, ``aio_send`` /
``aio_recv``, ``co_execute`` / ``co_ping`` / ``co_wait`` (a cooperative scheduler over Python
generators, R5), ``Queue`` (R6), ``serialize`` / ``deserialize`` (R4) and the ``signal_*``
constants, and the PS tags ``tag_ps_*`` of asyncsgd/init.lua:3-10.
"""
from __future__ import annotations

from collections import deque
from typing import Optional

import torch

from . import comm as _c
from . import datatypes as _dt
from . import dynamic as _dyn
from . import group as _g
from . import io as _io
from . import misc as _m
from . import runtime as _rt
from . import topology as _topo
from .parallel.ps import (tag_ps_recv_grad, tag_ps_recv_grad_tail, tag_ps_recv_header, tag_ps_recv_init,  # noqa: F401
                          tag_ps_recv_param, tag_ps_recv_param_tail, tag_ps_recv_stop, tag_ps_send_param)
from .utils.serialize import deserialize, serialize  # noqa: F401
from .window import LOCK_EXCLUSIVE, LOCK_SHARED, Win  # noqa: F401

SUCCESS = 0
# ---------------------------------------------------------------- constants (lua-mpi.h:125-231)
from .datatypes import (BYTE, CHAR, DOUBLE, DOUBLE_INT, FLOAT, FLOAT_INT, INT, LB, LONG, LONG_DOUBLE,  # noqa: E402,F401
                        LONG_DOUBLE_INT, LONG_INT, LONG_LONG_INT, PACKED, SHORT, SHORT_INT, TWOINT, UB, UNSIGNED,
                        UNSIGNED_CHAR, UNSIGNED_LONG, UNSIGNED_SHORT)
from .comm import (ANY_SOURCE, ANY_TAG, BAND, BOR, BXOR, CONGRUENT, IDENT, LAND, LOR, LXOR, MAX, MAXLOC, MIN,  # noqa: E402,F401
                   MINLOC, PROC_NULL, PROD, ROOT, SIMILAR, SUM, UNDEFINED, UNEQUAL)
from .misc import (ERR_ARG, ERR_BUFFER, ERR_COMM, ERR_COUNT, ERR_DIMS, ERR_GROUP, ERR_IN_STATUS,  # noqa: E402,F401
                   ERR_INTERN, ERR_LASTCODE, ERR_OP, ERR_OTHER, ERR_PENDING, ERR_RANK, ERR_REQUEST, ERR_ROOT,
                   ERR_TAG, ERR_TOPOLOGY, ERR_TRUNCATE, ERR_TYPE, ERR_UNKNOWN, KEYVAL_INVALID)
from .topology import CART, GRAPH  # noqa: E402,F401

globals()["2INT"] = TWOINT
MAX_PROCESSOR_NAME = 256
MAX_ERROR_STRING = 256
MAX_OBJECT_NAME = 64
COMM_NULL = OP_NULL = GROUP_NULL = DATATYPE_NULL = REQUEST_NULL = ERRHANDLER_NULL = INFO_NULL = None
GROUP_EMPTY = _g.GROUP_EMPTY
ERRORS_ARE_FATAL, ERRORS_RETURN = _m.ERRORS_ARE_FATAL, _m.ERRORS_RETURN


def __getattr__(name):
    # COMM_WORLD / COMM_SELF resolve after Init (lua-mpi.h:194-195)
    if name == "COMM_WORLD":
        return _c.COMM_WORLD()
    if name == "COMM_SELF":
        return _c.COMM_SELF()
    raise AttributeError(name)


def _buf(buf, count, datatype):
    """(tensor, count, datatype) -> (tensor or packed bytes, count for the comm layer)."""
    return buf, (None if count is None else int(count)), datatype if (datatype is not None and not datatype.is_contiguous_basic()) else None


# ---------------------------------------------------------------- environment (N4, R1)
Init = _rt.Init
Initialized = _rt.Initialized
Finalize = _rt.Finalize
Finalized = _rt.Finalized
Abort = lambda comm=None, errorcode=1: _rt.Abort(errorcode)  # noqa: E731
Wtime, Wtick = _rt.Wtime, _rt.Wtick
Get_processor_name = _rt.Get_processor_name
Get_version = _rt.Get_version
Query_thread = _rt.Query_thread
Is_thread_main = _rt.Is_thread_main


def Init_thread(required=_rt.THREAD_MULTIPLE):
    return _rt.Init_thread(required)


def Init_MTF():
    return _rt.Init_thread(_rt.THREAD_FUNNELED)


def Init_MTS():
    return _rt.Init_thread(_rt.THREAD_SERIALIZED)


def Init_MTM():
    return _rt.Init_thread(_rt.THREAD_MULTIPLE)


def get_rank(comm=None):
    return (comm or _c.COMM_WORLD()).Get_rank()


def get_size(comm=None):
    return (comm or _c.COMM_WORLD()).Get_size()


Comm_rank = lambda comm: comm.Get_rank()  # noqa: E731
Comm_size = lambda comm: comm.Get_size()  # noqa: E731

# errors / handlers / memory / buffers / profiling
Error_class, Error_string = _m.Error_class, _m.Error_string
Add_error_class, Add_error_code, Add_error_string = _m.Add_error_class, _m.Add_error_code, _m.Add_error_string
Comm_create_errhandler, Win_create_errhandler, File_create_errhandler = (_m.Comm_create_errhandler,) * 3
Errhandler_free = _m.Errhandler_free
Comm_set_errhandler, Comm_get_errhandler, Comm_call_errhandler = (_m.Comm_set_errhandler, _m.Comm_get_errhandler,
                                                                  _m.Comm_call_errhandler)
Win_set_errhandler = lambda w, eh: w.Set_errhandler(eh)  # noqa: E731
Win_get_errhandler = lambda w: w.Get_errhandler()  # noqa: E731
Win_call_errhandler = lambda w, code: w.Call_errhandler(code)  # noqa: E731
File_set_errhandler = lambda f, eh: f.Set_errhandler(eh)  # noqa: E731
File_get_errhandler = lambda f: f.Get_errhandler()  # noqa: E731
File_call_errhandler = lambda f, code: f.Call_errhandler(code)  # noqa: E731
Alloc_mem, Free_mem = _m.Alloc_mem, _m.Free_mem
Buffer_attach, Buffer_detach = _m.Buffer_attach, _m.Buffer_detach
Pcontrol = _m.Pcontrol

# ---------------------------------------------------------------- point-to-point


def Send(buf, count, datatype, dest, tag, comm):
    comm.Send(buf, dest, tag, count=count, datatype=_buf(buf, count, datatype)[2])
    return SUCCESS


# buffered / ready sends are standard sends on this engine (see Comm.Ibsend)
Bsend = Rsend = Send


def Ssend(buf, count, datatype, dest, tag, comm):
    comm.Ssend(buf, dest, tag, count=count, datatype=_buf(buf, count, datatype)[2])
    return SUCCESS


def Recv(buf, count, datatype, source, tag, comm, status=None):
    return comm.Recv(buf, source, tag, status, count=count, datatype=_buf(buf, count, datatype)[2])


def Isend(buf, count, datatype, dest, tag, comm):
    return comm.Isend(buf, dest, tag, count=count, datatype=_buf(buf, count, datatype)[2])


Ibsend = Irsend = Isend  # see Bsend


def Issend(buf, count, datatype, dest, tag, comm):
    return comm.Issend(buf, dest, tag, count=count, datatype=_buf(buf, count, datatype)[2])


def Irecv(buf, count, datatype, source, tag, comm):
    return comm.Irecv(buf, source, tag, count=count, datatype=_buf(buf, count, datatype)[2])


def Sendrecv(sendbuf, sendcount, sendtype, dest, sendtag, recvbuf, recvcount, recvtype, source, recvtag, comm, status=None):
    _, sc, st = _buf(sendbuf, sendcount, sendtype)
    _, rc, rt = _buf(recvbuf, recvcount, recvtype)
    return comm.Sendrecv(sendbuf, dest, sendtag, recvbuf, source, recvtag, status, sc, st, rc, rt)


def Sendrecv_replace(buf, count, datatype, dest, sendtag, source, recvtag, comm, status=None):
    _, c, dt = _buf(buf, count, datatype)
    return comm.Sendrecv_replace(buf, dest, sendtag, source, recvtag, status, c, dt)


def Send_init(buf, count, datatype, dest, tag, comm):
    _, c, dt = _buf(buf, count, datatype)
    return comm.Send_init(buf, dest, tag, c, dt)


Bsend_init = Rsend_init = Send_init


def Ssend_init(buf, count, datatype, dest, tag, comm):
    _, c, dt = _buf(buf, count, datatype)
    return comm.Ssend_init(buf, dest, tag, c, dt)


def Recv_init(buf, count, datatype, source, tag, comm):
    _, c, dt = _buf(buf, count, datatype)
    return comm.Recv_init(buf, source, tag, c, dt)


def Start(request):
    request.Start()
    return SUCCESS


def Startall(requests):
    for r in requests:
        r.Start()
    return SUCCESS


def Iprobe(source, tag, comm, status=None):
    return comm.Iprobe(source, tag, status)


def Probe(source, tag, comm, status=None):
    return comm.Probe(source, tag, status)


def Test(request, status=None):
    return request.Test(status)


def Wait(request, status=None):
    return request.Wait(status)


def Cancel(request):
    request.Cancel()
    return SUCCESS


def Test_cancelled(status):
    return status.Is_cancelled()


def Request_free(request):
    request.Free()
    return SUCCESS


def Request_get_status(request, status=None):
    return request.Get_status(status)


def Get_count(status, datatype):
    return status.Get_count(datatype)


Get_elements = _dt.Get_elements
Testall, Waitall = _c.Request.Testall, _c.Request.Waitall
Testany, Waitany = _c.Request.Testany, _c.Request.Waitany
Testsome, Waitsome = _c.Request.Testsome, _c.Request.Waitsome
Grequest_start, Grequest_complete = _c.Grequest_start, _c.Grequest_complete


def Status_set_cancelled(status, flag):
    status.Set_cancelled(flag)
    return SUCCESS


def Status_set_elements(status, datatype, count):
    status.Set_elements(datatype, count)
    return SUCCESS


# ---------------------------------------------------------------- collectives


def Barrier(comm):
    comm.Barrier()
    return SUCCESS


def Bcast(buf, count, datatype, root, comm):
    comm.Bcast(buf if count is None else buf.reshape(-1)[:count], root)
    return SUCCESS


def Reduce(sendbuf, recvbuf, count, datatype, op, root, comm):
    comm.Reduce(sendbuf.reshape(-1)[:count], recvbuf.reshape(-1)[:count] if recvbuf is not None else None, op, root)
    return SUCCESS


def Allreduce(sendbuf, recvbuf, count, datatype, op, comm):
    """mpifuncs.c:83 — ``sendbuf is recvbuf`` works as MPI_IN_PLACE."""
    s = sendbuf.reshape(-1)[:count]
    r = recvbuf.reshape(-1)[:count]
    comm.Allreduce(s, r, op)
    return SUCCESS


def Iallreduce(sendbuf, recvbuf, count, datatype, op, comm):
    return comm.Iallreduce(sendbuf.reshape(-1)[:count], recvbuf.reshape(-1)[:count], op)


def Gather(sendbuf, sendcount, sendtype, recvbuf, recvcount, recvtype, root, comm):
    comm.Gather(sendbuf.reshape(-1)[:sendcount], recvbuf, root)
    return SUCCESS


def Gatherv(sendbuf, sendcount, sendtype, recvbuf, recvcounts, displs, recvtype, root, comm):
    comm.Gatherv(sendbuf.reshape(-1)[:sendcount], recvbuf, recvcounts, displs, root)
    return SUCCESS


def Scatter(sendbuf, sendcount, sendtype, recvbuf, recvcount, recvtype, root, comm):
    comm.Scatter(sendbuf, recvbuf.reshape(-1)[:recvcount], root)
    return SUCCESS


def Scatterv(sendbuf, sendcounts, displs, sendtype, recvbuf, recvcount, recvtype, root, comm):
    comm.Scatterv(sendbuf, recvbuf.reshape(-1)[:recvcount], sendcounts, displs, root)
    return SUCCESS


def Allgather(sendbuf, sendcount, sendtype, recvbuf, recvcount, recvtype, comm):
    comm.Allgather(sendbuf.reshape(-1)[:sendcount], recvbuf)
    return SUCCESS


def Allgatherv(sendbuf, sendcount, sendtype, recvbuf, recvcounts, displs, recvtype, comm):
    comm.Allgatherv(sendbuf.reshape(-1)[:sendcount], recvbuf, recvcounts, displs)
    return SUCCESS


def Alltoall(sendbuf, sendcount, sendtype, recvbuf, recvcount, recvtype, comm):
    comm.Alltoall(sendbuf, recvbuf)
    return SUCCESS


def Alltoallv(sendbuf, sendcounts, sdispls, sendtype, recvbuf, recvcounts, rdispls, recvtype, comm):
    comm.Alltoallv(sendbuf, sendcounts, sdispls, recvbuf, recvcounts, rdispls)
    return SUCCESS


def Alltoallw(sendbufs, recvbufs, comm):
    comm.Alltoallw(sendbufs, recvbufs)
    return SUCCESS


def Reduce_scatter(sendbuf, recvbuf, recvcounts, datatype, op, comm):
    comm.Reduce_scatter(sendbuf, recvbuf, recvcounts, op)
    return SUCCESS


def Scan(sendbuf, recvbuf, count, datatype, op, comm):
    comm.Scan(sendbuf.reshape(-1)[:count], recvbuf.reshape(-1)[:count], op)
    return SUCCESS


def Exscan(sendbuf, recvbuf, count, datatype, op, comm):
    comm.Exscan(sendbuf.reshape(-1)[:count], recvbuf.reshape(-1)[:count], op)
    return SUCCESS


Op_create = _c.Op_create
Reduce_local = _c.Reduce_local


def Op_free(op):
    op.Free()
    return SUCCESS


def Op_commutative(op):
    return op.Is_commutative()


# ---------------------------------------------------------------- groups / communicators
Comm_group = lambda comm: comm.Get_group()  # noqa: E731
Comm_dup = lambda comm: comm.Dup()  # noqa: E731
Comm_create = lambda comm, group: comm.Create(group)  # noqa: E731
Comm_split = lambda comm, color, key: comm.Split(color, key)  # noqa: E731
Comm_compare = lambda a, b: a.Compare(b)  # noqa: E731
Comm_free = lambda comm: comm.Free()  # noqa: E731
Comm_get_name = lambda comm: comm.Get_name()  # noqa: E731
Comm_set_name = lambda comm, name: comm.Set_name(name)  # noqa: E731
Comm_test_inter = _dyn.Comm_test_inter
Comm_remote_size, Comm_remote_group = _dyn.Comm_remote_size, _dyn.Comm_remote_group
Intercomm_create, Intercomm_merge = _dyn.Intercomm_create, _dyn.Intercomm_merge
Group_size = lambda g: g.Get_size()  # noqa: E731
Group_rank = lambda g: g.Get_rank()  # noqa: E731
Group_incl = lambda g, ranks: g.Incl(ranks)  # noqa: E731
Group_excl = lambda g, ranks: g.Excl(ranks)  # noqa: E731
Group_range_incl = lambda g, ranges: g.Range_incl(ranges)  # noqa: E731
Group_range_excl = lambda g, ranges: g.Range_excl(ranges)  # noqa: E731
Group_union, Group_intersection, Group_difference = _g.Group_union, _g.Group_intersection, _g.Group_difference
Group_translate_ranks = lambda g1, ranks, g2: g1.Translate_ranks(ranks, g2)  # noqa: E731
Group_compare = lambda a, b: a.Compare(b)  # noqa: E731
Group_free = lambda g: g.Free()  # noqa: E731
# caching
Comm_create_keyval, Type_create_keyval, Win_create_keyval = (_m.Comm_create_keyval,) * 3
Comm_free_keyval, Type_free_keyval, Win_free_keyval = (_m.Comm_free_keyval,) * 3
Comm_set_attr, Comm_get_attr, Comm_delete_attr = _m.Comm_set_attr, _m.Comm_get_attr, _m.Comm_delete_attr
Type_set_attr, Type_get_attr, Type_delete_attr = _m.Type_set_attr, _m.Type_get_attr, _m.Type_delete_attr
Win_set_attr, Win_get_attr, Win_delete_attr = _m.Win_set_attr, _m.Win_get_attr, _m.Win_delete_attr
Type_get_name, Type_set_name = _dt.Type_get_name, _dt.Type_set_name
Win_get_name = lambda w: w.Get_name()  # noqa: E731
Win_set_name = lambda w, n: w.Set_name(n)  # noqa: E731

# ---------------------------------------------------------------- datatypes
for _n in ("Type_contiguous", "Type_vector", "Type_create_hvector", "Type_indexed", "Type_create_hindexed",
           "Type_create_indexed_block", "Type_create_struct", "Type_create_subarray", "Type_create_darray",
           "Type_create_resized", "Type_dup", "Type_commit", "Type_free", "Type_size", "Type_get_extent",
           "Type_get_true_extent", "Type_get_envelope", "Type_get_contents", "Type_match_size", "Pack", "Unpack",
           "Pack_size", "Pack_external", "Unpack_external", "Pack_external_size", "Get_address", "Register_datarep"):
    globals()[_n] = getattr(_dt, _n)

# ---------------------------------------------------------------- topologies
for _n in ("Cart_create", "Cart_coords", "Cart_rank", "Cart_get", "Cartdim_get", "Cart_shift", "Cart_sub", "Cart_map",
           "Dims_create", "Graph_create", "Graph_get", "Graphdims_get", "Graph_neighbors", "Graph_neighbors_count",
           "Graph_map", "Topo_test"):
    globals()[_n] = getattr(_topo, _n)

# ---------------------------------------------------------------- info
Info_create = _m.Info_create
Info_set = lambda info, k, v: info.Set(k, v)  # noqa: E731
Info_get = lambda info, k, valuelen=None: info.Get(k, valuelen)  # noqa: E731
Info_delete = lambda info, k: info.Delete(k)  # noqa: E731
Info_dup = lambda info: info.Dup()  # noqa: E731
Info_free = lambda info: info.Free()  # noqa: E731
Info_get_nkeys = lambda info: info.Get_nkeys()  # noqa: E731
Info_get_nthkey = lambda info, n: info.Get_nthkey(n)  # noqa: E731
Info_get_valuelen = lambda info, k: info.Get_valuelen(k)  # noqa: E731

# ---------------------------------------------------------------- one-sided


def Win_create(base, size=None, disp_unit=None, info=None, comm=None):
    return Win.Create(base, comm, disp_unit, info)


def _origin_stream(origin, count, dtype):
    """The origin buffer's `count` instances of `dtype` as one contiguous byte stream (packed
    when the type is derived, as the two-sided path does) and its element dtype."""
    flat = origin.contiguous().reshape(-1)
    if dtype is None or dtype.is_contiguous_basic():
        es = dtype.Get_size() if dtype is not None else flat.element_size()
        n = int(count) * es
        raw = flat.view(torch.uint8)
        if n > raw.numel():
            raise ValueError(f"one-sided origin: {count} elements exceed the buffer")
        return raw[:n], flat.dtype
    return dtype.pack(flat, count), dtype.element_dtype()


def _target_runs(win, target_disp, target_count, target_type, nbytes):
    """Byte runs (window offset, length) the target (disp, count, datatype) names."""
    base = int(target_disp) * win.disp_unit
    if target_type is None or target_type.is_contiguous_basic():
        size = (target_type.Get_size() if target_type is not None else win.tensor.element_size()) * int(target_count)
        runs = [(0, size)]
    else:
        runs = target_type.runs(target_count)
        size = sum(n for _, n in runs)
    if size != nbytes:  # the type signatures must carry the same bytes (MPI_ERR_TRUNCATE / _TYPE)
        raise ValueError(f"one-sided: origin carries {nbytes} bytes, target (count {target_count}, {target_type}) {size}")
    return [(base + o, n) for o, n in runs]


def Put(origin, origin_count, origin_type, target_rank, target_disp, target_count, target_type, win):
    """MPI_Put (mpifuncs.c:1656): origin (count, datatype) packed, scattered over the target
    datatype's runs in the target window (one peer copy per contiguous run)."""
    data, _ = _origin_stream(origin, origin_count, origin_type)
    pos = 0
    for off, n in _target_runs(win, target_disp, target_count, target_type, data.numel()):
        win._put_bytes(data[pos:pos + n], target_rank, off)
        pos += n
    return SUCCESS


def Get(origin, origin_count, origin_type, target_rank, target_disp, target_count, target_type, win):
    """MPI_Get (mpifuncs.c:1131): the target datatype's runs gathered, unpacked into the origin
    by the origin datatype. Complete after the epoch's synchronisation (Fence / Flush /
    Unlock), like MPI: a derived origin type is unpacked at that point."""
    if origin_type is None or origin_type.is_contiguous_basic():
        es = origin_type.Get_size() if origin_type is not None else origin.element_size()
        if not origin.is_contiguous():
            raise ValueError("Get: contiguous origin buffer needed for a basic datatype")
        stage = origin.reshape(-1).view(torch.uint8)[:int(origin_count) * es]
        unpack = None
    else:
        stage = origin_type.staging(origin, origin_count)
        unpack = (origin_type, stage, origin, int(origin_count))
    pos = 0
    for off, n in _target_runs(win, target_disp, target_count, target_type, stage.numel()):
        win._get_bytes(stage[pos:pos + n], target_rank, off)
        pos += n
    if unpack is not None:  # derived origin: scatter once the data has landed
        win.Flush()
        t, st, buf, cnt = unpack
        t.unpack(st, buf, cnt)
    return SUCCESS


def Accumulate(origin, origin_count, origin_type, target_rank, target_disp, target_count, target_type, op, win):
    """MPI_Accumulate (mpifuncs.c:9): SUM / REPLACE of fp32 / bf16 elements, per contiguous
    run of the target datatype; both type maps must hold that one element type."""
    from .comm import REPLACE, SUM

    data, edt = _origin_stream(origin, origin_count, origin_type)
    tdt = target_type.element_dtype() if target_type is not None else win.tensor.dtype
    if edt not in (torch.float32, torch.bfloat16) or tdt != edt:
        raise TypeError(f"Accumulate: fp32 / bf16 elements of one type on both sides (origin {edt}, target {tdt})")
    op = op or SUM
    if op is SUM:
        a, b = 1.0, 1.0
    elif op is REPLACE:
        a, b = 1.0, 0.0
    else:
        raise ValueError("Accumulate supports SUM and REPLACE")
    vals = data.view(edt)
    es = vals.element_size()
    pos = 0
    for off, n in _target_runs(win, target_disp, target_count, target_type, data.numel()):
        win._acc_elems(vals[pos // es:(pos + n) // es], target_rank, off, a, b)
        pos += n
    return SUCCESS


Win_fence = lambda assertion, win: win.Fence(assertion)  # noqa: E731
Win_free = lambda win: win.Free()  # noqa: E731
Win_get_group = lambda win: win.Get_group()  # noqa: E731
Win_lock = lambda lock_type, rank, assertion, win: win.Lock(rank, lock_type, assertion)  # noqa: E731
Win_unlock = lambda rank, win: win.Unlock(rank)  # noqa: E731
Win_post = lambda group, assertion, win: win.Post(group, assertion)  # noqa: E731
Win_start = lambda group, assertion, win: win.Start(group, assertion)  # noqa: E731
Win_complete = lambda win: win.Complete()  # noqa: E731
Win_wait = lambda win: win.Wait()  # noqa: E731
Win_test = lambda win: win.Test()  # noqa: E731

# ---------------------------------------------------------------- I/O
File_open, File_delete = _io.File_open, _io.File_delete
for _meth in ("close", "get_amode", "get_atomicity", "get_byte_offset", "get_group", "get_info", "get_position",
              "get_position_shared", "get_size", "get_type_extent", "get_view", "iread", "iread_at", "iread_shared",
              "iwrite", "iwrite_at", "iwrite_shared", "preallocate", "read", "read_all", "read_all_begin",
              "read_all_end", "read_at", "read_at_all", "read_at_all_begin", "read_at_all_end", "read_ordered",
              "read_ordered_begin", "read_ordered_end", "read_shared", "seek", "seek_shared", "set_atomicity",
              "set_info", "set_size", "set_view", "sync", "write", "write_all", "write_all_begin", "write_all_end",
              "write_at", "write_at_all", "write_at_all_begin", "write_at_all_end", "write_ordered",
              "write_ordered_begin", "write_ordered_end", "write_shared"):
    _m_name = _meth[0].upper() + _meth[1:]  # File_read_at -> File.Read_at
    globals()["File_" + _meth] = (lambda mn: (lambda f, *a, **k: getattr(f, mn)(*a, **k)))(_m_name)

# ---------------------------------------------------------------- dynamic processes
for _n in ("Open_port", "Close_port", "Publish_name", "Lookup_name", "Unpublish_name", "Comm_accept", "Comm_connect",
           "Comm_join", "Comm_get_parent", "Comm_spawn", "Comm_spawn_multiple", "Comm_disconnect"):
    globals()[_n] = getattr(_dyn, _n)


# ---------------------------------------------------------------- aio / coroutine runtime (init.lua)
signal_INIT, signal_EXEC, signal_OK, signal_ERR, signal_DONE = 0, 1, 2, 3, 4


class Queue:
    """FIFO run queue of coroutines (queue.lua:3-47)."""

    def __init__(self):
        self._q = deque()

    def push(self, x):
        self._q.append(x)

    def pop(self):
        return self._q.popleft() if self._q else None

    def empty(self):
        return not self._q

    def len(self):
        return len(self._q)

    def clear(self):
        self._q.clear()


def aio_send(buf, size, datatype, dest, tag, comm, state=None, cb=None):
    """Generator-coroutine send (init.lua:41-67): yields signal_EXEC while the send is in
    flight; cancels it when ``state['io']`` turns false."""
    req = comm.Isend(buf.reshape(-1)[:size] if size is not None else buf, dest, tag)
    while not req.Test():
        if state is not None and not state.get("io", True):
            req.Cancel()
            req.Wait()
            break
        yield signal_EXEC
    if cb is not None:
        cb(state)
    yield signal_OK


def aio_recv(buf, size, datatype, source, tag, comm, state=None, cb=None):
    """Generator-coroutine receive (init.lua:70-108), with the receive actually
    cancellable when ``state['io']`` turns false (the reference's branch is unreachable)."""
    req = comm.Irecv(buf.reshape(-1)[:size] if size is not None else buf, source, tag)
    while not req.Test():
        if state is not None and not state.get("io", True):
            req.Cancel()
            req.Wait()
            yield signal_DONE
            return
        yield signal_EXEC
    if cb is not None:
        cb(state)
    yield signal_OK


def co_execute(fn, args=()):
    """Create a coroutine from a generator function and run it to its first yield
    (init.lua:139-150)."""
    co = fn(*args)
    try:
        next(co)
    except StopIteration:
        return None
    return co


def co_ping(q: Queue):
    """Resume the head coroutine once; re-queue it unless it finished (init.lua:154-181)."""
    co = q.pop()
    if co is None:
        return
    try:
        sig = next(co)
    except StopIteration:
        return
    if sig == signal_DONE:
        try:
            next(co)
        except StopIteration:
            pass
        return
    q.push(co)


def co_wait(q: Queue, usec: float = 0):
    """Drain the queue (init.lua:185-192); default usec 0 (README.md:65)."""
    import time

    while not q.empty():
        co_ping(q)
        if usec:
            time.sleep(usec * 1e-6)


def type(obj):  # noqa: A001 - mpiT.type (an empty stub in the reference, init.lua:121-123)
    return None if obj is None else obj.__class__

"""MPI datatypes: the 22 basic types of the reference (lua-mpi.h:130-151) and derived
type constructors (mpifuncs.c Type_* / Pack* wrappers, SURVEY Appendix A "Datatypes").

A :class:`Datatype` is a *typemap*: a list of (byte displacement, basic type) plus lower
bound and extent. ``pack`` / ``unpack`` move ``count`` instances between a tensor (viewed
as bytes) and a contiguous byte stream with one gather / scatter index op, so they work
unchanged on host tensors and on HBM tensors (the index tensor is cached per type).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import torch

_BASIC: Dict[str, Tuple[int, Optional[torch.dtype]]] = {
    "CHAR": (1, torch.int8), "BYTE": (1, torch.uint8), "SHORT": (2, torch.int16), "INT": (4, torch.int32),
    "LONG": (8, torch.int64), "FLOAT": (4, torch.float32), "DOUBLE": (8, torch.float64),
    "UNSIGNED_CHAR": (1, torch.uint8), "UNSIGNED_SHORT": (2, torch.int16), "UNSIGNED": (4, torch.int32),
    "UNSIGNED_LONG": (8, torch.int64), "LONG_DOUBLE": (16, None), "LONG_LONG_INT": (8, torch.int64),
    "FLOAT_INT": (8, None), "LONG_INT": (16, None), "DOUBLE_INT": (16, None), "SHORT_INT": (8, None),
    "2INT": (8, None), "LONG_DOUBLE_INT": (32, None), "PACKED": (1, torch.uint8), "UB": (0, None), "LB": (0, None),
    "BFLOAT16": (2, torch.bfloat16), "HALF": (2, torch.float16), "BOOL": (1, torch.bool),
}


class Datatype:
    def __init__(self, typemap: List[Tuple[int, str]], lb: int, extent: int, name: str = "",
                 envelope=("NAMED", (), ()), committed=True):
        self.typemap = typemap  # [(disp_bytes, basic_name)]
        self.lb = lb
        self.extent = extent
        self._name = name
        self.envelope = envelope
        self.committed = committed
        self._attrs = {}
        self._idx_cache = {}

    # ---------------------------------------------------------------- queries
    def Get_size(self) -> int:
        return sum(_BASIC[b][0] for _, b in self.typemap)

    def Get_extent(self) -> Tuple[int, int]:
        return self.lb, self.extent

    def Get_true_extent(self) -> Tuple[int, int]:
        if not self.typemap:
            return 0, 0
        lo = min(d for d, _ in self.typemap)
        hi = max(d + _BASIC[b][0] for d, b in self.typemap)
        return lo, hi - lo

    def Get_envelope(self):
        kind, ints, types = self.envelope
        return len(ints), 0, len(types), kind

    def Get_contents(self):
        return self.envelope

    def Get_name(self) -> str:
        return self._name

    def Set_name(self, n: str):
        self._name = n

    def Commit(self):
        self.committed = True
        return self

    def Free(self):
        self._idx_cache.clear()

    def Dup(self) -> "Datatype":
        return Datatype(list(self.typemap), self.lb, self.extent, self._name, ("DUP", (), (self,)))

    def Set_attr(self, k, v):
        self._attrs[k] = v

    def Get_attr(self, k):
        return self._attrs.get(k)

    def Delete_attr(self, k):
        self._attrs.pop(k, None)

    def is_contiguous_basic(self) -> bool:
        return len(self.typemap) == 1 and self.typemap[0][0] == 0 and self.extent == _BASIC[self.typemap[0][1]][0]

    @property
    def torch_dtype(self) -> Optional[torch.dtype]:
        if len(self.typemap) == 1:
            return _BASIC[self.typemap[0][1]][1]
        return None

    # ---------------------------------------------------------------- byte gather / scatter
    def _byte_index(self, count: int, device) -> torch.Tensor:
        key = (count, str(device))
        t = self._idx_cache.get(key)
        if t is None:
            idx = []
            for i in range(count):
                base = i * self.extent
                for d, b in self.typemap:
                    sz = _BASIC[b][0]
                    idx.extend(range(base + d, base + d + sz))
            t = torch.tensor(idx, dtype=torch.int64, device=device)
            self._idx_cache[key] = t
        return t

    def _count_for(self, buf: torch.Tensor, count: Optional[int]) -> int:
        if count is not None:
            return int(count)
        nbytes = buf.numel() * buf.element_size()
        return max(0, (nbytes - self.Get_true_extent()[1]) // max(1, self.extent) + 1) if self.extent else 1

    def pack(self, buf: torch.Tensor, count: Optional[int] = None) -> torch.Tensor:
        """Gather `count` instances from `buf` into a contiguous uint8 tensor."""
        count = self._count_for(buf, count)
        raw = buf.contiguous().reshape(-1).view(torch.uint8)
        return raw[self._byte_index(count, raw.device)]

    def staging(self, buf: torch.Tensor, count: Optional[int] = None) -> torch.Tensor:
        count = self._count_for(buf, count)
        return torch.empty(count * self.Get_size(), dtype=torch.uint8, device=buf.device)

    def unpack(self, packed: torch.Tensor, buf: torch.Tensor, count: Optional[int] = None):
        """Scatter a packed byte stream into `buf` (in place)."""
        count = self._count_for(buf, count)
        if not buf.is_contiguous():
            raise ValueError("unpack target must be contiguous")
        raw = buf.reshape(-1).view(torch.uint8)
        raw[self._byte_index(count, raw.device)] = packed.reshape(-1)[: count * self.Get_size()].to(raw.device)
        return buf

    def runs(self, count: int) -> List[Tuple[int, int]]:
        """The byte runs (offset, length) that `count` instances occupy, in type-map order
        (the order of the packed stream), adjacent segments merged: what a one-sided
        transfer moves with one copy each."""
        out: List[Tuple[int, int]] = []
        for i in range(int(count)):
            base = i * self.extent
            for d, b in self.typemap:
                sz = _BASIC[b][0]
                if not sz:
                    continue
                o = base + d
                if out and out[-1][0] + out[-1][1] == o:
                    out[-1] = (out[-1][0], out[-1][1] + sz)
                else:
                    out.append((o, sz))
        return out

    def element_dtype(self) -> Optional[torch.dtype]:
        """The one basic torch dtype every entry of the type map has (None: mixed / none)."""
        kinds = {b for _, b in self.typemap if _BASIC[b][0]}
        return _BASIC[kinds.pop()][1] if len(kinds) == 1 else None

    def __repr__(self):
        return f"Datatype({self._name or self.envelope[0]}, size={self.Get_size()}, extent={self.extent})"


def _basic(name: str) -> Datatype:
    sz = _BASIC[name][0]
    return Datatype([(0, name)] if sz else [], 0, sz, "MPI_" + name)


CHAR, BYTE, SHORT, INT, LONG, FLOAT, DOUBLE = (_basic(n) for n in ("CHAR", "BYTE", "SHORT", "INT", "LONG", "FLOAT", "DOUBLE"))
UNSIGNED_CHAR, UNSIGNED_SHORT, UNSIGNED, UNSIGNED_LONG = (_basic(n) for n in ("UNSIGNED_CHAR", "UNSIGNED_SHORT", "UNSIGNED", "UNSIGNED_LONG"))
LONG_DOUBLE, LONG_LONG_INT, PACKED, UB, LB = (_basic(n) for n in ("LONG_DOUBLE", "LONG_LONG_INT", "PACKED", "UB", "LB"))
BFLOAT16, HALF, BOOL = _basic("BFLOAT16"), _basic("HALF"), _basic("BOOL")


def _pair(vname: str, iname: str, name: str) -> Datatype:
    vs, is_ = _BASIC[vname][0], _BASIC[iname][0]
    al = max(vs, is_)
    ext = (vs + is_ + al - 1) // al * al
    return Datatype([(0, vname), (vs, iname)], 0, ext, name)


FLOAT_INT = _pair("FLOAT", "INT", "MPI_FLOAT_INT")
DOUBLE_INT = _pair("DOUBLE", "INT", "MPI_DOUBLE_INT")
LONG_INT = _pair("LONG", "INT", "MPI_LONG_INT")
SHORT_INT = _pair("SHORT", "INT", "MPI_SHORT_INT")
TWOINT = _pair("INT", "INT", "MPI_2INT")
LONG_DOUBLE_INT = Datatype([(0, "LONG_DOUBLE"), (16, "INT")], 0, 32, "MPI_LONG_DOUBLE_INT")
DATATYPE_NULL = None

_BY_TORCH = {torch.float32: FLOAT, torch.float64: DOUBLE, torch.int32: INT, torch.int64: LONG, torch.int16: SHORT,
             torch.int8: CHAR, torch.uint8: BYTE, torch.bfloat16: BFLOAT16, torch.float16: HALF, torch.bool: BOOL}


def from_torch(dtype: torch.dtype) -> Datatype:
    return _BY_TORCH[dtype]


# -------------------------------------------------------------------- constructors

def _concat(parts: List[Tuple[int, Datatype, int]]) -> List[Tuple[int, str]]:
    """parts: (byte displacement, type, count) -> flattened typemap."""
    tm = []
    for disp, t, cnt in parts:
        for i in range(cnt):
            base = disp + i * t.extent
            tm.extend((base + d, b) for d, b in t.typemap)
    return tm


def _bounds(tm, lb=None, ub=None):
    if not tm:
        return 0, 0
    lo = min(d for d, _ in tm) if lb is None else lb
    hi = max(d + _BASIC[b][0] for d, b in tm) if ub is None else ub
    return lo, hi - lo


def Type_contiguous(count: int, oldtype: Datatype) -> Datatype:
    tm = _concat([(0, oldtype, count)])
    return Datatype(tm, oldtype.lb, count * oldtype.extent, envelope=("CONTIGUOUS", (count,), (oldtype,)), committed=False)


def Type_vector(count: int, blocklength: int, stride: int, oldtype: Datatype) -> Datatype:
    return Type_create_hvector(count, blocklength, stride * oldtype.extent, oldtype, _kind="VECTOR")


def Type_create_hvector(count: int, blocklength: int, stride_bytes: int, oldtype: Datatype, _kind="HVECTOR") -> Datatype:
    tm = _concat([(i * stride_bytes, oldtype, blocklength) for i in range(count)])
    lb, ext = _bounds(tm)
    ext = (count - 1) * stride_bytes + blocklength * oldtype.extent if count else 0
    return Datatype(tm, 0, ext, envelope=(_kind, (count, blocklength, stride_bytes), (oldtype,)), committed=False)


def Type_indexed(blocklengths: Sequence[int], displacements: Sequence[int], oldtype: Datatype) -> Datatype:
    return Type_create_hindexed(blocklengths, [d * oldtype.extent for d in displacements], oldtype, _kind="INDEXED")


def Type_create_hindexed(blocklengths, displacements_bytes, oldtype: Datatype, _kind="HINDEXED") -> Datatype:
    tm = _concat([(d, oldtype, b) for b, d in zip(blocklengths, displacements_bytes)])
    ends = [d + b * oldtype.extent for b, d in zip(blocklengths, displacements_bytes)]
    lb = min(displacements_bytes) if displacements_bytes else 0
    ext = (max(ends) - lb) if ends else 0
    return Datatype(tm, lb, ext, envelope=(_kind, (tuple(blocklengths), tuple(displacements_bytes)), (oldtype,)),
                    committed=False)


def Type_create_indexed_block(blocklength: int, displacements: Sequence[int], oldtype: Datatype) -> Datatype:
    return Type_indexed([blocklength] * len(displacements), displacements, oldtype)


def Type_create_struct(blocklengths, displacements_bytes, types: Sequence[Datatype]) -> Datatype:
    tm = _concat([(d, t, b) for b, d, t in zip(blocklengths, displacements_bytes, types)])
    ends = [d + b * t.extent for b, d, t in zip(blocklengths, displacements_bytes, types)]
    lb = min(displacements_bytes) if displacements_bytes else 0
    ext = (max(ends) - lb) if ends else 0
    return Datatype(tm, lb, ext, envelope=("STRUCT", (tuple(blocklengths), tuple(displacements_bytes)), tuple(types)),
                    committed=False)


ORDER_C, ORDER_FORTRAN = 56, 57


def Type_create_subarray(sizes, subsizes, starts, order: int, oldtype: Datatype) -> Datatype:
    import itertools

    nd = len(sizes)
    # element strides: row-major (last dim fastest) for C, column-major for Fortran
    fastest_last = order == ORDER_C
    strides, s = [0] * nd, oldtype.extent
    for d in (reversed(range(nd)) if fastest_last else range(nd)):
        strides[d] = s
        s *= sizes[d]
    total = s
    tm = []
    for idx in itertools.product(*[range(starts[d], starts[d] + subsizes[d]) for d in range(nd)]):
        off = sum(i * st for i, st in zip(idx, strides))
        tm.append((off, idx))
    tm.sort()
    tm = [(off + dd, b) for off, _ in tm for dd, b in oldtype.typemap]
    return Datatype(tm, 0, total, envelope=("SUBARRAY", (tuple(sizes), tuple(subsizes), tuple(starts), order), (oldtype,)),
                    committed=False)


DISTRIBUTE_BLOCK, DISTRIBUTE_CYCLIC, DISTRIBUTE_NONE, DISTRIBUTE_DFLT_DARG = 121, 122, 123, -49767


def Type_create_darray(size, rank, gsizes, distribs, dargs, psizes, order, oldtype) -> Datatype:
    """Block (and block-cyclic) distribution of a global array over a process grid."""
    # process coordinates in row-major order of psizes
    coords, r = [], rank
    for p in reversed(psizes):
        coords.append(r % p)
        r //= p
    coords = coords[::-1]
    ranges = []
    for d, g in enumerate(gsizes):
        p, c = psizes[d], coords[d]
        if distribs[d] == DISTRIBUTE_NONE or p == 1:
            ranges.append(list(range(g)))
        elif distribs[d] == DISTRIBUTE_BLOCK:
            b = dargs[d] if dargs[d] not in (DISTRIBUTE_DFLT_DARG, 0) else -(-g // p)
            ranges.append(list(range(c * b, min(g, (c + 1) * b))))
        else:  # cyclic(b)
            b = dargs[d] if dargs[d] not in (DISTRIBUTE_DFLT_DARG, 0) else 1
            ranges.append([i for i in range(g) if (i // b) % p == c])
    import itertools

    strides, s = [0] * len(gsizes), oldtype.extent
    for d in reversed(range(len(gsizes))):
        strides[d] = s
        s *= gsizes[d]
    tm = []
    for idx in itertools.product(*ranges):
        off = sum(i * st for i, st in zip(idx, strides))
        tm.extend((off + dd, b) for dd, b in oldtype.typemap)
    return Datatype(tm, 0, s, envelope=("DARRAY", (size, rank, tuple(gsizes)), (oldtype,)), committed=False)


def Type_create_resized(oldtype: Datatype, lb: int, extent: int) -> Datatype:
    return Datatype(list(oldtype.typemap), lb, extent, envelope=("RESIZED", (lb, extent), (oldtype,)), committed=False)


def Type_dup(t: Datatype) -> Datatype:
    return t.Dup()


def Type_commit(t: Datatype) -> Datatype:
    return t.Commit()


def Type_free(t: Datatype):
    t.Free()


def Type_size(t: Datatype) -> int:
    return t.Get_size()


def Type_get_extent(t: Datatype):
    return t.Get_extent()


def Type_get_true_extent(t: Datatype):
    return t.Get_true_extent()


def Type_get_envelope(t: Datatype):
    return t.Get_envelope()


def Type_get_contents(t: Datatype):
    return t.Get_contents()


def Type_get_name(t: Datatype) -> str:
    return t.Get_name()


def Type_set_name(t: Datatype, name: str):
    t.Set_name(name)


TYPECLASS_INTEGER, TYPECLASS_REAL, TYPECLASS_COMPLEX = 1, 2, 3


def Type_match_size(typeclass: int, size: int) -> Datatype:
    table = {TYPECLASS_INTEGER: {1: CHAR, 2: SHORT, 4: INT, 8: LONG}, TYPECLASS_REAL: {2: HALF, 4: FLOAT, 8: DOUBLE}}
    try:
        return table[typeclass][size]
    except KeyError:
        raise ValueError(f"no datatype of class {typeclass} and size {size}") from None


# -------------------------------------------------------------------- Pack / Unpack

def Pack(inbuf: torch.Tensor, incount: int, datatype: Datatype, outbuf: torch.Tensor, position: int) -> int:
    """Append `incount` instances to the byte buffer `outbuf` at `position`; returns the
    new position (MPI_Pack)."""
    data = datatype.pack(inbuf, incount)
    out = outbuf.reshape(-1).view(torch.uint8)
    out[position: position + data.numel()] = data.to(out.device)
    return position + data.numel()


def Unpack(inbuf: torch.Tensor, position: int, outbuf: torch.Tensor, outcount: int, datatype: Datatype) -> int:
    src = inbuf.reshape(-1).view(torch.uint8)
    n = outcount * datatype.Get_size()
    datatype.unpack(src[position: position + n], outbuf, outcount)
    return position + n


def Pack_size(incount: int, datatype: Datatype) -> int:
    return incount * datatype.Get_size()


def Pack_external(datarep: str, inbuf, incount, datatype, outbuf, position) -> int:
    """"external32" = big-endian canonical representation."""
    if datarep not in ("external32", "native"):
        raise ValueError("supported data representations: external32, native")
    pos0 = position
    position = Pack(inbuf, incount, datatype, outbuf, position)
    if datarep == "external32":
        _byteswap_inplace(outbuf.reshape(-1).view(torch.uint8)[pos0:position], datatype, incount)
    return position


def Unpack_external(datarep: str, inbuf, position, outbuf, outcount, datatype) -> int:
    src = inbuf.reshape(-1).view(torch.uint8)
    n = outcount * datatype.Get_size()
    seg = src[position: position + n].clone()
    if datarep == "external32":
        _byteswap_inplace(seg, datatype, outcount)
    datatype.unpack(seg, outbuf, outcount)
    return position + n


def Pack_external_size(datarep: str, incount: int, datatype: Datatype) -> int:
    return Pack_size(incount, datatype)


def _byteswap_inplace(seg: torch.Tensor, datatype: Datatype, count: int):
    o = 0
    for _ in range(count):
        for _, b in datatype.typemap:
            sz = _BASIC[b][0]
            if sz > 1:
                seg[o: o + sz] = seg[o: o + sz].flip(0)
            o += sz


def Get_address(t: torch.Tensor) -> int:
    return t.data_ptr()


def Get_elements(status, datatype: Datatype) -> int:
    """Number of basic elements received."""
    per = len(datatype.typemap) or 1
    return (status.count // max(1, datatype.Get_size())) * per


_datareps = {}


def Register_datarep(name: str, read_fn, write_fn, extent_fn, extra_state=None):
    _datareps[name] = (read_fn, write_fn, extent_fn, extra_state)

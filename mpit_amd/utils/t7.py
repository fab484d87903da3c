"""Pure-data reader for Torch7's binary ``torch.save`` format (the reference's ``-preloadBinary``
caches, BiCNN/plaunch.lua:218-229, read there with ``torch.load``).

Only plain data is accepted: nil, numbers, strings, booleans and tables (with Torch7's
back-references for shared tables). A ``torch.*`` object (tensors, storages, any class) or a
serialised Lua function is REFUSED with :class:`T7RefusedObject` — nothing in the file can
make this loader construct an object or run code, so it is safe on untrusted files.

Format (little endian, as Torch7's File:writeObject with 4-byte ints): every object starts
with an int type tag — 0 nil, 1 number (double), 2 string (int length + bytes), 3 table
(int reference index; on first sight an int entry count then key / value objects), 4 torch
object, 5 boolean (int), 6 / 7 / 8 functions.
"""
from __future__ import annotations

import struct
from typing import Any, Dict

T_NIL, T_NUMBER, T_STRING, T_TABLE, T_TORCH, T_BOOLEAN, T_FUNCTION, T_RECUR_FUNCTION_LEGACY, T_RECUR_FUNCTION = range(9)


class T7RefusedObject(ValueError):
    """The file holds something other than plain data (a torch object or a function)."""


class _Reader:
    def __init__(self, data: bytes):
        self.d = data
        self.o = 0
        self.refs: Dict[int, Any] = {}

    def _take(self, n: int) -> bytes:
        if self.o + n > len(self.d):
            raise ValueError(f"t7: truncated file (need {n} bytes at offset {self.o})")
        b = self.d[self.o:self.o + n]
        self.o += n
        return b

    def int(self) -> int:
        return struct.unpack("<i", self._take(4))[0]

    def obj(self) -> Any:
        t = self.int()
        if t == T_NIL:
            return None
        if t == T_NUMBER:
            v = struct.unpack("<d", self._take(8))[0]
            return int(v) if v.is_integer() and abs(v) < 2 ** 53 else v
        if t == T_STRING:
            n = self.int()
            if n < 0:
                raise ValueError("t7: negative string length")
            return self._take(n).decode("utf-8", errors="surrogateescape")
        if t == T_BOOLEAN:
            return self.int() == 1
        if t == T_TABLE:
            idx = self.int()
            if idx in self.refs:
                return self.refs[idx]
            tab: Dict[Any, Any] = {}
            self.refs[idx] = tab
            n = self.int()
            if n < 0:
                raise ValueError("t7: negative table size")
            for _ in range(n):
                k = self.obj()
                tab[k] = self.obj()
            return tab
        if t == T_TORCH:
            raise T7RefusedObject(f"t7: torch object at offset {self.o - 4} refused (plain data only)")
        if t in (T_FUNCTION, T_RECUR_FUNCTION_LEGACY, T_RECUR_FUNCTION):
            raise T7RefusedObject(f"t7: serialised function at offset {self.o - 4} refused (plain data only)")
        raise ValueError(f"t7: unknown type tag {t} at offset {self.o - 4}")


def loads(data: bytes) -> Any:
    r = _Reader(data)
    v = r.obj()
    if r.o != len(data):
        raise ValueError(f"t7: {len(data) - r.o} trailing bytes after the object")
    return v


def load(path: str) -> Any:
    with open(path, "rb") as f:
        return loads(f.read())


def dumps(v: Any) -> bytes:
    """Writer for the same plain-data subset (test fixtures, caches for the reference)."""
    out = []
    nref = [0]

    def w(x):
        if x is None:
            out.append(struct.pack("<i", T_NIL))
        elif isinstance(x, bool):
            out.append(struct.pack("<ii", T_BOOLEAN, 1 if x else 0))
        elif isinstance(x, (int, float)):
            out.append(struct.pack("<id", T_NUMBER, float(x)))
        elif isinstance(x, str):
            b = x.encode("utf-8", errors="surrogateescape")
            out.append(struct.pack("<ii", T_STRING, len(b)) + b)
        elif isinstance(x, dict):
            nref[0] += 1
            out.append(struct.pack("<iii", T_TABLE, nref[0], len(x)))
            for k, val in x.items():
                w(k)
                w(val)
        else:
            raise TypeError(f"t7: cannot write {type(x).__name__}")

    w(v)
    return b"".join(out)

"""MPI_Group: ordered sets of world ranks (mpifuncs.c Group_* wrappers, plus the
Group_range_incl / Group_range_excl the reference's generator dropped, readspec.py:79-84)."""
from __future__ import annotations

from typing import List, Sequence, Tuple

UNDEFINED = -32766
IDENT, SIMILAR, UNEQUAL = 0, 2, 3


class Group:
    def __init__(self, world_ranks: Sequence[int]):
        self._r = list(world_ranks)

    @property
    def world_ranks(self) -> List[int]:
        return list(self._r)

    def Get_size(self) -> int:
        return len(self._r)

    def Get_rank(self) -> int:
        from . import runtime as _rt

        me = _rt.state().rank
        return self._r.index(me) if me in self._r else UNDEFINED

    def Incl(self, ranks: Sequence[int]) -> "Group":
        return Group([self._r[i] for i in ranks])

    def Excl(self, ranks: Sequence[int]) -> "Group":
        ex = set(ranks)
        return Group([w for i, w in enumerate(self._r) if i not in ex])

    @staticmethod
    def _expand(ranges: Sequence[Tuple[int, int, int]]) -> List[int]:
        out = []
        for first, last, stride in ranges:
            if stride == 0:
                raise ValueError("range stride must be non-zero")
            out.extend(range(first, last + (1 if stride > 0 else -1), stride))
        return out

    def Range_incl(self, ranges: Sequence[Tuple[int, int, int]]) -> "Group":
        return self.Incl(self._expand(ranges))

    def Range_excl(self, ranges: Sequence[Tuple[int, int, int]]) -> "Group":
        return self.Excl(self._expand(ranges))

    def Union(self, other: "Group") -> "Group":
        return Group(self._r + [w for w in other._r if w not in self._r])

    def Intersection(self, other: "Group") -> "Group":
        s = set(other._r)
        return Group([w for w in self._r if w in s])

    def Difference(self, other: "Group") -> "Group":
        s = set(other._r)
        return Group([w for w in self._r if w not in s])

    def Translate_ranks(self, ranks: Sequence[int], other: "Group") -> List[int]:
        return [other._r.index(self._r[i]) if self._r[i] in other._r else UNDEFINED for i in ranks]

    def Compare(self, other: "Group") -> int:
        if self._r == other._r:
            return IDENT
        if sorted(self._r) == sorted(other._r):
            return SIMILAR
        return UNEQUAL

    def Free(self):
        pass

    def __repr__(self):
        return f"Group({self._r})"


GROUP_EMPTY = Group([])
GROUP_NULL = None


def Group_union(a, b):
    return a.Union(b)


def Group_intersection(a, b):
    return a.Intersection(b)


def Group_difference(a, b):
    return a.Difference(b)

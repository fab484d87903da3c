"""Process topologies: Cartesian and graph communicators (mpifuncs.c Cart_* / Graph_* /
Dims_create / Topo_test, SURVEY Appendix A "Process Topologies")."""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

from .comm import PROC_NULL, UNDEFINED, Comm

CART, GRAPH, DIST_GRAPH = 1, 2, 3


class CartTopo:
    def __init__(self, dims: Sequence[int], periods: Sequence[bool]):
        self.dims = list(dims)
        self.periods = [bool(p) for p in periods]

    def coords(self, rank: int) -> List[int]:
        c = []
        for d in reversed(self.dims):
            c.append(rank % d)
            rank //= d
        return c[::-1]

    def rank(self, coords: Sequence[int]) -> int:
        r = 0
        for d, (c, n, per) in enumerate(zip(coords, self.dims, self.periods)):
            if per:
                c %= n
            elif not 0 <= c < n:
                return PROC_NULL
            r = r * n + c
        return r


class GraphTopo:
    def __init__(self, index: Sequence[int], edges: Sequence[int]):
        self.index = list(index)
        self.edges = list(edges)

    def neighbors(self, rank: int) -> List[int]:
        lo = self.index[rank - 1] if rank > 0 else 0
        return self.edges[lo: self.index[rank]]


def Dims_create(nnodes: int, dims: Sequence[int]) -> List[int]:
    """Balanced factorisation of nnodes over the zero entries of dims (non-increasing)."""
    dims = list(dims)
    fixed = 1
    for d in dims:
        if d > 0:
            fixed *= d
    if nnodes % fixed:
        raise ValueError("nnodes is not divisible by the fixed dimensions")
    free = [i for i, d in enumerate(dims) if d <= 0]
    rem = nnodes // fixed
    facs = []
    n, p = rem, 2
    while p * p <= n:
        while n % p == 0:
            facs.append(p)
            n //= p
        p += 1
    if n > 1:
        facs.append(n)
    out = [1] * len(free)
    for f in sorted(facs, reverse=True):
        i = min(range(len(out)), key=lambda k: out[k]) if out else None
        if i is None:
            if f != 1:
                raise ValueError("no free dimensions")
            continue
        out[i] *= f
    out.sort(reverse=True)
    for i, v in zip(free, out):
        dims[i] = v
    return dims


def Cart_create(comm: Comm, dims: Sequence[int], periods: Sequence[bool], reorder: bool = False) -> Optional[Comm]:
    n = 1
    for d in dims:
        n *= d
    if n > comm.Get_size():
        raise ValueError("cartesian grid larger than the communicator")
    color = 0 if comm.Get_rank() < n else UNDEFINED
    c = comm.Split(color, comm.Get_rank())
    if c is not None:
        c.topology = CartTopo(dims, periods)
    return c


def _cart(comm: Comm) -> CartTopo:
    if not isinstance(comm.topology, CartTopo):
        raise ValueError("communicator has no cartesian topology")
    return comm.topology


def Cart_coords(comm: Comm, rank: int) -> List[int]:
    return _cart(comm).coords(rank)


def Cart_rank(comm: Comm, coords: Sequence[int]) -> int:
    return _cart(comm).rank(coords)


def Cart_get(comm: Comm) -> Tuple[List[int], List[bool], List[int]]:
    t = _cart(comm)
    return list(t.dims), list(t.periods), t.coords(comm.Get_rank())


def Cartdim_get(comm: Comm) -> int:
    return len(_cart(comm).dims)


def Cart_shift(comm: Comm, direction: int, disp: int) -> Tuple[int, int]:
    t = _cart(comm)
    me = t.coords(comm.Get_rank())
    src, dst = list(me), list(me)
    src[direction] -= disp
    dst[direction] += disp
    return t.rank(src), t.rank(dst)


def Cart_sub(comm: Comm, remain_dims: Sequence[bool]) -> Comm:
    t = _cart(comm)
    me = t.coords(comm.Get_rank())
    color = 0
    for d, keep in enumerate(remain_dims):
        if not keep:
            color = color * t.dims[d] + me[d]
    key = 0
    for d, keep in enumerate(remain_dims):
        if keep:
            key = key * t.dims[d] + me[d]
    sub = comm.Split(color, key)
    sub.topology = CartTopo([n for n, k in zip(t.dims, remain_dims) if k],
                            [p for p, k in zip(t.periods, remain_dims) if k])
    return sub


def Cart_map(comm: Comm, dims: Sequence[int], periods: Sequence[bool]) -> int:
    n = 1
    for d in dims:
        n *= d
    r = comm.Get_rank()
    return r if r < n else UNDEFINED


def Graph_create(comm: Comm, index: Sequence[int], edges: Sequence[int], reorder: bool = False) -> Optional[Comm]:
    n = len(index)
    color = 0 if comm.Get_rank() < n else UNDEFINED
    c = comm.Split(color, comm.Get_rank())
    if c is not None:
        c.topology = GraphTopo(index, edges)
    return c


def _graph(comm: Comm) -> GraphTopo:
    if not isinstance(comm.topology, GraphTopo):
        raise ValueError("communicator has no graph topology")
    return comm.topology


def Graph_get(comm: Comm):
    g = _graph(comm)
    return list(g.index), list(g.edges)


def Graphdims_get(comm: Comm):
    g = _graph(comm)
    return len(g.index), len(g.edges)


def Graph_neighbors(comm: Comm, rank: int) -> List[int]:
    return _graph(comm).neighbors(rank)


def Graph_neighbors_count(comm: Comm, rank: int) -> int:
    return len(_graph(comm).neighbors(rank))


def Graph_map(comm: Comm, index, edges) -> int:
    r = comm.Get_rank()
    return r if r < len(index) else UNDEFINED


def Topo_test(comm: Comm) -> int:
    if isinstance(comm.topology, CartTopo):
        return CART
    if isinstance(comm.topology, GraphTopo):
        return GRAPH
    return UNDEFINED

"""Inter-communicators and the connect/accept name service (SURVEY Appendix A "Process
Creation and Management" + Intercomm_* / Comm_remote_* of "Groups, Contexts,
Communicators").

All processes of a job share one node-local runtime, so an inter-communicator connects
two disjoint groups of the same world: point-to-point ranks on it address the *remote*
group, collectives are not defined on it (``Merge`` it first). Ports and published names
live in a small directory under /dev/shm shared by the job. Spawning new processes
(``Comm_spawn``) would need a second runtime segment and is not provided; the reference's
generator did not produce those wrappers either (dropped specs).
"""
from __future__ import annotations

import os
import socket
import struct
import time
import zlib
from typing import List, Optional

import torch

from . import runtime as _rt
from .comm import ANY_SOURCE, MAX, Comm, Request, Status
from .group import Group

_PORT_CTX = (1 << 25)  # world-level context for connect/accept handshakes


class InterComm(Comm):
    def __init__(self, local: List[int], remote: List[int], ctx: int, name: str = "intercomm"):
        super().__init__(local, ctx, name)
        self._remote = list(remote)
        self._rw2c = {w: i for i, w in enumerate(self._remote)}

    def Is_inter(self) -> bool:
        return True

    def Get_remote_size(self) -> int:
        return len(self._remote)

    def Get_remote_group(self) -> Group:
        return Group(self._remote)

    def _to_world(self, r: int) -> int:
        if r < 0:
            return r
        return self._remote[r]

    def _from_world(self, w: int) -> int:
        return self._rw2c.get(w, w)

    def Merge(self, high: bool = False) -> Comm:
        """Intracommunicator over both groups; the group passing high=False goes first."""
        local_first = not high
        # agree on the order with the remote side: compare the lowest world ranks on ties
        me = torch.tensor([1 if high else 0, min(self._ranks)], dtype=torch.int64)
        other = torch.zeros(2, dtype=torch.int64)
        if self.Get_rank() == 0:
            r = self._irecv(other, 0, 77, self._ctx + 3)
            self._isend(me, 0, 77, self._ctx + 3).Wait()
            r.Wait()
        loc = Comm(self._ranks, self._ctx + 5)
        loc.Bcast(other, 0)
        if int(other[0]) == int(me[0]):
            local_first = min(self._ranks) < int(other[1])
        ranks = self._ranks + self._remote if local_first else self._remote + self._ranks
        return Comm(ranks, self._ctx + 7, "merged")

    def Barrier(self):
        Comm(self._ranks + self._remote if min(self._ranks) < min(self._remote) else self._remote + self._ranks,
             self._ctx + 9).Barrier()


def Intercomm_create(local_comm: Comm, local_leader: int, peer_comm: Comm, remote_leader: int, tag: int = 0) -> InterComm:
    mine = torch.tensor(local_comm.world_ranks + [-1] * (64 - local_comm.Get_size()), dtype=torch.int64)
    theirs = torch.full((64,), -1, dtype=torch.int64)
    ctx_mine = torch.tensor([_rt.state().next_ctx], dtype=torch.int64)
    ctx_theirs = torch.zeros(1, dtype=torch.int64)
    if local_comm.Get_rank() == local_leader:
        r1 = peer_comm.Irecv(theirs, remote_leader, tag)
        r2 = peer_comm.Irecv(ctx_theirs, remote_leader, tag + 1)
        peer_comm.Send(mine, remote_leader, tag)
        peer_comm.Send(ctx_mine, remote_leader, tag + 1)
        r1.Wait()
        r2.Wait()
    local_comm.Bcast(theirs, local_leader)
    local_comm.Bcast(ctx_theirs, local_leader)
    ctxl = torch.zeros(1, dtype=torch.int64)
    local_comm.Allreduce(ctx_mine, ctxl, MAX)
    ctx = max(int(ctxl.item()), int(ctx_theirs.item()))
    # both groups must pick the same id: take the max of both groups' maxima, exchanged by leaders
    both = torch.tensor([ctx], dtype=torch.int64)
    if local_comm.Get_rank() == local_leader:
        other = torch.zeros(1, dtype=torch.int64)
        r = peer_comm.Irecv(other, remote_leader, tag + 2)
        peer_comm.Send(both, remote_leader, tag + 2)
        r.Wait()
        both = torch.maximum(both, other)
    local_comm.Bcast(both, local_leader)
    ctx = int(both.item())
    _rt.state().next_ctx = max(_rt.state().next_ctx, ctx + 1)
    remote = [int(x) for x in theirs.tolist() if x >= 0]
    return InterComm(local_comm.world_ranks, remote, 2 * ctx + (1 << 26))


def Intercomm_merge(inter: InterComm, high: bool = False) -> Comm:
    return inter.Merge(high)


def Comm_test_inter(comm: Comm) -> bool:
    return comm.Is_inter()


def Comm_remote_size(comm) -> int:
    return comm.Get_remote_size()


def Comm_remote_group(comm) -> Group:
    return comm.Get_remote_group()


# ------------------------------------------------------------------ ports & names
def _ns_dir() -> str:
    d = f"/dev/shm/mpit_ns_{os.getuid()}"
    os.makedirs(d, exist_ok=True)
    return d


_port_seq = [0]


def Open_port(info=None) -> str:
    _port_seq[0] += 1
    return f"mpit-port:{_rt.state().rank}:{os.getpid()}:{_port_seq[0]}"


def Close_port(port: str):
    pass


def Publish_name(service: str, port: str, info=None):
    with open(os.path.join(_ns_dir(), service), "w") as f:
        f.write(port)


def Lookup_name(service: str, info=None) -> str:
    p = os.path.join(_ns_dir(), service)
    for _ in range(2000):
        if os.path.exists(p):
            return open(p).read()
        time.sleep(0.005)
    raise KeyError(f"service {service!r} is not published")


def Unpublish_name(service: str, port: str = "", info=None):
    try:
        os.unlink(os.path.join(_ns_dir(), service))
    except FileNotFoundError:
        pass


def _port_tag(port: str) -> int:
    return zlib.crc32(port.encode()) & 0x3FFFFFFF


def _world():
    from .comm import COMM_WORLD

    return COMM_WORLD()


def Comm_accept(port: str, info=None, root: int = 0, comm: Optional[Comm] = None) -> InterComm:
    comm = comm or _world()
    tag = _port_tag(port)
    theirs = torch.full((65,), -1, dtype=torch.int64)
    if comm.Get_rank() == root:
        w = _world()
        st = Status()
        w._irecv(theirs, ANY_SOURCE, tag, _PORT_CTX).Wait(st)
        own_ctx = _rt.state().next_ctx
        reply = torch.tensor(comm.world_ranks + [-1] * (64 - comm.Get_size()) + [own_ctx], dtype=torch.int64)
        w._isend(reply, st.source, tag, _PORT_CTX).Wait()
        theirs[64] = max(int(theirs[64]), own_ctx)  # the connector takes the same max
    comm.Bcast(theirs, root)
    remote = [int(x) for x in theirs[:64].tolist() if x >= 0]
    ctx = int(theirs[64])
    return InterComm(comm.world_ranks, remote, 2 * ctx + (1 << 27))


def Comm_connect(port: str, info=None, root: int = 0, comm: Optional[Comm] = None) -> InterComm:
    comm = comm or _world()
    tag = _port_tag(port)
    owner = int(port.split(":")[1])
    theirs = torch.full((65,), -1, dtype=torch.int64)
    if comm.Get_rank() == root:
        w = _world()
        mine = torch.tensor(comm.world_ranks + [-1] * (64 - comm.Get_size()) + [_rt.state().next_ctx], dtype=torch.int64)
        r = w._irecv(theirs, ANY_SOURCE, tag, _PORT_CTX)
        # the accepting root is the port's owner unless a different root accepts; send to owner
        w._isend(mine, owner, tag, _PORT_CTX).Wait()
        r.Wait()
        mine_ctx = int(mine[64])
        ctx = max(mine_ctx, int(theirs[64]))
        theirs[64] = ctx
    comm.Bcast(theirs, root)
    remote = [int(x) for x in theirs[:64].tolist() if x >= 0]
    return InterComm(comm.world_ranks, remote, 2 * int(theirs[64]) + (1 << 27))


def Comm_join(fd: int) -> InterComm:
    """Two processes connected by a socket form an inter-communicator."""
    s = socket.socket(fileno=os.dup(fd))
    me = _rt.state().rank
    s.sendall(struct.pack("<q", me))
    other = struct.unpack("<q", s.recv(8))[0]
    s.close()
    lo, hi = min(me, other), max(me, other)
    return InterComm([me], [other], 2 * (lo * 1024 + hi) + (1 << 28))


def Comm_get_parent():
    """No process of an mpit job was spawned by another job: COMM_NULL."""
    return None


def Comm_spawn(*args, **kw):
    raise NotImplementedError("Comm_spawn: dynamic process creation is not provided (one runtime segment per job; "
                              "launch all ranks with mpit_amd.launch / torch.distributed.run)")


Comm_spawn_multiple = Comm_spawn


def Comm_disconnect(comm: Comm):
    comm.Disconnect()

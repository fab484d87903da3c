"""Multi-rank checks of the MPI-style API (run under torch.distributed.run).

Each check prints ``OK <name>`` on rank 0; the pytest wrapper asserts all are present.
Mirrors the reference's MPI test programs with real assertions instead of printed values:
test.lua (ring Send/Recv), test/testreduceall.lua (Allreduce SUM), test/testireduceall.lua
(Iallreduce + Test before/after Wait), plus the rest of the API surface."""
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

import mpit_amd as mp
from mpit_amd import datatypes as dt
from mpit_amd import dynamic, io, mpiT, topology
from mpit_amd.comm import COMM_WORLD

mp.Init()
W = COMM_WORLD()
r, n = W.Get_rank(), W.Get_size()
dev = torch.device(os.environ.get("T_DEVICE", "cpu"))
if dev.type == "cuda":
    dev = mp.runtime.device()


def ok(name):
    W.Barrier()
    if r == 0:
        print("OK", name, flush=True)


# ---- X1 test.lua: ring Send/Recv of one float; rank 0 sends first
x = torch.tensor([float(r)], device=dev)
y = torch.zeros(1, device=dev)
if r == 0:
    W.Send(x, (r + 1) % n, 7)
    W.Recv(y, (r - 1) % n, 7)
else:
    W.Recv(y, (r - 1) % n, 7)
    W.Send(x, (r + 1) % n, 7)
assert y.item() == float((r - 1) % n)
ok("ring_send_recv")

# ---- large message (bulk stream through the shm ring, > bulk capacity)
big = torch.arange(3_000_000, dtype=torch.float32, device=dev) + r
got = torch.empty_like(big)
rq = W.Irecv(got, (r - 1) % n, 11)
W.Send(big, (r + 1) % n, 11)
st = rq.Wait()
assert torch.equal(got, torch.arange(3_000_000, dtype=torch.float32, device=dev) + (r - 1) % n)
assert st.Get_count(dt.FLOAT) == 3_000_000 and st.source == (r - 1) % n
ok("large_message")

# ---- ANY_SOURCE / ANY_TAG, Iprobe / Probe, tag matching order
if r != 0:
    W.Send(torch.tensor([r * 10], dtype=torch.int64), 0, 100 + r)
else:
    seen = set()
    for _ in range(n - 1):
        s = mp.Status()
        W.Probe(mp.ANY_SOURCE, mp.ANY_TAG, s)
        buf = torch.zeros(1, dtype=torch.int64)
        W.Recv(buf, s.source, s.tag)
        assert buf.item() == s.source * 10 and s.tag == 100 + s.source
        seen.add(s.source)
    assert seen == set(range(1, n))
ok("probe_any_source")

# non-overtaking on the same (source, tag); different tags matched out of order
if r == 1 % n and n > 1:
    for i in range(5):
        W.Send(torch.tensor([i]), 0, 3)
    W.Send(torch.tensor([99]), 0, 4)
if r == 0 and n > 1:
    t4 = torch.zeros(1, dtype=torch.int64)
    W.Recv(t4, 1, 4)
    assert t4.item() == 99
    for i in range(5):
        t = torch.zeros(1, dtype=torch.int64)
        W.Recv(t, 1, 3)
        assert t.item() == i
ok("message_ordering")

# ---- Cancel an unmatched receive (reference bug: unreachable cancel, init.lua:94-102)
req = W.Irecv(torch.zeros(4), mp.ANY_SOURCE, 999)
assert req.Cancel()
st = req.Wait()
assert st.Is_cancelled()
ok("cancel_recv")

# ---- Ssend completes only once matched; Sendrecv; persistent requests
if n > 1:
    if r == 0:
        q = W.Issend(torch.ones(2), 1, 21)
        W.Barrier()
        q.Wait()
    elif r == 1:
        W.Barrier()
        W.Recv(torch.zeros(2), 0, 21)
    else:
        W.Barrier()
ok("ssend")
s_out, s_in = torch.tensor([float(r)]), torch.zeros(1)
W.Sendrecv(s_out, (r + 1) % n, 5, s_in, (r - 1) % n, 5)
assert s_in.item() == float((r - 1) % n)
pr = W.Recv_init(s_in, (r - 1) % n, 6)
ps = W.Send_init(s_out, (r + 1) % n, 6)
for _ in range(3):
    pr.Start()
    ps.Start()
    mp.Waitall([ps, pr])
ok("sendrecv_persistent")

# ---- the mpiT facade honours count and datatype on Sendrecv / Sendrecv_replace / persistent
# requests: 3 of 8 floats, and a strided vector type (every other element)
f_out = torch.arange(8, dtype=torch.float32) + 100 * r
f_in = torch.full((8,), -1.0)
mpiT.Sendrecv(f_out, 3, mpiT.FLOAT, (r + 1) % n, 31, f_in, 3, mpiT.FLOAT, (r - 1) % n, 31, W)
src = (r - 1) % n
assert f_in[:3].tolist() == [100.0 * src + i for i in range(3)] and f_in[3:].eq(-1).all(), f_in
vec = dt.Type_vector(4, 1, 2, dt.FLOAT)
vec.Commit()
rep = torch.arange(8, dtype=torch.float32) + 100 * r
mpiT.Sendrecv_replace(rep, 1, vec, (r + 1) % n, 32, (r - 1) % n, 32, W)
want = torch.arange(8, dtype=torch.float32) + 100 * r
want[0::2] = torch.arange(0, 8, 2, dtype=torch.float32) + 100 * src
assert torch.equal(rep, want), rep
p_in = torch.full((8,), -1.0)
pr = mpiT.Recv_init(p_in, 2, mpiT.FLOAT, (r - 1) % n, 33, W)
ps = mpiT.Send_init(f_out, 2, mpiT.FLOAT, (r + 1) % n, 33, W)
pr.Start()
ps.Start()
mp.Waitall([ps, pr])
assert p_in[:2].tolist() == [100.0 * src, 100.0 * src + 1] and p_in[2:].eq(-1).all(), p_in
ok("facade_count_datatype")

# ---- X2/X3: Allreduce, Iallreduce (Test before Wait false-or-true, after Wait true)
a = torch.full((1 << 16,), float(r + 1), device=dev)
W.Allreduce(a, a, mp.SUM)
assert torch.all(a == n * (n + 1) / 2)
ia = torch.full((1000,), 2.0, device=dev)
req = W.Iallreduce(ia, ia, mp.SUM)
if req._work is not None and r == 0:
    print("DIST_WORK_REQUEST", flush=True)  # the torch.distributed branch (RCCL / gloo) ran
req.Wait()
assert req.Test() and torch.all(ia == 2.0 * n)
# ring all-reduce (host point-to-point path for n > 2): odd length, every element checked
big = torch.arange(100003, dtype=torch.float64, device=dev) * (r + 1)
W.Allreduce(big, big, mp.SUM)
assert torch.equal(big, torch.arange(100003, dtype=torch.float64, device=dev) * (n * (n + 1) / 2))
ok("allreduce_iallreduce")

# ---- reductions: MAX MIN PROD LAND BOR MAXLOC MINLOC, Reduce to root, user op
v = torch.tensor([float(r), float(-r), 2.0], device=dev)
out = torch.zeros(3, device=dev)
W.Allreduce(v, out, mp.MAX)
assert out.tolist() == [n - 1, 0.0, 2.0]
W.Allreduce(v, out, mp.MIN)
assert out.tolist() == [0.0, -(n - 1), 2.0]
W.Allreduce(torch.tensor([2.0], device=dev), out[:1], mp.PROD)
assert out[0].item() == 2.0 ** n
bits = torch.tensor([1 << r], dtype=torch.int64)
ob = torch.zeros(1, dtype=torch.int64)
W.Allreduce(bits, ob, mp.BOR)
assert ob.item() == (1 << n) - 1
loc = torch.tensor([[float((r * 7) % n), float(r)]], device=dev)
ol = torch.zeros_like(loc)
W.Allreduce(loc, ol, mp.MAXLOC)
vals = [((q * 7) % n, q) for q in range(n)]
best = max(vals, key=lambda t: (t[0], -t[1]))
assert ol.tolist()[0] == [float(best[0]), float(best[1])]
W.Allreduce(loc, ol, mp.MINLOC)
assert ol[0, 0].item() == 0.0
myop = mp.Op_create(lambda a, b: a * 2 + b, commute=False)
red = torch.zeros(1)
W.Reduce(torch.tensor([1.0]), red, myop, root=0)
if r == 0:
    e = 1.0
    for _ in range(n - 1):
        e = e * 2 + 1.0
    assert red.item() == e
ok("reductions")

# ---- Bcast / Gather(v) / Scatter(v) / Allgather(v) / Alltoall(v) / Reduce_scatter / Scan / Exscan
b = torch.arange(5, dtype=torch.float32, device=dev) * (r == 1 % n)
W.Bcast(b, root=1 % n)
assert b.tolist() == [0.0, 1.0, 2.0, 3.0, 4.0]
g = torch.zeros(2 * n, device=dev)
W.Gather(torch.tensor([r, r], dtype=torch.float32, device=dev), g, root=0)
if r == 0:
    assert g.tolist() == sum([[q, q] for q in range(n)], [])
sc = torch.zeros(2, device=dev)
W.Scatter(torch.arange(2 * n, dtype=torch.float32, device=dev), sc, root=0)
assert sc.tolist() == [2 * r, 2 * r + 1]
counts = [q + 1 for q in range(n)]
agv = torch.zeros(sum(counts), device=dev)
W.Allgatherv(torch.full((r + 1,), float(r), device=dev), agv, counts)
assert agv.tolist() == sum([[float(q)] * (q + 1) for q in range(n)], [])
ag = torch.zeros(n, device=dev)
W.Allgather(torch.tensor([float(r)], device=dev), ag)
assert ag.tolist() == list(map(float, range(n)))
a2a = torch.zeros(n, device=dev)
W.Alltoall(torch.tensor([float(100 * r + q) for q in range(n)], device=dev), a2a)
assert a2a.tolist() == [float(100 * q + r) for q in range(n)]
rs = torch.zeros(2, device=dev)
W.Reduce_scatter(torch.ones(2 * n, device=dev), rs, [2] * n, mp.SUM)
assert rs.tolist() == [float(n)] * 2
scn = torch.zeros(1, device=dev)
W.Scan(torch.tensor([float(r + 1)], device=dev), scn, mp.SUM)
assert scn.item() == (r + 1) * (r + 2) / 2
exs = torch.full((1,), -5.0, device=dev)
W.Exscan(torch.tensor([float(r + 1)], device=dev), exs, mp.SUM)
assert exs.item() == (-5.0 if r == 0 else r * (r + 1) / 2)
ok("collectives")

# ---- groups, Comm_split / Dup / Create / Compare, sub-communicator collectives
sub = W.Split(r % 2, key=-r)
assert sub.Get_size() == len([q for q in range(n) if q % 2 == r % 2])
assert sub.world_ranks == sorted([q for q in range(n) if q % 2 == r % 2], reverse=True)
t = torch.tensor([1.0])
sub.Allreduce(t, t, mp.SUM)
assert t.item() == sub.Get_size()
sub.Barrier()
d = W.Dup()
assert d.Compare(W) == mp.CONGRUENT
G = W.Get_group()
ev = G.Range_incl([(0, n - 1, 2)])
assert ev.world_ranks == list(range(0, n, 2))
assert G.Difference(ev).world_ranks == list(range(1, n, 2))
c2 = W.Create(ev)
if r % 2 == 0:
    assert c2.Get_size() == len(ev.world_ranks)
else:
    assert c2 is None
ok("groups_comms")

# ---- topologies
dims = topology.Dims_create(n, [0, 0])
cart = topology.Cart_create(W, dims, [True, False])
co = topology.Cart_coords(cart, cart.Get_rank())
assert topology.Cart_rank(cart, co) == cart.Get_rank()
src, dst = topology.Cart_shift(cart, 0, 1)
assert topology.Topo_test(cart) == topology.CART
rowc = topology.Cart_sub(cart, [False, True])
assert rowc.Get_size() == dims[1]
ok("topologies")

# ---- derived datatypes through p2p and Pack/Unpack
vec = dt.Type_vector(3, 1, 2, dt.FLOAT).Commit()
if n > 1:
    if r == 0:
        W.Send(torch.arange(6, dtype=torch.float32), 1, 40, count=1, datatype=vec)
    elif r == 1:
        dst6 = torch.full((6,), -1.0)
        W.Recv(dst6, 0, 40, count=1, datatype=vec)
        assert dst6.tolist() == [0.0, -1.0, 2.0, -1.0, 4.0, -1.0]
buf = torch.zeros(64, dtype=torch.uint8)
pos = dt.Pack(torch.arange(6, dtype=torch.float32), 1, vec, buf, 0)
outv = torch.zeros(6)
dt.Unpack(buf, 0, outv, 1, vec)
assert pos == 12 and outv.tolist() == [0.0, 0.0, 2.0, 0.0, 4.0, 0.0]
ok("datatypes")

# ---- one-sided windows: Put / Get / Accumulate / Fence / Lock
win = mp.Win.Create(torch.zeros(n, device=dev), W)
win.Fence()
win.Put(torch.tensor([float(r)], device=dev), (r + 1) % n, r)
win.Fence()
loc_t = win.tensor
assert loc_t[(r - 1) % n].item() == float((r - 1) % n)
gt = torch.zeros(1, device=dev)
win.Get(gt, (r + 1) % n, r)
win.Flush()
assert gt.item() == float(r)
acc = mp.Win.Allocate(4, torch.float32, W, device=(dev.type == "cuda"))
acc.Fence()
acc.Accumulate(torch.ones(4, device=dev), 0, 0)
acc.Fence()
if r == 0:
    assert acc.tensor.tolist() == [float(n)] * 4
acc.Lock(0, mp.LOCK_EXCLUSIVE)
acc.Unlock(0)
win.Free()
acc.Free()
# derived datatypes through the facade (mpifuncs.c:1656,1131,9): origin / target (count,
# datatype) both honoured — a vector target scatters, a vector origin gathers / unpacks
vt = mpiT.Type_commit(mpiT.Type_vector(3, 1, 2, mpiT.FLOAT))
dw = mpiT.Win_create(torch.zeros(8, device=dev), comm=W)
mpiT.Win_fence(0, dw)
src = torch.tensor([r + 1.0, r + 2.0, r + 3.0], device=dev)
assert mpiT.Put(src, 3, mpiT.FLOAT, (r + 1) % n, 1, 1, vt, dw) == mpiT.SUCCESS
mpiT.Win_fence(0, dw)
q = (r - 1) % n
assert dw.tensor.tolist() == [0.0, q + 1.0, 0.0, q + 2.0, 0.0, q + 3.0, 0.0, 0.0], dw.tensor.tolist()
got = torch.full((6,), -1.0, device=dev)
assert mpiT.Get(got, 1, vt, (r + 1) % n, 1, 1, vt, dw) == mpiT.SUCCESS
mpiT.Win_fence(0, dw)
assert got.tolist() == [r + 1.0, -1.0, r + 2.0, -1.0, r + 3.0, -1.0], got.tolist()
assert mpiT.Accumulate(torch.ones(3, device=dev), 3, mpiT.FLOAT, 0, 1, 1, vt, mpiT.SUM, dw) == mpiT.SUCCESS
mpiT.Win_fence(0, dw)
if r == 0:
    q = n - 1
    assert dw.tensor.tolist() == [0.0, q + 1.0 + n, 0.0, q + 2.0 + n, 0.0, q + 3.0 + n, 0.0, 0.0], dw.tensor.tolist()
# 1,000 Fence-synchronised datatype-faithful Puts: each closed epoch releases its origin
# buffers (Win._keep_all), so retained memory stays flat instead of growing per Put
mem0 = torch.cuda.memory_allocated(dev) if dev.type == "cuda" else 0
for _ in range(1000):
    mpiT.Put(src * 1.0, 3, mpiT.FLOAT, (r + 1) % n, 1, 1, vt, dw)
    mpiT.Win_fence(0, dw)
    assert not getattr(dw, "_keep_all", []), len(dw._keep_all)
if dev.type == "cuda":
    assert torch.cuda.memory_allocated(dev) <= mem0 + (1 << 20), (mem0, torch.cuda.memory_allocated(dev))
q = (r - 1) % n
assert dw.tensor[1].item() == q + 1.0 and dw.tensor[5].item() == q + 3.0
try:  # signatures that do not carry the same bytes are refused, not silently truncated
    mpiT.Put(src, 2, mpiT.FLOAT, (r + 1) % n, 1, 1, vt, dw)
    raise AssertionError("mismatched one-sided signature accepted")
except ValueError:
    pass
mpiT.Win_fence(0, dw)
mpiT.Win_free(dw)
ok("windows")

# ---- MPI-IO: ordered / shared / explicit-offset writes
tmpd = W.bcast_obj(tempfile.mkdtemp() if r == 0 else None, 0)
path = os.path.join(tmpd, "io.bin")
fh = io.File.Open(W, path, io.MODE_CREATE | io.MODE_RDWR)
fh.Write_at(r * 4, torch.tensor([r], dtype=torch.int32))
fh.Sync()
rd = torch.zeros(n, dtype=torch.int32)
fh.Read_at_all(0, rd)
assert rd.tolist() == list(range(n))
fh.Set_view(4 * n, dt.INT, dt.INT)
fh.Write_ordered(torch.full((r + 1,), r, dtype=torch.int32))
fh.Sync()
allv = torch.zeros(n * (n + 1) // 2, dtype=torch.int32)
fh.Read_at(0, allv)
assert allv.tolist() == sum([[q] * (q + 1) for q in range(n)], [])
fh.Close()
ok("mpi_io")

# ---- inter-communicator (two halves) + merge, connect/accept
if n >= 2:
    half = W.Split(0 if r < n // 2 else 1, r)
    peer_leader = n // 2 if r < n // 2 else 0
    inter = dynamic.Intercomm_create(half, 0, W, peer_leader, tag=555)
    assert inter.Is_inter() and inter.Get_remote_size() == (n - n // 2 if r < n // 2 else n // 2)
    if inter.Get_rank() == 0:
        inter.Send(torch.tensor([float(r)]), 0, 9)
        rb = torch.zeros(1)
        inter.Recv(rb, 0, 9)
        assert rb.item() == float(peer_leader)
    merged = inter.Merge(high=(r >= n // 2))
    assert merged.Get_size() == n
    mt = torch.ones(1)
    merged.Allreduce(mt, mt, mp.SUM)
    assert mt.item() == n
ok("intercomm")

# ---- mpiT functional API (reference call convention)
mt = torch.tensor([1.0, 2.0])
mo = torch.zeros(2)
assert mpiT.Allreduce(mt, mo, 2, mpiT.FLOAT, mpiT.SUM, mpiT.COMM_WORLD) == mpiT.SUCCESS
assert mo.tolist() == [float(n), 2.0 * n]
assert mpiT.get_size() == n and mpiT.Comm_rank(mpiT.COMM_WORLD) == r
q = mpiT.Queue()
state = {"io": True}
rb2 = torch.zeros(1)
q.push(mpiT.co_execute(mpiT.aio_recv, (rb2, 1, mpiT.FLOAT, (r - 1) % n, 61, W, state)))
q.push(mpiT.co_execute(mpiT.aio_send, (torch.tensor([float(r)]), 1, mpiT.FLOAT, (r + 1) % n, 61, W, state)))
mpiT.co_wait(q)
assert rb2.item() == float((r - 1) % n)
ok("mpiT_api")

# ---- objects
objs = W.allgather_obj({"rank": r, "t": torch.tensor([r])})
assert [o["rank"] for o in objs] == list(range(n))
if n > 1:
    if r == 0:
        W.send_obj({"w": torch.arange(3)}, 1, 8)
    elif r == 1:
        o = W.recv_obj(0, 8)
        assert torch.equal(o["w"], torch.arange(3))
ok("objects")

if r == 0:
    print("ALL_DONE", flush=True)
mp.Finalize()

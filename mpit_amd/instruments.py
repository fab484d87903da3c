"""The reference's measuring instruments as library functions, so the headline benchmark
(bench.py) can report them from the same job as the training number:

* :func:`ps_pingpong` — parameter-server ping-pong bandwidth, asyncsgd/ptest.lua:3,58-67
  (640 MiB, 100 x (recv_param + send_grad + wait), bi-directional MB/s) and
  asyncsgd/testreduceall.lua:58-66 / BiCNN/ptest2.lua:53-73 (``straggle``);
* :func:`allreduce_time` — Allreduce / Iallreduce wall time of MEGS x 2^20 floats,
  test/testreduceall.lua:8-29 and test/testireduceall.lua:27-36.

Both run on the calling job's ranks (every rank must call them) and return the same dict
on every rank. benchmarks/ps_pingpong.py and benchmarks/allreduce_bench.py are thin CLIs
over them.
"""
from __future__ import annotations

import time
from typing import Optional, Sequence

import torch

from . import runtime as _rt
from .comm import COMM_WORLD, SUM


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def ps_pingpong(mib: float = 640.0, iters: int = 100, warmup: int = 3, servers: Optional[Sequence[int]] = None,
                clients: Optional[Sequence[int]] = None, ps_id: int = 7, straggle: bool = False,
                datapath: int = 2, time_budget_s: Optional[float] = None) -> dict:
    """Each client pulls every shard and pushes its gradient per iteration (2 x payload
    bytes over the fabric per client per iteration). Default roles: first half of the
    ranks serve, second half are clients (asyncsgd/ptest.lua:20-26); one rank serves and
    trains. ``time_budget_s`` caps the timed iterations (estimated from the warm-up)."""
    from .launch import colocated, half_half
    from .parallel.ps import PClient, PServer, ServerOpt

    W = COMM_WORLD()
    rank, size = W.Get_rank(), W.Get_size()
    dev = _rt.device() or torch.device("cpu")
    if servers is None or clients is None:
        servers, clients, _ = colocated(size) if size == 1 else half_half(size)
    servers, clients = list(servers), list(clients)
    plong = int(mib * (1 << 20)) // 4
    conf = dict(rank=rank, sranks=servers, cranks=clients, plong=plong, opt=ServerOpt("sum"), datapath=datapath,
                ps_id=ps_id)
    srv = None
    if rank in servers:
        srv = PServer(conf)
        srv.start(block=False)
    # every client agrees on the iteration count (budget from the slowest warm-up)
    res, n_it = None, iters
    pc = None
    if rank in clients:
        p = torch.zeros(plong, device=dev)
        g = torch.full((plong,), 1e-6, device=dev)
        pc = PClient(conf).start(p, g)
        t0 = time.perf_counter()
        for _ in range(max(1, warmup)):
            pc.async_recv_param()
            pc.async_send_grad()
            pc.wait()
        _sync(dev)
        per = (time.perf_counter() - t0) / max(1, warmup)
        if time_budget_s is not None:
            n_it = max(3, min(iters, int(time_budget_s / max(per, 1e-6))))
    n_it = int(max(v for v in W.allgather_obj(n_it if rank in clients else 0)) or iters)
    W.Barrier()
    if pc is not None:
        extra = max(0, (rank + 1 - size // 2)) ** 2 if straggle else 0
        scratch = torch.zeros(1 << 20, device=dev)
        _sync(dev)
        t0 = time.perf_counter()
        for _ in range(n_it):
            for _ in range(extra):
                scratch.mul_(1.0001)
            pc.async_recv_param()
            pc.async_send_grad()
            pc.wait()
        _sync(dev)
        dt = time.perf_counter() - t0
        res = dict(rank=rank, seconds=round(dt, 4), GBps_bidir=round(2 * plong * 4 * n_it / dt / 1e9, 2),
                   ms_per_iter=round(1000 * dt / n_it, 3), extra_passes=extra)
        pc.stop()
    if srv is not None:
        srv.wait_done()
    rs = [r for r in W.allgather_obj(res) if r]
    return {"payload_MiB": mib, "iters": n_it, "servers": len(servers), "clients": len(clients), "device": str(dev),
            "per_client": rs, "aggregate_GBps_bidir": round(sum(r["GBps_bidir"] for r in rs), 2)}


def allreduce_time(megs: float = 10.0, iters: int = 10, host: bool = False) -> dict:
    """Allreduce SUM of megs x 2^20 fp32 on every rank (HBM tensors ride RCCL when every rank
    owns its GPU), then one Iallreduce with Test before / after Wait; checked for
    correctness against a float64 reduction of one element."""
    W = COMM_WORLD()
    dev = torch.device("cpu") if host or _rt.device() is None else _rt.device()
    n = int(megs * (1 << 20))
    x = torch.rand(n, device=dev)
    ref = x.clone()
    W.Allreduce(ref, ref, SUM)  # warm-up (communicator init)
    _sync(dev)
    W.Barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        W.Allreduce(x, ref, SUM)
    _sync(dev)
    t_ar = (time.perf_counter() - t0) / iters
    W.Barrier()
    t0 = time.perf_counter()
    req = W.Iallreduce(x, ref, SUM)
    before = req.Test()
    req.Wait()
    after = req.Test()
    _sync(dev)
    t_iar = time.perf_counter() - t0
    tot = torch.zeros(1, dtype=torch.float64)
    W.Allreduce(torch.tensor([float(x[:1].double().item())], dtype=torch.float64), tot, SUM)
    ok = abs(float(ref[0].item()) - float(tot.item())) <= 1e-4 * max(1.0, abs(float(tot.item())))
    nb = n * 4
    size = W.Get_size()
    rccl = bool(dev.type == "cuda" and W._use_rccl(x))
    return {"MiB": nb / (1 << 20), "ranks": size, "device": str(dev), "backend": "rccl" if rccl else "mpit-p2p",
            "allreduce_ms": round(1000 * t_ar, 3), "iallreduce_ms": round(1000 * t_iar, 3),
            "busbw_GBps": round(2 * (size - 1) / size * nb / t_ar / 1e9, 2) if size > 1 else None,
            "test_before_wait": bool(before), "test_after_wait": bool(after), "correct": ok}

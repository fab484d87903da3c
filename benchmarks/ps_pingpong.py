"""Parameter-server ping-pong bandwidth (the reference's asyncsgd/ptest.lua:3,58-67 and
asyncsgd/testreduceall.lua:58-66 instruments; BiCNN/ptest2.lua:53-73 with --straggle).

    python -m mpit_amd.launch -n 2 benchmarks/ps_pingpong.py --mib 640 --iters 100

First half of the ranks serve, second half are clients (ptest.lua:20-26), or
``--colocated``. Each iteration a client pulls every shard and pushes its gradient
(recv_param + send_grad + wait), i.e. 2 x payload bytes cross the fabric per client per
iteration; the reported number is that bi-directional volume per second per client, and
summed over clients. ``--straggle`` adds ``(rank+1-size/2)^2`` extra elementwise passes per
iteration on each client (ptest2.lua:66-70) to show the asynchronous server is not held
back by slow clients.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import mpit_amd as mp
from mpit_amd.launch import colocated, half_half
from mpit_amd.parallel.ps import PClient, PServer, ServerOpt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=float, default=640.0)
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--colocated", action="store_true")
    ap.add_argument("--straggle", action="store_true")
    ap.add_argument("--datapath", type=int, default=2)
    a = ap.parse_args()
    mp.Init()
    W = mp.COMM_WORLD()
    rank, size = W.Get_rank(), W.Get_size()
    dev = mp.runtime.device() or torch.device("cpu")
    servers, clients, _ = colocated(size) if (a.colocated or size == 1) else half_half(size)
    plong = int(a.mib * (1 << 20)) // 4
    conf = dict(rank=rank, sranks=servers, cranks=clients, plong=plong, opt=ServerOpt("sum"), datapath=a.datapath)
    srv = None
    if rank in servers:
        srv = PServer(conf)
        srv.start(block=rank not in clients)
    res = None
    if rank in clients:
        p = torch.zeros(plong, device=dev)
        g = torch.full((plong,), 1e-6, device=dev)
        pc = PClient(conf).start(p, g)
        extra = max(0, (rank + 1 - size // 2)) ** 2 if a.straggle else 0
        scratch = torch.zeros(1 << 20, device=dev)
        for _ in range(a.warmup):
            pc.async_recv_param()
            pc.async_send_grad()
            pc.wait()
        if dev.type == "cuda":
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            for _ in range(extra):
                scratch.mul_(1.0001)
            pc.async_recv_param()
            pc.async_send_grad()
            pc.wait()
        if dev.type == "cuda":
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        gbps = 2 * plong * 4 * a.iters / dt / 1e9
        res = dict(rank=rank, seconds=round(dt, 4), GBps_bidir=round(gbps, 2), ms_per_iter=round(1000 * dt / a.iters, 3),
                   extra_passes=extra)
        pc.stop()
    allr = W.allgather_obj(res)
    if srv is not None and rank in clients:
        srv.wait_done()
    if rank == 0:
        rs = [r for r in allr if r]
        print(json.dumps({"benchmark": "ps_pingpong", "payload_MiB": a.mib, "iters": a.iters, "servers": len(servers),
                          "clients": len(clients), "device": str(dev), "per_client": rs,
                          "aggregate_GBps_bidir": round(sum(r["GBps_bidir"] for r in rs), 2)}), flush=True)
    mp.Finalize()


if __name__ == "__main__":
    main()

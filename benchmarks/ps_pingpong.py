"""Parameter-server ping-pong bandwidth (the reference's asyncsgd/ptest.lua:3,58-67 and
asyncsgd/testreduceall.lua:58-66 instruments; BiCNN/ptest2.lua:53-73 with --straggle).

    python -m mpit_amd.launch -n 2 benchmarks/ps_pingpong.py --mib 640 --iters 100

First half of the ranks serve, second half are clients (ptest.lua:20-26), or
``--colocated``. Each iteration a client pulls every shard and pushes its gradient
(recv_param + send_grad + wait), i.e. 2 x payload bytes cross the fabric per client per
iteration; the reported number is that bi-directional volume per second per client, and
summed over clients. ``--straggle`` adds ``(rank+1-size/2)^2`` extra elementwise passes per
iteration on each client (ptest2.lua:66-70) to show the asynchronous server is not held
back by slow clients. The measurement itself is mpit_amd.instruments.ps_pingpong.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import mpit_amd as mp
from mpit_amd.instruments import ps_pingpong
from mpit_amd.launch import colocated, half_half


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
    size = W.Get_size()
    servers, clients, _ = colocated(size) if (a.colocated or size == 1) else half_half(size)
    r = ps_pingpong(a.mib, a.iters, a.warmup, servers, clients, straggle=a.straggle, datapath=a.datapath)
    if W.Get_rank() == 0:
        print(json.dumps(dict(benchmark="ps_pingpong", **r)), flush=True)
    mp.Finalize()


if __name__ == "__main__":
    main()

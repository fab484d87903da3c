"""Allreduce / Iallreduce wall time (the reference's test/testreduceall.lua:8-29 and
test/testireduceall.lua:27-36 instruments): MEGS x 2^20 floats (default 10 -> 40 MiB),
SUM, checked for correctness, timed over --iters calls. HBM tensors use RCCL when every
rank owns a distinct GPU, host tensors the shm point-to-point layer (ring all-reduce).
The measurement itself is mpit_amd.instruments.allreduce_time.

    MEGS=10 python -m torch.distributed.run --nproc-per-node 8 benchmarks/allreduce_bench.py
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import mpit_amd as mp
from mpit_amd.instruments import allreduce_time


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--megs", type=float, default=float(os.environ.get("MEGS", "10")))
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--host", action="store_true")
    a = ap.parse_args()
    mp.Init()
    r = allreduce_time(a.megs, a.iters, a.host)
    if mp.COMM_WORLD().Get_rank() == 0:
        print(json.dumps(dict(benchmark="allreduce", **r)), flush=True)
    mp.Finalize()


if __name__ == "__main__":
    main()

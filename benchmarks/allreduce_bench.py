"""Allreduce / Iallreduce wall time (the reference's test/testreduceall.lua:8-29 and
test/testireduceall.lua:27-36 instruments): MEGS x 2^20 floats (default 10 -> 40 MiB),
SUM, checked for correctness, timed over --iters calls. HBM tensors use RCCL when every
rank owns a distinct GPU, host tensors the shm point-to-point layer.

    MEGS=10 python -m torch.distributed.run --nproc-per-node 8 benchmarks/allreduce_bench.py
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import mpit_amd as mp


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--megs", type=float, default=float(os.environ.get("MEGS", "10")))
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--host", action="store_true")
    a = ap.parse_args()
    mp.Init()
    W = mp.COMM_WORLD()
    dev = torch.device("cpu") if a.host or mp.runtime.device() is None else mp.runtime.device()
    n = int(a.megs * (1 << 20))
    x = torch.rand(n, device=dev, generator=None)
    ref = x.clone()
    W.Allreduce(ref, ref, mp.SUM)  # warm-up (RCCL communicator init)
    sync = (lambda: torch.cuda.synchronize()) if dev.type == "cuda" else (lambda: None)
    sync()
    W.Barrier()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        W.Allreduce(x, ref, mp.SUM)
    sync()
    t_ar = (time.perf_counter() - t0) / a.iters
    W.Barrier()
    t0 = time.perf_counter()
    req = W.Iallreduce(x, ref, mp.SUM)
    before = req.Test()
    req.Wait()
    after = req.Test()
    sync()
    t_iar = time.perf_counter() - t0
    tot = torch.zeros(1, dtype=torch.float64)
    W.Allreduce(torch.tensor([float(x[:1].double().item())], dtype=torch.float64), tot, mp.SUM)
    ok = abs(float(ref[0].item()) - float(tot.item())) <= 1e-4 * max(1.0, abs(float(tot.item())))
    if W.Get_rank() == 0:
        nb = n * 4
        print(json.dumps({"benchmark": "allreduce", "MiB": nb / (1 << 20), "ranks": W.Get_size(), "device": str(dev),
                          "allreduce_ms": round(1000 * t_ar, 3), "iallreduce_ms": round(1000 * t_iar, 3),
                          "busbw_GBps": round(2 * (W.Get_size() - 1) / W.Get_size() * nb / t_ar / 1e9, 2),
                          "test_before_wait": bool(before), "test_after_wait": bool(after), "correct": ok}), flush=True)
    mp.Finalize()


if __name__ == "__main__":
    main()

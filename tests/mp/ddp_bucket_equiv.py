"""Bucketed synchronous DP (parallel/ddp.py) against one bucket (BASELINE config 3;
test/testreduceall.lua:28, test/testireduceall.lua:32-38 are the reference's primitives).

Part A (T_TRAIN=1, 2 ranks: a sum of two is order-free, so any bucketing must give the same
bits): two allreduce trainers from one init, one with tiny buckets (many non-blocking
all-reduces launched from the backward's hooks), one with a single bucket; final parameters
bitwise equal on every rank.
Part B (any rank count): gradients of exactly representable values (multiples of 2^-8, sums
exact in fp32) through BucketedAllreduce with tiny buckets and with one bucket: bitwise equal
to each other and to the exact sum (every element reduced exactly once, padding untouched).
Prints one RESULT line from rank 0."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

import mpit_amd as mp
from mpit_amd.models import get_model
from mpit_amd.parallel.ddp import BucketedAllreduce
from mpit_amd.train import TrainConfig, Trainer, timed_steps
from mpit_amd.utils.flat import FlatParams

mp.Init()
W = mp.COMM_WORLD()
r, n = W.Get_rank(), W.Get_size()
res = {}
if os.environ.get("T_TRAIN", "0") == "1":
    finals = {}
    for name, mb in (("tiny", 0.02), ("one", 1e6)):
        tr = Trainer(TrainConfig(model="cnn7", batch=8, num_classes=10, optimizer="allreduce", lr=0.05,
                                 bucket_mb=mb))
        nb = len(tr.ddp.buckets)
        timed_steps(tr, 4, 1)
        finals[name] = (tr.flat.flat.detach().clone(), nb)
        tr.stop()
    a, b = finals["tiny"][0], finals["one"][0]
    res["train"] = {"same": bool(torch.equal(a.view(torch.int32), b.view(torch.int32))),
                    "buckets": (finals["tiny"][1], finals["one"][1])}
torch.manual_seed(5)
model = get_model("cnn7", num_classes=10)
out = {}
for name, mb in (("tiny", 0.02), ("one", 1e6)):
    fp = FlatParams(model)
    ar = BucketedAllreduce(model, fp, bucket_mb=mb, first_bucket_mb=0.01 if mb < 1 else 0.0)
    g = torch.Generator().manual_seed(100 + r)
    vals = torch.randint(-512, 512, (fp.numel,), generator=g).float() / 256.0
    fp.grad.zero_()
    for p, off in zip(fp.params, fp.offsets):
        fp.grad[off:off + p.numel()].copy_(vals[off:off + p.numel()])
    for b in range(len(ar.buckets)):  # as the backward hooks would, last bucket first
        ar._launch(len(ar.buckets) - 1 - b)
    ar.finish()
    out[name] = (fp.grad.clone(), len(ar.buckets))
    ar.remove()
exp = torch.zeros_like(out["one"][0])
for q in range(n):
    g = torch.Generator().manual_seed(100 + q)
    exp += torch.randint(-512, 512, (exp.numel(),), generator=g).float() / 256.0
fp = FlatParams(model)
mask = torch.zeros_like(exp, dtype=torch.bool)
for p, off in zip(fp.params, fp.offsets):
    mask[off:off + p.numel()] = True
ta, tb = out["tiny"][0], out["one"][0]
res["exact"] = {"same": bool(torch.equal(ta.view(torch.int32), tb.view(torch.int32))),
                "exact": bool(torch.equal(ta[mask], exp[mask])), "buckets": (out["tiny"][1], out["one"][1])}
allr = W.allgather_obj(res)
if r == 0:
    print("RESULT", allr, flush=True)
mp.Finalize()

"""How far ahead of the GPU the host runs in one ResNet-50 Downpour step (N=1).

Times, per step, when the host has finished issuing the forward and the backward (CPU
timestamps, no device sync) against the full step (which ends with the PS wait, i.e. the GPU).
If "backward issued" approaches the step time the step is host-bound.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import mpit_amd as mp
from mpit_amd.train import TrainConfig, Trainer

mp.Init()
# T_AMP=1: the bf16 autocast step (the one whose host can fall behind the GPU)
tr = Trainer(TrainConfig(model=sys.argv[1] if len(sys.argv) > 1 else "resnet50", batch=256,
                         amp=os.environ.get("T_AMP") == "1"))
marks = {}
orig_forward = tr.model.forward


def fwd(*a, **k):
    out = orig_forward(*a, **k)
    marks["fwd"] = time.perf_counter()
    return out


tr.model.forward = fwd
orig_feval = tr._feval


def feval(w):
    r = orig_feval(w)
    marks["bwd"] = time.perf_counter()
    return r


tr._feval = feval
for _ in range(5):
    tr.step()
torch.cuda.synchronize()
rows = []
for _ in range(10):
    t0 = time.perf_counter()
    tr.step()
    t1 = time.perf_counter()
    rows.append((marks["fwd"] - t0, marks["bwd"] - t0, t1 - t0))
torch.cuda.synchronize()
n = len(rows)
print(json.dumps({"forward_issued_ms": round(1e3 * sum(r[0] for r in rows) / n, 2),
                  "backward_issued_ms": round(1e3 * sum(r[1] for r in rows) / n, 2),
                  "step_ms": round(1e3 * sum(r[2] for r in rows) / n, 2)}))
tr.stop()
mp.Finalize()

"""Sync all-reduce DP on the GPU with the parameter-server path's step machinery (stolen
gradients, weight gradients written into their flat slots on the side stream, per-bucket
gather, next step's weight casts queued early: train.py ``ar_steal``) must give the same bits
as the plain path (autograd accumulating into the flat gradient, no side stream). The plain
arm runs first in the process (nothing has enabled the side stream yet). RESULT line."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

import mpit_amd as mp
from mpit_amd.train import TrainConfig, Trainer, timed_steps

torch.backends.cudnn.deterministic = True
torch.backends.cudnn.benchmark = False
model = os.environ.get("T_MODEL", "resnet18")
mp.Init()
res = {}
for amp in (False, True):
    finals = {}
    for arm in ("plain", "steal"):
        os.environ["MPIT_AR_STEAL"] = "1" if arm == "steal" else "0"
        tr = Trainer(TrainConfig(model=model, batch=8, num_classes=10, optimizer="allreduce", lr=0.05, amp=amp))
        assert getattr(tr, "ar_steal", False) == (arm == "steal")
        timed_steps(tr, 6, 1)
        finals[arm] = tr.flat.flat.detach().clone()
        tr.stop()
        del tr
    a, b = finals["plain"], finals["steal"]
    res["bf16" if amp else "fp32"] = (bool(torch.equal(a.view(torch.int32), b.view(torch.int32))),
                                      float((a - b).abs().max()))
print("RESULT", res, flush=True)
mp.Finalize()

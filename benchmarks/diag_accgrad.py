"""Diagnostic: which trainer configuration makes autograd warn that an AccumulateGrad
node's stream does not match the producing node's stream?

Builds small ResNet-50 trainers (batch 16) under a few switches and reports, per step,
whether the warning fired. Prints one JSON line per variant."""
import json
import os
import sys
import warnings

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import mpit_amd as mp
from mpit_amd.train import TrainConfig, Trainer


def run(name, env, amp=False, steps=3, **extra):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        tr = Trainer(TrainConfig(model="resnet50", batch=16, amp=amp, extra=dict(ps_id=len(seen), **extra)))
        per = []
        for _ in range(steps):
            with warnings.catch_warnings(record=True) as w:
                warnings.simplefilter("always")
                tr.step()
                torch.cuda.synchronize()
            per.append(sum("AccumulateGrad" in str(x.message) for x in w))
        tr.stop()
        print(json.dumps({"variant": name, "warnings_per_step": per}), flush=True)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


seen = []
mp.Init()
for name, env, kw in [("default", {}, {}), ("no_hp_stream", {"MPIT_HP_STREAM": "0"}, {}),
                      ("no_overlap_push", {}, {"overlap_push": False}),
                      ("no_wgrad_stream", {"MPIT_WGRAD_STREAM": "0"}, {}),
                      ("bf16", {}, {"_amp": True})]:
    amp = kw.pop("_amp", False)
    run(name, env, amp=amp, **kw)
    seen.append(name)
mp.Finalize()

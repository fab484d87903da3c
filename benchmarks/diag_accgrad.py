"""Diagnostic: which trainer configuration makes autograd warn that an AccumulateGrad
node's stream does not match the producing node's stream?

The warning fires once per process, so every variant runs in its own process:
    python benchmarks/diag_accgrad.py            # all variants, one JSON line each
    python benchmarks/diag_accgrad.py <variant>  # one variant (child)"""
import json
import os
import subprocess
import sys
import warnings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VARIANTS = {
    "default": ({}, {}, False),
    "no_hp_stream": ({"MPIT_HP_STREAM": "0"}, {}, False),
    "hp_init": ({"MPIT_HP_INIT": "1"}, {}, False),
    "no_overlap_push": ({}, {"overlap_push": False}, False),
    "no_wgrad_stream": ({"MPIT_WGRAD_STREAM": "0"}, {}, False),
    "bf16": ({}, {}, True),
}


def child(name):
    sys.path.insert(0, ROOT)
    import torch

    import mpit_amd as mp
    from mpit_amd.train import TrainConfig, Trainer

    env, extra, amp = VARIANTS[name]
    mp.Init()
    tr = Trainer(TrainConfig(model="resnet50", batch=16, amp=amp, extra=extra))
    per = []
    for _ in range(4):
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            tr.step()
            torch.cuda.synchronize()
        per.append(sum("AccumulateGrad" in str(x.message) for x in w))
    tr.stop()
    print(json.dumps({"variant": name, "warnings_per_step": per}), flush=True)
    mp.Finalize()


if __name__ == "__main__":
    if len(sys.argv) > 1:
        child(sys.argv[1])
    else:
        for name, (env, _, _) in VARIANTS.items():
            r = subprocess.run([sys.executable, os.path.abspath(__file__), name], env=dict(os.environ, **env),
                               capture_output=True, text=True, timeout=240)
            line = [x for x in r.stdout.splitlines() if x.startswith("{")]
            print(line[-1] if line else json.dumps({"variant": name, "rc": r.returncode, "err": r.stderr[-400:]}),
                  flush=True)

#!/usr/bin/env python3
"""Headline benchmark: images/sec (whole node) of ResNet-50 async-SGD (Downpour) through
the mpit_amd parameter server on 1/2/4/8 MI355X (BASELINE.json).

    python bench.py --gpus 1 --steps 20 --warmup 5
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8 --steps 20 --warmup 5

One process per GPU. Every rank trains a ResNet-50 replica on a synthetic ImageNet batch
(random bf16 images, random labels, random-init weights) AND serves one shard of the
flat parameter vector (co-located sharded parameter servers). Each step: forward +
backward (bf16 autocast, channels_last), fused Downpour scale into the push window, push
of every gradient shard to its server + pull of every refreshed shard (one fused HIP
kernel per shard reading / writing the worker's HBM over xGMI), wait. Weak scaling: the
per-GPU batch is fixed. The timed region is exactly `--steps` full steps bracketed by a
barrier + device synchronize on both sides; the reported time is the max over ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

METRIC = "images/sec (whole node) ResNet-50 async-SGD at 1/2/4/8 MI355X"
_REPO = os.path.dirname(os.path.abspath(__file__))
# MIOpen find / perf databases are kept in-tree (miopen_db/) so a fresh box reuses the
# algorithm choices of earlier runs instead of re-searching every convolution.
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(_REPO, "miopen_db"))
os.environ.setdefault("MIOPEN_CUSTOM_CACHE_DIR", os.path.join(_REPO, "miopen_db", "kcache"))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--optimizer", default="downpour", choices=["downpour", "eamsgd", "easgd", "msgd", "allreduce"])
    ap.add_argument("--topology", default="colocated", choices=["colocated", "dedicated"])
    ap.add_argument("--servers", type=int, default=1)
    ap.add_argument("--su", type=int, default=1)
    ap.add_argument("--lr", type=float, default=0.05,
                    help="learning rate; Downpour divides it by the number of workers (every worker's "
                         "push is applied, so N pushes per round then add up to one step of this size)")
    ap.add_argument("--datapath", type=int, default=2)
    ap.add_argument("--staleness", type=int, default=-1, help="bounded staleness (SSP); -1 = fully async")
    ap.add_argument("--wire", default="fp32", choices=["fp32", "bf16"], help="EASGD elastic-difference dtype")
    ap.add_argument("--no-amp", action="store_true")
    ap.add_argument("--no-channels-last", action="store_true")
    ap.add_argument("--miopen-find", action="store_true",
                    help="exhaustive MIOpen algorithm search (measured: same steady-state speed as the "
                         "heuristics for ResNet-50 bf16 NHWC on MI355X, but minutes of warm-up)")
    a = ap.parse_args(argv)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}; launch N>1 with torch.distributed.run",
              file=sys.stderr)
        return 2

    import torch

    torch.backends.cudnn.benchmark = a.miopen_find
    import mpit_amd as mp
    from mpit_amd.train import TrainConfig, Trainer, timed_steps

    mp.Init()
    mva = 0.9 / max(1, a.gpus) if a.optimizer in ("eamsgd", "easgd") else 0.0
    nw = a.gpus if a.topology == "colocated" else max(1, a.gpus - a.servers)
    lr = a.lr / max(1, nw) if a.optimizer == "downpour" else a.lr
    cfg = TrainConfig(model=a.model, batch=a.batch, optimizer=a.optimizer, topology=a.topology, servers=a.servers,
                      su=a.su, lr=lr, mva=mva, mom=0.0, amp=not a.no_amp, channels_last=not a.no_channels_last,
                      datapath=a.datapath, staleness=a.staleness, wire_dtype=a.wire)
    tr = Trainer(cfg)
    secs, loss = timed_steps(tr, a.steps, a.warmup)
    nworkers = len(tr.cranks)
    from mpit_amd.models.cnn import INPUT_SHAPES

    shape = INPUT_SHAPES.get(a.model, (3, 224, 224))
    images = a.steps * a.batch * nworkers
    value = images / secs
    import math

    lossv = float(loss.float().item()) if loss is not None else None
    if lossv is not None and not math.isfinite(lossv):
        lossv = None  # keep the line strict JSON
    tr.stop()
    if tr.rank == 0:
        par = {"downpour": "async-ps", "eamsgd": "easgd-ps", "easgd": "easgd-ps", "msgd": "local",
               "allreduce": "dp"}[a.optimizer]
        if a.optimizer != "allreduce" and a.optimizer != "msgd":
            par += f"-{a.topology}-{len(tr.sranks)}srv-{nworkers}wrk"
        else:
            par += str(a.gpus)
        out = {
            "metric": METRIC if (a.model == "resnet50" and a.optimizer == "downpour") else
                      f"images/sec (whole node) {a.model} {a.optimizer}",
            "value": round(value, 2),
            "unit": "images/sec",
            "n_gpus": a.gpus,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1000.0 * secs / a.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if (tr.on_gpu and not a.no_amp) else "fp32",
            "data": f"synthetic (random images {shape[0]}x{shape[1]}x{shape[2]}, random labels, random-init weights)",
            "config": {"model": a.model, "global_batch": a.batch * nworkers, "seq_len": None, "image_size": shape[-1],
                       "parallelism": par, "optimizer": a.optimizer, "su": a.su, "per_gpu_batch": a.batch,
                       "master_weights": "fp32", "loss_last": lossv},
        }
        print(json.dumps(out), flush=True)
    mp.Finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main())

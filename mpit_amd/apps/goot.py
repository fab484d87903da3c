"""CIFAR-10 trainer with the 7-layer CNN through the parameter server
(asyncsgd/goot.lua + asyncsgd/mlaunch.lua / claunch.lua / glaunch.lua).

    python -m mpit_amd.launch -n 4 -m mpit_amd.apps.goot --optimizer eamsgd --epochs 2
    python -m mpit_amd.apps.goot --optimizer msgd          # single process (claunch/glaunch)

Roles follow mlaunch (even ranks serve, odd ranks train) unless ``--topology colocated``.
Defaults follow mlaunch's EAMSGD config: su=2, mva=0.9/p, lr=1e-2, mom=0.99
(asyncsgd/mlaunch.lua:48-67). Data: CIFAR-10 from ``--data`` (an ``.npz`` with
``x_train`` [N,32,32,3] uint8, ``y_train``, ``x_test``, ``y_test``) or a deterministic
synthetic stand-in with the same shapes. Training applies a per-sample random 28x28 crop,
testing a center crop (asyncsgd/goot.lua:160-184, :265-322); the batch goes through the
model at once instead of one sample at a time. Seeds are per rank (the reference's
same-second ``os.time()`` seeds are a defect).

Reference defects fixed: claunch's single-process EASGD run fails (asyncsgd/claunch.lua:10)
— here a single process runs EASGD against a co-located server; mlaunch's GPU branch is
disabled (asyncsgd/mlaunch.lua:76-77) — here workers use the GPU when present.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F

import mpit_amd as mp
from mpit_amd.launch import colocated, even_odd
from mpit_amd.models import get_model
from mpit_amd.optim import ALL as OPTIMS
from mpit_amd.parallel.ps import PClient, PServer, ServerOpt
from mpit_amd.utils import checkpoint
from mpit_amd.utils.flat import FlatParams
from mpit_amd.utils.metrics import ConfusionMatrix, JsonLogger
from mpit_amd.utils.trace import Timers


def load_cifar(path: str, subset: bool, seed: int):
    if path and os.path.exists(path):
        d = np.load(path, allow_pickle=False)
        xtr, ytr, xte, yte = d["x_train"], d["y_train"], d["x_test"], d["y_test"]
    else:
        g = np.random.default_rng(seed)
        # synthetic stand-in: class-dependent colour means so the task is learnable
        ntr, nte = (2000, 1000) if subset else (50000, 10000)
        ytr, yte = g.integers(0, 10, ntr), g.integers(0, 10, nte)
        means = g.integers(40, 215, (10, 1, 1, 3))
        xtr = np.clip(means[ytr] + g.normal(0, 40, (ntr, 32, 32, 3)), 0, 255).astype(np.uint8)
        xte = np.clip(means[yte] + g.normal(0, 40, (nte, 32, 32, 3)), 0, 255).astype(np.uint8)
    if subset:
        xtr, ytr, xte, yte = xtr[:2000], ytr[:2000], xte[:1000], yte[:1000]
    to_t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).permute(0, 3, 1, 2).float().div_(255.0)  # noqa: E731
    return to_t(xtr), torch.from_numpy(np.asarray(ytr)).long(), to_t(xte), torch.from_numpy(np.asarray(yte)).long()


def random_crop(x: torch.Tensor, size: int, gen: torch.Generator) -> torch.Tensor:
    n, c, h, w = x.shape
    i = torch.randint(0, h - size + 1, (n,), generator=gen)
    j = torch.randint(0, w - size + 1, (n,), generator=gen)
    rows = (i[:, None] + torch.arange(size)[None, :])  # [n, size]
    cols = (j[:, None] + torch.arange(size)[None, :])
    return x[torch.arange(n)[:, None, None, None], torch.arange(c)[None, :, None, None], rows[:, None, :, None],
             cols[:, None, None, :]]


def center_crop(x: torch.Tensor, size: int) -> torch.Tensor:
    h, w = x.shape[-2:]
    i, j = (h - size) // 2, (w - size) // 2
    return x[..., i: i + size, j: j + size]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--optimizer", default="eamsgd", choices=["eamsgd", "easgd", "downpour", "msgd"])
    ap.add_argument("--topology", default="even_odd", choices=["even_odd", "colocated"])
    ap.add_argument("--lr", type=float, default=1e-2)
    ap.add_argument("--mom", type=float, default=0.99)
    ap.add_argument("--su", type=int, default=2)
    ap.add_argument("--mva", type=float, default=None)
    ap.add_argument("--l2wd", type=float, default=0.0)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--max-steps", type=int, default=0, help="stop each epoch after this many steps (0: full)")
    ap.add_argument("--data", default="")
    ap.add_argument("--subset", action="store_true", help="2k/1k subset (asyncsgd/goot.lua:48-54)")
    ap.add_argument("--save", default="goot_out")
    ap.add_argument("--saveep", type=int, default=10)
    ap.add_argument("--resume", action="store_true")
    a = ap.parse_args(argv)

    mp.Init()
    W = mp.COMM_WORLD()
    rank, size = W.Get_rank(), W.Get_size()
    dev = mp.runtime.device() or torch.device("cpu")
    if size == 1 or a.topology == "colocated":
        sranks, cranks, _ = colocated(size)
    else:
        sranks, cranks, _ = even_odd(size)
    p = len(cranks)
    mva = a.mva if a.mva is not None else 0.9 / p
    torch.manual_seed(1)  # identical model init everywhere
    model = get_model("cnn7").to(dev)
    flat = FlatParams(model)
    plong = flat.numel
    conf = dict(rank=rank, sranks=sranks, cranks=cranks, plong=plong, opt=ServerOpt("sum"))
    server = client = None
    if rank in sranks and a.optimizer != "msgd":
        server = PServer(conf)
        server.start(block=rank not in cranks)
    timers = Timers()
    if rank in cranks:
        log = JsonLogger(os.path.join(a.save, f"train_rank{rank}.jsonl"), rank)
        tlog = JsonLogger(os.path.join(a.save, f"test_rank{rank}.jsonl"), rank)
        gen = torch.Generator().manual_seed(1000 + rank)
        xtr, ytr, xte, yte = load_cifar(a.data, a.subset, seed=7)
        state = {}
        config = dict(lr=a.lr, mom=a.mom, su=a.su, mva=mva, l2wd=a.l2wd)
        if a.optimizer != "msgd":
            client = PClient(conf)
            if a.optimizer in ("eamsgd", "easgd"):
                client.start(torch.zeros(plong, device=dev), torch.zeros(plong, device=dev), init=flat.flat)
            else:
                client.start(flat.flat, torch.zeros(plong, device=dev))
                if client.rx.data_ptr() != flat.flat.data_ptr():
                    flat.rebind(client.rx)
            config["pclient"] = client
        opti = OPTIMS[a.optimizer]
        if a.resume:
            ck = checkpoint.latest(a.save, rank)
            if ck:
                checkpoint.load(ck, flat, state)
        cm = ConfusionMatrix(10)
        t_start = time.perf_counter()
        nsamples = 0
        for ep in range(a.epochs):
            perm = torch.randperm(xtr.shape[0], generator=gen)
            cm.zero()
            model.train()
            nb = xtr.shape[0] // a.batch
            if a.max_steps:
                nb = min(nb, a.max_steps)
            for b in range(nb):
                idx = perm[b * a.batch: (b + 1) * a.batch]
                xb = random_crop(xtr[idx], 28, gen).to(dev)
                yb = ytr[idx].to(dev)

                def feval(w):
                    with timers("feval"):
                        flat.zero_grad()
                        out = model(xb)
                        loss = F.nll_loss(out, yb)
                        loss.backward()
                        cm.batch_add(out.detach(), yb)
                    return loss.detach(), flat.grad

                _, (fx,) = opti(feval, flat.flat, config, state)
                nsamples += xb.shape[0]
            log.log(epoch=ep, train_acc=cm.total_valid, loss=float(fx) if fx is not None else None)
            # test (center crop)
            model.eval()
            tc = ConfusionMatrix(10)
            with torch.no_grad():
                for s in range(0, xte.shape[0], 500):
                    xb = center_crop(xte[s: s + 500], 28).to(dev)
                    tc.batch_add(model(xb), yte[s: s + 500].to(dev))
            tlog.log(epoch=ep, test_acc=tc.total_valid)
            if rank == cranks[0]:
                print(f"[goot] epoch {ep} train {100 * cm.total_valid:.2f}% test {100 * tc.total_valid:.2f}%", flush=True)
            if (ep + 1) % a.saveep == 0 or ep == a.epochs - 1:
                checkpoint.save(a.save, ep + 1, rank, flat, state)
        total = time.perf_counter() - t_start
        if client is not None:
            client.stop()
        fe = timers.total["feval"]
        print(f"[goot] rank {rank}: total {total:.2f}s feval {fe:.2f}s per-sample {1000 * fe / max(1, nsamples):.3f}ms "
              f"sync {state.get('dusync', 0.0):.2f}s", flush=True)
        log.close()
        tlog.close()
    if server is not None and rank in cranks:
        server.wait_done()
    W.Barrier()
    mp.Finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main())

#!/usr/bin/env python3
"""Headline benchmark: images/sec (whole node) of ResNet-50 async-SGD (Downpour) through
the mpit_amd parameter server on 1/2/4/8 MI355X (BASELINE.json).

    python bench.py --gpus 1 --steps 20 --warmup 5
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8 --steps 20 --warmup 5

One process per GPU. Every rank trains a ResNet-50 replica on a synthetic ImageNet batch
(random images, random labels, random-init weights) AND serves one shard of the flat
parameter vector (co-located sharded parameter servers). Each step: forward + backward,
fused Downpour scale into the push window, push of every gradient shard to its server +
pull of every refreshed shard (overlapped with the backward, shard by shard), wait. Weak
scaling: the per-GPU batch is fixed. The timed region is exactly ``--steps`` full steps
bracketed by a barrier + device synchronize on both sides; the reported time is the max
over ranks.

Precision: the headline is **fp32** — the reference trains fp32 Float/CudaTensors
(asyncsgd/glaunch.lua:11, BiCNN/plaunch.lua:200) — with fp32 weights, activations and
gradients on the hand-written gfx950 kernels. Every GEMM-shaped op runs as fp16x3 split
products on the fp16 MFMA (``"fp32_gemm": "fp16x3"`` in the JSON; ops/conv.py,
csrc/kernels/gemm.hip FM 11): each operand is scaled by a power of two from a device-side
bound and split exactly into two fp16 planes (22 significant bits), three MFMAs per product
with fp32 accumulation. Measured closer to fp64 than PyTorch's fp32 GEMMs on every
ResNet-50 shape (tests/test_fp32_path.py). ``MPIT_F32_SPLIT=bf16x6`` selects the 6-MFMA bf16
split instead. bf16 autocast (fp32 master weights) is reported as the secondary field
``secondary.bf16_autocast`` of the same job.

The last pulls of a step are waited for at the end of that step (the reference's
push, pull, wait: asyncsgd/optim-downpour.lua:50-53); ``--defer-ps-wait`` retires them at
the next step's first read of the weights instead (measured slower, off by default).

``peak_mem_gib``: the device memory peak of the headline run (torch.cuda.max_memory_allocated).
The next step's weight casts are queued as soon as a step's pulls have landed (the weights
change only by the pulls; mpit_amd/train.py precast): that is part of each timed step.

Also reported, outside the timed region (``--no-secondary`` skips them):
* ``ps_check``: after the run every worker pulls every shard again and the exact bit-sums
  of each shard must agree between all workers and the owning server (exit status 3 if
  not); ``world`` / ``rccl``: the ranks and the collective backend actually seen;
* at N > 1: ``secondary.dedicated``: the same step in BASELINE config 2's topology (1
  dedicated pserver + N-1 workers); ``secondary.ps_pingpong``: the reference's
  asyncsgd/ptest.lua instrument (640 MiB pull + push, bi-directional GB/s);
  ``secondary.allreduce``: test/testreduceall.lua's 40 MiB Allreduce time.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

METRIC = "images/sec (whole node) ResNet-50 async-SGD at 1/2/4/8 MI355X"
_REPO = os.path.dirname(os.path.abspath(__file__))
# MIOpen find / perf databases are kept in-tree (miopen_db/) so a fresh box reuses the
# algorithm choices of earlier runs (only the fc layer and fallbacks still reach MIOpen).
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(_REPO, "miopen_db"))
os.environ.setdefault("MIOPEN_CUSTOM_CACHE_DIR", os.path.join(_REPO, "miopen_db", "kcache"))
# a benchmark has no slow straggler to wait for: a PS reply missing for 5 minutes is a stuck
# job, so the bench fails with the missing replies named (the library default is no limit)
os.environ.setdefault("MPIT_PS_TIMEOUT_S", "300")


def _par(a, tr, nworkers) -> str:
    par = {"downpour": "async-ps", "eamsgd": "easgd-ps", "easgd": "easgd-ps", "msgd": "local",
           "allreduce": "dp"}[a.optimizer]
    if a.optimizer not in ("allreduce", "msgd"):
        return par + f"-{tr.cfg.topology}-{len(tr.sranks)}srv-{nworkers}wrk"
    return par + str(a.gpus)


def _make(a, mp_train, amp: bool, topology: str, servers: int, ps_id: int):
    nw_world = int(os.environ.get("WORLD_SIZE", "1"))
    nw = nw_world if topology == "colocated" else max(1, nw_world - servers)
    mva = 0.9 / max(1, nw_world) if a.optimizer in ("eamsgd", "easgd") else 0.0
    lr = a.lr / max(1, nw) if a.optimizer == "downpour" else a.lr
    cfg = mp_train.TrainConfig(model=a.model, batch=a.batch, optimizer=a.optimizer, topology=topology,
                               servers=servers, su=a.su, lr=lr, mva=mva, mom=0.0, amp=amp,
                               channels_last=not a.no_channels_last, datapath=a.datapath, staleness=a.staleness,
                               wire_dtype=a.wire, extra={"ps_id": ps_id, "shards_per_server": a.emulate_shards,
                                                         "defer_ps_wait": a.defer_ps_wait})
    return mp_train.Trainer(cfg)


def _fp32_gemm() -> str:
    """How the fp32 step's GEMMs use the matrix cores (ops/conv.py MPIT_F32_SPLIT)."""
    from mpit_amd.ops import conv

    # "+planes": activations and gradients that only GEMMs read are written as the two fp16
    # planes by their producers (ops/conv.py _F32_PLANES, gemm.hip FM 13)
    return conv._F32_SPLIT + ("+planes" if conv._F32_PLANES else "")


def _gemm_counters() -> dict:
    from mpit_amd.ops import conv

    return dict(conv.COUNTERS)


def _devices(W, tr) -> list:
    """[(rank, device index, PCI bus id)] of every rank: the record itself shows which GPUs ran."""
    import torch

    mine = (W.Get_rank(), None, None)
    if tr.on_gpu:
        p = torch.cuda.get_device_properties(tr.device)
        mine = (W.Get_rank(), tr.device.index, f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}")
    return [list(x) for x in W.allgather_obj(mine)]


def _rccl_probe(W, tr, st) -> dict:
    """A live check, not a predicate: one dist.all_reduce over every rank on the NCCL (RCCL)
    process group, and what came back."""
    import torch
    import torch.distributed as dist

    out = {"backend": None, "ranks": None, "ok": False}
    if not (tr.on_gpu and dist.is_initialized()) or st.shared_devices:
        out["reason"] = "ranks share a GPU (RCCL needs one GPU per rank)" if st.shared_devices else "no GPU group"
        return out
    try:
        x = torch.ones(1, device=tr.device)
        dist.all_reduce(x)
        torch.cuda.synchronize(tr.device)
        seen = W.allgather_obj(float(x.item()))
        out.update(backend=dist.get_backend(), ranks=dist.get_world_size(), ok=all(v == st.world for v in seen),
                   sums=seen)
    except Exception as e:  # reported, never fatal to the headline
        out["error"] = f"{type(e).__name__}: {e}"
    return out


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
    ap.add_argument("--datapath", type=int, default=2,
                    help="PS data plane: 2 = one-sided xGMI peer copies on per-client link streams (default), "
                         "0 = fused remote kernel, 1 = serial SDMA, 3 = two-sided RCCL send/recv (the automatic "
                         "fallback when the pre-flight check finds a broken peer mapping)")
    ap.add_argument("--staleness", type=int, default=-1, help="bounded staleness (SSP); -1 = fully async")
    ap.add_argument("--wire", default="fp32", choices=["fp32", "bf16"], help="EASGD elastic-difference dtype")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"],
                    help="headline compute precision (fp32 = the reference's; bf16 = autocast, fp32 master)")
    ap.add_argument("--no-amp", action="store_true", help="alias of --dtype fp32 (kept for old scripts)")
    ap.add_argument("--no-secondary", action="store_true", help="headline only")
    ap.add_argument("--no-channels-last", action="store_true")
    ap.add_argument("--emulate-shards", type=int, default=1,
                    help="K > 1: split the (single) server's shard into K shards, each pushed from inside the "
                         "backward and served through the remote-client pipeline (link stream, inbox / outbox) — "
                         "one GPU carrying the per-worker shard traffic of an N=K job (diagnostic, not the headline)")
    ap.add_argument("--no-rccl-fallback", action="store_true",
                    help="fail (exit 3) when the pre-flight check fails instead of switching to datapath 3")
    ap.add_argument("--defer-ps-wait", action="store_true",
                    help="retire a step's last pulls at the next step's first weight read instead of at the "
                         "end of the step (profiles/defer_ps_wait_ab_r03.md: slower; off by default)")
    ap.add_argument("--miopen-find", action="store_true",
                    help="exhaustive MIOpen algorithm search for what still runs on MIOpen (the fc layer)")
    a = ap.parse_args(argv)
    if a.no_amp:
        a.dtype = "fp32"

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}; launch N>1 with torch.distributed.run",
              file=sys.stderr)
        return 2

    if a.emulate_shards > 1:
        os.environ["MPIT_PS_FORCE_PIPE"] = "1"  # the local client takes the remote-client pipeline
    import torch

    torch.backends.cudnn.benchmark = a.miopen_find
    import mpit_amd as mp
    from mpit_amd import train as mp_train
    from mpit_amd.models.cnn import INPUT_SHAPES

    mp.Init()
    W = mp.COMM_WORLD()
    amp = a.dtype == "bf16"
    from mpit_amd.parallel.ps import PSMapError

    fallback = None
    try:
        tr = _make(a, mp_train, amp, a.topology, a.servers, 0)
    except PSMapError as e:  # a peer window could not be mapped (every rank raised it)
        if a.datapath == 3 or mp.runtime.state().shared_devices or a.no_rccl_fallback:
            raise
        fallback = {"from_datapath": a.datapath, "reason": f"window mapping: {e}",
                    "unverified": "datapath 3's RCCL device path is exercised here for the first time"}
        a.datapath = 3
        tr = _make(a, mp_train, amp, a.topology, a.servers, 2)
    preflight = None
    if world > 1 and (tr.pc is not None or tr.ps_server is not None):
        # every (worker, server) data path exercised once BEFORE the timed region: peer
        # access per pair, one pull of every shard, exact bit-sums against the owning server
        # (asyncsgd/ptest.lua's ping-pong before training). A broken one-sided path switches
        # the job to the two-sided RCCL data plane (datapath 3, csrc/core/link.h) and checks
        # again; a pair still broken ends the run here, named, before any timing.
        preflight = tr.preflight()
        if (not preflight["ok"] and a.datapath != 3 and not mp.runtime.state().shared_devices
                and not a.no_rccl_fallback):
            # datapath 3 is deadlock-free by construction (csrc/core/link.h) and the bench's
            # clients wait at most MPIT_PS_TIMEOUT_S (300 s, set above) before failing with a
            # named error; its RCCL device path had not run on distinct GPUs before such a job, so
            # the JSON says so
            fallback = {"from_datapath": a.datapath, "reason": f"pre-flight: no peer access {preflight['no_peer']}, "
                                                                 f"pulled shard bits differ {preflight['mismatches']}",
                        "unverified": "datapath 3's RCCL device path is exercised here for the first time"}
            tr.stop()
            a.datapath = 3
            tr = _make(a, mp_train, amp, a.topology, a.servers, 2)
            preflight = tr.preflight()
        if not preflight["ok"]:
            if W.Get_rank() == 0:
                print(f"bench.py: pre-flight failed: no peer access {preflight['no_peer']}, pulled shard bits "
                      f"differ for (worker, server) {preflight['mismatches']}; devices {preflight['devices']}",
                      file=sys.stderr, flush=True)
            mp.Finalize()
            return 3
        if fallback is not None:
            preflight["fallback"] = fallback
    secs, loss = mp_train.timed_steps(tr, a.steps, a.warmup)
    peak_gib = round(torch.cuda.max_memory_allocated(tr.device) / 2 ** 30, 2) if tr.on_gpu else None
    nworkers = len(tr.cranks)
    shape = INPUT_SHAPES.get(a.model, (3, 224, 224))
    value = a.steps * a.batch * nworkers / secs
    lossv = float(loss.float().item()) if loss is not None else None
    if lossv is not None and not math.isfinite(lossv):
        lossv = None  # keep the line strict JSON
    par = _par(a, tr, nworkers)
    secondary = {}
    t_sec = time.perf_counter()
    sec_steps, sec_warm = max(3, min(a.steps, 20)), max(4, a.warmup)
    if not a.no_secondary and tr.on_gpu:
        # the other precision on the same replicas / PS (bf16 autocast when the headline is fp32)
        tr.set_amp(not amp)
        s2, _ = mp_train.timed_steps(tr, sec_steps, sec_warm)
        secondary["bf16_autocast" if not amp else "fp32"] = {
            "value": round(sec_steps * a.batch * nworkers / s2, 2), "unit": "images/sec",
            "ms_per_step": round(1000.0 * s2 / sec_steps, 3), "steps": sec_steps, "warmup": sec_warm,
            "dtype": "bf16" if not amp else "fp32", "parallelism": par}
        tr.set_amp(amp)
    check = tr.verify_ps() if (tr.pc is not None or tr.ps_server is not None) else None
    tr.stop()
    st = mp.runtime.state()
    devices = _devices(W, tr)
    rccl = _rccl_probe(W, tr, st) if world > 1 else None
    if not a.no_secondary and world > 1 and a.optimizer != "allreduce":
        from mpit_amd.instruments import allreduce_time, ps_pingpong

        try:
            # BASELINE config 2: one dedicated pserver, N-1 workers (second PS instance)
            td = _make(a, mp_train, amp, "dedicated", 1, 1)
            sd, _ = mp_train.timed_steps(td, sec_steps, sec_warm)
            nwd = len(td.cranks)
            cd = td.verify_ps()
            td.stop()
            secondary["dedicated"] = {"value": round(sec_steps * a.batch * nwd / sd, 2), "unit": "images/sec",
                                      "ms_per_step": round(1000.0 * sd / sec_steps, 3), "steps": sec_steps,
                                      "dtype": a.dtype, "parallelism": _par(a, td, nwd), "ps_check": cd}
            del td
            secondary["ps_pingpong"] = ps_pingpong(640.0, iters=100, warmup=2, ps_id=7, time_budget_s=8.0)
            secondary["allreduce"] = allreduce_time(10.0, iters=10)
        except Exception as e:  # secondary fields never take the headline down
            secondary["error"] = f"{type(e).__name__}: {e}"
    if W.Get_rank() == 0:
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
            "dtype": "fp32" if not (tr.on_gpu and amp) else "bf16",
            "data": f"synthetic (random images {shape[0]}x{shape[1]}x{shape[2]}, random labels, random-init weights)",
            "config": {"model": a.model, "global_batch": a.batch * nworkers, "seq_len": None, "image_size": shape[-1],
                       "parallelism": par, "optimizer": a.optimizer, "su": a.su, "per_gpu_batch": a.batch,
                       "master_weights": "fp32", "loss_last": lossv, "defer_ps_wait": a.defer_ps_wait,
                       "datapath": a.datapath},
            "fp32_gemm": _fp32_gemm() if not (tr.on_gpu and amp) else None,
            # operand-path counters over the whole run (ops/conv.py COUNTERS): planes GEMMs, and the
            # fallbacks that must stay 0 on the flagship (decoded planes, mixed pairs, amax passes)
            "gemm_counters": _gemm_counters(),
            "world": st.world, "shared_devices": st.shared_devices, "devices": devices, "rccl": rccl,
            "ps_check": check, "preflight": preflight, "peak_mem_gib": peak_gib,
            **({"emulate_shards": a.emulate_shards} if a.emulate_shards > 1 else {}),
            "secondary": secondary,
            "secondary_s": round(time.perf_counter() - t_sec, 2),
        }
        print(json.dumps(out), flush=True)
    ok = check is None or check["ok"]
    mp.Finalize()
    return 0 if ok else 3


if __name__ == "__main__":
    sys.exit(main())

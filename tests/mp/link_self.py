"""Datapath 3 (two-sided RCCL send / recv, csrc/core/link.h) on ONE rank through the link's
self-loop (MPIT_LINK_SELF=1, set by the caller): the co-located client's shard travels as a
grouped RCCL send to itself + receive on the link stream, with the server's inbox / outbox
events and continuations exactly as for a remote client. The reference moves every shard as
an Isend / Irecv pair of the storage's data pointer (init.lua:41-108).

For each precision, two PS instances train the same Downpour replica from the same init on
the same data: datapath 2 (the local fused path) and datapath 3 (self-loop). The final
parameters must be bit-identical. Then the reference's ptest.lua instrument (640 MiB pull +
push, asyncsgd/ptest.lua:40-67) runs over the self-loop. Prints one RESULT line."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

import mpit_amd as mp
from mpit_amd.instruments import ps_pingpong
from mpit_amd.train import TrainConfig, Trainer, timed_steps

torch.backends.cudnn.deterministic = True
torch.backends.cudnn.benchmark = False
model = os.environ.get("T_MODEL", "resnet18")
steps = int(os.environ.get("T_STEPS", "20"))
batch = int(os.environ.get("T_BATCH", "8"))
precs = os.environ.get("T_PRECS", "fp32,bf16").split(",")
mp.Init()
W = mp.COMM_WORLD()
assert W.Get_size() == 1, "the self-loop test runs on one rank"
res = {}
pid = 40
for prec in precs:
    finals, stats = {}, None
    for dp in (2, 3):
        tr = Trainer(TrainConfig(model=model, batch=batch, num_classes=10, optimizer="downpour", topology="colocated",
                                 lr=0.05, amp=prec == "bf16", datapath=dp, extra={"ps_id": pid}))
        pid += 1
        timed_steps(tr, steps, 0)
        chk = tr.verify_ps()
        assert chk["ok"], chk
        finals[dp] = tr.flat.flat.detach().clone()
        if dp == 3:
            assert tr.pc.link is not None
            stats = tr.pc.link.stats()
        else:
            assert tr.pc.link is None
        tr.stop()
    a, b = finals[2], finals[3]
    same = bool(torch.equal(a.view(torch.int32), b.view(torch.int32)))
    res[prec] = {"same": same, "maxdiff": float((a - b).abs().max()), "link": stats,
                 "finite": bool(torch.isfinite(a).all())}
if os.environ.get("T_PINGPONG", "1") == "1":
    mib = float(os.environ.get("T_PP_MIB", "640"))
    res["pingpong"] = ps_pingpong(mib, iters=int(os.environ.get("T_PP_ITERS", "20")), warmup=2, ps_id=pid,
                                  datapath=3)
print("RESULT", res, flush=True)
mp.Finalize()

"""Downpour with the ShardPusher overlap (shards pushed and refreshed shards pulled into the
model while the backward of earlier layers still runs, parallel/overlap.py) must produce
bit-identical parameters to the non-overlapped path (push + pull after the backward).

Run under torch.distributed.run with 3 ranks: 2 dedicated servers, 1 worker. For each
precision (fp32, bf16 autocast) two PS instances train the same model from the same init on
the same data, one with overlap, one without; the final pulled parameters are compared
bit for bit (int64 sums of the fp32 words and an exact tensor compare on the worker). A third
instance runs the overlap with the deferred wait (the last pulls retired at the next forward,
extra["defer_ps_wait"], what bench.py runs) and must match too."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

import mpit_amd as mp
from mpit_amd.train import TrainConfig, Trainer, timed_steps

# bitwise comparison: layers still on MIOpen (the classifier) must pick deterministic solvers
torch.backends.cudnn.deterministic = True
torch.backends.cudnn.benchmark = False
model = os.environ.get("T_MODEL", "resnet18")
steps = int(os.environ.get("T_STEPS", "4"))
mp.Init()
W = mp.COMM_WORLD()
results = {}
ps_id = 0
for amp in (False, True):
    finals = {}
    for arm in ("overlap", "plain", "defer"):
        overlap = arm != "plain"
        tr = Trainer(TrainConfig(model=model, batch=8, num_classes=10, optimizer="downpour", topology="dedicated",
                                 servers=2, lr=0.05, amp=amp,
                                 extra={"ps_id": ps_id, "overlap_push": overlap, "defer_ps_wait": arm == "defer"}))
        ps_id += 1
        if tr.is_worker:
            assert ("pusher" in tr.opt_config) == overlap
        if os.environ.get("T_DEBUG"):
            # per step: loss, bit-sum of the pushed window (scaled gradients) and of the pulled
            # parameters, to find the first step / quantity where the arms part
            # (snapshots queued on the stream, no host sync inside the loop: the timing stays
            # the test's)
            snaps = []
            w_init = tr.flat.flat.clone() if tr.is_worker else None
            for k in range(steps if tr.is_worker else 0):
                loss = tr.step()
                snaps.append((loss.clone(), tr.pc.tx.clone(), tr.flat.flat.clone()))
            tr.sync()
            bs = lambda t: int(t.detach().reshape(-1).view(torch.int32).to(torch.int64).sum().item())
            prev = w_init
            for k, (loss, txs, ws) in enumerate(snaps):
                # one worker, server rule p += g: the pulled w must be exactly prev + pushed tx
                exact = bool(torch.equal(ws, prev + txs)) if arm != "defer" else None
                print(f"STEP {('bf16' if amp else 'fp32')} {arm} {k} loss={float(loss):.9g} tx={bs(txs)} "
                      f"w={bs(ws)} txmax={float(txs.abs().max()):.4g} w0={bs(w_init)} pull_exact={exact}", flush=True)
                prev = ws
            tr.barrier()
        else:
            timed_steps(tr, steps, 0)
        chk = tr.verify_ps()
        assert chk["ok"], chk
        if tr.is_worker:
            finals[arm] = tr.flat.flat.detach().clone()
            names = [(n, off, p.numel()) for (n, p), off in zip(tr.model.named_parameters(), tr.flat.offsets)]
        tr.stop()
    for arm in ("overlap", "defer"):
        if not finals:
            break
        a, b = finals[arm], finals["plain"]
        same = bool(torch.equal(a.view(torch.int32), b.view(torch.int32)))
        diff = float((a - b).abs().max())
        key = ("bf16" if amp else "fp32") + ("" if arm == "overlap" else "_defer")
        results[key] = (same, diff)
        if not same:  # which parameters differ (diagnostics)
            bad = [(n, float((a[o:o + k] - b[o:o + k]).abs().max())) for n, o, k in names
                   if not torch.equal(a[o:o + k], b[o:o + k])]
            print(f"DIFF {key} {len(bad)}/{len(names)}: {bad[:12]}", flush=True)
allr = [r for r in W.allgather_obj(results) if r]
if W.Get_rank() == 0:
    print("RESULT", allr, flush=True)
mp.Finalize()

"""Checkpoint / resume equivalence (run under torch.distributed.run, CPU or GPU):
6 training steps == 3 steps + save_checkpoint + a fresh job state + load_checkpoint +
3 steps, bit for bit, including the dedicated server's shard and rule state.

T_OPT: downpour | eamsgd | adam (server-side Adam with stepDivAdam: its step counter must
survive the restart). T_TOPO: colocated | dedicated."""
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

import mpit_amd as mp
from mpit_amd.parallel.ps import ServerOpt
from mpit_amd.train import TrainConfig, Trainer

# bitwise equality needs deterministic library kernels: cnn7's convolutions run on MIOpen,
# whose default backward-weight solvers may reduce with atomics
torch.backends.cudnn.deterministic = True
torch.backends.cudnn.benchmark = False
opt = os.environ.get("T_OPT", "downpour")
topo = os.environ.get("T_TOPO", "dedicated")
mp.Init()
W = mp.COMM_WORLD()
rule = None
optimizer = opt
if opt == "adam":
    rule = ServerOpt("adam", lr=1e-3, step_div=2)
    optimizer = "downpour"  # raw gradients pushed, the server runs Adam
ckdir = W.allgather_obj(tempfile.mkdtemp(prefix="mpit_ck_") if W.Get_rank() == 0 else None)[0]


def make(ps_id):
    torch.manual_seed(99)
    return Trainer(TrainConfig(model="cnn7", batch=8, num_classes=10, optimizer=optimizer, topology=topo, servers=1,
                               lr=0.05, mva=0.45, su=1 if optimizer == "downpour" else 2, server_rule=rule,
                               extra={"ps_id": ps_id, "steal_grads": False}))


def run(tr, n):
    for _ in range(n):
        if tr.is_worker:
            tr.step()
    tr.sync()
    tr.barrier()


def final(tr):
    chk = tr.verify_ps()  # final pull; shards == worker copies
    assert chk["ok"], chk
    out = tr.flat.flat.detach().clone() if tr.is_worker else None
    srv = tr.ps_server.p.detach().clone() if tr.ps_server is not None else None
    tr.stop()
    return out, srv


a = make(0)
run(a, 6)
wa, sa = final(a)
b = make(1)
run(b, 3)
b.save_checkpoint(ckdir)
b.stop()
c = make(2)
c.load_checkpoint(ckdir)
run(c, 3)
wc, sc = final(c)
res = {}
if wa is not None:
    res["worker_equal"] = bool(torch.equal(wa.view(torch.int32), wc.view(torch.int32)))
    res["worker_maxdiff"] = float((wa - wc).abs().max())
if sa is not None:
    res["server_equal"] = bool(torch.equal(sa.view(torch.int32), sc.view(torch.int32)))
allr = W.allgather_obj(res)
if W.Get_rank() == 0:
    print("RESULT", allr, flush=True)
mp.Finalize()

"""EAMSGD leaves its last elastic push in flight (asyncsgd/optim-eamsgd.lua:65-67):
verify_ps / save_checkpoint must retire it before comparing / saving shards. Run on 3+
ranks (1 dedicated server + workers) under torch.distributed.run."""
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

import mpit_amd as mp
from mpit_amd.train import TrainConfig, Trainer

mp.Init()
W = mp.COMM_WORLD()
tr = Trainer(TrainConfig(model="cnn7", batch=8, num_classes=10, optimizer="eamsgd", topology="dedicated", servers=1,
                         lr=0.05, mva=0.3, su=1, extra={"steal_grads": False}))
oks = []
for rnd in range(4):
    for _ in range(2):
        if tr.is_worker:
            tr.step()  # leaves the elastic push in flight
    oks.append(tr.verify_ps()["ok"])
ckdir = W.allgather_obj(tempfile.mkdtemp(prefix="mpit_ck_") if W.Get_rank() == 0 else None)[0]
tr.save_checkpoint(ckdir)
# after save: the saved server shard must equal what every worker now pulls
srv = tr.ps_server.p.detach().clone() if tr.ps_server is not None else None
chk = tr.verify_ps()
tr.stop()
res = W.allgather_obj({"rank": W.Get_rank(), "oks": oks, "final": chk["ok"]})
if W.Get_rank() == 0:
    print("RESULT", res, flush=True)
mp.Finalize()

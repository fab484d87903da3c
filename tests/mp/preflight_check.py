"""bench.py's pre-timing check (Trainer.preflight) on a co-located CPU job: with a broken
(worker, server) data path injected (MPIT_PS_FAULT=badpull: server MPIT_PS_FAULT_RANK corrupts
every pull it serves to client MPIT_PS_FAULT_CLIENT) the report names exactly that pair."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ["MPIT_CPU_ONLY"] = "1"

import mpit_amd as mp
from mpit_amd.train import TrainConfig, Trainer

mp.Init()
W = mp.COMM_WORLD()
tr = Trainer(TrainConfig(model="cnn7", batch=4, num_classes=10, optimizer="downpour", topology="colocated", lr=0.01))
rep = tr.preflight()
if tr.is_worker:
    tr.step()
tr.stop()
if W.Get_rank() == 0:
    print("PREFLIGHT", {k: rep[k] for k in ("ok", "mismatches", "no_peer", "shards", "workers")}, flush=True)
mp.Finalize()

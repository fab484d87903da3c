"""Multi-rank PS training check (run under torch.distributed.run)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

import mpit_amd as mp
from mpit_amd.train import TrainConfig, Trainer, timed_steps

model = os.environ.get("T_MODEL", "lenet")
opt = os.environ.get("T_OPT", "downpour")
topo = os.environ.get("T_TOPO", "colocated")
batch = int(os.environ.get("T_BATCH", "16"))
steps = int(os.environ.get("T_STEPS", "6"))
dp = int(os.environ.get("T_DATAPATH", "0"))
mp.Init()
nc = 10 if model in ("lenet", "cnn7") else 1000
rule = None
if os.environ.get("T_RULE"):
    from mpit_amd.parallel.ps import ServerOpt

    rule = ServerOpt(os.environ["T_RULE"], lr=1e-3, step_div=2)
tr = Trainer(TrainConfig(model=model, batch=batch, num_classes=nc, optimizer=opt, topology=topo, lr=0.05,
                         mva=0.45, su=int(os.environ.get("T_SU", "1")), datapath=dp, servers=1,
                         wire_dtype=os.environ.get("T_WIRE", "fp32"), server_rule=rule,
                         extra={"shards_per_server": int(os.environ.get("T_SPS", "1"))}))
secs, loss = timed_steps(tr, steps, 2)
# every push has been acked before the barrier inside timed_steps: one more pull gives
# every worker the final server state — compare a checksum across ranks
if tr.pc is not None and opt == "downpour":
    tr.pc.async_recv_param()
    tr.pc.wait()
cs = torch.tensor([float(tr.flat.flat.double().sum())], dtype=torch.float64)
bits = int(tr.flat.flat.view(torch.int32).to(torch.int64).sum())
allcs = torch.zeros(mp.get_size(), dtype=torch.float64)
mp.COMM_WORLD().Allgather(cs, allcs)
ls = torch.tensor([float(loss) if loss is not None else float("nan")], dtype=torch.float64)
all_loss = torch.zeros(mp.get_size(), dtype=torch.float64)
mp.COMM_WORLD().Allgather(ls, all_loss)
stats = tr.ps_server.stats() if tr.ps_server is not None else {}
tr.stop()
if mp.get_rank() == 0:
    print(f"RESULT opt={opt} topo={topo} secs={secs:.4f} loss={float(loss) if loss is not None else -1:.4f} "
          f"checksums={allcs.tolist()} losses={all_loss.tolist()} stats={stats} bits={bits}", flush=True)
mp.Finalize()

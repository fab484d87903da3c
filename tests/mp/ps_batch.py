"""One rank, HBM server, its co-located client pushing the shard as K pieces per step and
waiting for the pull: deterministic, so MPIT_PS_BATCH=1 (pieces found queued in one progress
sweep applied by ONE multi-segment launch) and MPIT_PS_BATCH=0 (one launch per piece) must
leave the same parameters, bit for bit."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

import mpit_amd as mp
from mpit_amd.parallel.ps import PClient, PServer

mp.Init()
rank = mp.get_rank()
plong = 3 * 1000003 + 5
conf = dict(rank=rank, sranks=[0], cranks=[0], plong=plong, shards_per_server=int(os.environ.get("T_SPS", "4")))
srv = PServer(conf)
srv.start(block=False)
pc = PClient(conf)
gen = torch.Generator().manual_seed(3)
p = torch.randn(plong, generator=gen).cuda()
g = torch.zeros(plong).cuda()
pc.start(p, g)
for step in range(6):
    g.copy_(torch.randn(plong, generator=gen))
    torch.cuda.synchronize()
    pc.async_send_grad(pull=True)
    pc.wait()
torch.cuda.synchronize()
bits = int(p.view(torch.int32).to(torch.int64).sum())
pc.stop()
srv.wait_done()
st = srv.stats()
print(f"RESULT bits={bits} stats={dict(st)}", flush=True)
mp.Finalize()

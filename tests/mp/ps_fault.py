"""A PS job whose server fails (MPIT_PS_FAULT) must end on every rank, non-zero, with the
reason — never hang (the reference's co_ping assert(false), init.lua:168-171)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ["MPIT_CPU_ONLY"] = "1"
import torch

import mpit_amd as mp
from mpit_amd.parallel.ps import PClient, PServer

mp.Init()
rank, world = mp.get_rank(), mp.get_size()
plong = 4096
conf = dict(rank=rank, sranks=list(range(world)), cranks=list(range(world)), plong=plong, datapath=0)
srv = PServer(conf)
srv.start(block=False)
pc = PClient(conf)
p = torch.zeros(plong)
g = torch.full((plong,), 1e-3)
pc.start(p, g)
for step in range(20):
    pc.async_send_grad(pull=True)
    pc.wait()
print(f"rank {rank}: should not get here", flush=True)
pc.stop()
mp.Finalize()

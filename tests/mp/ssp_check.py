"""Bounded staleness: rank 0 serves, ranks 1 and 2 are clients, staleness 0.
Client 1 pushes with a pull; the pull must wait for client 2's first push, and the
parameters it then receives must include that push: 0 + 1 + 1 = 2 everywhere (sum rule,
both gradients all ones)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

import mpit_amd as mp
from mpit_amd.parallel.ps import PClient, PServer, ServerOpt

mp.Init()
W = mp.COMM_WORLD()
r = W.Get_rank()
conf = dict(rank=r, sranks=[0], cranks=[1, 2], plong=64, opt=ServerOpt("sum"), staleness=0,
            datapath=int(os.environ.get("T_DATAPATH", "2")))
if r == 0:
    s = PServer(conf)
    s.start(block=True)
    st = s.stats()
    assert st["deferred"] >= 1, st
    print("RESULT SSP_OK", st, flush=True)
else:
    pc = PClient(conf).start(torch.zeros(64), torch.ones(64))
    pc.tx.fill_(1.0)  # the push window (host: a view of the client's shm window)
    if r == 1:
        pc.async_send_grad(pull=True)
        pc.wait()  # clocks (1, 0): 1 - 0 > 0 -> deferred until client 2 pushes
        got = pc.rx.clone()
        assert torch.equal(got, torch.full_like(got, 2.0)), got[:8].tolist()
        print("RESULT SSP_PULL_OK", flush=True)
    if r == 2:
        time.sleep(0.5)
        pc.async_send_grad(pull=True)
        pc.wait()
    pc.stop()
mp.COMM_WORLD().Barrier()
mp.Finalize()

"""PS datapath 3 under BLOCKING rendezvous semantics (csrc/core/link.h, MPIT_LINK_RDV=1): every
rank's link ops run in ONE FIFO, and a send completes only once the receiver's matching
receive has reached the head of the receiver's FIFO — what an RCCL send / recv pair at the
head of a hardware queue does, with all of a rank's streams merged into one queue.

Every step each client pushes its gradient shards (with pulls) to the servers in a random
shard order, with random control-message timing (MPIT_LINK_JITTER_US, seeded per rank) and
random sleeps, sometimes followed by extra plain pulls. T_STEPS steps (default 200): every
step is a fresh random arrival order of control messages at the servers and the sequencer.

T_TOPO=colocated  every rank is a worker and serves one shard (the N = 8 node layout);
T_TOPO=dedicated  rank 0 serves alone, the other ranks are workers (BASELINE config 2).

Result: RESULT RDV_OK when every worker's final pull equals the closed form (exact dyadic
sums). With MPIT_LINK_LEGACY=1 (the pre-sequencer layout: a client queues its ops when it
sends its control message, a server when the message arrives) the ranks' FIFOs deadlock;
the clients' finite wait (MPIT_PS_TIMEOUT_S) then reports RESULT RDV_TIMEOUT.
"""
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ["MPIT_CPU_ONLY"] = "1"
import torch

import mpit_amd as mp
from mpit_amd.parallel.ps import PClient, PServer, ServerOpt

mp.Init()
W = mp.COMM_WORLD()
rank, world = W.Get_rank(), W.Get_size()
topo = os.environ.get("T_TOPO", "colocated")
steps = int(os.environ.get("T_STEPS", "200"))
sranks = list(range(world)) if topo == "colocated" else [0]
cranks = list(range(world)) if topo == "colocated" else list(range(1, world))
plong = 4099 * len(sranks) + 3
rng = random.Random(1000 + rank)
# T_STALE >= 0: bounded staleness, so deferred pulls are released (and ordered) by other
# clients' pushes
conf = dict(rank=rank, sranks=sranks, cranks=cranks, plong=plong, datapath=3, ps_id=31, opt=ServerOpt("sum", a=1.0),
            staleness=int(os.environ.get("T_STALE", "-1")))
srv = None
if rank in sranks:
    srv = PServer(conf)
    srv.start(block=False)
pc = None
status = "RDV_OK"
t0 = time.time()
try:
    if rank in cranks:
        pc = PClient(conf)
        p0 = torch.arange(plong, dtype=torch.float32) * 0.25
        pc.start(p0.clone(), torch.zeros(plong))
        nsh = len(sranks)
        for s in range(steps):
            pc.tx.fill_((rank + 1) * 0.125)
            order = list(range(nsh))
            rng.shuffle(order)
            for k in order:
                if rng.random() < 0.3:
                    time.sleep(rng.random() * 2e-4)
                pc.async_send_grad_shard(k, pull=True)
            pc.wait()
            if rng.random() < 0.25:
                pc.async_recv_param()
                pc.wait()
        pc.wait()
    W.Barrier()
    if pc is not None:
        pc.async_recv_param()
        pc.wait()
        want = torch.arange(plong, dtype=torch.float32) * 0.25 + steps * 0.125 * sum(c + 1 for c in cranks)
        if not torch.equal(pc.rx, want):
            status = f"RDV_WRONG maxdiff={float((pc.rx - want).abs().max())}"
except RuntimeError as e:
    if "MPIT_PS_TIMEOUT_S" not in str(e):
        raise
    # a deadlocked FIFO: report and leave without the stop protocol (it cannot complete)
    print(f"RANK {rank} RESULT RDV_TIMEOUT after {time.time() - t0:.1f}s", flush=True)
    sys.stdout.flush()
    os._exit(0)
stats = srv.stats() if srv is not None else None
if pc is not None:
    pc.stop()
if srv is not None:
    srv.wait_done()
W.Barrier()
print(f"RANK {rank} RESULT {status} steps={steps} t={time.time() - t0:.1f}s stats={stats}", flush=True)
mp.Finalize()

"""PS datapath 3 (two-sided messages, csrc/core/link.h) on CPU ranks, the engine's tagged host
messages standing in for RCCL: the op sequences of every (client, server) pair must match
(deadlock-free) and the results must equal the one-sided datapath's.

T_CASE=sum:      co-located (every rank worker + server): each client pushes exact dyadic
                 gradients with a pull for 12 steps, interleaved with plain pulls; the final
                 shards are order independent (exact sums) -> compare to the closed form.
T_CASE=train:    Trainer Downpour (cnn7), topology from T_TOPO, datapath 3 vs datapath 0 from
                 the same init: final pulled parameters bit-equal when there is ONE worker
                 (deterministic order), equal to the server's shards in any case.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ["MPIT_CPU_ONLY"] = "1"
import torch

import mpit_amd as mp
from mpit_amd.parallel.ps import PClient, PServer, ServerOpt

mp.Init()
W = mp.COMM_WORLD()
rank, world = W.Get_rank(), W.Get_size()
case = os.environ.get("T_CASE", "sum")
out = {}
if case == "sum":
    plong, steps = 10007, 12
    for dp in (3, 0):
        conf = dict(rank=rank, sranks=list(range(world)), cranks=list(range(world)), plong=plong, datapath=dp,
                    ps_id=10 + dp, opt=ServerOpt("sum", a=1.0))
        srv = PServer(conf)
        srv.start(block=False)
        pc = PClient(conf)
        p0 = torch.arange(plong, dtype=torch.float32) * 0.5
        p = p0.clone()
        g = torch.zeros(plong)
        pc.start(p, g)
        for s in range(steps):
            pc.tx.fill_((rank + 1) * 0.125)
            pc.async_send_grad(pull=True)
            pc.wait()
            if s % 3 == 2:
                pc.async_recv_param()
                pc.wait()
        W.Barrier()
        pc.async_recv_param()
        pc.wait()
        want = p0 + steps * 0.125 * sum(range(1, world + 1))
        out[dp] = bool(torch.equal(pc.rx, want))
        if not out[dp]:
            d = (pc.rx - want)
            print("DBG", dp, rank, float(d.abs().max()), d[:4].tolist(), d[-4:].tolist(), flush=True)
        srv_stats = srv.stats()
        pc.stop()
        srv.wait_done()
        W.Barrier()
    print(f"RANK {rank} equal={out} stats={srv_stats}", flush=True)
else:
    from mpit_amd.train import TrainConfig, Trainer, timed_steps

    topo = os.environ.get("T_TOPO", "dedicated")
    finals = {}
    for i, dp in enumerate((3, 0)):
        tr = Trainer(TrainConfig(model="cnn7", batch=4, num_classes=10, optimizer="downpour", topology=topo,
                                 servers=int(os.environ.get("T_SERVERS", "2")), lr=0.05, datapath=dp,
                                 extra={"ps_id": 20 + i}))
        timed_steps(tr, 4, 1)
        chk = tr.verify_ps()
        if tr.is_worker:
            finals[dp] = tr.flat.flat.detach().clone()
        stats = tr.ps_server.stats() if tr.ps_server is not None else None
        tr.stop()
        out[dp] = chk["ok"]
    same = bool(torch.equal(finals[3], finals[0])) if finals else None
    print(f"RANK {rank} ok={out} same={same} stats={stats}", flush=True)
W.Barrier()
mp.Finalize()

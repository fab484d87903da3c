"""BiCNN question-answer training through the parameter server
(BiCNN/plaunch.lua + BiCNN/bicnn.lua).

    python -m mpit_amd.launch -n 5 mpit_amd/apps/bicnn.py --optimization adam --testerfirst --masterFreq 2

Roles: BiCNN/plaunch.lua's masterFreq assignment with the tester first or last. The
tester pulls the center parameters in a loop, evaluates GESD ranking accuracy on the
validation pools, keeps the best parameters, and — unlike the reference, whose tester
never terminates (BiCNN/bicnn.lua:582) — stops once every worker has finished.
Optimizers: every BiCNN optimizer (sgd / downpour / eamsgd / rmsprop / adam / adamax /
adagrad / adadelta, global or local, and the *single parameter-push variants); the
server-side rule follows the same flags (ServerOpt.from_bicnn_opt).
"""
from __future__ import annotations

import argparse
import os
import random
import sys
import time

import torch

import mpit_amd as mp
from mpit_amd import ops
from mpit_amd.apps.qa_data import pad_batch, synthetic_qa, load_files
from mpit_amd.launch import master_freq
from mpit_amd.models.bicnn import BiCNN, gesd, margin_ranking_loss
from mpit_amd.optim import ALL as OPTIMS
from mpit_amd.parallel.ps import PClient, PServer, ServerOpt
from mpit_amd.utils.flat import FlatParams
from mpit_amd.utils.metrics import JsonLogger, RunningAverage
from mpit_amd.utils.trace import Timers

TAG_WORKER_DONE = 9001


def build_args(argv=None):
    ap = argparse.ArgumentParser()
    # data (BiCNN/plaunch.lua:7-30)
    ap.add_argument("--embeddingFile", default="none")
    ap.add_argument("--trainFile", default="none")
    ap.add_argument("--validFile", default="none")
    ap.add_argument("--label2answFile", default="none")
    ap.add_argument("--embeddingDim", type=int, default=100)
    ap.add_argument("--wordHiddenDim", type=int, default=200)
    ap.add_argument("--numFilters", type=int, default=3000)
    ap.add_argument("--contConvWidth", type=int, default=2)
    ap.add_argument("--mmode", type=int, default=1)
    ap.add_argument("--margin", type=float, default=0.009)
    ap.add_argument("--maxnegsample", type=int, default=50)
    ap.add_argument("--batchSize", type=int, default=64)
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--maxSteps", type=int, default=0)
    # regularisation (BiCNN/bicnn.lua:398-409)
    ap.add_argument("--L1reg", type=float, default=0.0)
    ap.add_argument("--L2reg", type=float, default=0.0)
    ap.add_argument("--gradClip", type=float, default=0.0)
    # optimisation
    ap.add_argument("--optimization", default="adam")
    ap.add_argument("--learningRate", type=float, default=0.01)
    ap.add_argument("--commperiod", type=int, default=1)
    ap.add_argument("--modeRMSProp", default="global")
    ap.add_argument("--decayRMSProp", type=float, default=0.95)
    ap.add_argument("--lrRMSProp", type=float, default=1e-3)
    ap.add_argument("--momentumRMSProp", type=float, default=0.9)
    ap.add_argument("--epsilonRMSProp", type=float, default=1e-4)
    ap.add_argument("--modeAdam", default="global")
    ap.add_argument("--lrAdam", type=float, default=1e-3)
    ap.add_argument("--beta1Adam", type=float, default=0.9)
    ap.add_argument("--beta2Adam", type=float, default=0.999)
    ap.add_argument("--epsilonAdam", type=float, default=1e-8)
    ap.add_argument("--stepDivAdam", type=int, default=72)
    ap.add_argument("--modeAdagrad", default="global")
    ap.add_argument("--lrAdagrad", type=float, default=1e-2)
    ap.add_argument("--lrDecayAdagrad", type=float, default=0.0)
    ap.add_argument("--epsilonAdagrad", type=float, default=1e-10)
    ap.add_argument("--modeAdadelta", default="global")
    ap.add_argument("--rhoAdadelta", type=float, default=0.95)
    ap.add_argument("--epsilonAdadelta", type=float, default=1e-6)
    ap.add_argument("--lrAdadelta", type=float, default=1.0)
    ap.add_argument("--mva", type=float, default=0.0)
    ap.add_argument("--momentum", type=float, default=0.0)
    # topology (BiCNN/plaunch.lua:37-70)
    ap.add_argument("--masterFreq", type=int, default=2)
    ap.add_argument("--testerfirst", action="store_true")
    ap.add_argument("--testerlast", action="store_true")
    ap.add_argument("--validMode", default="additionalTester", choices=["additionalTester", "lastClient", "none"])
    ap.add_argument("--testerPeriod", type=float, default=0.5, help="seconds between tester evaluations")
    ap.add_argument("--save", default="bicnn_out")
    ap.add_argument("--synthetic", type=int, default=200, help="synthetic answers when no data files are given")
    return ap.parse_args(argv)


def optim_config(a, pc):
    o = a.optimization
    c = dict(pclient=pc, su=a.commperiod)
    if o in ("sgd", "msgd"):
        c.update(lr=a.learningRate, push_param=True)
    elif o == "downpour":
        c.update(lr=a.learningRate)
    elif o in ("eamsgd", "easgd"):
        c.update(lr=a.learningRate, mva=a.mva or 0.3, mom=a.momentum)
    elif o.startswith("rmsprop"):
        c.update(mode=a.modeRMSProp, decay=a.decayRMSProp, lr=a.lrRMSProp, momentum=a.momentumRMSProp,
                 epsilon=a.epsilonRMSProp)
    elif o.startswith("adam"):
        c.update(lr=a.lrAdam, beta1=a.beta1Adam, beta2=a.beta2Adam, epsilon=a.epsilonAdam)
    elif o.startswith("adagrad"):
        c.update(lr=a.lrAdagrad, lrd=a.lrDecayAdagrad, epsilon=a.epsilonAdagrad)
    elif o.startswith("adadelta"):
        c.update(rho=a.rhoAdadelta, epsilon=a.epsilonAdadelta, lr=a.lrAdadelta)
    return c


@torch.no_grad()
def evaluate(model, data, dev, max_q=None) -> float:
    model.eval()
    labs = sorted(data.answers)
    emb = []
    for s in range(0, len(labs), 256):
        emb.append(model.encode(pad_batch([data.answers[x] for x in labs[s: s + 256]]).to(dev)))
    emb = torch.cat(emb)
    pos = {x: i for i, x in enumerate(labs)}
    correct = total = 0
    items = data.valid[:max_q] if max_q else data.valid
    for s in range(0, len(items), 256):
        chunk = items[s: s + 256]
        eq = model.encode(pad_batch([q for _, q, _ in chunk]).to(dev))
        for (labels, _, pool), e in zip(chunk, eq):
            cand = torch.tensor([pos[p] for p in pool], device=dev)
            sims = gesd(e.unsqueeze(0).expand(len(pool), -1), emb[cand])
            correct += int(pool[int(sims.argmax())] in labels)
            total += 1
    model.train()
    return correct / max(1, total)


def main(argv=None) -> int:
    a = build_args(argv)
    mp.Init()
    W = mp.COMM_WORLD()
    rank, size = W.Get_rank(), W.Get_size()
    dev = mp.runtime.device() or torch.device("cpu")
    if size == 1:
        servers, workers, testers = [0], [0], []
    else:
        servers, workers, testers = master_freq(size, a.masterFreq, "last" if a.testerlast else "first")
        if a.validMode == "lastClient":
            testers = []
    cranks = sorted(testers + workers)
    random.seed(rank)
    torch.manual_seed(rank)
    if a.trainFile != "none":
        data = load_files(a.embeddingFile, a.trainFile, a.label2answFile, a.validFile if a.validFile != "none" else None,
                          emb_dim=a.embeddingDim, conv_width=a.contConvWidth)
    else:
        data = synthetic_qa(n_answers=a.synthetic, emb_dim=a.embeddingDim, conv_width=a.contConvWidth)
    torch.manual_seed(1)  # identical initial weights
    model = BiCNN(len(data.word2idx), a.embeddingDim, a.wordHiddenDim, a.numFilters, a.contConvWidth, a.mmode).to(dev)
    with torch.no_grad():
        model.embed.weight.copy_(data.embedding_matrix().to(dev))
    flat = FlatParams(model)
    plong = flat.numel
    sopt = ServerOpt.from_bicnn_opt(vars(a))
    if a.optimization.endswith("single") or a.optimization in ("sgd", "msgd"):
        sopt = ServerOpt("sum")
    conf = dict(rank=rank, sranks=servers, cranks=cranks, plong=plong, opt=sopt)
    server = None
    if rank in servers:
        server = PServer(conf)
        server.start(block=rank not in cranks)
    if rank in cranks:
        pc = PClient(conf)
        pc.start(flat.flat, torch.zeros(plong, device=dev))
        if pc.rx.data_ptr() != flat.flat.data_ptr():
            flat.rebind(pc.rx)
        log = JsonLogger(os.path.join(a.save, f"rank{rank}.jsonl"), rank)
        if rank in testers:
            best, done, t0 = -1.0, 0, time.time()
            probe = mp.Status()
            while done < len(workers):
                while W.Iprobe(mp.ANY_SOURCE, TAG_WORKER_DONE, probe):
                    W.Recv(torch.zeros(1, dtype=torch.int64), probe.source, TAG_WORKER_DONE)
                    done += 1
                pc.async_recv_param()
                pc.wait()
                acc = evaluate(model, data, dev, max_q=200)
                log.log(kind="valid", acc=acc, elapsed=time.time() - t0)
                if acc > best:
                    best = acc
                    os.makedirs(a.save, exist_ok=True)
                    torch.save(flat.flat[:plong].cpu(), os.path.join(a.save, "best_params.pt"))
                time.sleep(a.testerPeriod)
            print(f"[bicnn tester] best valid acc {100 * best:.2f}%", flush=True)
        else:
            opti = OPTIMS[a.optimization]
            config = optim_config(a, pc)
            state = {}
            timers = Timers()
            avg = RunningAverage(every=50)
            n = len(data.train)
            steps = 0
            labs = sorted(data.answers)
            for ep in range(a.epochs):
                order = list(range(n))
                random.shuffle(order)
                for s in range(0, n - a.batchSize + 1, a.batchSize):
                    batch = [data.train[i] for i in order[s: s + a.batchSize]]
                    q = pad_batch([b[1] for b in batch]).to(dev)
                    ap_ = pad_batch([b[2] for b in batch]).to(dev)
                    negs = []
                    for labels, _, _ in batch:
                        cand = [x for x in random.sample(labs, min(len(labs), a.maxnegsample)) if x not in labels]
                        negs.append(cand[: max(1, min(len(cand), 8))])
                    k = min(len(x) for x in negs)
                    an = pad_batch([data.answers[x] for ng in negs for x in ng[:k]]).to(dev).view(len(batch), k, -1)

                    def feval(w):
                        with timers("feval"):
                            flat.zero_grad()
                            sp, sn = model(q, ap_, an)
                            loss = margin_ranking_loss(sp, sn, a.margin)
                            loss.backward()
                            if a.L1reg or a.L2reg or a.gradClip:
                                nm = ops.norms(flat.flat[:plong])
                                loss = loss + a.L1reg * nm[0] + 0.5 * a.L2reg * nm[1]
                                ops.regclip_(flat.grad, flat.flat, 1.0, a.L1reg, a.L2reg, a.gradClip)
                        return loss.detach(), flat.grad

                    _, (fx,) = opti(feval, flat.flat, config, state)
                    r = avg.add(float(fx))
                    if r is not None:
                        log.log(kind="train", step=steps, loss=r)
                    steps += 1
                    if a.maxSteps and steps >= a.maxSteps:
                        break
            pc.wait()
            if a.validMode == "lastClient" and rank == cranks[-1]:
                pc.async_recv_param()
                pc.wait()
                print(f"[bicnn lastClient] valid acc {100 * evaluate(model, data, dev):.2f}%", flush=True)
            print(f"[bicnn worker {rank}] steps {steps} feval {timers.total['feval']:.2f}s sync "
                  f"{state.get('dusync', 0.0):.2f}s", flush=True)
            for t in testers:
                W.Send(torch.ones(1, dtype=torch.int64), t, TAG_WORKER_DONE)
        pc.stop()
        log.close()
    if server is not None and rank in cranks:
        server.wait_done()
    W.Barrier()
    mp.Finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main())

"""BiCNN question-answer training through the parameter server
(BiCNN/plaunch.lua + BiCNN/bicnn.lua).

    python -m mpit_amd.launch -n 5 mpit_amd/apps/bicnn.py --optimization adam --testerfirst --masterFreq 2

Every plaunch.lua flag is accepted, with one or two leading dashes (``-testerfirst`` as in
the reference, or ``--testerfirst``); defaults are plaunch.lua:10-68's except ``epoch``
(1 here) and ``batchSize`` (64 here: the reference's default of 1 leaves an MI355X idle).

Roles (plaunch.lua:117-177): masterFreq assignment with the tester first or last;
``-maxrank`` caps the job at ranks 0..maxrank and leaves the rest idle (plaunch.lua:90-96;
here they join the final barrier instead of spinning forever). ``-validMode`` =
``additionalTester`` (a dedicated tester rank pulls the center parameters, evaluates
valid / test1 / test2 and writes a timestamped parameter file each round,
bicnn.lua:580-596), ``lastClient`` (the last client trains and also evaluates + saves
every ``commperiod`` steps, bicnn.lua:625-633) or ``none``. Unlike the reference, whose
tester never terminates (bicnn.lua:581), the tester stops once every worker finished.

Negative sampling (``-negMode parity``, the default): per example, draw negatives until
the first margin violation within ``maxnegsample`` draws and skip examples without one;
the summed hinge loss of the selected examples is back-propagated
(bicnn.lua:321-397, see models/bicnn.py::first_violations). ``-negMode hardest`` keeps the
batched hardest-of-8 shortcut of round 1.

Continuation: ``-loadmodel`` loads a parameter file (bicnn.lua:259-261), ``-prevtime``
offsets every reported / file-name time (plaunch.lua:61), ``-preloadBinary`` reads the
prepared-data cache written by ``-saveBinary`` instead of the text files
(plaunch.lua:218-229). ``-singlemode`` (pserver.lua:280-289): the server takes
parameters, not gradients, from ONE pusher (the first worker, which must run a ``*single``
optimizer or ``sgd``) and serves pulls to the tester; the other workers stop at once. The
reference's singlemode never queued its ``recvstop`` coroutine, so its server could not
stop; here the server counts every client's stop as in the normal mode.
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
from mpit_amd.apps.qa_data import (T7_VOCAB, load_binary, load_files, load_t7_vocab, pad_batch, qa_from_vocab,
                                   save_binary, synthetic_qa)
from mpit_amd.launch import master_freq
from mpit_amd.models.bicnn import (BiCNN, draw_negatives, first_violations, gesd, margin_ranking_loss, parity_grad_,
                                   parity_loss)
from mpit_amd.optim import ALL as OPTIMS
from mpit_amd.parallel.ps import PClient, PServer, ServerOpt
from mpit_amd.utils.flat import FlatParams
from mpit_amd.utils.metrics import JsonLogger, RunningAverage
from mpit_amd.utils.trace import Timers

TAG_WORKER_DONE = 9001
PUSH_ONLY = ("sgd", "msgd")


def _flag(ap, name, **kw):
    """plaunch.lua spelling (-name) and the usual --name."""
    ap.add_argument("--" + name, "-" + name, dest=name, **kw)


def _bool(s):
    return str(s).lower() in ("1", "true", "yes", "on")


def build_args(argv=None):
    ap = argparse.ArgumentParser(description="BiCNN QA training (BiCNN/plaunch.lua flags)")
    f = lambda n, **kw: _flag(ap, n, **kw)  # noqa: E731
    # data (plaunch.lua:40-50)
    f("embeddingFile", default="none")
    f("trainFile", default="none")
    f("validFile", default="none")
    f("testFile1", default="none")
    f("testFile2", default="none")
    f("label2answFile", default="none")
    f("embeddingDim", type=int, default=100)
    f("wordHiddenDim", type=int, default=200)
    f("numFilters", type=int, default=3000)
    f("contConvWidth", type=int, default=2)
    f("mmode", type=int, default=1)
    f("margin", type=float, default=0.02)
    f("maxnegsample", type=int, default=100)
    f("negMode", default="parity", choices=["parity", "hardest"])
    f("batchSize", type=int, default=64)
    f("epoch", type=int, default=1)
    ap.add_argument("--epochs", dest="epoch", type=int)
    f("maxSteps", type=int, default=0)
    f("threads", type=int, default=1)
    f("type", default="cuda", choices=["float", "double", "cuda"])
    # regularisation (bicnn.lua:398-409)
    f("L1reg", type=float, default=0.0)
    f("L2reg", type=float, default=1e-4)
    f("gradClip", type=float, default=0.5)
    # parity (default): regularise + clamp the accumulated gradient after every violating
    # example, as the reference does (bicnn.lua:398-409); batch: once per mini-batch
    f("clipMode", default="parity", choices=["parity", "batch"])
    f("weightDecay", type=float, default=1e-6)
    # optimisation (plaunch.lua:11-38)
    f("optimization", default="downpour")
    f("learningRate", type=float, default=1e-2)
    f("commperiod", type=int, default=1)
    f("movingrate", type=float, default=0.05)
    f("modeRMSProp", default="global")
    f("decayRMSProp", type=float, default=0.95)
    f("lrRMSProp", type=float, default=1e-4)
    f("momentumRMSProp", type=float, default=0.9)
    f("epsilonRMSProp", type=float, default=1e-4)
    f("modeAdam", default="global")
    f("lrAdam", type=float, default=1e-3)
    f("beta1Adam", type=float, default=0.9)
    f("beta2Adam", type=float, default=0.999)
    f("epsilonAdam", type=float, default=1e-8)
    f("stepDivAdam", type=int, default=72)
    f("modeAdagrad", default="global")
    f("lrAdagrad", type=float, default=1e-3)
    f("lrDecayAdagrad", type=float, default=1e-6)
    f("epsilonAdagrad", type=float, default=1e-10)
    f("modeAdadelta", default="global")
    f("rhoAdadelta", type=float, default=0.9)
    f("epsilonAdadelta", type=float, default=1e-6)
    f("lrAdadelta", type=float, default=1.0)
    f("mva", type=float, default=0.0)
    f("momentum", type=float, default=0.0)
    # topology / roles (plaunch.lua:37-70)
    f("masterFreq", type=int, default=2)
    f("testerfirst", action="store_true")
    f("testerlast", action="store_true")
    f("maxrank", type=int, default=-1, help="ranks above this stay idle (-1: all ranks work)")
    f("singlemode", action="store_true")
    f("servRecvgrad", type=_bool, default=True)
    f("servSendparam", type=_bool, default=True)
    f("validMode", default="additionalTester", choices=["additionalTester", "lastClient", "none"])
    f("validSleepTime", type=float, default=0.5, help="seconds between tester evaluations")
    ap.add_argument("--testerPeriod", dest="validSleepTime", type=float)
    f("evalMax", type=int, default=0, help="evaluate at most this many questions per set (0: all)")
    # continuation / output
    f("outputprefix", default="none")
    f("prevtime", type=float, default=0.0)
    f("loadmodel", default="none")
    f("preloadBinary", action="store_true")
    f("saveBinary", action="store_true", help="write the prepared-data cache and continue")
    f("binaryFile", default="binary_qadata.pt")
    f("binaryDir", default=".", help="-preloadBinary: directory of the reference's Torch7 caches (binary_map*)")
    f("save", default="bicnn_out")
    f("synthetic", type=int, default=200, help="synthetic answers when no data files are given")
    a = ap.parse_args(argv)
    if a.mva == 0.0:
        a.mva = a.movingrate
    return a


def optim_config(a, pc):
    o = a.optimization
    c = dict(pclient=pc, su=a.commperiod)
    if o in PUSH_ONLY:
        c.update(lr=a.learningRate, mom=a.momentum, push_param=True)
    elif o == "downpour":
        c.update(lr=a.learningRate)
    elif o in ("eamsgd", "easgd"):
        c.update(lr=a.learningRate, mva=a.mva, mom=a.momentum)
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


def assign_roles(a, size: int):
    """(servers, workers, testers, active) for a world of ``size`` ranks
    (plaunch.lua:90-177)."""
    if a.maxrank >= 0:
        size = min(size, a.maxrank + 1)
    active = list(range(size))
    if size == 1:
        return [0], [0], [], active
    servers, workers, testers = master_freq(size, a.masterFreq, "last" if a.testerlast else "first")
    if a.validMode != "additionalTester":
        # lastClient / none: the 'pe' rank is an ordinary training client (plaunch.lua:166-177)
        workers, testers = sorted(workers + testers), []
    return servers, workers, testers, active


@torch.no_grad()
def evaluate(model, data, items, dev, max_q=0) -> float:
    """Ranking accuracy over a pool per question (bicnn.lua:422-462): argmax GESD of the
    question vs every pool answer; ties go to the later pool entry (``simi >= most_simi``)."""
    model.eval()
    labs = sorted(data.answers)
    emb = []
    for s in range(0, len(labs), 256):
        emb.append(model.encode(pad_batch([data.answers[x] for x in labs[s: s + 256]]).to(dev)))
    emb = torch.cat(emb)
    pos = {x: i for i, x in enumerate(labs)}
    correct = total = 0
    items = items[:max_q] if max_q else items
    for s in range(0, len(items), 256):
        chunk = items[s: s + 256]
        eq = model.encode(pad_batch([q for _, q, _ in chunk]).to(dev))
        for (labels, _, pool), e in zip(chunk, eq):
            cand = torch.tensor([pos[p] for p in pool], device=dev)
            sims = gesd(e.unsqueeze(0).expand(len(pool), -1), emb[cand])
            best = len(pool) - 1 - int(sims.flip(0).argmax())  # last maximum
            correct += int(pool[best] in labels)
            total += 1
    model.train()
    return correct / max(1, total)


class Evaluator:
    """test3 (bicnn.lua:465-571): valid, test1, test2 with best-so-far per set."""

    def __init__(self, model, data, dev, rank, log, a, t0):
        self.model, self.data, self.dev, self.rank, self.log, self.a, self.t0 = model, data, dev, rank, log, a, t0
        self.sets = [("valid", data.valid)] + [(f"test{i + 1}", t) for i, t in enumerate(data.tests)]
        self.best = {n: 0.0 for n, _ in self.sets}

    def now(self) -> float:
        return time.time() - self.t0 + self.a.prevtime

    def __call__(self):
        accs = {}
        for i, (name, items) in enumerate(self.sets):
            if not items:
                continue
            acc = evaluate(self.model, self.data, items, self.dev, self.a.evalMax)
            self.best[name] = max(self.best[name], acc)
            accs[name] = acc
            print(f"Client {self.rank}: curr time: {self.now():.2f}, Accuracy: {acc:.4f}, best Accuracy: "
                  f"{self.best[name]:.4f} on file{i + 1}", flush=True)
        self.log.log(kind="eval", time=self.now(), **accs)
        return accs

    def save(self, flat, plong):
        if self.a.outputprefix != "none":
            d = os.path.dirname(self.a.outputprefix)
            if d:
                os.makedirs(d, exist_ok=True)
            torch.save(flat.flat[:plong].detach().cpu(), f"{self.a.outputprefix}_{self.now():010.2f}_model")


def load_data(a):
    if a.preloadBinary:
        # this package's cache (-saveBinary's --binaryFile) whenever it exists; otherwise the
        # reference's own Torch7 caches (plaunch.lua:221-228) in --binaryDir. Only the two
        # vocabulary maps of those ship (the other six are .MISSING_LARGE_BLOBS), so that
        # mode trains on SYNTHETIC questions / answers and random embeddings over the
        # reference's vocabulary — said loudly, never silently
        if os.path.exists(a.binaryFile):
            return load_binary(a.binaryFile)
        if all(os.path.exists(os.path.join(a.binaryDir, f)) for f in T7_VOCAB):
            print(f"bicnn: -preloadBinary: {a.binaryFile!r} not found; using the Torch7 vocabulary maps in "
                  f"{a.binaryDir!r} with SYNTHETIC questions/answers and random embeddings (the reference's "
                  f"dataset caches are not shipped)", file=sys.stderr, flush=True)
            return qa_from_vocab(load_t7_vocab(a.binaryDir), emb_dim=a.embeddingDim, conv_width=a.contConvWidth,
                                 n_answers=a.synthetic)
        return load_binary(a.binaryFile)
    if a.trainFile != "none":
        tests = [t for t in (a.testFile1, a.testFile2) if t != "none"]
        data = load_files(a.embeddingFile, a.trainFile, a.label2answFile, a.validFile if a.validFile != "none" else None,
                          tests=tests, emb_dim=a.embeddingDim, conv_width=a.contConvWidth)
    else:
        data = synthetic_qa(n_answers=a.synthetic, emb_dim=a.embeddingDim, conv_width=a.contConvWidth)
    if a.saveBinary:
        save_binary(data, a.binaryFile)
    return data


def main(argv=None) -> int:
    a = build_args(argv)
    mp.Init()
    W = mp.COMM_WORLD()
    rank, world = W.Get_rank(), W.Get_size()
    servers, workers, testers, active = assign_roles(a, world)
    if rank not in active:
        print(f"rank {rank} do nothing", flush=True)  # plaunch.lua:91-96
        W.Barrier()
        mp.Finalize()
        return 0
    dev = (mp.runtime.device() if a.type == "cuda" else None) or torch.device("cpu")
    cranks = sorted(testers + workers)
    pusher = workers[0] if workers else None
    if a.singlemode and not (a.optimization.endswith("single") or a.optimization in PUSH_ONLY):
        raise SystemExit("-singlemode: the server receives parameters, use a *single optimizer or sgd")
    random.seed(rank)
    torch.manual_seed(rank)
    data = load_data(a)  # servers too: the shard sizes follow the vocabulary
    torch.manual_seed(1)  # identical initial weights
    model = BiCNN(len(data.word2idx), a.embeddingDim, a.wordHiddenDim, a.numFilters, a.contConvWidth, a.mmode).to(dev)
    with torch.no_grad():
        model.embed.weight.copy_(data.embedding_matrix().to(dev))
    flat = FlatParams(model)
    plong = flat.numel
    if a.loadmodel != "none":
        with torch.no_grad():
            flat.flat[:plong].copy_(torch.load(a.loadmodel, weights_only=True).reshape(-1).to(flat.flat))
    sopt = ServerOpt.from_bicnn_opt(vars(a))
    if a.optimization.endswith("single") or a.optimization in PUSH_ONLY:
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
        t0 = time.time()
        ev = Evaluator(model, data, dev, rank, log, a, t0)
        if rank in testers:
            done = 0
            probe = mp.Status()
            n_workers = 1 if a.singlemode else len(workers)
            while done < n_workers:
                while W.Iprobe(mp.ANY_SOURCE, TAG_WORKER_DONE, probe):
                    W.Recv(torch.zeros(1, dtype=torch.int64), probe.source, TAG_WORKER_DONE)
                    done += 1
                t1 = time.perf_counter()
                pc.async_recv_param()
                pc.wait()
                print(f"Client {rank}: communication time: {time.perf_counter() - t1:.2f}", flush=True)
                ev()
                ev.save(flat, plong)
                time.sleep(a.validSleepTime)
            print(f"[bicnn tester] best valid acc {100 * ev.best['valid']:.2f}%", flush=True)
        elif a.singlemode and rank != pusher:
            print(f"[bicnn worker {rank}] singlemode: only rank {pusher} pushes parameters", flush=True)
        else:
            train(a, rank, model, flat, plong, data, dev, pc, log, ev, cranks)
            for t in testers:
                W.Send(torch.ones(1, dtype=torch.int64), t, TAG_WORKER_DONE)
        pc.stop()
        log.close()
    if server is not None and rank in cranks:
        server.wait_done()
    W.Barrier()
    mp.Finalize()
    return 0


def train(a, rank, model, flat, plong, data, dev, pc, log, ev, cranks):
    opti = OPTIMS[a.optimization]
    config = optim_config(a, pc)
    state = {}
    timers = Timers()
    avg = RunningAverage(every=50)
    n = len(data.train)
    steps = 0
    labs = sorted(data.answers)
    lpos = {x: i for i, x in enumerate(labs)}
    rng = random.Random(rank)
    last_client = a.validMode == "lastClient" and rank == cranks[-1]
    for ep in range(a.epoch):
        te = time.time()
        order = list(range(n))
        random.shuffle(order)
        for s in range(0, n, a.batchSize):  # the last partial batch too (bicnn.lua:614-618)
            batch = [data.train[i] for i in order[s: s + a.batchSize]]
            q = pad_batch([b[1] for b in batch]).to(dev)
            ap_ = pad_batch([b[2] for b in batch]).to(dev)
            if a.negMode == "hardest":
                negs = []
                for labels, _, _ in batch:
                    cand = [x for x in rng.sample(labs, min(len(labs), a.maxnegsample)) if x not in labels]
                    negs.append(cand[: max(1, min(len(cand), 8))])
                k = min(len(x) for x in negs)
                an = pad_batch([data.answers[x] for ng in negs for x in ng[:k]]).to(dev).view(len(batch), k, -1)
            else:
                draws = [[labs[j] for j in draw_negatives(rng, len(labs), [lpos[x] for x in labels if x in lpos],
                                                           a.maxnegsample)] for labels, _, _ in batch]

            def feval(w):
                with timers("feval"):
                    flat.zero_grad()
                    if a.negMode == "hardest":
                        sp, sn = model(q, ap_, an)
                        loss = margin_ranking_loss(sp, sn, a.margin)
                        nviol = len(batch)
                    else:
                        with torch.no_grad():
                            eq = model.encode(q)
                            sp0 = gesd(eq, model.encode(ap_))
                        chosen = first_violations(model, eq, sp0, draws, data.answers, a.margin, pad_batch)
                        sel = [i for i, c in enumerate(chosen) if c is not None]
                        nviol = len(sel)
                        if not sel:
                            return torch.zeros((), device=dev), flat.grad  # every example skipped
                        idx = torch.tensor(sel, device=dev)
                        an1 = pad_batch([data.answers[chosen[i]] for i in sel]).to(dev)
                        if a.clipMode == "parity" and (a.L1reg or a.L2reg or a.gradClip > 0):
                            loss = parity_grad_(model, flat, q[idx], ap_[idx], an1, a.margin, a.L1reg, a.L2reg,
                                                a.gradClip)
                            return loss.detach(), flat.grad
                        loss = parity_loss(model, q[idx], ap_[idx], an1, a.margin)
                    loss.backward()
                    if a.L1reg or a.L2reg or a.gradClip:
                        # per violating example in the reference (bicnn.lua:398-409): the
                        # regulariser is added once per example that produced a gradient
                        nm = ops.norms(flat.flat[:plong])
                        loss = loss + nviol * (a.L1reg * nm[0] + 0.5 * a.L2reg * nm[1])
                        ops.regclip_(flat.grad, flat.flat, 1.0, nviol * a.L1reg, nviol * a.L2reg, a.gradClip)
                return loss.detach(), flat.grad

            _, (fx,) = opti(feval, flat.flat, config, state)
            r = avg.add(float(fx))
            if r is not None:
                log.log(kind="train", step=steps, loss=r, time=ev.now())
            if last_client and steps % a.commperiod == 0:
                print(f"Client {rank} will also run testing", flush=True)
                ev()
                ev.save(flat, plong)
            steps += 1
            if a.maxSteps and steps >= a.maxSteps:
                break
        print(f"client {rank}: epoch {ep + 1} done, for {time.time() - te:.2f} seconds", flush=True)
        if a.maxSteps and steps >= a.maxSteps:
            break
    pc.wait()
    print(f"[bicnn worker {rank}] steps {steps} feval {timers.total['feval']:.2f}s sync "
          f"{state.get('dusync', 0.0):.2f}s", flush=True)


if __name__ == "__main__":
    sys.exit(main())

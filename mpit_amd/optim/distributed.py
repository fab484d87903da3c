"""Distributed optimizers of mpiT (SURVEY §2.4 O1–O3), Torch-optim calling convention.

``optim_fn(opfunc, w, config, state=None) -> (w, [fx])`` where ``opfunc(w)`` runs
forward + backward and returns ``(fx, dfdx)`` with ``dfdx`` the flat gradient tensor.
``config['pclient']`` is a started :class:`~mpit_amd.parallel.ps.PClient`.

Every tensor update is one fused native pass (mpit_amd.ops); the semantics, including
``state['pversion']`` starting at 0 so that step 0 is always a sync step, follow the
reference exactly. ``state['dusync']`` accumulates the time spent blocked on the
parameter server, as in the reference.
"""
from __future__ import annotations

import time

import torch

from ..utils import trace as _trace

from .. import ops


def _cfg(config, k, d):
    v = config.get(k, d)
    return d if v is None else v


def msgd(opfunc, w, config, state=None):
    """Nesterov momentum SGD, local only (asyncsgd/optim-msgd.lua:6-42)."""
    state = config if state is None else state
    lr, lrd, lrp = _cfg(config, "lr", 0.0), _cfg(config, "lrd", 0.0), _cfg(config, "lrp", 0.0)
    mom, mmax, mlrd = _cfg(config, "mom", 0.0), _cfg(config, "mommax", 1.0), _cfg(config, "momdecay", 0.0)
    l2wd = _cfg(config, "l2wd", 0.0)
    gscale = _cfg(config, "gscale", 1.0)
    pv = state.setdefault("pversion", 0)
    vt = None
    if mom > 0:
        if mlrd > 0:
            mom = min(mmax, 1 - 0.5 / (1 + pv / mlrd))
        vt = state.get("vt")
        if vt is None:
            vt = state["vt"] = torch.zeros_like(w)
        ops.nesterov_pre_(vt, w, mom)
    fx, dfdx = opfunc(w)
    clr = lr / (1 + pv * lrd) ** lrp if (lrd > 0 and lrp > 0) else lr
    ops.nesterov_post_(w, dfdx, vt, None, clr=clr, gscale=gscale, l2wd=l2wd)
    state["pversion"] = pv + 1
    pc = config.get("pclient")
    if pc is not None and config.get("push_param", False):
        # BiCNN "sgd" (BiCNN/optim-msgd.lua:47-48): push the parameters every step
        pc.async_send_param()
        t0 = time.perf_counter()
        pc.wait()
        state["dusync"] = state.get("dusync", 0.0) + time.perf_counter() - t0
    return w, [fx]


def downpour(opfunc, w, config, state=None):
    """Downpour / async SGD (asyncsgd/optim-downpour.lua:6-60); su == 1 is Hogwild-style
    async SGD. The worker's w must be the pClient's parameter window (pulled shards land
    in it); with su == 1 the scaled gradient is written straight into the push window."""
    state = config if state is None else state
    lr, lrd, l2wd = _cfg(config, "lr", 0.0), _cfg(config, "lrd", 0.0), _cfg(config, "l2wd", 0.0)
    gscale = _cfg(config, "gscale", 1.0)
    pc = config.get("pclient")
    su = _cfg(config, "su", 0)
    pv = state.setdefault("pversion", 0)
    state.setdefault("dusync", 0.0)
    if lrd != 0:
        lr = lr / (1 + pv * lrd)
    pusher = config.get("pusher")
    if pusher is not None and pc is not None and su == 1:
        # shards pushed (with their pulls) from inside the backward as they complete
        # (parallel/overlap.py); what is left here is the last shards' round trip
        with _trace.range("push_arm"):
            pusher.arm(-lr * gscale, w if l2wd else None, -lr * l2wd)
        try:
            fx, _ = opfunc(w)
        except BaseException:
            pusher.abort()  # no pushes of half-computed shards
            raise
        pusher.finish()
        pusher.reset()  # the next step's counters, while the pulls are still in flight
        if config.get("defer_wait"):
            # the caller retires the pulls right before its next read of w (mpit_amd/train.py
            # Trainer._feval / sync): the host's step bookkeeping then overlaps the servers'
            # apply + pull instead of following the reply
            state["wait_pending"] = True
        else:
            t0 = time.perf_counter()
            pc.wait()
            state["dusync"] += time.perf_counter() - t0
        state["pversion"] = pv + 1
        return w, [fx]
    fx, dfdx = opfunc(w)
    from ..utils.flat import StolenGrads

    if isinstance(dfdx, StolenGrads):
        if pc is not None and su == 1:
            # K12+K9 fused: gather every parameter's gradient straight into the push
            # window with the -lr scale (and weight decay) applied, one launch
            dfdx.gather(pc.tx, -lr * gscale, w if l2wd else None, -lr * l2wd)
            pc.async_send_grad(pull=True)
            t0 = time.perf_counter()
            pc.wait()
            state["dusync"] += time.perf_counter() - t0
            state["pversion"] = pv + 1
            return w, [fx]
        dfdx = dfdx.materialize()
    if pc is not None and su > 1:
        acc = pc.tx  # the push window doubles as the accumulator (reference: config.dfdx)
        if not config.get("_acc_init"):
            acc.zero_()
            config["_acc_init"] = True
        if pv % su == 0:
            ops.downpour_(dfdx, w, acc, lr, mode=1, gscale=gscale, l2wd=l2wd)
            pc.async_send_grad(pull=True)
            t0 = time.perf_counter()
            pc.wait()
            state["dusync"] += time.perf_counter() - t0
            acc.zero_()
        else:
            ops.downpour_(dfdx, w, acc, lr, mode=2, gscale=gscale, l2wd=l2wd)
    elif pc is not None and su == 1:
        ops.downpour_(dfdx, w, pc.tx, lr, mode=0, gscale=gscale, l2wd=l2wd)
        pc.async_send_grad(pull=True)
        t0 = time.perf_counter()
        pc.wait()
        state["dusync"] += time.perf_counter() - t0
    else:
        raise ValueError("downpour needs config['pclient'] and su >= 1")
    state["pversion"] = pv + 1
    return w, [fx]


def eamsgd(opfunc, w, config, state=None):
    """Elastic averaging (momentum) SGD (asyncsgd/optim-eamsgd.lua:7-79); mom == 0 is
    EASGD. Every ``su`` steps: pull the center w~ into the client's rx window, push
    ``sug = mva*(w - w~)`` (left in flight), run the local step, then ``w -= sug`` fused
    into the local step's kernel."""
    state = config if state is None else state
    lr, lrd, lrp = _cfg(config, "lr", 0.0), _cfg(config, "lrd", 0.0), _cfg(config, "lrp", 0.0)
    mom, l2wd = _cfg(config, "mom", 0.0), _cfg(config, "l2wd", 0.0)
    gscale = _cfg(config, "gscale", 1.0)
    pc, mva, su = config.get("pclient"), _cfg(config, "mva", 0.0), _cfg(config, "su", 1)
    state.setdefault("pversion", 0)
    state.setdefault("dusync", 0.0)
    out = {}

    def localupdate(sug=None):
        if lr == 0:
            # no local step (and no pversion increment), but the elastic correction still
            # applies: w -= sug (asyncsgd/optim-eamsgd.lua:69-70 runs it whatever the lr)
            if sug is not None:
                ops.axpby_(w, sug, -1.0, 1.0)
            return
        pv = state["pversion"]
        vt = None
        if mom > 0:
            vt = state.get("vt")
            if vt is None:
                vt = state["vt"] = torch.zeros_like(w)
            ops.nesterov_pre_(vt, w, mom)
        fx, dfdx = opfunc(w)
        out["fx"] = fx
        clr = lr / (1 + pv * lrd) ** lrp if (lrd != 0 and lrp > 0) else lr
        ops.nesterov_post_(w, dfdx, vt, sug, clr=clr, gscale=gscale, l2wd=l2wd)
        state["pversion"] = pv + 1

    if not (pc is not None and su > 0 and mva > 0):
        raise ValueError("eamsgd needs config['pclient'], su > 0 and mva > 0")
    if state["pversion"] % su == 0:
        suw, sug = pc.rx, pc.tx
        pc.async_recv_param()  # suw = w~
        t0 = time.perf_counter()
        pc.wait()  # also retires the previous in-flight push
        state["dusync"] += time.perf_counter() - t0
        ops.elastic_(w, suw, sug, mva)  # sug = mva*(w - w~)
        pc.async_send_grad()  # w~ += sug on the servers, overlapped with the local step
        pc.ping()
        localupdate(sug)  # ... w -= clr*g' + sug
    else:
        localupdate()
    return w, [out.get("fx")]


easgd = eamsgd

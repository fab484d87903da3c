"""BiCNN's adaptive distributed optimizers (SURVEY §2.4 O4–O13; BiCNN/optim-*.lua).

Three families, all with the Torch-optim signature ``f(opfunc, w, config, state)``:

* ``global`` mode (``rmsprop`` / ``adam`` / ``adamax`` / ``adagrad`` / ``adadelta``): the worker
  pushes its raw gradient (su == 1) or the sum of its last ``su`` gradients (su > 1) and
  pulls the parameters; the server applies the adaptive rule on its shard
  (:class:`~mpit_amd.parallel.ps.ServerOpt`, csrc/core/ps.cpp). On non-sync steps the
  worker does not move (BiCNN/optim-adam.lua:27-43).
* ``local`` RMSProp (BiCNN/optim-rmsprop.lua:48-66,74-90): the worker runs RMSProp and
  pushes the update ``u`` (su == 1) or the accumulated updates (su > 1, moving locally
  in between); the server just adds (rule 'sum').
* ``*single`` (BiCNN/optim-*-single.lua): a full local optimizer step, then the parameters
  are pushed to the server every step (parameter-push / single-writer mode).

Each tensor update is one fused kernel (mpit_amd.ops).
"""
from __future__ import annotations

import time

import torch

from .. import ops


def _sync(pc, state, pull=True):
    t0 = time.perf_counter()
    pc.wait()
    state["dusync"] = state.get("dusync", 0.0) + time.perf_counter() - t0


def _global_step(opfunc, w, config, state):
    """Shared body of the 'global' modes: push raw / accumulated gradients."""
    state = config if state is None else state
    pc, su = config.get("pclient"), config.get("su", 1) or 1
    pv = state.setdefault("pversion", 0)
    fx, dfdx = opfunc(w)
    if pc is None:
        raise ValueError("global-mode optimizers need config['pclient']")
    acc = pc.tx
    if su > 1:
        if not config.get("_acc_init"):
            acc.zero_()
            config["_acc_init"] = True
        ops.axpby_(acc, dfdx, 1.0, 1.0)  # accumulated += dfdx
        if pv % su == 0:
            pc.async_send_grad(pull=True)
            _sync(pc, state)
            acc.zero_()
    else:
        ops.copy_(acc, dfdx)
        pc.async_send_grad(pull=True)
        _sync(pc, state)
    state["pversion"] = pv + 1
    return w, [fx]


def adam(opfunc, w, config, state=None):
    """BiCNN/optim-adam.lua (global): server-side Adam with stepDivAdam."""
    return _global_step(opfunc, w, config, state)


adamax = adagrad = adadelta = adam


def rmsprop(opfunc, w, config, state=None):
    """BiCNN/optim-rmsprop.lua: mode 'global' (server RMSProp) or 'local'."""
    mode = config.get("mode", "global")
    if mode == "global":
        return _global_step(opfunc, w, config, state)
    if mode != "local":
        raise ValueError(f"Incorrect mode: {mode}")
    state = config if state is None else state
    pc, su = config.get("pclient"), config.get("su", 1) or 1
    decay, lr, mom, eps = config["decay"], config["lr"], config["momentum"], config["epsilon"]
    for k in ("gradAccum", "gradSqAccum", "update"):
        if k not in state:
            state[k] = torch.zeros_like(w)
    pv = state.setdefault("pversion", 0)
    fx, dfdx = opfunc(w)
    u = state["update"]
    # local mode: produce the update u only (p operand unused)
    ops.rmsprop_(u, dfdx, state["gradAccum"], state["gradSqAccum"], u, decay, lr, mom, eps, add=False)
    if su > 1:
        acc = pc.tx
        if not config.get("_acc_init"):
            acc.zero_()
            config["_acc_init"] = True
        ops.axpby_(acc, u, 1.0, 1.0)
        if pv % su == 0:
            pc.async_send_grad(pull=True)
            _sync(pc, state)
            acc.zero_()
        else:
            ops.axpby_(w, u, 1.0, 1.0)  # w += update
    else:
        ops.copy_(pc.tx, u)
        pc.async_send_grad(pull=True)
        _sync(pc, state)
    state["pversion"] = pv + 1
    return w, [fx]


# ------------------------------------------------------------------ single (parameter push)

def _push_params(config, state, w):
    pc = config.get("pclient")
    if pc is not None:
        pc.async_send_param(w)
        _sync(pc, state)


def rmspropsingle(opfunc, w, config, state=None):
    """BiCNN/optim-rmsprop-single.lua:6-39."""
    state = config if state is None else state
    for k in ("gradAccum", "gradSqAccum", "update"):
        if k not in state:
            state[k] = torch.zeros_like(w)
    fx, dfdx = opfunc(w)
    ops.rmsprop_(w, dfdx, state["gradAccum"], state["gradSqAccum"], state["update"], config["decay"], config["lr"],
                 config["momentum"], config["epsilon"], add=True)
    state["pversion"] = state.get("pversion", 0) + 1
    _push_params(config, state, w)
    return w, [fx]


def adamsingle(opfunc, w, config, state=None):
    """BiCNN/optim-adam-single.lua:6-38 (standard bias correction, k = t)."""
    state = config if state is None else state
    fx, dfdx = opfunc(w)
    for k in ("adam_m", "adam_v"):
        if k not in state:
            state[k] = torch.zeros_like(w)
    state["adam_t"] = state.get("adam_t", 0) + 1
    b1, b2 = config["beta1"], config["beta2"]
    lr_t = ops.adam_lr_t(config["lr"], b1, b2, state["adam_t"] - 1, 1)  # k = t
    ops.adam_(w, dfdx, state["adam_m"], state["adam_v"], b1, b2, config["epsilon"], lr_t)
    state["pversion"] = state.get("pversion", 0) + 1
    _push_params(config, state, w)
    return w, [fx]


def adamaxsingle(opfunc, w, config, state=None):
    """BiCNN/optim-adamax-single.lua:6-38."""
    state = config if state is None else state
    fx, dfdx = opfunc(w)
    for k in ("adamax_m", "adamax_u"):
        if k not in state:
            state[k] = torch.zeros_like(w)
    state["adamax_t"] = state.get("adamax_t", 0) + 1
    b1 = config["beta1"]
    lr_t = config["lr"] / (1 - b1 ** state["adamax_t"])
    ops.adamax_(w, dfdx, state["adamax_m"], state["adamax_u"], b1, config["beta2"], config["epsilon"], lr_t)
    state["pversion"] = state.get("pversion", 0) + 1
    _push_params(config, state, w)
    return w, [fx]


def adagradsingle(opfunc, w, config, state=None):
    """BiCNN/optim-adagrad-single.lua:6-33."""
    state = config if state is None else state
    pv = state.setdefault("pversion", 0)
    clr = config["lr"] / (1 + pv * config.get("lrd", 0.0))
    fx, dfdx = opfunc(w)
    if "paramVariance" not in state:
        state["paramVariance"] = torch.zeros_like(w)
    ops.adagrad_(w, dfdx, state["paramVariance"], config["epsilon"], clr)
    state["pversion"] = pv + 1
    _push_params(config, state, w)
    return w, [fx]


def adadeltasingle(opfunc, w, config, state=None):
    """BiCNN/optim-adadelta-single.lua:6-35."""
    state = config if state is None else state
    fx, dfdx = opfunc(w)
    for k in ("paramVariance", "accDelta"):
        if k not in state:
            state[k] = torch.zeros_like(w)
    ops.adadelta_(w, dfdx, state["paramVariance"], state["accDelta"], config["rho"], config["epsilon"],
                  config.get("lr", 1.0))
    state["pversion"] = state.get("pversion", 0) + 1
    _push_params(config, state, w)
    return w, [fx]

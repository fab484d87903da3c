"""Pure-PyTorch fp32 oracles of every fused rule, written from the reference's Lua
tensor-call chains (cited per function). Used only by tests and for debugging — the
framework never calls these on its hot path.
"""
from __future__ import annotations

import torch


def apply(p, g, a=1.0):
    return p + a * g.float()


def rmsprop(p, g, ga, gs, u, decay, lr, mom, eps, add=True):
    # BiCNN/pserver.lua:130-136
    g = g.float()
    ga = ga * decay + (1 - decay) * g
    gs = gs * decay + (1 - decay) * g * g
    rms = torch.sqrt(gs - ga * ga + eps)
    u = u * mom - lr * (g / rms)
    if add:
        p = p + u
    return p, ga, gs, u


def adam(p, g, m, v, b1, b2, eps, lr_t):
    # BiCNN/pserver.lua:147-154 (lr_t from the host)
    g = g.float()
    m = m * b1 + (1 - b1) * g
    v = v * b2 + (1 - b2) * g * g
    d = torch.sqrt(v) + eps
    return p - lr_t * m / d, m, v


def adamax(p, g, m, u, b1, b2, eps, lr_t):
    # BiCNN/pserver.lua:163-170
    g = g.float()
    m = m * b1 + (1 - b1) * g
    u = torch.maximum(u * b2, g.abs() + eps)
    return p - lr_t * m / u, m, u


def adagrad(p, g, var, eps, clr):
    # BiCNN/pserver.lua:177-182
    g = g.float()
    var = var + g * g
    return p - clr * g / (torch.sqrt(var) + eps), var


def adadelta(p, g, var, acc, rho, eps, lr):
    # BiCNN/pserver.lua:189-193
    g = g.float()
    var = var * rho + (1 - rho) * g * g
    std = torch.sqrt(var + eps)
    d = torch.sqrt(acc + eps) / std * g
    p = p - lr * d
    acc = acc * rho + (1 - rho) * d * d
    return p, var, acc


def nesterov_pre(vt, w, mom):
    # asyncsgd/optim-msgd.lua:27-28
    vt = vt * mom
    return vt, w + vt


def nesterov_post(w, g, vt, sug, clr, gscale=1.0, l2wd=0.0):
    # asyncsgd/optim-msgd.lua:31-39 ; optim-eamsgd.lua:36-44 then :70
    g = gscale * g.float() + l2wd * w
    w = w - clr * g
    if sug is not None:
        w = w - sug
    if vt is not None:
        vt = vt - clr * g
    return w, vt


def downpour(g, w, acc, lr, mode=0, gscale=1.0, l2wd=0.0):
    # asyncsgd/optim-downpour.lua:24-48
    d = -lr * (gscale * g.float() + l2wd * w)
    if mode == 0:
        acc = d
    else:
        acc = acc + d
    if mode == 2:
        w = w + d
    return acc, w


def elastic(w, c, mva):
    # asyncsgd/optim-eamsgd.lua:62-64
    return mva * (w - c)


def regclip(g, p, gscale=1.0, l1=0.0, l2=0.0, clip=0.0):
    # BiCNN/bicnn.lua:398-409
    g = gscale * g.float() + l1 * torch.sign(p) + l2 * p
    if clip > 0:
        g = g.clamp(-clip, clip)
    return g

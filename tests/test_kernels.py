"""Numerics of every fused update rule (K1–K14) against the pure-PyTorch fp32 oracles
written from the reference's Lua tensor chains (mpit_amd/ops/reference.py).

Runs on the host twins (CPU) always and on the gfx950 HIP kernels when a GPU is present
(``-m gpu``). Sizes include non-multiples of 4 and misaligned views, which exercise the
scalar tail and the unaligned-kernel paths."""
import math

import pytest
import torch

from mpit_amd import ops
from mpit_amd.ops import reference as R

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]
SIZES = [1, 7, 1024, 100003]


def _dev(d):
    if d == "cuda" and not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device(d)


def rnd(n, d, lo=-1.0, hi=1.0, dtype=torch.float32):
    g = torch.Generator().manual_seed(n * 31 + 7)
    return (torch.rand(n, generator=g) * (hi - lo) + lo).to(dtype).to(d)


def close(a, b, tol=2e-6):
    assert a.shape == b.shape
    err = (a.float().cpu() - b.float().cpu()).abs().max().item() if a.numel() else 0.0
    scale = max(1.0, b.float().abs().max().item() if b.numel() else 1.0)
    assert err <= tol * scale, f"max err {err} (scale {scale})"


@pytest.mark.parametrize("d", DEVICES)
@pytest.mark.parametrize("n", SIZES)
def test_apply(d, n):
    d = _dev(d)
    p, g = rnd(n, d), rnd(n + 1, d)[1:]  # g misaligned view
    out = torch.empty(n, device=d)
    ref = R.apply(p.clone(), g, 0.37)
    ops.apply_(p, g.contiguous() if n % 4 == 0 else g, 0.37, out=out)
    close(p, ref)
    close(out, ref)


@pytest.mark.parametrize("d", DEVICES)
def test_apply_bf16_grad_and_out(d):
    d = _dev(d)
    n = 4099
    p, g = rnd(n, d), rnd(n, d, dtype=torch.bfloat16)
    out = torch.empty(n, device=d, dtype=torch.bfloat16)
    ref = R.apply(p.clone(), g, -0.5)
    ops.apply_(p, g, -0.5, out=out)
    close(p, ref)
    close(out, ref.to(torch.bfloat16), tol=1e-2)


@pytest.mark.parametrize("d", DEVICES)
@pytest.mark.parametrize("out", [False, True])
def test_apply_multi_segment_equals_per_segment(d, out):
    """One multi-segment launch over disjoint pieces (sizes with n % 4 tails, a one-element
    piece, bf16 gradients) == one apply_ per piece, bit for bit."""
    d = _dev(d)
    sizes = [100003, 1, 4096, 7, 33333, 1024]
    base = rnd(sum(sizes), d)
    gb = rnd(sum(sizes) + 5, d, dtype=torch.bfloat16)[:sum(sizes)]
    offs = [sum(sizes[:i]) for i in range(len(sizes))]
    # 16-B aligned piece starts (the multi kernel's vector path) and an unaligned set (fallback)
    for align in (True, False):
        o, at = [], 0
        for n in sizes:  # aligned: each piece starts at the next multiple of 4 after the last
            at = (at + 3) // 4 * 4 if align else at
            o.append(at)
            at += n
        p1 = torch.zeros(o[-1] + sizes[-1] + 8, device=d)
        p2 = p1.clone()
        segs1 = [p1[a:a + n] for a, n in zip(o, sizes)]
        segs2 = [p2[a:a + n] for a, n in zip(o, sizes)]
        for s1, s2, a, n in zip(segs1, segs2, offs, sizes):
            s1.copy_(base[a:a + n])
            s2.copy_(base[a:a + n])
        gs = [gb[a:a + n].clone() for a, n in zip(offs, sizes)]
        o1 = [torch.empty(n, device=d) for n in sizes] if out else None
        o2 = [torch.empty(n, device=d) for n in sizes] if out else None
        ops.apply_multi_(segs1, gs, -0.3, outs=o1)
        for i, (s2, g) in enumerate(zip(segs2, gs)):
            ops.apply_(s2, g, -0.3, out=o2[i] if out else None)
        assert torch.equal(p1, p2)
        if out:
            for u, v in zip(o1, o2):
                assert torch.equal(u, v)


@pytest.mark.parametrize("d", DEVICES)
@pytest.mark.parametrize("ng", [1, 2, 3, 8])
def test_apply_sum(d, ng):
    d = _dev(d)
    n = 5003
    p = rnd(n, d)
    gs = [rnd(n, d) * (k + 1) for k in range(ng)]
    ref = p.clone() + 0.25 * sum(gs)
    ops.apply_sum_(p, gs, 0.25)
    close(p, ref, 1e-5)


@pytest.mark.parametrize("d", DEVICES)
@pytest.mark.parametrize("add", [True, False])
def test_rmsprop(d, add):
    d = _dev(d)
    n = 10007
    p, g = rnd(n, d), rnd(n, d)
    ga, gs, u = rnd(n, d) * 0.1, rnd(n, d, 0.5, 1.0), rnd(n, d) * 0.01
    rp, rga, rgs, ru = R.rmsprop(p.clone(), g, ga.clone(), gs.clone(), u.clone(), 0.95, 1e-3, 0.9, 1e-4, add)
    p0 = p.clone()
    ops.rmsprop_(p, g, ga, gs, u, 0.95, 1e-3, 0.9, 1e-4, add=add)
    close(ga, rga)
    close(gs, rgs)
    close(u, ru, 1e-5)
    close(p, rp if add else p0)


@pytest.mark.parametrize("d", DEVICES)
def test_adam_and_lr_t(d):
    d = _dev(d)
    n = 4097
    p, g, m, v = rnd(n, d), rnd(n, d), rnd(n, d) * 0.1, rnd(n, d, 0.0, 0.01)
    lr_t = ops.adam_lr_t(1e-3, 0.9, 0.999, t=150, step_div=72)
    assert math.isclose(lr_t, 1e-3 * math.sqrt(1 - 0.999 ** 3) / (1 - 0.9 ** 3))
    rp, rm, rv = R.adam(p.clone(), g, m.clone(), v.clone(), 0.9, 0.999, 1e-8, lr_t)
    ops.adam_(p, g, m, v, 0.9, 0.999, 1e-8, lr_t)
    close(m, rm)
    close(v, rv)
    close(p, rp, 1e-5)


@pytest.mark.parametrize("d", DEVICES)
def test_adamax(d):
    d = _dev(d)
    n = 3001
    p, g, m, u = rnd(n, d), rnd(n, d), rnd(n, d) * 0.1, rnd(n, d, 0.0, 0.5)
    rp, rm, ru = R.adamax(p.clone(), g, m.clone(), u.clone(), 0.9, 0.999, 1e-8, 2e-3)
    ops.adamax_(p, g, m, u, 0.9, 0.999, 1e-8, 2e-3)
    close(m, rm)
    close(u, ru)
    close(p, rp, 1e-5)


@pytest.mark.parametrize("d", DEVICES)
def test_adagrad(d):
    d = _dev(d)
    n = 2049
    p, g, var = rnd(n, d), rnd(n, d), rnd(n, d, 0.0, 1.0)
    rp, rv = R.adagrad(p.clone(), g, var.clone(), 1e-10, 0.01)
    ops.adagrad_(p, g, var, 1e-10, 0.01)
    close(var, rv)
    close(p, rp, 1e-5)


@pytest.mark.parametrize("d", DEVICES)
def test_adadelta(d):
    d = _dev(d)
    n = 2051
    p, g, var, acc = rnd(n, d), rnd(n, d), rnd(n, d, 0.0, 1.0), rnd(n, d, 0.0, 1.0)
    rp, rv, ra = R.adadelta(p.clone(), g, var.clone(), acc.clone(), 0.95, 1e-6, 1.0)
    ops.adadelta_(p, g, var, acc, 0.95, 1e-6, 1.0)
    close(var, rv)
    close(acc, ra, 1e-5)
    close(p, rp, 1e-5)


@pytest.mark.parametrize("d", DEVICES)
@pytest.mark.parametrize("vt", [True, False])
@pytest.mark.parametrize("sug", [True, False])
def test_nesterov(d, vt, sug):
    d = _dev(d)
    n = 6007
    w, g = rnd(n, d), rnd(n, d)
    v = rnd(n, d) * 0.1 if vt else None
    s = rnd(n, d) * 0.01 if sug else None
    if vt:
        rv, rw = R.nesterov_pre(v.clone(), w.clone(), 0.9)
        ops.nesterov_pre_(v, w, 0.9)
        close(v, rv)
        close(w, rw)
    rw, rv = R.nesterov_post(w.clone(), g, v.clone() if vt else None, s, 0.01, gscale=0.5, l2wd=1e-4)
    ops.nesterov_post_(w, g, v, s, clr=0.01, gscale=0.5, l2wd=1e-4)
    close(w, rw)
    if vt:
        close(v, rv)


@pytest.mark.parametrize("d", DEVICES)
@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("l2wd", [0.0, 1e-3])
def test_downpour(d, mode, l2wd):
    d = _dev(d)
    n = 8191
    g, w, acc = rnd(n, d), rnd(n, d), rnd(n, d)
    racc, rw = R.downpour(g, w.clone(), acc.clone(), 0.1, mode, gscale=0.25, l2wd=l2wd)
    ops.downpour_(g, w, acc, 0.1, mode=mode, gscale=0.25, l2wd=l2wd)
    close(acc, racc)
    close(w, rw)


@pytest.mark.parametrize("d", DEVICES)
def test_downpour_nan_safe_without_w(d):
    # mode 0 without weight decay must not read w (it may hold garbage / NaN)
    d = _dev(d)
    n = 4096
    g, acc = rnd(n, d), torch.zeros(n, device=d)
    w = torch.full((n,), float("nan"), device=d)
    ops.downpour_(g, w, acc, 0.5, mode=0)
    assert torch.isfinite(acc).all()
    close(acc, -0.5 * g)


@pytest.mark.parametrize("d", DEVICES)
def test_elastic_regclip_scale_copy_fill(d):
    d = _dev(d)
    n = 5000
    w, c = rnd(n, d), rnd(n, d)
    sug = torch.empty(n, device=d)
    ops.elastic_(w, c, sug, 0.45)
    close(sug, R.elastic(w, c, 0.45))
    g, p = rnd(n, d), rnd(n, d)
    rg = R.regclip(g.clone(), p, 0.5, 1e-3, 1e-2, 0.3)
    ops.regclip_(g, p, 0.5, 1e-3, 1e-2, 0.3)
    close(g, rg)
    x = rnd(n, d)
    r = x * 3.0
    ops.scale_(x, 3.0)
    close(x, r)
    b = torch.empty(n, device=d, dtype=torch.bfloat16)
    ops.copy_(b, x)
    close(b, x.to(torch.bfloat16), 0)
    y = torch.empty(n, device=d)
    ops.copy_(y, b, 2.0)
    close(y, 2.0 * b.float(), 0)
    ops.fill_(y, -1.5)
    assert (y == -1.5).all()
    z = rnd(n, d)
    rz = 0.5 * x + 2.0 * z
    ops.axpby_(z, x, 0.5, 2.0)
    close(z, rz)


@pytest.mark.parametrize("d", DEVICES)
@pytest.mark.parametrize("n", [3, 1 << 20])
def test_norms_dot(d, n):
    d = _dev(d)
    x, y = rnd(n, d), rnd(n, d)
    nm = ops.norms(x).cpu()
    xd = x.double().cpu()
    assert math.isclose(nm[0].item(), xd.abs().sum().item(), rel_tol=1e-4)
    assert math.isclose(nm[1].item(), (xd * xd).sum().item(), rel_tol=1e-4)
    assert nm[2].item() == x.abs().max().item()
    dt = ops.dot(x, y).cpu()
    assert math.isclose(dt.item(), (xd * y.double().cpu()).sum().item(), rel_tol=1e-3, abs_tol=1e-3)
    # deterministic: bitwise identical on repeat
    assert torch.equal(ops.norms(x).cpu(), nm)


@pytest.mark.parametrize("d", DEVICES)
@pytest.mark.parametrize("l2wd", [0.0, 1e-2])
def test_stolen_grads_gather_scale(d, l2wd):
    """K12+K9: autograd's own gradient tensors gathered into the push buffer with the
    Downpour scale in one launch, channels_last conv weights included."""
    d = _dev(d)
    from mpit_amd.utils.flat import FlatParams

    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3), torch.nn.ReLU(), torch.nn.Flatten(),
                            torch.nn.Linear(8 * 6 * 6, 5)).to(d)
    cl = d.type == "cuda"
    if cl:
        m = m.to(memory_format=torch.channels_last)
    fp = FlatParams(m, channels_last=cl)
    x = torch.randn(4, 3, 8, 8, device=d)
    # reference: accumulate into the flat gradient views
    m(x).square().sum().backward()
    ref = -0.1 * (fp.grad.clone() + l2wd / 1.0 * 0) - 0.1 * l2wd * fp.flat
    fp.steal_grads()
    m(x).square().sum().backward()
    out = torch.full((fp.numel,), 7.0, device=d)
    fp.stolen().gather(out, -0.1, fp.flat if l2wd else None, -0.1 * l2wd)
    # padding between parameters is not written by the gather; compare parameter ranges
    for p, off in zip(fp.params, fp.offsets):
        close(out[off: off + p.numel()], ref[off: off + p.numel()], 1e-5)
    assert all(p.grad is None for p in fp.params)


@pytest.mark.parametrize("d", DEVICES)
def test_pack_unpack(d):
    d = _dev(d)
    shapes = [(64, 3, 7, 7), (1000,), (3,), (256, 1024), (70001,)]
    ts = [rnd(int(torch.tensor(s).prod()), d).view(s) for s in shapes]
    total = sum(t.numel() for t in ts)
    flat = torch.zeros(total, device=d)
    plan = ops.PackPlan(ts, flat)
    plan.pack(scale=0.5)
    close(flat, 0.5 * torch.cat([t.reshape(-1) for t in ts]))
    # unpack into bf16 model copies
    bts = [torch.zeros(s, device=d, dtype=torch.bfloat16) for s in shapes]
    plan2 = ops.PackPlan(bts, flat)
    plan2.unpack(scale=2.0)
    for t, b in zip(ts, bts):
        close(b, t.to(torch.bfloat16), 1e-2)


@pytest.mark.parametrize("d", DEVICES)
@pytest.mark.parametrize("n", SIZES)
def test_clamp_scan(d, n):
    """K11 per example: G = clamp(G + g_k + l1 sign(p) + l2 p, -c, c) for k in order, vs a
    plain PyTorch fp32 loop (HIP kernel on the GPU, host twin on the CPU)."""
    dev = _dev(d)
    rows, ldg = 5, n + (-n % 4) + 8
    g = torch.zeros(rows, ldg)
    for k in range(rows):
        g[k, :n] = rnd(n + k, "cpu", -0.4, 0.4)[:n]
    p = rnd(n + 11, "cpu")[:n].contiguous()
    G0 = rnd(n + 13, "cpu", -0.3, 0.3)[:n].contiguous()
    l1, l2, c = 1e-3, 1e-2, 0.25
    ref = G0.clone()
    for k in range(rows):
        ref = (ref + g[k, :n] + l1 * torch.sign(p) + l2 * p).clamp(-c, c)
    G = G0.to(dev)
    ops.clamp_scan_(G, g.to(dev), p.to(dev), l1, l2, c)
    close(G, ref)

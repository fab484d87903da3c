"""fp16x3 split products for the fp32 GEMMs (csrc/kernels/gemm.hip FM 11): the power-of-two
operand scales come from device-side bounds of |x| that the producers write — the BN apply
passes (forward y, backward dx, the bn_pair passes, the finalize folded into a backward-data
GEMM) and the weight plan. A bound below the true max |x| would overflow the fp16 planes, so
every producer's bound is checked to equal max |x| exactly."""
import pytest
import torch

from mpit_amd.ops import conv as C

gpu = pytest.mark.gpu


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def test_exp2i_exact_cpu():
    e = torch.arange(-126, 128)
    got = C._exp2i(e)
    want = torch.tensor([2.0 ** int(k) for k in e.tolist()], dtype=torch.float64)
    assert torch.equal(got.double(), want)


def test_f16_exp_places_bound_cpu():
    for a in (1e-30, 3e-8, 0.0625, 0.07, 1.0, 13.5, 1e6, 3e38):
        e = int(C._f16_exp(torch.tensor([a])).item())
        assert 2.0 ** 13 <= a * 2.0 ** e < 2.0 ** 14 or e in (-126, 116), (a, e)
    assert int(C._f16_exp(torch.tensor([0.0])).item()) == 0
    assert int(C._f16_exp(torch.tensor([float("inf")])).item()) == 0


def test_f16_planes_match_exact_split_cpu():
    """f16_planes == the exact residual split, element by element (h = RNE(s), l = RNE(2^11 (s - h)))."""
    torch.manual_seed(1)
    w = torch.randn(2000) * 0.05
    amax = C.bound_of_value(w.abs().max())
    p = C.f16_planes(w, amax)
    e = int(C._f16_exp(C.bound_value(amax)).item())
    s = w.double() * 2.0 ** e
    h = s.half().double()
    assert torch.equal(p[0].double(), h)
    assert torch.equal(p[1].double(), ((s - h) * 2048).half().double())


def test_park_grad_keeps_bound_cpu():
    x = torch.randn(4, 8)
    a = C.bound_of_value(x.abs().max())
    C.set_amax(x, a)
    v = C.park_grad(x, C.GradSlot())
    assert C.amax_of(v) is a
    x.add_(1.0)  # a new version: the bound no longer holds
    assert C.amax_of(x) is None


def _bound(t):
    a = C.amax_of(t)
    assert a is not None, "no bound attached"
    return C.bound_value(a).item()


@gpu
@pytest.mark.parametrize("res,relu", [(False, True), (True, True), (False, False)])
def test_bn_forward_backward_bounds_exact(res, relu):
    from mpit_amd.ops.bn import BatchNormAct2d

    torch.manual_seed(3)
    bn = BatchNormAct2d(64, act=relu).cuda()
    bn.weight.data.uniform_(0.5, 2.0)
    bn.bias.data.uniform_(-1.0, 1.0)
    x = _cl(torch.randn(4, 64, 9, 9, device="cuda") * 3).requires_grad_(True)
    r = _cl(torch.randn(4, 64, 9, 9, device="cuda")) if res else None
    got = []
    x.register_hook(lambda g: got.append(g))
    y = bn(x, r)
    torch.cuda.synchronize()
    assert _bound(y) == y.detach().abs().max().item()
    y.backward(torch.randn_like(y) * 1e-6)
    torch.cuda.synchronize()
    assert _bound(got[0]) == got[0].abs().max().item()


@gpu
def test_bn_pair_bounds_exact():
    from mpit_amd.ops.bn import BatchNormAct2d, bn_pair

    torch.manual_seed(4)
    b1, b2 = BatchNormAct2d(128).cuda(), BatchNormAct2d(128, act=False).cuda()
    x1 = _cl(torch.randn(2, 128, 7, 7, device="cuda")).requires_grad_(True)
    x2 = _cl(torch.randn(2, 128, 7, 7, device="cuda")).requires_grad_(True)
    g1, g2 = [], []
    x1.register_hook(lambda g: g1.append(g))
    x2.register_hook(lambda g: g2.append(g))
    y = bn_pair(b1, x1, b2, x2)
    torch.cuda.synchronize()
    assert _bound(y) == y.detach().abs().max().item()
    y.backward(torch.randn_like(y))
    torch.cuda.synchronize()
    assert _bound(g1[0]) == g1[0].abs().max().item()
    assert _bound(g2[0]) == g2[0].abs().max().item()


@gpu
def test_folded_finalize_bound_exact():
    """BN -> Conv1x1: the conv's backward-data GEMM folds the BN backward's finalize and zeroes
    the bound that the BN's apply pass then raises to max |dx|; repeated steps reuse nothing stale."""
    from mpit_amd.ops.bn import COUNTERS, BatchNormAct2d

    torch.manual_seed(5)
    bn = BatchNormAct2d(128).cuda()
    conv = C.Conv1x1(128, 256).cuda().to(memory_format=torch.channels_last)
    for step in range(3):
        x = _cl(torch.randn(2, 128, 14, 14, device="cuda") * (10.0 ** -step)).requires_grad_(True)
        got = []
        x.register_hook(lambda g: got.append(g))
        n0 = COUNTERS["bwd_folded"]
        z = conv(bn(x))
        z.backward(torch.randn_like(z))
        torch.cuda.synchronize()
        assert COUNTERS["bwd_folded"] == n0 + 1
        assert _bound(got[0]) == got[0].abs().max().item()


@gpu
def test_resnet50_f16x3_step_uses_producer_bounds():
    """One fp32 ResNet-50 step through the weight plan: every fp16x3 GEMM operand has its
    producer's bound (no fallback reduction), and the backward-weight GEMMs run fp16x3."""
    from mpit_amd.models.resnet import resnet50

    if C._F32_SPLIT != "f16x3":
        pytest.skip("MPIT_F32_SPLIT=bf16x6")
    torch.manual_seed(0)
    net = resnet50(num_classes=10).cuda().to(memory_format=torch.channels_last)
    plan = C.WeightCastPlan(net, torch.float32)
    x = _cl(torch.randn(4, 3, 64, 64, device="cuda"))
    c0 = dict(C.COUNTERS)
    plan.run()
    out = net(x)
    out.float().sum().backward()
    plan.invalidate()
    torch.cuda.synchronize()
    d = {k: C.COUNTERS[k] - c0[k] for k in C.COUNTERS}
    assert d["amax_fallback"] == 0
    # every conv but the stem, on fp32 operands (FM 12) or on fp16 planes (FM 13, the
    # activations / gradients the BN passes write as planes: ops/conv.py _F32_PLANES)
    assert d["wgrad_f16x3"] + d["wgrad_planes"] == 52, d
    assert d["wgrad_mixed"] == 0 and d["unplanes"] == 0, d
    if C._F32_PLANES:
        assert d["wgrad_planes"] >= 45, d
    for m in net.modules():
        if isinstance(m, torch.nn.Conv2d):
            assert torch.isfinite(m.weight.grad).all()


@gpu
def test_stem_f16x3_vs_fp64():
    """The row-tap stem on fp16x3 (32-deep tiles, one kernel row per k-tile), forward and, with
    the stem BN's backward bound on dy, the backward-weight GEMM: within 2x of PyTorch fp32."""
    import torch.nn.functional as F

    from mpit_amd.ops.bn import BatchNormAct2d

    torch.manual_seed(6)
    conv = C.StemConv(3, 64, 7, 2, 3).cuda().to(memory_format=torch.channels_last)
    bn = BatchNormAct2d(64).cuda()
    x = _cl(torch.randn(4, 3, 64, 64, device="cuda"))
    assert conv.fused(x)
    y = bn(conv(x))
    g = torch.randn_like(y)
    y.backward(g)

    def ref(dev, dt):
        xx = x.to(dev, dt)
        ww = conv.weight.detach().to(dev, dt).clone().requires_grad_(True)
        z = F.conv2d(xx, ww, stride=2, padding=3)
        yy = F.relu(F.batch_norm(z, None, None, bn.weight.detach().to(dev, dt), bn.bias.detach().to(dev, dt),
                                 training=True, eps=bn.eps))
        yy.backward(g.to(dev, dt))
        return yy.detach(), ww.grad

    (yr, gr), (yl, gl) = ref("cpu", torch.float64), ref("cuda", torch.float32)

    def rel(a, b):
        a, b = a.double().cpu(), b.double().cpu()
        return ((a - b).norm() / b.norm()).item()

    assert rel(y, yr) <= 2 * rel(yl, yr) + 1e-9
    assert rel(conv.weight.grad, gr) <= 2 * rel(gl, gr) + 1e-9


@gpu
def test_folded_finalize_on_many_streams():
    """The BN finalize fold takes its ticket sets per (device, stream): a process that runs the
    fold from more than the static table's 8 streams (one priority stream per Trainer, test
    sessions) gets a zeroed allocation per extra stream instead of an exception, with the same
    bits on every stream (round-3 verdict: an 8-stream process-lifetime cap)."""
    from mpit_amd.ops.bn import COUNTERS, BatchNormAct2d

    torch.manual_seed(7)
    bn = BatchNormAct2d(128).cuda()
    conv = C.Conv1x1(128, 256).cuda().to(memory_format=torch.channels_last)
    x0 = _cl(torch.randn(2, 128, 14, 14, device="cuda"))
    g = None
    outs = []
    for k in range(12):
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            x = x0.clone().requires_grad_(True)
            n0 = COUNTERS["bwd_folded"]
            z = conv(bn(x))
            if g is None:
                g = torch.randn_like(z)
            bn.zero_grad(set_to_none=True)
            z.backward(g)
            outs.append((x.grad.clone(), bn.weight.grad.clone()))
        torch.cuda.current_stream().wait_stream(st)
        torch.cuda.synchronize()
        assert COUNTERS["bwd_folded"] == n0 + 1
    for dx, dgam in outs[1:]:
        assert torch.equal(dx, outs[0][0]) and torch.equal(dgam, outs[0][1])

"""The fp32 training path (the reference's precision: asyncsgd/glaunch.lua:11 trains
CudaTensors, BiCNN/plaunch.lua:200 likewise) on the hand-written gfx950 kernels:
``v_mfma_f32_32x32x2_f32`` GEMMs / implicit-GEMM convolutions (csrc/kernels/gemm.hip),
fp32 fused BN (bn_act.hip) and max pooling (pool.hip).

Every GEMM-shaped op is held to at most 2x the error of PyTorch's own fp32 op (rocBLAS /
MIOpen) against an fp64 reference of the same math, computed on the CPU."""
import pytest
import torch
import torch.nn.functional as F

from mpit_amd.ops import conv as C

gpu = pytest.mark.gpu


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-300)).item()


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def test_mfma_dtype_selection_cpu():
    x = torch.randn(2, 64, 4, 4)
    assert C.mfma_dtype(x) == torch.float32
    assert C.mfma_dtype(x.to(torch.bfloat16)) == torch.bfloat16
    assert C.mfma_dtype(x.half()) is None
    # CPU tensors never take the MFMA path
    assert not C.conv_supported(x, torch.randn(64, 64, 3, 3))


@gpu
@pytest.mark.parametrize("M,N,K", [(128, 64, 64), (1000, 192, 128), (4096, 256, 512), (333, 64, 1024),
                                   (12544, 512, 2048), (50176, 128, 576)])
def test_gemm_nt_fp32_vs_fp64(M, N, K):
    torch.manual_seed(M + N + K)
    a = torch.randn(M, K, device="cuda")
    b = torch.randn(N, K, device="cuda") * 0.05
    ref = a.double().cpu() @ b.double().cpu().t()
    c = C.gemm_nt(a, b)
    assert c.dtype == torch.float32 and c.shape == (M, N)
    lib = a @ b.t()
    e, el = _rel(c, ref), _rel(lib, ref)
    assert e <= 2.0 * el + 1e-9, (e, el)
    assert e < 2e-6


def test_f16_planes_carry_22_bits_cpu():
    """fp16x3 weight planes: (h + l / 2^11) / 2^e == w to 2^-22 relative for |w| 2^e >= 2^-14
    (within 2^27 of the bound; the scale places the bound in [2^13, 2^14)); smaller values keep
    their absolute error below 2^-48 of the bound."""
    torch.manual_seed(0)
    w = torch.randn(4096) * torch.exp(torch.randn(4096) * 3)
    amax = w.abs().max().reshape(1)
    p = C.f16_planes(w, C.bound_of_value(amax))
    assert p.dtype == torch.float16 and p.shape == (2, 4096)
    e = int(C._f16_exp(amax).item())
    assert 2.0 ** 13 <= amax.item() * 2.0 ** e < 2.0 ** 14
    back = C._unsplit(p)
    err = (back.double() - w.double()).abs()
    big = w.abs() * 2.0 ** e >= 2.0 ** -14
    assert (err[big] <= w.double().abs()[big] * 2.0 ** -22).all()
    assert (err[~big] <= amax.item() * 2.0 ** -48).all()
    assert torch.isfinite(p.float()).all()


@gpu
@pytest.mark.parametrize("M,N,K", [(128, 64, 64), (1000, 192, 128), (4096, 256, 512), (333, 64, 1024),
                                   (12544, 512, 2048), (50176, 128, 576)])
def test_gemm_nt_f16x3_vs_fp64(M, N, K):
    """fp16x3 split products (FM 11): within 2x of PyTorch fp32's error against fp64, also for
    a gradient-sized operand (1e-7 scale: the power-of-two scale keeps it in fp16 range)."""
    torch.manual_seed(M + N + K)
    for sa in (1.0, 1e-7):
        a = torch.randn(M, K, device="cuda") * sa
        b = torch.randn(N, K, device="cuda") * 0.05
        ref = a.double().cpu() @ b.double().cpu().t()
        c = C.gemm_nt(a, b, f16x3=True)
        lib = a @ b.t()
        e, el = _rel(c, ref), _rel(lib, ref)
        assert e <= 2.0 * el + 1e-9, (sa, e, el)
        assert e < 2e-6


@gpu
@pytest.mark.parametrize("M,N,K", [(64, 64, 64), (1000, 64, 128), (4096, 128, 128), (200704, 256, 64),
                                   (12544, 512, 2048), (5000, 192, 320)])
def test_gemm_tn_f16x3_vs_fp64(M, N, K):
    torch.manual_seed(M % 97 + N + K)
    y, x = torch.randn(M, N, device="cuda") * 1e-6, torch.relu(torch.randn(M, K, device="cuda"))
    ref = y.double().cpu().t() @ x.double().cpu()
    out = C.gemm_tn(y, x, f16x3=True)
    lib = y.t() @ x
    e, el = _rel(out, ref), _rel(lib, ref)
    assert e <= 2.0 * el + 1e-9, (e, el)


@gpu
@pytest.mark.parametrize("M,N,K", [(256, 64, 64), (1000, 128, 192)])
def test_gemm_nt_fp32_stats(M, N, K):
    torch.manual_seed(1)
    a, b = torch.randn(M, K, device="cuda"), torch.randn(N, K, device="cuda") * 0.05
    c, st = C.gemm_nt(a, b, stats=True)
    cd = c.double()
    torch.testing.assert_close(st[0].double(), cd.sum(0), rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(st[1].double(), (cd * cd).sum(0), rtol=1e-5, atol=1e-4)


@gpu
@pytest.mark.parametrize("M,N,K", [(64, 64, 64), (1000, 64, 128), (4096, 128, 128), (200704, 256, 64),
                                   (12544, 512, 2048), (5000, 192, 320)])
def test_gemm_tn_fp32_vs_fp64(M, N, K):
    torch.manual_seed(M % 97 + N + K)
    y, x = torch.randn(M, N, device="cuda"), torch.randn(M, K, device="cuda")
    ref = y.double().cpu().t() @ x.double().cpu()
    out = C.gemm_tn(y, x)
    lib = y.t() @ x
    e, el = _rel(out, ref), _rel(lib, ref)
    assert e <= 2.0 * el + 1e-9, (e, el)
    base = torch.randn(N, K, device="cuda")
    out2 = C.gemm_tn(y, x, out=base.clone(), beta=1.0)
    assert _rel(out2, ref + base.double().cpu()) < 4 * el + 1e-7


@gpu
def test_cast_transpose_fp32_taps():
    w = _cl(torch.randn(128, 64, 3, 3, device="cuda"))
    wb, wt = C.conv_weights(w, dgrad=True, dtype=torch.float32)
    ref = w.permute(0, 2, 3, 1)  # [Co][R][S][C]
    assert wb.data_ptr() == w.data_ptr() and torch.equal(wb, ref)
    assert wt.dtype == torch.float32
    assert torch.equal(wt, ref.flip(1, 2).permute(3, 1, 2, 0).contiguous())
    wb2, wt2 = C.cast_transpose(torch.randn(192, 320, device="cuda"), torch.float32)
    assert torch.equal(wt2, wb2.t().contiguous())


def _conv_case(n, ci, co, hw, k, stride, mod_cls):
    torch.manual_seed(n * ci + co + k + stride)
    pad = k // 2
    if mod_cls is C.Conv1x1:
        mod = C.Conv1x1(ci, co)
    else:
        mod = C.ConvNHWC(ci, co, k, stride=stride, padding=pad)
    mod = mod.cuda().to(memory_format=torch.channels_last)
    x = _cl(torch.randn(n, ci, hw, hw, device="cuda"))
    x1 = x.clone().requires_grad_(True)
    y1 = mod(x1)
    assert y1.dtype == torch.float32
    g = torch.randn_like(y1)
    y1.backward(g)
    ours = (y1.detach(), x1.grad, mod.weight.grad)
    # PyTorch fp32 (MIOpen) and fp64 (CPU) references
    w = mod.weight.detach()

    def run(dev, dt):
        xx = x.detach().to(dev, dt).clone().requires_grad_(True)
        ww = w.to(dev, dt).clone().requires_grad_(True)
        yy = F.conv2d(xx, ww, stride=mod.stride, padding=mod.padding)
        yy.backward(g.to(dev, dt))
        return yy.detach(), xx.grad, ww.grad

    lib = run("cuda", torch.float32)
    ref = run("cpu", torch.float64)
    return ours, lib, ref


@gpu
@pytest.mark.parametrize("n,ci,co,hw,k,stride", [(2, 64, 64, 28, 3, 1), (2, 128, 128, 28, 3, 2),
                                                 (2, 256, 256, 14, 3, 1), (2, 64, 128, 9, 3, 2),
                                                 (2, 128, 64, 13, 5, 1), (2, 256, 512, 14, 1, 2),
                                                 (2, 64, 64, 12, 3, 3)])
def test_conv_fp32_within_2x_of_pytorch_fp32(n, ci, co, hw, k, stride):
    """fwd, dgrad (stride 1 and the strided parity classes), wgrad on v_mfma_f32_32x32x2_f32."""
    ours, lib, ref = _conv_case(n, ci, co, hw, k, stride, C.ConvNHWC)
    for name, a, b, r in zip(("y", "dx", "dw"), ours, lib, ref):
        e, el = _rel(a, r), _rel(b, r)
        assert e <= 2.0 * el + 1e-9, (name, e, el)


@gpu
@pytest.mark.parametrize("n,ci,co,hw", [(4, 64, 256, 14), (2, 256, 64, 9), (3, 128, 128, 7)])
def test_conv1x1_fp32_within_2x_of_pytorch_fp32(n, ci, co, hw):
    ours, lib, ref = _conv_case(n, ci, co, hw, 1, 1, C.Conv1x1)
    for name, a, b, r in zip(("y", "dx", "dw"), ours, lib, ref):
        e, el = _rel(a, r), _rel(b, r)
        assert e <= 2.0 * el + 1e-9, (name, e, el)


@gpu
def test_stem_fp32():
    torch.manual_seed(5)
    mod = C.StemConv(3, 64, 7, 2, 3).cuda().to(memory_format=torch.channels_last)
    x = _cl(torch.randn(2, 3, 64, 64, device="cuda"))
    assert mod.fused(x)
    y = mod(x)
    assert y.dtype == torch.float32
    g = torch.randn_like(y)
    y.backward(g)
    w = mod.weight.detach()
    xx = x.double().cpu()
    ww = w.double().cpu().requires_grad_(True)
    yr = F.conv2d(xx, ww, stride=2, padding=3)
    yr.backward(g.double().cpu())
    xl = x.clone()
    wl = w.clone().requires_grad_(True)
    yl = F.conv2d(xl, wl, stride=2, padding=3)
    yl.backward(g)
    assert _rel(y, yr) <= 2 * _rel(yl, yr) + 1e-9
    assert _rel(mod.weight.grad, ww.grad) <= 2 * _rel(wl.grad, ww.grad) + 1e-9


@gpu
def test_maxpool_fp32_exact():
    from mpit_amd.ops.pool import MaxPool2dNHWC

    torch.manual_seed(2)
    x = _cl(torch.randn(2, 64, 17, 17, device="cuda")).requires_grad_(True)
    p = MaxPool2dNHWC(3, stride=2, padding=1)
    assert p.fused(x)
    y = p(x)
    x2 = x.detach().clone().requires_grad_(True)
    y2 = F.max_pool2d(x2, 3, 2, 1)
    assert torch.equal(y, y2)
    g = torch.randn_like(y)
    y.backward(g)
    y2.backward(g)
    torch.testing.assert_close(x.grad, x2.grad, rtol=1e-6, atol=1e-6)


def _ref_block(blk, x):
    """The bottleneck's math on plain PyTorch ops in x's dtype."""
    def bn(mod, t):
        return F.batch_norm(t, None, None, mod.weight.to(t.dtype), mod.bias.to(t.dtype), training=True, eps=mod.eps)

    def conv(mod, t):
        return F.conv2d(t, mod.weight.to(t.dtype), stride=mod.stride, padding=mod.padding)

    out = F.relu(bn(blk.bn1, conv(blk.conv1, x)))
    out = F.relu(bn(blk.bn2, conv(blk.conv2, out)))
    out = bn(blk.bn3, conv(blk.conv3, out))
    idt = x if blk.downsample is None else bn(blk.downsample[1], conv(blk.downsample[0], x))
    return F.relu(out + idt)


def planes_input(x):
    """x (fp32, channels_last) as an fp16-planes tensor (ops/conv.py set_planes), and the
    values those planes carry (exact decode)."""
    b = C.bound_of_value(torch.linalg.vector_norm(x, float("inf")))
    n, c, h, w = x.shape
    p = C.f16_planes(x.permute(0, 2, 3, 1).reshape(-1).contiguous(), b)
    xp = p.reshape(-1).view(torch.float32).view(n, h, w, c).permute(0, 3, 1, 2)
    C.set_planes(xp, b)
    return xp, C.unplanes(xp).contiguous(memory_format=torch.channels_last)


@gpu
@pytest.mark.parametrize("plan,pl", [(False, False), (True, False), (True, True)])
@pytest.mark.parametrize("inp,planes,stride", [(256, 64, 1), (256, 128, 2)])
def test_bottleneck_fp32_vs_fp64(inp, planes, stride, plan, pl):
    """A whole fused bottleneck block in fp32 (GEMM-epilogue BN statistics and backward
    reductions, parked shortcut gradients, bn_pair) against fp64 on the CPU: within 2x of
    the same block on PyTorch's fp32 ops. With the weight plan (the trainer's setting) every
    GEMM runs the fp16x3 split products on the bounds the BN passes wrote. ``pl``: as inside
    ResNet-50's fp32 step — the block input, its BN outputs and their input gradients as fp16
    planes (gemm.hip FM 13; the residual add decodes its planes), the reference on the values
    the input planes carry."""
    from mpit_amd.models.resnet import Bottleneck, conv1x1
    from mpit_amd.ops.bn import BatchNormAct2d

    torch.manual_seed(inp + planes + stride)
    down = None
    if stride != 1 or inp != planes * 4:
        down = torch.nn.Sequential(conv1x1(inp, planes * 4, stride), BatchNormAct2d(planes * 4, act=False))
    blk = Bottleneck(inp, planes, stride, down).cuda().to(memory_format=torch.channels_last)
    for m in blk.modules():
        if isinstance(m, BatchNormAct2d):
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.2, 0.2)
            # (the block output stays fp32: the test reads it; its gradient comes from the test)
            m.out_planes = m.grad_planes = pl and m is not blk.bn3
    blk.bn3.grad_planes = pl
    x = _cl(torch.randn(4, inp, 14, 14, device="cuda"))
    if pl:
        xp, x = planes_input(x)
        x1 = xp.detach().requires_grad_(True)
        C.set_planes(x1, C.planes_of(xp))
    else:
        x1 = x.clone().requires_grad_(True)
    wp = C.WeightCastPlan(blk, torch.float32) if plan else None
    n16 = C.COUNTERS["wgrad_f16x3"] + C.COUNTERS["wgrad_planes"]
    npl, nmix = C.COUNTERS["wgrad_planes"], C.COUNTERS["wgrad_mixed"]
    if wp is not None:
        wp.run()
    y1 = blk(x1)
    assert y1.dtype == torch.float32
    g = torch.randn(y1.shape, device="cuda")
    y1.backward(g)
    if wp is not None:
        wp.invalidate()
        if C._F32_SPLIT == "f16x3":
            # bounds reached the backward-weight GEMMs
            assert C.COUNTERS["wgrad_f16x3"] + C.COUNTERS["wgrad_planes"] > n16
    if pl and C._F32_PLANES:
        # conv1, conv2 (and the shortcut conv) take both operands as planes; conv3's gradient
        # comes from the test's fp32 g through bn3 (not linked): decoded, counted
        assert C.COUNTERS["wgrad_planes"] - npl >= 2, C.COUNTERS
    ours = {n: p.grad.detach().clone() for n, p in blk.named_parameters()}
    ours.update(y=y1.detach(), dx=x1.grad)
    blk.zero_grad(set_to_none=True)
    x3 = x.clone().requires_grad_(True)
    y3 = _ref_block(blk, x3)
    y3.backward(g)
    lib = {n: p.grad.detach().clone() for n, p in blk.named_parameters()}
    lib.update(y=y3.detach(), dx=x3.grad)
    blk.zero_grad(set_to_none=True)
    bd = blk.double().cpu()
    x2 = x.double().cpu().requires_grad_(True)
    y2 = _ref_block(bd, x2)
    y2.backward(g.double().cpu())
    ref = {n: p.grad.detach().clone() for n, p in bd.named_parameters()}
    ref.update(y=y2.detach(), dx=x2.grad)
    for k in ref:
        e, el = _rel(ours[k], ref[k]), _rel(lib[k], ref[k])
        assert e <= 2.0 * el + 1e-7, (k, e, el)


@gpu
def test_weight_cast_plan_fp32():
    """The fp32 plan writes exactly the per-call fp32 transposes and forwards read the master."""
    from mpit_amd.models.resnet import Bottleneck, conv1x1
    from mpit_amd.ops.bn import BatchNormAct2d

    torch.manual_seed(3)
    down = torch.nn.Sequential(conv1x1(256, 512, 2), BatchNormAct2d(512, act=False))
    net = torch.nn.Sequential(Bottleneck(256, 128, 2, down), Bottleneck(512, 128)).cuda().to(
        memory_format=torch.channels_last)
    old = C._F32_BSPLIT
    C._F32_BSPLIT = False  # the round-2 fp32 plan: forwards read the master, fp32 transposes
    try:
        plan = C.WeightCastPlan(net, torch.float32)
    finally:
        C._F32_BSPLIT = old
    plan.run()
    for mod, _, (wb, wt) in plan.mods:
        w = mod.weight
        assert wb.data_ptr() == w.data_ptr()
        if isinstance(mod, C.Conv1x1):
            _, rt = C.cast_transpose(w, torch.float32)
        elif mod.stride[0] > 1 and C.strided_dgrad_supported(w.shape[1], w.shape[0], mod.stride[0]):
            _, rt = C.strided_dgrad_weights(w, mod.stride[0], mod.padding[0], torch.float32)
        elif mod.stride[0] > 1:
            rt = None
        else:
            _, rt = C.conv_weights(w, True, torch.float32)
        assert (wt is None) == (rt is None)
        if wt is not None:
            assert torch.equal(wt.reshape(-1), rt.reshape(-1))
    x = _cl(torch.randn(2, 256, 14, 14, device="cuda"))
    y1 = net(x)
    plan.invalidate()
    y2 = net(x)
    assert torch.equal(y1, y2)


@gpu
def test_resnet50_fp32_step_runs_native():
    """One fp32 ResNet-50 forward/backward: every convolution on the MFMA kernels (no MIOpen
    conv), finite loss and gradients."""
    from mpit_amd.models.resnet import resnet50

    torch.manual_seed(0)
    net = resnet50(num_classes=10).cuda().to(memory_format=torch.channels_last)
    convs = [m for m in net.modules() if isinstance(m, torch.nn.Conv2d)]
    x = _cl(torch.randn(4, 3, 64, 64, device="cuda"))
    assert net.conv1.fused(x)
    plan = C.WeightCastPlan(net, torch.float32)  # the trainer's per-step weight planes
    plan.run()
    out = net(x)
    assert out.dtype == torch.float32
    n0 = dict(C.COUNTERS)
    loss = F.cross_entropy(out, torch.randint(0, 10, (4,), device="cuda"))
    loss.backward()
    assert torch.isfinite(loss)
    for m in convs:
        assert m.weight.grad is not None and torch.isfinite(m.weight.grad).all()
    plan.invalidate()
    if C._F32_PLANES:  # activations / gradients as fp16 planes wherever only GEMMs read them
        assert C.COUNTERS["wgrad_planes"] - n0["wgrad_planes"] >= 45, C.COUNTERS
        assert C.COUNTERS["wgrad_mixed"] == n0["wgrad_mixed"], C.COUNTERS
        assert C.COUNTERS["unplanes"] == n0["unplanes"], C.COUNTERS


@pytest.mark.gpu
def test_fp32_training_tracks_fp64_like_stock_pytorch():
    """ResNet-50 on the fp32 mpit kernels: forward loss and first-step gradients as close to
    an fp64 CPU reference as the same network in stock PyTorch fp32 (benchmarks/loss_parity.py)."""
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "benchmarks"))
    import loss_parity

    r = loss_parity.run(batch=8, size=64, steps=2, lr=0.02, classes=10)
    print(r["step0_grad_rel_err"], r["step0_grad_worst_tensor_rel_err"], r["loss_fp64_cpu"], r["loss_mpit_fp32"])
    assert all(l == l for l in r["loss_mpit_fp32"]), r["loss_mpit_fp32"]
    # the forward loss at the shared starting point and the first gradients are the
    # precision measures (later steps amplify any fp32 rounding chaotically)
    assert abs(r["loss_mpit_fp32"][0] - r["loss_fp64_cpu"][0]) <= 1e-5 * abs(r["loss_fp64_cpu"][0])
    ours, stock = r["step0_grad_rel_err"]["mpit_fp32"], r["step0_grad_rel_err"]["stock_fp32"]
    assert ours <= 4 * stock + 1e-6, (ours, stock)


def _bottleneck_net(seed=5):
    from mpit_amd.models.resnet import Bottleneck, conv1x1
    from mpit_amd.ops.bn import BatchNormAct2d

    torch.manual_seed(seed)
    down = torch.nn.Sequential(conv1x1(256, 512, 2), BatchNormAct2d(512, act=False))
    return torch.nn.Sequential(Bottleneck(256, 128, 2, down), Bottleneck(512, 128)).cuda().to(
        memory_format=torch.channels_last)


@gpu
def test_weight_cast_plan_fp32_planes_exact():
    """The pre-split plan (default): every weight operand as three bf16 planes whose sum is
    the fp32 master (forward) / its fp32 transpose (backward-data), exactly."""
    net = _bottleneck_net()
    assert C._F32_BSPLIT
    plan = C.WeightCastPlan(net, torch.float32)
    plan.run()
    torch.cuda.synchronize()

    def same(got, want):  # bf16x6 planes: exact; fp16x3 planes: 22 bits (f16_planes' arithmetic)
        if got.dtype == torch.float16:
            assert torch.equal(got, C.f16_planes(want, got._mpit_wamax).view(got.shape))
            return torch.allclose(C._unsplit(got), want.view(got.shape[1:]), rtol=2.0 ** -22,
                                  atol=C.bound_value(got._mpit_wamax).item() * 2.0 ** -47)
        return torch.equal(C._unsplit(got).reshape(-1), want.reshape(-1))

    for mod, _, (wb, wt) in plan.mods:
        w = mod.weight.detach()
        if wb.dtype in (torch.bfloat16, torch.float16):
            assert wb.shape[0] == (2 if wb.dtype == torch.float16 else 3) and w.shape[0] % C._F32_PLANES_N == 0
            assert same(wb, C._as_rsc(w).contiguous())
        else:
            assert wb.data_ptr() == w.data_ptr()
        if isinstance(mod, C.Conv1x1):
            _, rt = C.cast_transpose(w, torch.float32)
        elif mod.stride[0] > 1 and C.strided_dgrad_supported(w.shape[1], w.shape[0], mod.stride[0]):
            _, rt = C.strided_dgrad_weights(w, mod.stride[0], mod.padding[0], torch.float32)
        elif mod.stride[0] > 1:
            rt = None
        else:
            _, rt = C.conv_weights(w, True, torch.float32)
        assert (wt is None) == (rt is None)
        if wt is not None and wt.dtype in (torch.bfloat16, torch.float16):
            assert same(wt, rt.contiguous())
        elif wt is not None:
            assert torch.equal(wt.reshape(-1), rt.reshape(-1))
    if plan.wlist:  # the plan's bound covers every plane weight
        assert C.bound_value(plan.amax).item() == max(w.abs().max().item() for w in plan.wlist)


@gpu
def test_presplit_weights_bitwise_equal_register_split():
    """GEMMs reading the pre-split weight planes (FM 4) give bit for bit what the in-register
    split of the fp32 weights gives (FM 3): same planes, same MFMA sequence. Two bottleneck
    blocks forward + backward (1x1, 3x3, strided dgrad classes, downsample)."""
    def run(planes):
        old = C._F32_BSPLIT, C._F32_SPLIT, C._F32_PLANES_N
        C._F32_BSPLIT, C._F32_SPLIT, C._F32_PLANES_N = planes, "bf16x6", 128  # the bf16x6 kernels
        try:
            net = _bottleneck_net()
            plan = C.WeightCastPlan(net, torch.float32)
        finally:
            C._F32_BSPLIT = old[0]
        torch.manual_seed(11)
        x = _cl(torch.randn(4, 256, 14, 14, device="cuda")).requires_grad_(True)
        try:
            plan.run()
            y = net(x)
            y.backward(torch.randn_like(y))
            plan.invalidate()
            torch.cuda.synchronize()
        finally:
            C._F32_SPLIT, C._F32_PLANES_N = old[1], old[2]
        return [y.detach(), x.grad] + [p.grad for p in net.parameters()]

    a, b = run(True), run(False)
    for u, v in zip(a, b):
        assert torch.equal(u.view(torch.int32), v.view(torch.int32))


@gpu
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_convact_weight_plan_bitwise(dt):
    """VGG / AlexNet conv(+bias)+ReLU layers take their per-step weight operands from the
    model's WeightCastPlan (bf16 casts, or fp32 pre-split planes): bit for bit the result of
    casting / splitting per call."""
    torch.manual_seed(2)
    net = torch.nn.Sequential(C.ConvAct2d(64, 128, 3, padding=1), C.ConvAct2d(128, 128, 3, padding=1),
                              C.ConvAct2d(128, 256, 3, stride=2, padding=1)).cuda().to(
        memory_format=torch.channels_last)
    x0 = _cl(torch.randn(4, 64, 20, 20, device="cuda"))

    def run(plan):
        net.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        if plan is not None:
            plan.run()
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=dt == torch.bfloat16):
            y = net(x)
        y.float().sum().backward()
        if plan is not None:
            plan.invalidate()
        torch.cuda.synchronize()
        return [y.detach().float(), x.grad] + [p.grad.clone() for p in net.parameters()]

    old = C._F32_SPLIT, C._F32_PLANES_N
    try:
        # bitwise: the bf16x6 planes split like the per-call path; fp16x3: within fp32 rounding
        for mode in ("bf16x6", "f16x3") if dt == torch.float32 else ("bf16x6",):
            C._F32_SPLIT, C._F32_PLANES_N = mode, 128 if mode == "bf16x6" else 64
            plan = C.WeightCastPlan(net, dt)
            assert plan.njobs == 3
            a, b = run(plan), run(None)
            for u, v in zip(a, b):
                if mode == "bf16x6":
                    assert torch.equal(u, v)
                else:
                    assert _rel(u, v) < 1e-5, _rel(u, v)
    finally:
        C._F32_SPLIT, C._F32_PLANES_N = old


_WGRAD_CHILD = r"""
import sys, torch
sys.path.insert(0, sys.argv[2])
from mpit_amd.ops import conv as C
torch.manual_seed(5)
outs = []
for M, N, K in [(5000, 256, 128), (12544, 512, 1024), (333, 128, 128)]:
    y, x = torch.randn(M, N, device="cuda"), torch.randn(M, K, device="cuda")
    outs.append(C.gemm_tn(y, x))
    outs.append(C.gemm_tn(y, x, out=torch.ones(N, K, device="cuda"), beta=1.0))
for n, ci, co, hw, k, s in [(4, 128, 128, 14, 3, 1), (2, 128, 256, 15, 3, 2), (4, 256, 128, 14, 1, 1)]:
    mod = C.ConvNHWC(ci, co, k, stride=s, padding=k // 2).cuda().to(memory_format=torch.channels_last)
    xx = torch.randn(n, ci, hw, hw, device="cuda").contiguous(memory_format=torch.channels_last)
    mod(xx).backward(torch.randn_like(mod(xx)))
    outs.append(mod.weight.grad)
torch.cuda.synchronize()
torch.save([o.cpu() for o in outs], sys.argv[1])
"""


@gpu
def test_wgrad_split_once_bitwise_equal_per_tile_split(tmp_path):
    """The split-once fp32 wgrad kernel (gemm_tn_f32s_kernel: each staged element split into
    bf16 h/m/l once, planes kept in LDS) gives bit for bit gemm_tn_kernel's bf16x6 result
    (MPIT_TN_F32S=0): same planes, same MFMA order. The knob is read once per process, so
    each side runs in its own process."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = []
    for knob in ("1", "0"):
        f = str(tmp_path / f"w{knob}.pt")
        subprocess.run([sys.executable, "-c", _WGRAD_CHILD, f, root], check=True, timeout=300,
                       env=dict(os.environ, MPIT_TN_F32S=knob))
        res.append(torch.load(f, weights_only=True))
    for i, (u, v) in enumerate(zip(*res)):
        assert torch.equal(u.view(torch.int32), v.view(torch.int32)), (i, _rel(u, v))


# ---- fp16x3 on hostile operands (verdict r03 #8): heavy tails and a 2^20 outlier row, judged
# per output row against fp64 (a Frobenius norm over the whole output hides per-row loss)

def _row_rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return (a - b).norm(dim=1) / (b.norm(dim=1) + 1e-300)


def _hostile(dist, shape, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    if dist == "student_t2":  # nu = 2: infinite variance, |x| up to ~1e3 x the median
        z = torch.randn(shape, generator=g)
        chi2 = torch.randn(shape, generator=g) ** 2 + torch.randn(shape, generator=g) ** 2
        t = z / torch.sqrt(chi2 / 2)
    else:  # gaussian with one row 2^20 above the rest
        t = torch.randn(shape, generator=g)
        t[shape[0] // 3] *= 2.0 ** 20
    return (t * scale).cuda()


# Per-row acceptance. The split GEMMs carry 22 (fp16x3) / 24 (bf16x6) significant bits per
# operand and accumulate the split products on the MFMA; PyTorch's fp32 runs FMA chains. On a row
# whose result one product dominates (heavy tails) PyTorch's row error is ~2^-24 while both splits
# measure ~2^-21 — a dot-product error bounded by the magnitudes of the terms, not of the result
# (|err| <= c * sum_k |a_k b_k|). So every row must be within 2x of PyTorch's row error plus
# 2^-19 * kappa_row, kappa_row = || |A||B|^T row || / || AB^T row || (the row's condition: 1 without
# cancellation, large where an outlier column cancels), AND the worst row within 2x of PyTorch's
# worst row. Measured ratios: profiles/fp16x3_hostile_rows_r04.md.
_ROW_FLOOR = 2.0 ** -19


def _row_cond(a_abs_prod, ref):
    return a_abs_prod.double().norm(dim=1) / (ref.double().norm(dim=1) + 1e-300)


def _check_rows(tag, ours, theirs, mode, cond):
    worst = int(torch.argmax(ours / (theirs + 2.0 ** -24)))
    print(f"{tag} [{mode}]: max row err ours {ours.max():.3e} lib {theirs.max():.3e}; worst ratio row {worst}: "
          f"{ours[worst]:.3e} vs {theirs[worst]:.3e} ({ours[worst] / theirs[worst]:.2f}x, kappa {cond[worst]:.3g})")
    assert (ours <= 2.0 * theirs + _ROW_FLOOR * cond).all(), (worst, ours[worst].item(), theirs[worst].item())
    assert ours.max() <= 2.0 * theirs.max() + 2.0 ** -24, (ours.max().item(), theirs.max().item())


@gpu
@pytest.mark.parametrize("mode", ["f16x3", "bf16x6"])
@pytest.mark.parametrize("dist", ["student_t2", "outlier_row"])
@pytest.mark.parametrize("M,N,K", [(1000, 192, 128), (4096, 256, 512), (12544, 512, 2048)])
def test_gemm_nt_hostile_rows(dist, M, N, K, mode):
    a = _hostile(dist, (M, K), M + K)
    b = _hostile("student_t2", (N, K), N + K, 0.05)
    ref = a.double().cpu() @ b.double().cpu().t()
    c = C.gemm_nt(a, b, f16x3=mode == "f16x3")
    assert torch.isfinite(c).all()
    cond = _row_cond(a.abs().double().cpu() @ b.abs().double().cpu().t(), ref)
    _check_rows(f"nt {dist} {M}x{N}x{K}", _row_rel(c, ref), _row_rel(a @ b.t(), ref), mode, cond)


@gpu
@pytest.mark.parametrize("mode", ["f16x3", "bf16x6"])
@pytest.mark.parametrize("dist", ["student_t2", "outlier_row"])
@pytest.mark.parametrize("M,N,K", [(5000, 192, 320), (12544, 512, 256)])
def test_gemm_tn_hostile_rows(dist, M, N, K, mode):
    """The backward-weight shape: dW[N, K] = dY^T X with heavy-tailed gradients and an outlier
    activation column (a 2^20 row of X^T)."""
    y = _hostile("student_t2", (M, N), M + N, 1e-6)
    x = _hostile(dist, (K, M), K + M).t().contiguous()
    ref = y.double().cpu().t() @ x.double().cpu()
    out = C.gemm_tn(y, x, f16x3=mode == "f16x3")
    assert torch.isfinite(out).all()
    cond = _row_cond(y.abs().double().cpu().t() @ x.abs().double().cpu(), ref)
    _check_rows(f"tn {dist} {M}x{N}x{K}", _row_rel(out, ref), _row_rel(y.t() @ x, ref), mode, cond)


def _loose_planes(t, factor):
    """fp16 planes of ``t`` (its memory order) scaled by a bound ``factor`` x max |t| — a producer
    bound that overshoots (the BN apply passes bound their output from coefficient and input
    maxima, never below the true maximum, up to a few times above it)."""
    bnd = C.bound_of_value(torch.linalg.vector_norm(t.float(), float("inf")) * factor)
    return C.f16_planes(t.reshape(-1).contiguous(), bnd), bnd


@gpu
@pytest.mark.parametrize("factor", [1.0, 4.0, 16.0])
@pytest.mark.parametrize("dist", ["student_t2", "outlier_row"])
@pytest.mark.parametrize("M,N,K", [(4096, 256, 512), (12544, 512, 2048)])
def test_gemm_nt_hostile_rows_planes(dist, M, N, K, factor):
    """FM 13: the activation operand arrives as fp16 planes whose bound overshoots max |A| by
    ``factor`` (the precision floor moves up by log2(factor) bits: 22 bits down to 2^-27 of the
    bound) — same per-row acceptance as the in-kernel split."""
    from mpit_amd._ext import native

    a = _hostile(dist, (M, K), M + K)
    b = _hostile("student_t2", (N, K), N + K, 0.05)
    ref = a.double().cpu() @ b.double().cpu().t()
    ap, abnd = _loose_planes(a, factor)
    bp = C.f16_planes(b.contiguous(), C.bound_of_value(torch.linalg.vector_norm(b, float("inf"))))
    c = torch.empty(M, N, device="cuda")
    native().gemm_nt(0, torch.cuda.current_stream().cuda_stream, M, N, K, ap.data_ptr(), K, bp.data_ptr(), K,
                     c.data_ptr(), N, 0, f32=True, bps=bp[0].numel(), amax_a=abnd.data_ptr(),
                     amax_b=bp._mpit_wamax.data_ptr(), aps=ap[0].numel())
    torch.cuda.synchronize()
    assert torch.isfinite(c).all()
    cond = _row_cond(a.abs().double().cpu() @ b.abs().double().cpu().t(), ref)
    _check_rows(f"nt planes x{factor} {dist} {M}x{N}x{K}", _row_rel(c, ref), _row_rel(a @ b.t(), ref), "planes",
                cond)


@gpu
@pytest.mark.parametrize("factor", [1.0, 4.0, 16.0])
@pytest.mark.parametrize("dist", ["student_t2", "outlier_row"])
@pytest.mark.parametrize("M,N,K", [(5000, 192, 320), (12544, 512, 256)])
def test_gemm_tn_hostile_rows_planes(dist, M, N, K, factor):
    """FM 13 backward-weight: dY and X both as fp16 planes with overshooting bounds."""
    from mpit_amd._ext import native

    y = _hostile("student_t2", (M, N), M + N, 1e-6)
    x = _hostile(dist, (K, M), K + M).t().contiguous()
    ref = y.double().cpu().t() @ x.double().cpu()
    yp, yb = _loose_planes(y, factor)
    xp, xb = _loose_planes(x, factor)
    m = native()
    out = torch.empty(N, K, device="cuda")
    ws = torch.empty(max(1, m.gemm_tn_ws_floats(0, M, N, K)), device="cuda")
    m.gemm_tn(0, torch.cuda.current_stream().cuda_stream, M, N, K, yp.data_ptr(), N, xp.data_ptr(), K,
              out.data_ptr(), ws.data_ptr(), 0.0, f32=True, amax_y=yb.data_ptr(), amax_x=xb.data_ptr(),
              yps=yp[0].numel(), xps=xp[0].numel())
    torch.cuda.synchronize()
    assert torch.isfinite(out).all()
    cond = _row_cond(y.abs().double().cpu().t() @ x.abs().double().cpu(), ref)
    _check_rows(f"tn planes x{factor} {dist} {M}x{N}x{K}", _row_rel(out, ref), _row_rel(y.t() @ x, ref), "planes",
                cond)


@gpu
def test_conv_f16x3_hostile_input_rows():
    """A 3x3 convolution through the fp32 weight plan (fp16x3 planes) on a heavy-tailed input
    with one outlier image: per (image, output channel) row against fp64, vs MIOpen fp32."""
    torch.manual_seed(9)
    mod = C.ConvNHWC(128, 128, 3, stride=1, padding=1).cuda().to(memory_format=torch.channels_last)
    plan = C.WeightCastPlan(mod, torch.float32)
    x = _hostile("student_t2", (4, 128, 14, 14), 77)
    x[1] *= 2.0 ** 20
    x = _cl(x)
    plan.run()
    y = mod(x)
    plan.invalidate()
    w = mod.weight.detach()
    ref = F.conv2d(x.double().cpu(), w.double().cpu(), padding=1)
    lib = F.conv2d(x, w, padding=1)

    def rows(t):  # one row per (image, output channel)
        return t.reshape(t.shape[0] * t.shape[1], -1)

    absref = F.conv2d(x.double().cpu().abs(), w.double().cpu().abs(), padding=1)
    _check_rows("conv 3x3 hostile", _row_rel(rows(y), rows(ref)), _row_rel(rows(lib), rows(ref)),
                "f16x3" if C._F32_SPLIT == "f16x3" else "bf16x6", _row_cond(rows(absref), rows(ref)))

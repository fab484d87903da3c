"""ResNet bottleneck blocks on the fused GPU path (MFMA 1x1 convs, fused BN+add+ReLU with
mask bits, shortcut gradient added inside conv1's backward-data GEMM) against the same
block computed with plain fp32 PyTorch ops."""
import pytest
import torch
import torch.nn.functional as F

from mpit_amd.models.resnet import Bottleneck, conv1x1
from mpit_amd.ops.bn import BatchNormAct2d


def _ref_block(blk, x):
    def bn(mod, t):
        return F.batch_norm(t, None, None, mod.weight.float(), mod.bias.float(), training=True, eps=mod.eps)

    def conv(mod, t):
        return F.conv2d(t, mod.weight.float(), stride=mod.stride, padding=mod.padding)

    out = F.relu(bn(blk.bn1, conv(blk.conv1, x)))
    out = F.relu(bn(blk.bn2, conv(blk.conv2, out)))
    out = bn(blk.bn3, conv(blk.conv3, out))
    if blk.downsample is not None:
        idt = bn(blk.downsample[1], conv(blk.downsample[0], x))
    else:
        idt = x
    return F.relu(out + idt)


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def test_block_cpu_matches_reference():
    torch.manual_seed(0)
    blk = Bottleneck(64, 16)
    x = torch.randn(2, 64, 6, 6, requires_grad=True)
    y = blk(x)
    x2 = x.detach().clone().requires_grad_(True)
    y2 = _ref_block(blk, x2)
    assert torch.allclose(y, y2, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("inp,planes,stride", [(256, 64, 1), (64, 64, 1), (256, 128, 2)])
def test_bottleneck_fused_matches_fp32(inp, planes, stride):
    torch.manual_seed(inp + planes + stride)
    down = None
    if stride != 1 or inp != planes * 4:
        down = torch.nn.Sequential(conv1x1(inp, planes * 4, stride), BatchNormAct2d(planes * 4, act=False))
    blk = Bottleneck(inp, planes, stride, down).cuda().to(memory_format=torch.channels_last)
    for m in blk.modules():
        if isinstance(m, BatchNormAct2d):
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.2, 0.2)
    x = torch.randn(4, inp, 14, 14, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x1 = x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y1 = blk(x1)
    g = torch.randn(y1.shape, device="cuda")
    y1.backward(g.to(y1.dtype))
    grads1 = {n: p.grad.detach().clone() for n, p in blk.named_parameters()}
    blk.zero_grad(set_to_none=True)

    # the same block through the plain library path in bf16 autocast: the bf16 error floor
    x3 = x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y3 = _ref_block(blk, x3)
    y3.backward(g.to(y3.dtype))
    grads3 = {n: p.grad.detach().clone() for n, p in blk.named_parameters()}
    blk.zero_grad(set_to_none=True)

    x2 = x.float().clone().requires_grad_(True)
    y2 = _ref_block(blk, x2)
    y2.backward(g)
    errs = {"y": (_rel(y1, y2), _rel(y3, y2)), "x.grad": (_rel(x1.grad, x2.grad), _rel(x3.grad, x2.grad))}
    for n, p in blk.named_parameters():
        errs[n] = (_rel(grads1[n], p.grad), _rel(grads3[n], p.grad))
    print(errs)
    for k, (fused, lib) in errs.items():
        assert fused < 1.5 * lib + 1e-2, (k, fused, lib)


@pytest.mark.gpu
@pytest.mark.parametrize("stride", [1, 2])
def test_chained_blocks_fold_bn_passes(stride):
    """Two chained bottlenecks: every BN takes its statistics from the producing conv's
    GEMM epilogue, and every BN whose output feeds a conv gets its backward reduction from
    that conv's backward-data epilogue (bn1 -> 3x3 incl. the strided parity classes, bn2
    -> 1x1, block-1 bn3 -> block-2 conv1 with the parked shortcut gradient). Checked
    against fp32 and the bf16 library floor, and the fused hand-overs must have fired."""
    from mpit_amd.ops import bn as bnmod

    torch.manual_seed(7 + stride)
    inp, planes = 256, 64 * stride
    down = None
    if stride != 1 or inp != planes * 4:
        down = torch.nn.Sequential(conv1x1(inp, planes * 4, stride), BatchNormAct2d(planes * 4, act=False))
    b1 = Bottleneck(inp, planes, stride, down)
    b2 = Bottleneck(planes * 4, planes)
    net = torch.nn.Sequential(b1, b2).cuda().to(memory_format=torch.channels_last)
    for m in net.modules():
        if isinstance(m, BatchNormAct2d):
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.2, 0.2)
    x = torch.randn(4, inp, 14, 14, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    c0 = dict(bnmod.COUNTERS)
    x1 = x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y1 = net(x1)
    g = torch.randn(y1.shape, device="cuda")
    y1.backward(g.to(y1.dtype))
    fired = {k: bnmod.COUNTERS[k] - c0[k] for k in c0}
    nbn = sum(isinstance(m, BatchNormAct2d) for m in net.modules())
    assert fired["fwd_tile_stats"] == nbn, fired
    # bn1, bn2 of both blocks + bn3 of block 1 (block 2's bn3 output is the loss input); with
    # a downsample shortcut block 1's bn3 and shortcut BN are one pair, both linked
    assert fired["bwd_linked"] == (6 if down is not None else 5), fired
    # the finalize runs inside the producing GEMM for single-launch backward-data GEMMs of a
    # single BN (not the strided parity classes, not a bn_pair)
    assert fired["bwd_folded"] == (3 if down is not None else 5), fired
    grads1 = {n: p.grad.detach().clone() for n, p in net.named_parameters()}
    net.zero_grad(set_to_none=True)

    def ref(t):
        return _ref_block(b2, _ref_block(b1, t))

    x3 = x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y3 = ref(x3)
    y3.backward(g.to(y3.dtype))
    grads3 = {n: p.grad.detach().clone() for n, p in net.named_parameters()}
    net.zero_grad(set_to_none=True)
    x2 = x.float().clone().requires_grad_(True)
    y2 = ref(x2)
    y2.backward(g)
    errs = {"y": (_rel(y1, y2), _rel(y3, y2)), "x.grad": (_rel(x1.grad, x2.grad), _rel(x3.grad, x2.grad))}
    for n, p in net.named_parameters():
        errs[n] = (_rel(grads1[n], p.grad), _rel(grads3[n], p.grad))
    print(errs)
    for k, (fused, lib) in errs.items():
        assert fused < 1.5 * lib + 1e-2, (k, fused, lib)


@pytest.mark.gpu
def test_weight_cast_plan_matches_per_call_casts():
    """One batched launch produces exactly the bf16 weights (plain, tap-flipped transposes,
    strided parity classes) the convolutions would cast per call."""
    from mpit_amd.ops import conv as C

    torch.manual_seed(3)
    down = torch.nn.Sequential(conv1x1(256, 512, 2), BatchNormAct2d(512, act=False))
    net = torch.nn.Sequential(Bottleneck(256, 128, 2, down), Bottleneck(512, 128)).cuda().to(
        memory_format=torch.channels_last)
    plan = C.WeightCastPlan(net)
    assert plan.njobs == 7
    plan.run()
    for mod, _, (wb, wt) in plan.mods:
        w = mod.weight
        if isinstance(mod, C.Conv1x1):
            rb, rt = C.cast_transpose(w)
        elif mod.stride[0] > 1 and C.strided_dgrad_supported(w.shape[1], w.shape[0], mod.stride[0]):
            rb, rt = C.strided_dgrad_weights(w, mod.stride[0], mod.padding[0])
        elif mod.stride[0] > 1:
            rb, rt = C.conv_weights(w, dgrad=False)
        else:
            rb, rt = C.conv_weights(w, dgrad=True)
        assert torch.equal(wb.view(-1), rb.reshape(-1))
        assert (wt is None) == (rt is None)
        if wt is not None:
            assert torch.equal(wt.view(-1), rt.reshape(-1))
    # a forward inside the plan's window uses the cast weights and gives the same output
    x = torch.randn(2, 256, 14, 14, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y1 = net(x)
        plan.invalidate()
        y2 = net(x)
    assert torch.equal(y1, y2)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_folded_bn_finalize_matches_separate_launch(dtype):
    """BN backward finalize inside the backward-data GEMM (ops/conv.py _red_args fold) vs the
    separate bn_tiles_finalize launch: same gradients up to summation order, on a tall layer
    (12544 rows: several fold groups) and the downsample / 3x3 / 1x1 mix of two blocks."""
    from mpit_amd.ops import bn as bnmod
    from mpit_amd.ops import conv as convmod

    torch.manual_seed(11)
    b1 = Bottleneck(256, 64)
    b2 = Bottleneck(256, 64)
    net = torch.nn.Sequential(b1, b2).cuda().to(memory_format=torch.channels_last)
    for m in net.modules():
        if isinstance(m, BatchNormAct2d):
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.2, 0.2)
    x = torch.randn(16, 256, 28, 28, device="cuda").contiguous(memory_format=torch.channels_last)
    g = torch.randn(16, 256, 28, 28, device="cuda").contiguous(memory_format=torch.channels_last)

    def run(fold):
        saved = convmod._BN_FOLD
        convmod._BN_FOLD = fold
        try:
            c0 = bnmod.COUNTERS["bwd_folded"]
            xi = x.clone().to(dtype).requires_grad_(True)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=dtype == torch.bfloat16):
                y = net(xi)
            y.backward(g.to(y.dtype))
            torch.cuda.synchronize()
            grads = {n: p.grad.detach().float().clone() for n, p in net.named_parameters()}
            grads["x"] = xi.grad.detach().float().clone()
            net.zero_grad(set_to_none=True)
            return grads, bnmod.COUNTERS["bwd_folded"] - c0
        finally:
            convmod._BN_FOLD = saved

    g_sep, n_sep = run(False)
    g_fold, n_fold = run(True)
    assert n_sep == 0 and n_fold == 5, (n_sep, n_fold)
    tol = 2e-5 if dtype == torch.float32 else 2e-2
    for n in g_sep:
        assert torch.isfinite(g_fold[n]).all(), n
        assert _rel(g_fold[n], g_sep[n]) < tol, (n, _rel(g_fold[n], g_sep[n]))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_folded_bn_forward_finalize_matches_separate_launch(dtype):
    """BN forward finalize inside the producing GEMM (gemm.hip stats_fold, ops/bn.py BNFold)
    vs the separate bn_tiles_finalize launch: same outputs, running statistics and gradients
    up to summation order, on the stem-free two-block mix (1x1, 3x3, strided downsample pair)
    at a height with several fold groups; every BN of the net took the folded path."""
    from mpit_amd.ops import bn as bnmod

    torch.manual_seed(13)
    down = torch.nn.Sequential(conv1x1(256, 512, 2), BatchNormAct2d(512, act=False))
    net = torch.nn.Sequential(Bottleneck(256, 128, 2, down), Bottleneck(512, 128)).cuda()
    net = net.to(memory_format=torch.channels_last)
    for m in net.modules():
        if isinstance(m, BatchNormAct2d):
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.2, 0.2)
    x = torch.randn(16, 256, 56, 56, device="cuda").contiguous(memory_format=torch.channels_last)
    g = torch.randn(16, 512, 28, 28, device="cuda").contiguous(memory_format=torch.channels_last)
    nbn = sum(isinstance(m, BatchNormAct2d) for m in net.modules())
    state0 = {k: v.clone() for k, v in net.state_dict().items()}

    def run(fold):
        saved = bnmod._FWD_FOLD
        bnmod._FWD_FOLD = fold
        try:
            net.load_state_dict(state0)
            c0 = bnmod.COUNTERS["fwd_folded"]
            xi = x.clone().to(dtype).requires_grad_(True)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=dtype == torch.bfloat16):
                y = net(xi)
            y.backward(g.to(y.dtype))
            torch.cuda.synchronize()
            out = {n: p.grad.detach().float().clone() for n, p in net.named_parameters()}
            out.update({"y": y.detach().float().clone(), "x": xi.grad.detach().float().clone()})
            out.update({k: v.float().clone() for k, v in net.state_dict().items() if "running" in k})
            net.zero_grad(set_to_none=True)
            return out, bnmod.COUNTERS["fwd_folded"] - c0
        finally:
            bnmod._FWD_FOLD = saved

    r_sep, n_sep = run(False)
    r_fold, n_fold = run(True)
    assert n_sep == 0 and n_fold == nbn, (n_sep, n_fold, nbn)
    # fp32: the two summation orders agree to a few ulps everywhere. bf16: the statistics
    # still agree that closely, but a statistic that moves by an ulp flips bf16 roundings of
    # the activations, and those propagate into the gradients of the later layers
    for k in r_sep:
        assert torch.isfinite(r_fold[k]).all(), k
        tol = 2e-5 if dtype == torch.float32 else (1e-3 if "running" in k else 5e-2)
        assert _rel(r_fold[k], r_sep[k]) < tol, (k, _rel(r_fold[k], r_sep[k]))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_tagged_fold_protocol_is_bitwise_the_ticket_protocol(dtype):
    """The tagged fold protocol (ops/conv.py _FOLD_TAG: fold ticket before the output stores,
    (value, epoch) partials in persistent buffers) against the first one (every block drains
    its own stores, then takes its ticket): the same sums in the same order, so the outputs,
    running statistics and every gradient are bitwise equal, for both folds at once, over
    three steps (the persistent buffers then hold an earlier epoch's pairs)."""
    from mpit_amd.ops import bn as bnmod
    from mpit_amd.ops import conv as convmod

    torch.manual_seed(17)
    down = torch.nn.Sequential(conv1x1(256, 512, 2), BatchNormAct2d(512, act=False))
    net = torch.nn.Sequential(Bottleneck(256, 128, 2, down), Bottleneck(512, 128)).cuda()
    net = net.to(memory_format=torch.channels_last)
    x = torch.randn(16, 256, 56, 56, device="cuda").contiguous(memory_format=torch.channels_last)
    g = torch.randn(16, 512, 28, 28, device="cuda").contiguous(memory_format=torch.channels_last)
    state0 = {k: v.clone() for k, v in net.state_dict().items()}

    def run(tag):
        saved = (bnmod._FWD_FOLD, convmod._BN_FOLD, convmod._FOLD_TAG)
        bnmod._FWD_FOLD, convmod._BN_FOLD, convmod._FOLD_TAG = True, True, tag
        try:
            net.load_state_dict(state0)
            outs = []
            for _ in range(3):
                f0, b0 = bnmod.COUNTERS["fwd_folded"], bnmod.COUNTERS["bwd_folded"]
                xi = x.clone().to(dtype).requires_grad_(True)
                with torch.autocast("cuda", dtype=torch.bfloat16, enabled=dtype == torch.bfloat16):
                    y = net(xi)
                y.backward(g.to(y.dtype))
                torch.cuda.synchronize()
                assert bnmod.COUNTERS["fwd_folded"] > f0 and bnmod.COUNTERS["bwd_folded"] > b0
                out = {n: p.grad.detach().clone() for n, p in net.named_parameters()}
                out.update({"y": y.detach().clone(), "x": xi.grad.detach().clone()})
                out.update({k: v.clone() for k, v in net.state_dict().items() if "running" in k})
                net.zero_grad(set_to_none=True)
                outs.append(out)
            return outs
        finally:
            bnmod._FWD_FOLD, convmod._BN_FOLD, convmod._FOLD_TAG = saved

    first, tagged = run(False), run(True)
    for step, (a, b) in enumerate(zip(first, tagged)):
        for k in a:
            assert torch.equal(a[k], b[k]), (step, k)

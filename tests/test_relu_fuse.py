"""ReLU / bias backward fused into the kernel that produces a conv(+bias)+ReLU layer's output
gradient (ops/conv.py ReluLink): the next conv's backward-data GEMM epilogue (EPI_RELUB) or
the max pool's backward. Gradients against fp32 PyTorch, and fused == unfused."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F


def test_relu_link_take_semantics():
    from mpit_amd.ops.conv import ReluLink

    link = ReluLink(True)
    dz, db = torch.randn(2, 8, 4, 4), torch.randn(8)
    link.give(dz, db)
    ok, got = link.take(dz)
    assert ok and got is db
    assert link.take(dz) == (False, None)  # handed once
    link.give(dz, db)
    assert link.take(dz.clone()) == (False, None)  # another tensor (e.g. autograd's sum): not taken
    link.give(dz, None)
    assert link.take(dz.view(2, 8, 16)) == (False, None)  # same storage, other shape


def _vgg_block(c_in=3):
    from mpit_amd.ops.conv import ConvAct2d
    from mpit_amd.ops.pool import MaxPool2dNHWC

    return nn.Sequential(ConvAct2d(c_in, 64, 3, padding=1), ConvAct2d(64, 64, 3, padding=1), MaxPool2dNHWC(2, 2),
                         ConvAct2d(64, 128, 3, padding=1), ConvAct2d(128, 128, 3, padding=1), MaxPool2dNHWC(2, 2))


def _ref_forward(mods, x):
    y = x
    for m in mods:
        if isinstance(m, nn.Conv2d):
            y = F.relu(F.conv2d(y, m.weight.float(), m.bias.float(), padding=m.padding))
        else:
            y = F.max_pool2d(y, 2, 2)
    return y


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_vgg_block_fused_relu_backward(dt):
    from mpit_amd.ops.conv import ReluLink

    torch.manual_seed(0)
    net = _vgg_block().cuda().to(memory_format=torch.channels_last)
    with torch.no_grad():
        for m in net:
            if isinstance(m, nn.Conv2d):
                m.bias.uniform_(-0.2, 0.2)
    x = torch.randn(4, 3, 32, 32, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
    g = None
    grads = {}
    for fuse in (True, False):
        ReluLink.enabled = fuse
        try:
            net.zero_grad(set_to_none=True)
            h0 = ReluLink.hits
            y = net(x)
            if g is None:
                g = torch.randn_like(y.float()).to(dt).contiguous(memory_format=torch.channels_last)
            y.backward(g)
            torch.cuda.synchronize()
            # 4 conv+ReLU layers: 2 handed over by the pools, 2 by the next conv's dgrad epilogue
            assert ReluLink.hits - h0 == (4 if fuse else 0)
            grads[fuse] = [p.grad.detach().clone() for p in net.parameters()]
        finally:
            ReluLink.enabled = True
    # the fp32 reference on the same (rounded) weights and input
    ref = _vgg_block().cuda()
    ref.load_state_dict({k: v.to(dt).float() for k, v in net.state_dict().items()})
    xr = x.float().requires_grad_(False)
    yr = _ref_forward(list(ref), xr)
    yr.backward(g.float())
    # bf16: the 4-layer chain against an fp32 forward differs by 5-17 % of max (r05h): bf16
    # rounding makes near-ties in the 2x2 pools pick other argmax pixels and flips ReLU masks
    # near 0, so the gradient lands on other pixels. Each layer alone is held to the fp32
    # reference in test_conv_act / test_stem; the claim here is fused == unfused, and a sanity
    # bound against fp32.
    tol = 0.25 if dt == torch.bfloat16 else 2e-3
    report, bad = [], []
    for (name, p), a, b in zip(ref.named_parameters(), grads[True], grads[False]):
        r = p.grad
        scale = r.abs().max().item() + 1e-6
        ea, eb, eab = ((a - r).abs().max().item() / scale, (b - r).abs().max().item() / scale,
                       (a - b).abs().max().item() / scale)
        report.append(f"{name}: fused {ea:.2e} unfused {eb:.2e} fused-unfused {eab:.2e}")
        # fused vs unfused: the same math on the same kernels (the bias sums differ in order only)
        if ea > tol or eab > (1e-2 if dt == torch.bfloat16 else 1e-4):
            bad.append(name)
    assert not bad, "; ".join(report)

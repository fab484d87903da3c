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


def _ref_forward(mods, x, masks, idxs):
    """fp32 forward on the SAME routing as the run under test: each ReLU is the run's own
    mask (y > 0 of its output) and each 2x2 max pool takes the run's own argmax pixels, so
    the backward sends every gradient to the same pixels and a bf16 near-tie or a ReLU flip
    near 0 cannot move it (the pools' first-max rule is PyTorch's: pool.hip, strict >)."""
    y = x
    for i, m in enumerate(mods):
        if isinstance(m, nn.Conv2d):
            y = F.conv2d(y, m.weight.float(), m.bias.float(), padding=m.padding) * masks[i]
        else:
            n, c, h, w = idxs[i].shape
            y = y.flatten(2).gather(2, idxs[i].flatten(2)).view(n, c, h, w)
    return y


def _routing(mods, x, outs):
    """(ReLU masks, pool argmax indices) of a run from its captured layer outputs."""
    masks, idxs, prev = {}, {}, x
    for i, m in enumerate(mods):
        if isinstance(m, nn.Conv2d):
            masks[i] = (outs[i].float() > 0).float()
        else:
            idxs[i] = F.max_pool2d(prev.float(), 2, 2, return_indices=True)[1]
        prev = outs[i]
    return masks, idxs


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
    grads, outs = {}, {}
    hooks = [m.register_forward_hook(lambda mod, inp, out, i=i: outs.__setitem__(i, out.detach().clone()))
             for i, m in enumerate(net)]
    for fuse in (True, False):
        ReluLink.enabled = fuse
        try:
            net.zero_grad(set_to_none=True)
            h0 = ReluLink.hits
            y = net(x)
            if fuse:
                for h in hooks:
                    h.remove()
            if g is None:
                g = torch.randn_like(y.float()).to(dt).contiguous(memory_format=torch.channels_last)
            y.backward(g)
            torch.cuda.synchronize()
            # 4 conv+ReLU layers: 2 handed over by the pools, 2 by the next conv's dgrad epilogue
            assert ReluLink.hits - h0 == (4 if fuse else 0)
            grads[fuse] = [p.grad.detach().clone() for p in net.parameters()]
        finally:
            ReluLink.enabled = True
    # the fp32 reference on the same (rounded) weights and input AND the fused run's routing
    # (its ReLU masks and pool argmax pixels): what is left is the run's bf16 / fp32 rounding
    ref = _vgg_block().cuda()
    ref.load_state_dict({k: v.to(dt).float() for k, v in net.state_dict().items()})
    masks, idxs = _routing(list(net), x, outs)
    yr = _ref_forward(list(ref), x.float(), masks, idxs)
    yr.backward(g.float())
    tol = 3e-2 if dt == torch.bfloat16 else 2e-3
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
    print("\n".join(report))
    assert not bad, "; ".join(report)

"""ConvAct2d (conv + bias + ReLU in the MFMA GEMM epilogue) against fp32 PyTorch, alone
(no ReLU hand-over: its output feeds a plain op) — forward, input / weight / bias gradients."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("c,co,k,pad", [(64, 128, 3, 1), (128, 64, 5, 2)])
def test_conv_act_alone(dt, c, co, k, pad):
    from mpit_amd.ops.conv import ConvAct2d, ReluLink

    torch.manual_seed(0)
    conv = ConvAct2d(c, co, k, padding=pad).cuda().to(memory_format=torch.channels_last)
    with torch.no_grad():
        conv.bias.uniform_(-0.3, 0.3)
    x = torch.randn(2, c, 14, 14, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    assert conv.fused(x)
    h0 = ReluLink.hits
    y = conv(x)
    wq = conv.weight.detach().to(dt).float()
    xr = x.detach().float().requires_grad_(True)
    wr = wq.clone().requires_grad_(True)
    br = conv.bias.detach().clone().requires_grad_(True)
    ref = F.relu(F.conv2d(xr, wr, br, padding=pad))
    tol = 2e-2 if dt == torch.bfloat16 else 1e-4
    assert (y.float() - ref).abs().max() <= tol * ref.abs().max()
    g = torch.randn_like(ref)
    (y.float() * g).sum().backward()  # the gradient reaches the layer through a plain multiply
    ref.backward(g)
    assert ReluLink.hits == h0  # nothing handed over: the layer's own ReLU backward ran
    for a, r in ((x.grad.float(), xr.grad), (conv.weight.grad, wr.grad), (conv.bias.grad, br.grad)):
        assert (a - r).abs().max() <= 2 * tol * r.abs().max() + 1e-4

"""NHWC max pooling kernels (csrc/kernels/pool.hip) against PyTorch's max_pool2d."""
import pytest
import torch
import torch.nn.functional as F

from mpit_amd.ops.pool import MaxPool2dNHWC


def test_maxpool_cpu_fallback():
    m = MaxPool2dNHWC(3, stride=2, padding=1)
    x = torch.randn(2, 16, 9, 9)
    assert torch.equal(m(x), F.max_pool2d(x, 3, 2, 1))


@pytest.mark.gpu
@pytest.mark.parametrize("n,c,hw,k,s,p", [(4, 64, 112, 3, 2, 1), (2, 16, 15, 3, 2, 1), (3, 8, 10, 2, 2, 0),
                                          (2, 32, 9, 3, 1, 1), (2, 24, 13, 5, 3, 2)])
def test_maxpool_fwd_bwd(n, c, hw, k, s, p):
    torch.manual_seed(hw + c)
    # distinct values per window so the argmax (and the routed gradient) is unambiguous
    x = torch.randperm(n * c * hw * hw, device="cuda").float().reshape(n, c, hw, hw) / (n * c * hw * hw)
    x = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    m = MaxPool2dNHWC(k, stride=s, padding=p)
    assert m.fused(x)
    x1 = x.clone().requires_grad_(True)
    x2 = x.float().clone().requires_grad_(True)
    y1, y2 = m(x1), F.max_pool2d(x2, k, s, p)
    assert torch.equal(y1.float(), y2)
    g = torch.randn_like(y2).to(torch.bfloat16)
    y1.backward(g)
    y2.backward(g.float())
    # bf16 rounding ties can route a gradient to a different (equal-valued) input
    close = (x1.grad.float() - x2.grad).abs() <= 1e-2 * (1 + x2.grad.abs())
    assert close.float().mean().item() > 0.999

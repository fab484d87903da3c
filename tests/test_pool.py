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
                                          (2, 32, 9, 3, 1, 1), (2, 24, 13, 5, 3, 2),
                                          # windows partitioning the input (K == stride): the
                                          # one-thread-per-window backward, with remainders
                                          (2, 16, 11, 2, 2, 0), (2, 8, 10, 3, 3, 0), (2, 64, 56, 2, 2, 0)])
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


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_maxpool_partition_backward_matches_gather(dt, monkeypatch):
    """The per-window backward (K == stride) writes exactly what the per-input-pixel gather
    writes (MPIT_POOL_GATHER forces the gather)."""
    torch.manual_seed(0)
    x = torch.randn(3, 64, 23, 23, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
    m = MaxPool2dNHWC(2, stride=2)
    grads = []
    for gather in (False, True):
        if gather:
            monkeypatch.setenv("MPIT_POOL_GATHER", "1")
        xx = x.clone().requires_grad_(True)
        y = m(xx)
        y.backward(torch.ones_like(y) * torch.arange(y.numel(), device="cuda").reshape(y.shape).to(dt) / y.numel())
        grads.append(xx.grad.clone())
    assert torch.equal(grads[0], grads[1])


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_global_avgpool_backward(dt):
    """GlobalAvgPoolNHWC: PyTorch's forward, the one-pass HIP backward (dy / HW per pixel)."""
    from mpit_amd.ops.pool import GlobalAvgPoolNHWC

    torch.manual_seed(0)
    x = torch.randn(4, 256, 7, 7, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
    m = GlobalAvgPoolNHWC()
    x1, x2 = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    assert m.fused(x1)
    y1, y2 = m(x1), F.adaptive_avg_pool2d(x2, 1)
    assert torch.equal(y1, y2)
    g = torch.randn_like(y2)
    y1.backward(g)
    y2.backward(g)
    assert x1.grad.is_contiguous(memory_format=torch.channels_last)
    assert torch.allclose(x1.grad.float(), x2.grad.float(), rtol=1e-2 if dt == torch.bfloat16 else 1e-6, atol=1e-6)

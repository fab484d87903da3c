"""Fused BN(+residual)(+ReLU) HIP kernels vs a plain PyTorch fp32 reference
(F.batch_norm in training mode + add + relu), forward, backward and running stats."""
import pytest
import torch
import torch.nn.functional as F

from mpit_amd.ops.bn import BatchNormAct2d

gpu = pytest.mark.gpu


def _ref(x, w, b, rm, rv, res, relu, mom, eps):
    y = F.batch_norm(x, rm, rv, w, b, True, mom, eps)
    if res is not None:
        y = y + res
    return F.relu(y) if relu else y


def test_cpu_path_matches_plain_modules():
    torch.manual_seed(0)
    m = BatchNormAct2d(16, act=True)
    ref = torch.nn.BatchNorm2d(16)
    x = torch.randn(4, 16, 5, 5)
    r = torch.randn(4, 16, 5, 5)
    torch.testing.assert_close(m(x, r), F.relu(ref(x) + r))


@gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("C", [64, 256, 2048])
@pytest.mark.parametrize("res", [False, True])
@pytest.mark.parametrize("relu", [True, False])
def test_bn_act_fwd_bwd(dtype, C, res, relu):
    _check(dtype, C, res, relu, (8, 7, 9))


@gpu
@pytest.mark.parametrize("C", [8, 24, 64, 512])
@pytest.mark.parametrize("shape", [(3, 5, 7), (1, 1, 3)])
def test_bn_act_fp32_lane_layouts(C, shape):
    """fp32 apply passes read each wave's 512-element chunk as two coalesced float4 halves
    (C | 2048) or one 32-byte vector per lane (other C): tails that end inside a wave's chunk,
    channel counts on both sides of the rule, the ReLU mask bytes two lanes share."""
    _check(torch.float32, C, True, True, shape)
    _check(torch.float32, C, False, True, shape)


def _check(dtype, C, res, relu, shape):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.manual_seed(C + res * 7 + relu)
    dev = torch.device("cuda")
    N, H, W = shape
    x32 = (torch.randn(N, C, H, W, device=dev) * 2 + 0.7).contiguous(memory_format=torch.channels_last)
    r32 = torch.randn(N, C, H, W, device=dev).contiguous(memory_format=torch.channels_last) if res else None
    x = x32.to(dtype).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    r = r32.to(dtype).contiguous(memory_format=torch.channels_last).requires_grad_(True) if res else None
    m = BatchNormAct2d(C, act=relu).to(dev)
    with torch.no_grad():
        m.weight.uniform_(0.5, 1.5)
        m.bias.uniform_(-0.5, 0.5)
    w = m.weight.detach().clone().requires_grad_(True)
    b = m.bias.detach().clone().requires_grad_(True)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    xr = x.detach().float().requires_grad_(True)
    rr = r.detach().float().requires_grad_(True) if res else None
    yref = _ref(xr, w, b, rm, rv, rr, relu, 0.1, 1e-5)
    y = m(x, r)
    assert y.dtype == dtype and y.is_contiguous(memory_format=torch.channels_last)
    tol = 3e-2 if dtype == torch.bfloat16 else 1e-4
    torch.testing.assert_close(y.float(), yref, atol=tol, rtol=tol)
    torch.testing.assert_close(m.running_mean, rm, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(m.running_var, rv, atol=1e-3, rtol=1e-3)
    gy = torch.randn_like(yref)
    yref.backward(gy)
    y.backward(gy.to(dtype).contiguous(memory_format=torch.channels_last))
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=5 * tol, rtol=5 * tol)
    torch.testing.assert_close(m.weight.grad, w.grad, atol=1e-2 * N * H * W ** 0.5, rtol=2e-2)
    torch.testing.assert_close(m.bias.grad, b.grad, atol=1e-2 * N * H, rtol=2e-2)
    if res:
        torch.testing.assert_close(r.grad.float(), rr.grad, atol=tol, rtol=tol)
    # eval path
    m.eval()
    with torch.no_grad():
        ye = m(x.detach(), r.detach() if res else None)
        yr = F.batch_norm(x.detach().float(), m.running_mean, m.running_var, m.weight, m.bias, False, 0.0, 1e-5)
        if res:
            yr = yr + r.detach().float()
        if relu:
            yr = F.relu(yr)
    torch.testing.assert_close(ye.float(), yr, atol=tol, rtol=tol)


@gpu
def test_bn_act_large_mean_stability():
    """|mean| >> std: shifted sums must not cancel catastrophically."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    dev = torch.device("cuda")
    x = (torch.randn(16, 64, 8, 8, device=dev) * 0.01 + 100.0).contiguous(memory_format=torch.channels_last)
    m = BatchNormAct2d(64, act=False).to(dev)
    y = m(x)
    ref = F.batch_norm(x, None, None, None, None, True, 0.1, 1e-5)
    torch.testing.assert_close(y, ref, atol=2e-3, rtol=2e-3)

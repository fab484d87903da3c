"""LinearAct (ops/linear.py): the classifier's Linear(+ReLU) on the MFMA kernels in bf16 and fp32
steps, against fp32 PyTorch on the same bf16-rounded operands; CPU fallback == F.linear."""
import pytest
import torch
import torch.nn.functional as F


def test_linear_act_cpu_fallback():
    from mpit_amd.ops.linear import LinearAct

    torch.manual_seed(0)
    lin = LinearAct(128, 64)
    x = torch.randn(8, 128)
    assert not lin.fused(x)
    assert torch.equal(lin(x), F.relu(F.linear(x, lin.weight, lin.bias)))
    lin.act = False
    assert torch.equal(lin(x), F.linear(x, lin.weight, lin.bias))


@pytest.mark.gpu
@pytest.mark.parametrize("act", [True, False])
@pytest.mark.parametrize("M,K,N", [(64, 25088, 4096), (128, 1024, 512), (64, 4096, 4096), (256, 2048, 1000)])
def test_linear_act_bf16(act, M, K, N):
    from mpit_amd.ops.linear import LinearAct

    torch.manual_seed(0)
    lin = LinearAct(K, N, act=act, pad_out=N % 64 != 0).cuda()
    with torch.no_grad():
        lin.bias.uniform_(-0.1, 0.1)
    x = torch.randn(M, K, device="cuda").requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        assert lin.fused(x)
        y = lin(x)
    assert y.dtype == torch.bfloat16 and y.shape == (M, N)
    xq = x.detach().to(torch.bfloat16).float().requires_grad_(True)
    wq = lin.weight.detach().to(torch.bfloat16).float().requires_grad_(True)
    bq = lin.bias.detach().clone().requires_grad_(True)
    ref = F.linear(xq, wq, bq)
    if act:
        ref = F.relu(ref)
    scale = ref.abs().max().item()
    assert (y.float() - ref).abs().max().item() <= 1e-2 * scale
    g = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    y.backward(g)
    ref.backward(g.float() * ((y.float() > 0).float() if act else 1.0))  # the same mask as the layer's
    for a, r, name in ((x.grad, xq.grad, "x"), (lin.weight.grad, wq.grad, "w"), (lin.bias.grad, bq.grad, "b")):
        assert a.dtype == torch.float32 and a.shape == r.shape, name
        assert (a - r).abs().max().item() <= 2e-2 * r.abs().max().item() + 1e-4, name


@pytest.mark.gpu
@pytest.mark.parametrize("act", [True, False])
@pytest.mark.parametrize("M,K,N", [(64, 4096, 4096), (256, 2048, 1000)])
def test_linear_act_fp32(act, M, K, N):
    """fp32 steps (and ResNet's fp32 classifier): the same GEMMs on fp32 operands (bf16x6
    split products), against fp64 — fp32-class error, and no library GEMM."""
    from mpit_amd.ops.linear import LinearAct

    torch.manual_seed(1)
    lin = LinearAct(K, N, act=act, pad_out=N % 64 != 0).cuda()
    with torch.no_grad():
        lin.bias.uniform_(-0.1, 0.1)
    x = torch.randn(M, K, device="cuda").requires_grad_(True)
    assert lin.fused(x)
    y = lin(x)
    assert y.dtype == torch.float32 and y.shape == (M, N)
    xd = x.detach().double().requires_grad_(True)
    wd = lin.weight.detach().double().requires_grad_(True)
    bd = lin.bias.detach().double().requires_grad_(True)
    ref = F.linear(xd, wd, bd)
    if act:
        ref = F.relu(ref)
    assert (y.double() - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()
    g = torch.randn(M, N, device="cuda")
    y.backward(g)
    ref.backward(g.double() * ((y > 0).double() if act else 1.0))
    for a, r, name in ((x.grad, xd.grad, "x"), (lin.weight.grad, wd.grad, "w"), (lin.bias.grad, bd.grad, "b")):
        assert a.dtype == torch.float32 and a.shape == r.shape, name
        assert (a.double() - r).abs().max().item() <= 1e-5 * r.abs().max().item() + 1e-7, name


def test_fused_xent_cpu_fallback():
    from mpit_amd.ops.loss import cross_entropy

    torch.manual_seed(0)
    x = torch.randn(8, 10, requires_grad=True)
    t = torch.randint(0, 10, (8,))
    assert torch.equal(cross_entropy(x, t), F.cross_entropy(x, t))


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,C", [(256, 1000), (64, 10), (3, 4097)])
def test_fused_xent_vs_pytorch(dt, B, C):
    """ops/loss.py: the one-launch softmax cross-entropy (loss and logits' gradient) against
    PyTorch's F.cross_entropy on the same (fp32-promoted) logits."""
    from mpit_amd.ops.loss import cross_entropy

    torch.manual_seed(3)
    x = (torch.randn(B, C, device="cuda") * 4).to(dt).requires_grad_(True)
    t = torch.randint(0, C, (B,), device="cuda")
    loss = cross_entropy(x, t)
    loss.backward(torch.tensor(0.5, device="cuda"))
    xr = x.detach().float().requires_grad_(True)
    ref = F.cross_entropy(xr, t)
    ref.backward(torch.tensor(0.5, device="cuda"))
    assert loss.dtype == torch.float32
    assert abs(loss.item() - ref.item()) <= 1e-5 * max(1.0, abs(ref.item()))
    assert x.grad.dtype == dt and x.grad.shape == x.shape
    tol = 1e-6 if dt == torch.float32 else 1e-2 * xr.grad.abs().max().item()
    assert (x.grad.float() - xr.grad).abs().max().item() <= tol

"""MFMA GEMM kernels (csrc/kernels/gemm.hip) and the 1x1-conv op built on them, against
plain PyTorch fp32 references of the same math."""
import os

import pytest
import torch
import torch.nn.functional as F

from mpit_amd.ops import conv as C

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_convnhwc_cpu_fallback_matches_conv2d():
    torch.manual_seed(0)
    m = C.ConvNHWC(64, 64, 3, stride=2, padding=1)
    x = torch.randn(2, 64, 9, 9)
    assert torch.allclose(m(x), F.conv2d(x, m.weight, stride=2, padding=1), atol=1e-5)
    assert not C.conv_supported(x, m.weight)


def test_conv1x1_cpu_fallback_matches_conv2d():
    torch.manual_seed(0)
    m = C.Conv1x1(64, 128)
    x = torch.randn(2, 64, 5, 5)
    assert torch.allclose(m(x), F.conv2d(x, m.weight), atol=1e-6)
    assert not C.conv1x1_supported(x, m.weight)


gpu = pytest.mark.gpu


def _bf(*shape, scale=1.0):
    return (torch.randn(*shape, device="cuda") * scale).to(torch.bfloat16)


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@gpu
@pytest.mark.parametrize("M,N,K", [(128, 64, 64), (256, 128, 64), (1000, 192, 128), (4096, 256, 512),
                                   (333, 64, 1024), (12544, 2048, 512), (50176, 256, 1024),
                                   (262144, 128, 1024), (262000, 256, 2048)])  # (auto 256x128 tiles)
def test_gemm_nt(M, N, K):
    torch.manual_seed(M + N + K)
    a, b = _bf(M, K), _bf(N, K, scale=0.05)
    ref = a.float() @ b.float().t()
    c = C.gemm_nt(a, b)
    assert c.shape == (M, N) and c.dtype == torch.bfloat16
    assert _rel(c, ref) < 8e-3


@gpu
@pytest.mark.parametrize("M,N,K", [(256, 64, 64), (1000, 128, 192), (4096, 256, 256), (262100, 128, 1024)])
def test_gemm_nt_stats(M, N, K):
    torch.manual_seed(1)
    a, b = _bf(M, K), _bf(N, K, scale=0.05)
    c, st = C.gemm_nt(a, b, stats=True)
    # the statistics are those of the stored (bf16) C
    cf = c.float()
    assert torch.allclose(st[0], cf.sum(0), rtol=1e-3, atol=1e-2)
    assert torch.allclose(st[1], (cf * cf).sum(0), rtol=1e-3, atol=1e-2)


@gpu
@pytest.mark.parametrize("M,N,K", [(64, 64, 64), (1000, 64, 128), (4096, 128, 128), (802816, 256, 64),
                                   (12544, 512, 2048), (5000, 192, 320)])
def test_gemm_tn(M, N, K):
    torch.manual_seed(M % 97 + N + K)
    y, x = _bf(M, N), _bf(M, K)
    ref = y.float().t() @ x.float()
    out = C.gemm_tn(y, x)
    assert out.dtype == torch.float32 and out.shape == (N, K)
    assert _rel(out, ref) < 1e-4
    # beta accumulate
    base = torch.randn(N, K, device="cuda")
    out2 = C.gemm_tn(y, x, out=base.clone(), beta=1.0)
    assert _rel(out2, ref + base) < 1e-4


@gpu
def test_cast_transpose():
    w = torch.randn(192, 320, device="cuda")
    wb, wt = C.cast_transpose(w)
    assert torch.equal(wb, w.to(torch.bfloat16))
    assert torch.equal(wt, w.t().contiguous().to(torch.bfloat16))


@gpu
@pytest.mark.parametrize("n,ci,co,hw", [(4, 64, 256, 14), (2, 256, 64, 9), (3, 128, 128, 7)])
def test_conv1x1_fwd_bwd(n, ci, co, hw):
    torch.manual_seed(n * ci + co)
    mod = C.Conv1x1(ci, co).cuda().to(memory_format=torch.channels_last)
    ref = torch.nn.Conv2d(ci, co, 1, bias=False).cuda()
    ref.weight.data.copy_(mod.weight.data)
    x = torch.randn(n, ci, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x1 = x.clone().requires_grad_(True)
    x2 = x.float().clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y1 = mod(x1)
    y2 = ref(x2)
    assert y1.dtype == torch.bfloat16
    assert _rel(y1, y2) < 8e-3
    g = torch.randn_like(y2)
    y1.backward(g.to(torch.bfloat16))
    y2.backward(g)
    assert _rel(x1.grad, x2.grad) < 1e-2
    assert mod.weight.grad.dtype == torch.float32
    assert _rel(mod.weight.grad, ref.weight.grad) < 1e-2


@gpu
def test_cast_transpose_taps():
    w = torch.randn(128, 64, 3, 3, device="cuda").contiguous(memory_format=torch.channels_last)
    wb, wt = C.conv_weights(w, dgrad=True)
    ref = w.permute(0, 2, 3, 1).to(torch.bfloat16)  # [Co][R][S][C]
    assert torch.equal(wb, ref)
    assert torch.equal(wt, ref.flip(1, 2).permute(3, 1, 2, 0).contiguous())  # [C][R'][S'][Co]


@gpu
@pytest.mark.parametrize("n,ci,co,hw,k,stride", [(2, 64, 64, 56, 3, 1), (3, 128, 128, 28, 3, 2), (4, 256, 256, 14, 3, 1),
                                                 (2, 512, 512, 7, 3, 1), (2, 64, 128, 9, 3, 2), (2, 128, 64, 13, 5, 1),
                                                 (5, 64, 192, 11, 3, 1), (2, 256, 512, 14, 1, 2), (2, 128, 256, 15, 1, 2),
                                                 (2, 64, 64, 11, 5, 2), (2, 64, 64, 12, 3, 3)])
def test_conv_nhwc_fwd_bwd(n, ci, co, hw, k, stride):
    """Implicit-GEMM conv (fwd, dgrad, wgrad) against fp32 PyTorch conv2d."""
    torch.manual_seed(n * ci + co + k)
    pad = k // 2
    mod = C.ConvNHWC(ci, co, k, stride=stride, padding=pad).cuda().to(memory_format=torch.channels_last)
    ref = torch.nn.Conv2d(ci, co, k, stride=stride, padding=pad, bias=False).cuda()
    ref.weight.data.copy_(mod.weight.data)
    x = torch.randn(n, ci, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x1 = x.clone().requires_grad_(True)
    x2 = x.float().clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y1 = mod(x1)
    y2 = ref(x2)
    assert y1.dtype == torch.bfloat16 and y1.shape == y2.shape
    assert _rel(y1, y2) < 8e-3
    g = torch.randn_like(y2)
    y1.backward(g.to(torch.bfloat16))
    y2.backward(g)
    assert _rel(x1.grad, x2.grad) < 1e-2
    assert mod.weight.grad.dtype == torch.float32
    assert _rel(mod.weight.grad, ref.weight.grad) < 1e-2


def test_park_grad_slot_protocol():
    # producer runs first: the gradient is parked, autograd gets none
    slot = C.GradSlot()
    x = torch.randn(3, 4, requires_grad=True)
    (C.park_grad(x, slot) * 2).sum().backward()
    assert x.grad is None
    g, m = slot.take()
    assert torch.equal(g, torch.full((3, 4), 2.0)) and m is None
    # consumer already ran (slot closed): the gradient goes back to autograd
    slot2 = C.GradSlot()
    slot2.take()
    x2 = torch.randn(3, 4, requires_grad=True)
    (C.park_grad(x2, slot2) * 3).sum().backward()
    assert torch.equal(x2.grad, torch.full((3, 4), 3.0))


@gpu
@pytest.mark.parametrize("n,ci,co,hw,k,relu", [(2, 64, 192, 13, 5, True), (3, 192, 384, 13, 3, True),
                                               (16, 64, 64, 56, 3, True),
                                               (2, 128, 64, 9, 3, False),
                                               (16, 128, 128, 128, 3, True)])  # (auto 256x128 tiles)
def test_conv_act_bias_relu(n, ci, co, hw, k, relu):
    """conv + bias + ReLU with the bias / ReLU in the GEMM epilogue and the one-pass
    ReLU/bias backward, against fp32 PyTorch; ReLU mask flips of near-zero outputs under
    bf16 make the gradient error data dependent, so it is held to the error of the same
    layer on the bf16 library path (MIOpen under autocast)."""
    torch.manual_seed(ci + co)
    pad = k // 2
    mod = C.ConvAct2d(ci, co, k, padding=pad, act=relu).cuda().to(memory_format=torch.channels_last)
    mod.bias.data.uniform_(-0.5, 0.5)
    x = torch.randn(n, ci, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g = torch.randn(n, co, hw, hw, device="cuda")

    def ref(xx, dtype):
        xx = xx.clone().to(dtype).requires_grad_(True)
        ww = mod.weight.detach().clone().requires_grad_(True)
        bb = mod.bias.detach().clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=dtype == torch.bfloat16):
            y = F.conv2d(xx, ww, bb, padding=pad)
            y = F.relu(y) if relu else y
        y.backward(g.to(y.dtype))
        return y, xx.grad, ww.grad, bb.grad

    x1 = x.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y1 = mod(x1)
    y1.backward(g.to(torch.bfloat16))
    got = (y1, x1.grad, mod.weight.grad, mod.bias.grad)
    lib = ref(x, torch.bfloat16)
    exact = ref(x, torch.float32)
    for name, a, b, e in zip(("y", "dx", "dw", "db"), got, lib, exact):
        err, floor = _rel(a, e), _rel(b, e)
        assert err < 1.5 * floor + 5e-3, (name, err, floor)


@gpu
@pytest.mark.parametrize("M", [1000, 70000])
def test_gemm_nt_tile_stats_large_mean(M):
    """Per-tile (mean, M2) statistics stay exact when |mean| >> std (no E[y^2]-E[y]^2
    cancellation): C = A . I reproduces A's columns, offset by 300 with unit spread."""
    torch.manual_seed(M)
    N = K = 64
    a = (torch.randn(M, K, device="cuda") + 300.0).to(torch.bfloat16)
    b = torch.eye(N, K, device="cuda", dtype=torch.bfloat16)
    m = C.native()
    c = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    st = torch.empty(m.gemm_nt_stats_floats(M, N), dtype=torch.float32, device="cuda")
    m.gemm_nt(0, torch.cuda.current_stream().cuda_stream, M, N, K, a.data_ptr(), K, b.data_ptr(), K, c.data_ptr(), N,
              st.data_ptr())
    p = st.view(-1, 2, N).double()
    n = (M - 128 * torch.arange(p.shape[0], device="cuda", dtype=torch.float64)).clamp(max=128)[:, None]
    mean = (n * p[:, 0]).sum(0) / M
    var = (p[:, 1] + n * (p[:, 0] - mean) ** 2).sum(0) / M
    cd = c.double()
    torch.testing.assert_close(mean, cd.mean(0), rtol=1e-7, atol=1e-4)
    torch.testing.assert_close(var, cd.var(0, unbiased=False), rtol=1e-4, atol=1e-5)


@gpu
def test_tn_fused_split_reduction_bitwise(tmp_path):
    """The in-kernel split reduction (MPIT_TN_FUSED=1) adds the partials in the order of
    the split_reduce launches: identical bits, for gemm_tn (one and two reduction levels,
    beta 0 and 1) and conv_wgrad, bf16 and fp32 operands."""
    import subprocess
    import sys

    res = {}
    for fused in ("0", "1"):
        path = str(tmp_path / f"tn{fused}.pt")
        env = dict(os.environ, MPIT_TN_FUSED=fused)
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "mp", "tn_fused_check.py"), path],
                           env=env, capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-3000:]
        res[fused] = torch.load(path, weights_only=True)
    assert res["0"].keys() == res["1"].keys()
    for k in res["0"]:
        assert torch.equal(res["0"][k].view(torch.int32), res["1"][k].view(torch.int32)), k

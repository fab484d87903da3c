"""fp16x3 GEMMs on operands that arrive as fp16 planes (csrc/kernels/gemm.hip FM 13).

A producer that knows a bound of its output writes it as two fp16 planes h, l of x * 2^e —
the split the fp16x3 kernels otherwise do in registers (gemm_nt FM 11: the activation, per
k16 fragment and per wave) or in LDS (gemm_tn FM 12: both operands, per staged step). Given
planes made with the same arithmetic (ops.conv.f16_planes = gemm.hip split1h), the planes
kernels must give the SAME BITS as the splitting ones: same planes, same MFMA sequence. Every
case below compares them bit for bit, on the ResNet-50 shapes of each kernel family (1x1,
3x3 implicit GEMM, strided 1x1 / 3x3, strided backward-data parity classes, backward-weight
1x1 and implicit), and once against fp64."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _m():
    from mpit_amd._ext import native

    return native()


def _st():
    return torch.cuda.current_stream().cuda_stream


def _bound(t):
    from mpit_amd.ops.conv import bound_of_value

    return bound_of_value(torch.linalg.vector_norm(t.float(), float("inf")))


def _planes(t, bnd):
    """[2, numel] fp16 planes of t in its memory order (t contiguous or channels_last)."""
    from mpit_amd.ops.conv import f16_planes

    flat = t.permute(0, 2, 3, 1).reshape(-1) if t.dim() == 4 else t.reshape(-1)
    return f16_planes(flat.contiguous(), bnd)


def _wplanes(w):
    from mpit_amd.ops.conv import f16_planes

    return f16_planes(w.contiguous(), _bound(w))


def _same(a, b):
    return bool(torch.equal(a.view(torch.int32), b.view(torch.int32)))


@pytest.mark.parametrize("M,N,K", [(4096, 256, 64), (2048, 512, 256), (1536, 128, 512), (1000, 1024, 256)])
def test_nt_planes_bitwise(M, N, K):
    torch.manual_seed(0)
    m = _m()
    a = torch.randn(M, K, device="cuda") * 3.0
    w = torch.randn(N, K, device="cuda") * 0.05
    wp = _wplanes(w)
    ab = _bound(a)
    ap = _planes(a, ab)
    c1 = torch.empty(M, N, device="cuda")
    c2 = torch.empty(M, N, device="cuda")
    kw = dict(f32=True, bps=wp[0].numel(), amax_a=ab.data_ptr(), amax_b=wp._mpit_wamax.data_ptr())
    m.gemm_nt(0, _st(), M, N, K, a.data_ptr(), K, wp.data_ptr(), K, c1.data_ptr(), N, 0, **kw)
    m.gemm_nt(0, _st(), M, N, K, ap.data_ptr(), K, wp.data_ptr(), K, c2.data_ptr(), N, 0, aps=ap[0].numel(), **kw)
    torch.cuda.synchronize()
    assert _same(c1, c2), (c1 - c2).abs().max().item()
    ref = a.double() @ w.double().t()
    err = ((c2.double() - ref).abs().max() / ref.abs().max()).item()
    assert err < 1e-5, err


@pytest.mark.parametrize("Nb,H,C,Co,R,S", [(4, 14, 256, 256, 3, 1), (4, 28, 128, 128, 3, 2), (4, 28, 256, 512, 1, 2),
                                           (2, 56, 64, 64, 3, 1)])
def test_conv_planes_bitwise(Nb, H, C, Co, R, S):
    torch.manual_seed(1)
    m = _m()
    pad = R // 2
    Ho = (H + 2 * pad - R) // S + 1
    x = torch.relu(torch.randn(Nb, C, H, H, device="cuda")).contiguous(memory_format=torch.channels_last)
    w = torch.randn(Co, R, R, C, device="cuda") * 0.05
    wp = _wplanes(w)
    xb = _bound(x)
    xp = _planes(x, xb)
    y1 = torch.empty(Nb, Ho, Ho, Co, device="cuda")
    y2 = torch.empty_like(y1)
    kw = dict(f32=True, bps=wp[0].numel(), amax_a=xb.data_ptr(), amax_b=wp._mpit_wamax.data_ptr())
    m.conv_fwd(0, _st(), Nb, H, H, C, Co, R, R, S, pad, x.data_ptr(), wp.data_ptr(), y1.data_ptr(), **kw)
    m.conv_fwd(0, _st(), Nb, H, H, C, Co, R, R, S, pad, xp.data_ptr(), wp.data_ptr(), y2.data_ptr(),
               aps=xp[0].numel(), **kw)
    torch.cuda.synchronize()
    assert _same(y1, y2), (y1 - y2).abs().max().item()


@pytest.mark.parametrize("M,N,K", [(8192, 256, 64), (3136, 512, 128), (6272, 128, 128)])
def test_tn_planes_bitwise(M, N, K):
    torch.manual_seed(2)
    m = _m()
    y = torch.randn(M, N, device="cuda") * 1e-3
    x = torch.relu(torch.randn(M, K, device="cuda"))
    yb, xb = _bound(y), _bound(x)
    yp, xp = _planes(y, yb), _planes(x, xb)
    o1 = torch.empty(N, K, device="cuda")
    o2 = torch.empty(N, K, device="cuda")
    nws = m.gemm_tn_ws_floats(0, M, N, K)
    ws = torch.empty(max(1, nws), device="cuda")
    kw = dict(f32=True, amax_y=yb.data_ptr(), amax_x=xb.data_ptr())
    m.gemm_tn(0, _st(), M, N, K, y.data_ptr(), N, x.data_ptr(), K, o1.data_ptr(), ws.data_ptr(), 0.0, **kw)
    m.gemm_tn(0, _st(), M, N, K, yp.data_ptr(), N, xp.data_ptr(), K, o2.data_ptr(), ws.data_ptr(), 0.0,
              yps=yp[0].numel(), xps=xp[0].numel(), **kw)
    torch.cuda.synchronize()
    assert _same(o1, o2), (o1 - o2).abs().max().item()
    ref = y.double().t() @ x.double()
    err = ((o2.double() - ref).abs().max() / ref.abs().max()).item()
    assert err < 1e-5, err


@pytest.mark.parametrize("Nb,H,C,Co,R,S", [(4, 14, 256, 256, 3, 1), (4, 28, 128, 128, 3, 2), (4, 28, 256, 512, 1, 2)])
def test_wgrad_planes_bitwise(Nb, H, C, Co, R, S):
    torch.manual_seed(3)
    m = _m()
    pad = R // 2
    Ho = (H + 2 * pad - R) // S + 1
    x = torch.relu(torch.randn(Nb, C, H, H, device="cuda")).contiguous(memory_format=torch.channels_last)
    dy = (torch.randn(Nb, Co, Ho, Ho, device="cuda") * 1e-2).contiguous(memory_format=torch.channels_last)
    xb, yb = _bound(x), _bound(dy)
    xp, yp = _planes(x, xb), _planes(dy, yb)
    d1 = torch.empty(Co, R, R, C, device="cuda")
    d2 = torch.empty_like(d1)
    nws = m.conv_wgrad_ws_floats(0, Nb, H, H, C, Co, R, R, S, pad)
    ws = torch.empty(max(1, nws), device="cuda")
    kw = dict(f32=True, amax_y=yb.data_ptr(), amax_x=xb.data_ptr())
    m.conv_wgrad(0, _st(), Nb, H, H, C, Co, R, R, S, pad, dy.data_ptr(), x.data_ptr(), d1.data_ptr(), ws.data_ptr(),
                 0.0, **kw)
    m.conv_wgrad(0, _st(), Nb, H, H, C, Co, R, R, S, pad, yp.data_ptr(), xp.data_ptr(), d2.data_ptr(), ws.data_ptr(),
                 0.0, yps=yp[0].numel(), xps=xp[0].numel(), **kw)
    torch.cuda.synchronize()
    assert _same(d1, d2), (d1 - d2).abs().max().item()


def test_dgrad_strided_planes_bitwise():
    """Strided backward-data (stride-2 3x3, parity classes) with dY as planes."""
    torch.manual_seed(4)
    m = _m()
    Nb, H, C, Co, R, S, pad = 4, 28, 128, 128, 3, 2, 1
    Ho = (H + 2 * pad - R) // S + 1
    w = torch.randn(Co, C, R, R, device="cuda") * 0.05
    from mpit_amd.ops.conv import strided_dgrad_weights

    _, wc32 = strided_dgrad_weights(w.contiguous(memory_format=torch.channels_last), S, pad, torch.float32)
    wcls = _wplanes(wc32.reshape(-1))  # the packed parity-class weights as fp16 planes
    dy = (torch.randn(Nb, Co, Ho, Ho, device="cuda") * 1e-2).contiguous(memory_format=torch.channels_last)
    yb = _bound(dy)
    yp = _planes(dy, yb)
    d1 = torch.empty(Nb, H, H, C, device="cuda")
    d2 = torch.empty_like(d1)
    kw = dict(f32=True, bps=wcls[0].numel(), amax_a=yb.data_ptr(), amax_b=wcls._mpit_wamax.data_ptr())
    m.conv_dgrad_strided(0, _st(), Nb, H, H, C, Co, R, R, S, pad, dy.data_ptr(), wcls.data_ptr(), d1.data_ptr(), **kw)
    m.conv_dgrad_strided(0, _st(), Nb, H, H, C, Co, R, R, S, pad, yp.data_ptr(), wcls.data_ptr(), d2.data_ptr(),
                         aps=yp[0].numel(), **kw)
    torch.cuda.synchronize()
    assert _same(d1, d2), (d1 - d2).abs().max().item()

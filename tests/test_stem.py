"""Row-tap stem convolution (ops/conv.py StemConv) against an fp32 PyTorch reference."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nb,h,co,k,stride,pad", [(4, 224, 64, 7, 2, 3), (2, 37, 128, 7, 2, 3), (3, 32, 64, 5, 1, 2)])
def test_stem_fwd_wgrad(nb, h, co, k, stride, pad):
    from mpit_amd.ops.conv import StemConv

    torch.manual_seed(0)
    conv = StemConv(3, co, k, stride, pad).cuda().to(memory_format=torch.channels_last)
    x = torch.randn(nb, 3, h, h, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    assert conv.fused(x)
    y = conv(x)
    wb = conv.weight.detach().to(torch.bfloat16).float()
    ref = F.conv2d(x.float(), wb, stride=stride, padding=pad)
    assert y.shape == ref.shape
    assert (y.float() - ref).abs().max() <= 2e-2 * ref.abs().max()
    g = torch.randn_like(ref).to(torch.bfloat16)
    y.backward(g.contiguous(memory_format=torch.channels_last))
    wref = torch.nn.grad.conv2d_weight(x.float(), conv.weight.shape, g.float(), stride=stride, padding=pad)
    err = (conv.weight.grad - wref).abs().max() / wref.abs().max()
    assert err < 1e-2, float(err)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("nb,h,co", [(2, 224, 64), (3, 30, 128)])
def test_first_layer_3x3_bias_relu(dt, nb, h, co):
    """VGG's 3-channel 3x3 first layer (ConvAct2d) on the 3-row row-tap kernel with the bias
    and ReLU in the epilogue: y, and the weight and bias gradients, against fp32 PyTorch."""
    from mpit_amd._ext import native
    from mpit_amd.ops.conv import ConvAct2d

    assert native().stem_wgrad_rows(3) == 4
    torch.manual_seed(0)
    conv = ConvAct2d(3, co, 3, padding=1).cuda().to(memory_format=torch.channels_last)
    with torch.no_grad():
        conv.bias.uniform_(-0.5, 0.5)
    x = torch.randn(nb, 3, h, h, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
    assert not conv.fused(x)  # (3 channels: not the implicit-GEMM path) -> the row-tap path
    y = conv(x)
    assert y.grad_fn is not None and "Stem" in type(y.grad_fn).__name__
    wq = conv.weight.detach().to(dt).float()
    ref = F.relu(F.conv2d(x.float(), wq, conv.bias.detach(), padding=1))
    assert y.shape == ref.shape and y.dtype == dt
    tol = 2e-2 if dt == torch.bfloat16 else 1e-4
    assert (y.float() - ref).abs().max() <= tol * ref.abs().max()
    g = torch.randn_like(ref).to(dt)
    y.backward(g.contiguous(memory_format=torch.channels_last))
    gz = g.float() * (y.float() > 0)
    wref = torch.nn.grad.conv2d_weight(x.float(), conv.weight.shape, gz, padding=1)
    err = (conv.weight.grad - wref).abs().max() / wref.abs().max()
    assert err < tol, float(err)
    bref = gz.sum(dim=(0, 2, 3))
    assert (conv.bias.grad - bref).abs().max() <= tol * bref.abs().max() + 1e-3


def test_stem_emits_bn_stats():
    from mpit_amd.ops.conv import StemConv, tile_stats_to_sums

    conv = StemConv(3, 64, 7, 2, 3).cuda().to(memory_format=torch.channels_last)
    conv.emit_stats = True
    x = torch.randn(2, 3, 64, 64, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = conv(x)
    part, nt, ptr, _fold = y._mpit_tstats
    assert ptr == y.data_ptr()
    M = y.shape[0] * y.shape[2] * y.shape[3]
    sums = tile_stats_to_sums(part, M, 64).double()
    yf = y.double().permute(0, 2, 3, 1).reshape(-1, 64)
    assert torch.allclose(sums[0], yf.sum(0), atol=1e-1, rtol=1e-3)
    assert torch.allclose(sums[1], (yf * yf).sum(0), atol=1e-1, rtol=1e-3)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_stem_pack_buffer_reuse(dt):
    """The padded stem input buffer kept across steps (_StemPackBuf) gives the same outputs
    and weight gradients as padding anew, across steps with new images, with two forwards
    before their backwards (the busy buffer is not reused) and with the backward on
    another stream."""
    from mpit_amd.ops import conv as C

    torch.manual_seed(3)
    conv = C.StemConv(3, 64, 7, 2, 3).cuda().to(memory_format=torch.channels_last)
    xs = [torch.randn(4, 3, 64, 64, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
          for _ in range(4)]

    def steps(reuse):
        C._StemPackBuf.enabled = reuse
        C._StemPackBuf.bufs.clear()
        out = []
        try:
            for x in xs[:2]:  # one forward + backward per step
                conv.weight.grad = None
                y = conv(x)
                y.float().square().sum().backward()
                out += [y.detach().float().clone(), conv.weight.grad.clone()]
            conv.weight.grad = None  # two forwards, then both backwards
            ya, yb = conv(xs[2]), conv(xs[3])
            (ya.float().square().sum() + yb.float().sum()).backward()
            out += [ya.detach().float().clone(), yb.detach().float().clone(), conv.weight.grad.clone()]
            conv.weight.grad = None  # backward on a side stream, then a forward on the main one
            y = conv(xs[0])
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                y.float().square().sum().backward()
            torch.cuda.current_stream().wait_stream(side)
            y2 = conv(xs[1])
            out += [conv.weight.grad.clone(), y2.detach().float().clone()]
            torch.cuda.synchronize()
            return out
        finally:
            C._StemPackBuf.enabled = True
            C._StemPackBuf.bufs.clear()

    a, b = steps(False), steps(True)
    for i, (u, v) in enumerate(zip(a, b)):
        assert torch.equal(u, v), i


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["randn", "zero", "nchw", "tiny"])
def test_stem_weight_planes_match_torch(case):
    """The one-launch fp16x3 planes of the stem's zero-extended weight image (stem_pack.hip)
    are bitwise the PyTorch-op planes (f16_planes of the packed image under max |w|), bound too."""
    from mpit_amd.ops import conv as C

    torch.manual_seed(11)
    w = torch.randn(64, 3, 7, 7, device="cuda") * 0.05
    if case == "zero":
        w.zero_()
    elif case == "tiny":
        w = w * 2.0 ** -40
    w[5, 1, 3, 2] = -0.9 if case != "zero" else 0.0
    if case != "nchw":
        w = w.contiguous(memory_format=torch.channels_last)
    p, b = C.stem_weight_planes(w)
    wp = torch.zeros(64, 8, 8, 4, device="cuda")
    wp[:, :7, :7, :3] = w.permute(0, 2, 3, 1)
    bref = C.bound_of_value(torch.linalg.vector_norm(w, float("inf")))
    ref = C.f16_planes(wp.reshape(64, -1), bref)
    torch.cuda.synchronize()
    assert torch.equal(b, bref)
    assert torch.equal(p.view(2, 64, -1).view(torch.int16), ref.view(2, 64, -1).view(torch.int16))

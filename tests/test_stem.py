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


def test_stem_emits_bn_stats():
    from mpit_amd.ops.conv import StemConv, tile_stats_to_sums

    conv = StemConv(3, 64, 7, 2, 3).cuda().to(memory_format=torch.channels_last)
    conv.emit_stats = True
    x = torch.randn(2, 3, 64, 64, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = conv(x)
    part, nt, ptr = y._mpit_tstats
    assert ptr == y.data_ptr()
    M = y.shape[0] * y.shape[2] * y.shape[3]
    sums = tile_stats_to_sums(part, M, 64).double()
    yf = y.double().permute(0, 2, 3, 1).reshape(-1, 64)
    assert torch.allclose(sums[0], yf.sum(0), atol=1e-1, rtol=1e-3)
    assert torch.allclose(sums[1], (yf * yf).sum(0), atol=1e-1, rtol=1e-3)

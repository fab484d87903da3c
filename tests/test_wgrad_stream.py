"""Weight gradients on the side stream (ops/conv.py WgradStream) equal the single-stream
ones bit for bit (the trainer path is exercised by bench.py and the GPU tier)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _grads(model, x, y, side):
    from mpit_amd.ops.conv import WgradStream

    WgradStream.enable(side)
    try:
        for p in model.parameters():
            p.grad = None
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = model(x)
        torch.nn.functional.cross_entropy(out.float(), y).backward()
        WgradStream.join()
        torch.cuda.synchronize()
        return [p.grad.clone() for p in model.parameters()]
    finally:
        WgradStream.enable(False)


def test_side_stream_wgrad_matches():
    from mpit_amd.models.resnet import resnet50

    torch.manual_seed(0)
    model = resnet50(num_classes=10).to(memory_format=torch.channels_last).cuda()
    x = torch.randn(8, 3, 64, 64, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device="cuda")
    names = [n for n, _ in model.named_parameters()]
    g0 = _grads(model, x, y, False)
    g1 = _grads(model, x, y, True)
    for n, a, c in zip(names, g0, g1):
        if n == "conv1.weight":  # the 7x7 stem's backward-weight is MIOpen's (atomics): not bitwise
            assert (a - c).abs().max() <= 1e-3 * a.abs().max(), n
        else:
            assert torch.equal(a, c), n


def test_cu_masked_side_stream_wgrad_matches(monkeypatch):
    """The side stream restricted to all but 32 CUs (MPIT_SIDE_CU_RESERVE) changes where the
    weight-gradient GEMMs run, not what they compute."""
    from mpit_amd.models.resnet import resnet50
    from mpit_amd.ops.conv import WgradStream

    torch.manual_seed(0)
    model = resnet50(num_classes=10).to(memory_format=torch.channels_last).cuda()
    x = torch.randn(8, 3, 64, 64, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device="cuda")
    g0 = _grads(model, x, y, False)
    saved = dict(WgradStream._side)
    monkeypatch.setenv("MPIT_SIDE_CU_RESERVE", "32")
    WgradStream._side.clear()
    try:
        g1 = _grads(model, x, y, True)
        assert isinstance(WgradStream._side[0], torch.cuda.ExternalStream)
    finally:
        WgradStream._side.clear()
        WgradStream._side.update(saved)
    for (n, _), a, c in zip(model.named_parameters(), g0, g1):
        if n == "conv1.weight":
            assert (a - c).abs().max() <= 1e-3 * a.abs().max(), n
        else:
            assert torch.equal(a, c), n

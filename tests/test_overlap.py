"""ShardPusher (parallel/overlap.py): shard-by-shard Downpour pushes from inside the
backward. Checked on CPU against the one-shot gather of every gradient, and on the GPU
(real pulls landing mid-backward) against the non-overlapped path, bit for bit."""
import re

import pytest
import torch

from mp_util import run_ranks

from mpit_amd.models import get_model
from mpit_amd.parallel.overlap import ShardPusher
from mpit_amd.parallel.ps import shard_ranges
from mpit_amd.utils.flat import FlatParams


class _FakeClient:
    def __init__(self, plong, nserv):
        self.sranks = list(range(nserv))
        self.sinfo = {s: r for s, r in zip(self.sranks, shard_ranges(plong, nserv))}
        self.entries = [(s, *self.sinfo[s]) for s in self.sranks]
        self.tx = torch.full((plong,), float("nan"))
        self.pushed = []

    def async_send_grad_shard(self, k, pull=False):
        lo, n = self.sinfo[self.sranks[k]]
        assert pull
        # everything this shard carries must already be written
        assert not torch.isnan(self.tx[lo:lo + n]).any() or self._gap(lo, n), k
        self.pushed.append(k)

    def _gap(self, lo, n):
        return False


def _grads_ref(model, x, y):
    model.zero_grad(set_to_none=True)
    torch.manual_seed(1)  # same dropout mask as the pushed pass
    torch.nn.functional.nll_loss(model(x), y).backward()
    return [p.grad.detach().clone() for p in model.parameters()]


def test_shard_pusher_matches_one_shot_gather():
    torch.manual_seed(0)
    model = get_model("cnn7", num_classes=10)
    x, y = torch.randn(4, 3, 28, 28), torch.randint(0, 10, (4,))
    ref = _grads_ref(model, x, y)
    flat = FlatParams(model)
    pc = _FakeClient(flat.numel, 3)
    pc.tx[:] = 0.0  # alignment gaps between parameters are never written
    flat.steal_grads()
    pusher = ShardPusher(flat, pc)
    a = -0.1
    pusher.arm(a)
    torch.manual_seed(1)
    torch.nn.functional.nll_loss(model(x), y).backward()
    pusher.finish()
    assert sorted(pc.pushed) == [0, 1, 2] and len(pc.pushed) == 3
    # the last layers' shard completes first in the backward
    assert pc.pushed[0] == 2, pc.pushed
    for p, off, g in zip(flat.params, flat.offsets, ref):
        torch.testing.assert_close(pc.tx[off:off + p.numel()].view_as(g), a * g)
        assert p.grad is None
    pusher.close()


@pytest.mark.gpu
def test_overlap_equals_non_overlapped_on_gpu_three_ranks():
    """1 worker + 2 dedicated servers on the box's GPU: ResNet-18 Downpour steps with the
    refreshed shards written into the model during the backward give exactly the parameters
    of pushing / pulling after the backward, in fp32 and in bf16 autocast — also with the
    last pulls' wait deferred to the next forward (defer_ps_wait)."""
    out = run_ranks("overlap_equiv.py", 3, {"MPIT_WGRAD_STREAM": "force"}, timeout=400)
    m = re.search(r"RESULT (.*)", out)
    assert m, out[-3000:]
    res = eval(m.group(1))
    assert len(res) == 1, res
    for prec in ("fp32", "bf16", "fp32_defer", "bf16_defer"):
        same, diff = res[0][prec]
        assert same, (prec, diff)


def test_shard_pusher_weight_decay_for_gradientless_params():
    """A parameter without a gradient this step still pushes its weight-decay term
    b*aux (asyncsgd/optim-downpour.lua:24 adds l2wd*w to the whole dfdx)."""
    torch.manual_seed(0)
    model = get_model("cnn7", num_classes=10)
    flat = FlatParams(model)
    pc = _FakeClient(flat.numel, 2)
    pc.tx[:] = 0.0
    flat.steal_grads()
    pusher = ShardPusher(flat, pc)
    aux = torch.randn(flat.numel)
    pusher.arm(-0.1, aux, 0.25)
    frozen = flat.params[0]
    frozen.requires_grad_(False)  # no gradient this step
    x, y = torch.randn(2, 3, 28, 28), torch.randint(0, 10, (2,))
    torch.nn.functional.nll_loss(model(x), y).backward()
    pusher.finish()
    off, n = flat.offsets[0], frozen.numel()
    torch.testing.assert_close(pc.tx[off:off + n], 0.25 * aux[off:off + n])
    frozen.requires_grad_(True)

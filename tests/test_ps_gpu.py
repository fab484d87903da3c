"""Parameter-server ordering on the GPU (the box's one device shared by the ranks)."""
import pytest

from mp_util import run_ranks


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 3])
def test_server_shard_init_ordered_after_fills(n):
    """The shard buffers' fills are ordered before the server's stream uses them: the first
    client's initial push survives a held-back PyTorch stream (round-3 overlap failure)."""
    out = run_ranks("ps_init_order.py", n, timeout=300)
    assert out.count("INIT_EXACT [True, True, True]") == n, out

"""Datapath 3's two-sided data plane (csrc/core/link.h) through the link's self-loop
(MPIT_LINK_SELF=1): a one-rank job routes its own shard through PsLink — on the GPU as grouped
RCCL send / recv to itself on the link stream (a 1-rank communicator), on the CPU through the
host FIFO. Downpour parameters after N steps must equal the local datapath 2 path bit for bit."""
import re

import pytest

from mp_util import run_ranks


def _result(out):
    m = re.search(r"RESULT (.*)", out)
    assert m, out[-3000:]
    return eval(m.group(1))


@pytest.mark.parametrize("rdv", ["0", "1"])
def test_link_self_loop_host_bitwise(rdv):
    res = _result(run_ranks("link_self.py", 1, {"MPIT_LINK_SELF": "1", "MPIT_CPU_ONLY": "1", "MPIT_LINK_RDV": rdv,
                                                "T_MODEL": "cnn7", "T_STEPS": "6", "T_PRECS": "fp32",
                                                "T_PP_MIB": "8", "T_PP_ITERS": "3"}, timeout=300))
    r = res["fp32"]
    assert r["same"] and r["finite"], r
    # every step: one gradient push and one pull per shard crossed the link (plus the init push)
    assert r["link"]["self_mode"] and r["link"]["ordered"] >= 2 * 6, r
    assert res["pingpong"]["aggregate_GBps_bidir"] > 0


@pytest.mark.gpu
def test_link_self_loop_rccl_bitwise_on_gpu():
    """20 ResNet-18 Downpour steps, fp32 and bf16 autocast, over grouped RCCL self send / recv
    (ncclGroupStart/End batches counted), bitwise equal to datapath 2; then the 640 MiB
    ptest.lua ping-pong over the same self-loop."""
    res = _result(run_ranks("link_self.py", 1, {"MPIT_LINK_SELF": "1"}, timeout=600))
    print(res)
    for prec in ("fp32", "bf16"):
        r = res[prec]
        assert r["same"] and r["finite"], (prec, r)
        assert r["link"]["groups"] >= 20 and r["link"]["bytes_recv"] > 0, (prec, r)
    assert res["pingpong"]["aggregate_GBps_bidir"] > 0, res["pingpong"]

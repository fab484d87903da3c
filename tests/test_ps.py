"""Parameter-server end to end: multi-process (gloo/CPU here; HBM + IPC on a GPU box)."""
import re

import pytest

from mp_util import run_ranks


def _result(out):
    m = re.search(r"RESULT (.*)", out)
    assert m, out
    return m.group(1)


@pytest.mark.parametrize("n", [1, 2, 3])
def test_downpour_colocated_cpu(n):
    r = _result(run_ranks("ps_train.py", n, {"MPIT_CPU_ONLY": "1"}))
    cs = eval(re.search(r"checksums=(\[.*?\])", r).group(1))
    # after the final synchronous pull every worker holds the server parameters
    assert max(cs) - min(cs) < 1e-6 * max(1.0, abs(cs[0])), cs


def test_downpour_dedicated_cpu():
    r = _result(run_ranks("ps_train.py", 3, {"MPIT_CPU_ONLY": "1", "T_TOPO": "dedicated"}))
    assert "grads" in r


@pytest.mark.parametrize("opt", ["eamsgd", "msgd"])
def test_other_optimizers_cpu(opt):
    r = _result(run_ranks("ps_train.py", 2, {"MPIT_CPU_ONLY": "1", "T_OPT": opt}))
    assert "loss=" in r


def test_downpour_su2_cpu():
    r = _result(run_ranks("ps_train.py", 2, {"MPIT_CPU_ONLY": "1", "T_SU": "2"}))
    assert "loss=" in r


@pytest.mark.gpu
@pytest.mark.parametrize("dp", [0, 1, 2])
def test_downpour_colocated_gpu_two_ranks_one_device(dp):
    # two ranks share the box's single GPU: exercises HIP IPC windows + fused remote kernels
    r = _result(run_ranks("ps_train.py", 2, {"T_MODEL": "cnn7", "T_DATAPATH": str(dp)}))
    cs = eval(re.search(r"checksums=(\[.*?\])", r).group(1))
    assert max(cs) - min(cs) < 1e-6 * max(1.0, abs(cs[0])), cs


@pytest.mark.parametrize("wire", ["fp32", "bf16"])
def test_sync_allreduce_dp_cpu(wire):
    r = _result(run_ranks("ps_train.py", 3, {"MPIT_CPU_ONLY": "1", "T_OPT": "allreduce", "T_WIRE": wire}))
    cs = eval(re.search(r"checksums=(\[.*?\])", r).group(1))
    # synchronous DP keeps every replica bit-identical (bf16 wire too: all ranks cast back the same sums)
    assert max(cs) == min(cs), cs


def test_baseline_config1_lenet_easgd_dedicated_cpu():
    """BASELINE.json config 1: LeNet EASGD, one dedicated parameter server + one worker, on
    the CPU (asyncsgd/mlaunch.lua's 2-rank layout)."""
    r = _result(run_ranks("ps_train.py", 2, {"MPIT_CPU_ONLY": "1", "T_MODEL": "lenet", "T_OPT": "eamsgd",
                                             "T_TOPO": "dedicated", "T_STEPS": "8"}))
    assert "opt=eamsgd topo=dedicated" in r
    losses = [float(x) for x in re.search(r"losses=\[(.*?)\]", r).group(1).split(",")]
    assert losses[1] == losses[1] and 0 < losses[1] < 10, r  # rank 1 trains
    stats = eval(re.search(r"stats=(\{.*\})", r).group(1))
    assert stats, r  # rank 0 is the dedicated server
    assert stats["grads"] + stats.get("params", 0) >= 1, stats


@pytest.mark.parametrize("rule", ["", "adam"])
def test_split_shard_entries_bitwise_cpu(rule):
    """A shard pushed / pulled as K pieces (bench.py --emulate-shards) gives the same
    parameters, bit for bit, as the whole shard: the pieces apply the same rule to disjoint
    ranges, and a server-side Adam advances its step counter once per push."""
    bits = []
    for k in (1, 3):
        r = _result(run_ranks("ps_train.py", 1, {"MPIT_CPU_ONLY": "1", "T_SPS": str(k), "T_RULE": rule}))
        bits.append(int(re.search(r"bits=(-?\d+)", r).group(1)))
    assert bits[0] == bits[1], bits


def test_split_shard_entries_two_ranks_cpu():
    r = _result(run_ranks("ps_train.py", 2, {"MPIT_CPU_ONLY": "1", "T_SPS": "4"}))
    cs = eval(re.search(r"checksums=(\[.*?\])", r).group(1))
    assert max(cs) - min(cs) < 1e-6 * max(1.0, abs(cs[0])), cs


@pytest.mark.gpu
def test_batched_server_updates_bitwise_gpu():
    """HBM server, its co-located client pushing 4 pieces per step: the pieces a progress
    sweep finds queued are applied by ONE multi-segment launch (PSServer::flush_grads); the
    parameters equal the one-launch-per-piece server's (MPIT_PS_BATCH=0) bit for bit."""
    res = []
    for b in ("1", "0"):
        r = _result(run_ranks("ps_batch.py", 1, {"MPIT_PS_BATCH": b}))
        res.append((int(re.search(r"bits=(-?\d+)", r).group(1)), eval(re.search(r"stats=(\{.*\})", r).group(1))))
    assert res[0][0] == res[1][0], res
    assert res[1][1].get("batches", 0) == 0 and res[0][1].get("batches", 0) >= 1, res


# ---- datapath 3: shard data as two-sided messages (csrc/core/link.h); on CPU ranks the
# engine's tagged host messages stand in for RCCL (same op order per (client, server) pair)

@pytest.mark.parametrize("n", [3, 8])
def test_datapath3_colocated_exact_sums(n):
    """n co-located ranks (8 = the N=8 node layout): pushes with pulls and plain pulls
    interleaved, deadlock-free; every worker's final pull equals the closed form, as with
    the one-sided datapath 0."""
    out = run_ranks("ps_link.py", n, {"MPIT_CPU_ONLY": "1", "T_CASE": "sum"}, timeout=300)
    assert out.count("equal={3: True, 0: True}") == n, out


def test_datapath3_trainer_bitwise_equals_datapath0():
    """1 worker + 2 dedicated servers: Downpour through the message data plane gives exactly
    the parameters of the one-sided data plane, and the servers' shards agree (verify_ps)."""
    out = run_ranks("ps_link.py", 3, {"MPIT_CPU_ONLY": "1", "T_CASE": "train", "T_SERVERS": "2"}, timeout=300)
    assert "same=True" in out and out.count("ok={3: True, 0: True}") == 3, out


def test_datapath3_one_server_seven_workers():
    """BASELINE config 2's layout (1 pserver + 7 workers) on the message data plane."""
    out = run_ranks("ps_link.py", 8, {"MPIT_CPU_ONLY": "1", "T_CASE": "train", "T_SERVERS": "1"}, timeout=300)
    assert out.count("ok={3: True, 0: True}") == 8, out


def test_datapath3_bounded_staleness():
    out = run_ranks("ssp_check.py", 3, {"MPIT_CPU_ONLY": "1", "T_DATAPATH": "3"})
    assert "SSP_OK" in out and "SSP_PULL_OK" in out, out


# ---- datapath 3 under blocking rendezvous semantics (MPIT_LINK_RDV=1): one FIFO per rank, a
# send completes only against a receive at the head of the peer's FIFO (an RCCL pair at the
# head of a hardware queue). 200 steps of randomised control-message timing each.

_RDV = {"MPIT_CPU_ONLY": "1", "MPIT_LINK_RDV": "1", "MPIT_LINK_JITTER_US": "300", "T_STEPS": "200"}


@pytest.mark.parametrize("stale", ["-1", "0"])
def test_datapath3_rendezvous_colocated_8(stale):
    """8 co-located ranks (worker + shard server each), random shard order per push, random
    timing, plain async and SSP (deferred pulls released by other clients' pushes): every
    step completes and the final shards equal the closed form."""
    out = run_ranks("ps_link_rdv.py", 8, dict(_RDV, T_TOPO="colocated", T_STALE=stale, MPIT_PS_TIMEOUT_S="60"),
                    timeout=300)
    assert out.count("RESULT RDV_OK") == 8, out


def test_datapath3_rendezvous_one_server_seven_workers():
    out = run_ranks("ps_link_rdv.py", 8, dict(_RDV, T_TOPO="dedicated", MPIT_PS_TIMEOUT_S="60"), timeout=300)
    assert out.count("RESULT RDV_OK") == 8, out


def test_datapath3_pre_sequencer_layout_deadlocks():
    """The layout before the sequencer (each client queues its ops when it sends its control
    message, each server when the message arrives; all on one FIFO per rank) deadlocks under
    the same blocking semantics: the clients' finite wait reports it."""
    # (the deadlock needs an unlucky arrival order; 1,000 random steps make one all but certain,
    # and the run ends at the first one)
    out = run_ranks("ps_link_rdv.py", 8, dict(_RDV, T_TOPO="colocated", MPIT_LINK_LEGACY="1", MPIT_PS_TIMEOUT_S="6",
                                              T_STEPS="1000"), timeout=300)
    assert "RESULT RDV_TIMEOUT" in out and "RESULT RDV_OK" not in out, out


def test_bucketed_allreduce_equals_one_bucket_training_two_ranks():
    """Sync DP with many buckets (non-blocking all-reduces launched from the backward) ends
    bit-identical to one bucket: 2 ranks, CNN-7, 4 steps (a two-term sum is order-free)."""
    res = eval(_result(run_ranks("ddp_bucket_equiv.py", 2, {"MPIT_CPU_ONLY": "1", "T_TRAIN": "1"}, timeout=300)))
    for rr in res:
        assert rr["train"]["same"], rr
        assert rr["train"]["buckets"][0] > 3 and rr["train"]["buckets"][1] == 1, rr
        assert rr["exact"]["same"] and rr["exact"]["exact"], rr


@pytest.mark.parametrize("n", [3, 4])
def test_bucketed_allreduce_exact_sums(n):
    """3-4 ranks: exactly representable gradients through tiny buckets and one bucket give
    the exact sum bit for bit (every element reduced once, whatever the bucket layout)."""
    res = eval(_result(run_ranks("ddp_bucket_equiv.py", n, {"MPIT_CPU_ONLY": "1"}, timeout=300)))
    assert len(res) == n
    for rr in res:
        assert rr["exact"]["same"] and rr["exact"]["exact"] and rr["exact"]["buckets"][0] > 3, rr


@pytest.mark.gpu
def test_allreduce_steal_machinery_bitwise_on_gpu():
    """BASELINE config 3 on the PS path's machinery (train.py ar_steal) == the plain path."""
    res = eval(_result(run_ranks("ar_steal_equiv.py", 1, {}, timeout=400)))
    for prec, (same, diff) in res.items():
        assert same, (prec, diff)

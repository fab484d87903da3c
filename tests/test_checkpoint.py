"""Checkpoint / resume of the whole job (workers + parameter-server shards + server
optimizer state + RNG): 6 steps == 3 steps + save + restart + load + 3 steps, bit for bit
(tests/mp/ckpt_resume.py). The reference never checkpoints servers."""
import re

import pytest

from mp_util import run_ranks


def _res(out):
    m = re.search(r"RESULT (.*)", out)
    assert m, out[-3000:]
    return eval(m.group(1))


@pytest.mark.parametrize("opt", ["downpour", "eamsgd", "adam"])
def test_resume_bitwise_dedicated_server_cpu(opt):
    res = _res(run_ranks("ckpt_resume.py", 2, {"MPIT_CPU_ONLY": "1", "T_OPT": opt, "T_TOPO": "dedicated"}))
    assert res[0]["server_equal"] and res[1]["worker_equal"], res


def test_resume_bitwise_colocated_cpu():
    # one rank serving its own shard (with two asynchronous workers the arrival order of
    # their pushes differs from run to run, checkpoint or not)
    res = _res(run_ranks("ckpt_resume.py", 1, {"MPIT_CPU_ONLY": "1", "T_OPT": "downpour", "T_TOPO": "colocated"}))
    for r in res:
        assert r["worker_equal"] and r["server_equal"], res


@pytest.mark.gpu
def test_resume_bitwise_gpu_two_ranks_one_device():
    res = _res(run_ranks("ckpt_resume.py", 2, {"T_OPT": "downpour", "T_TOPO": "dedicated"}))
    assert res[0]["server_equal"] and res[1]["worker_equal"], res


def test_eamsgd_in_flight_push_retired_three_ranks_cpu():
    """verify_ps / save_checkpoint retire EAMSGD's outstanding push first."""
    res = _res(run_ranks("eamsgd_verify.py", 3, {"MPIT_CPU_ONLY": "1"}))
    for r in res:
        assert all(r["oks"]) and r["final"], res

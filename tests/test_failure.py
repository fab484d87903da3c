"""Failure detection: a rank that dies without Finalize makes the survivors abort
instead of blocking forever (the reference has no failure detection)."""
import os
import subprocess
import sys

from mp_util import ROOT, free_port


def test_peer_crash_aborts_the_job():
    port = free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), MPIT_CPU_ONLY="1", PYTHONPATH=ROOT)
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "mp", "crash_peer.py")], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = [p.communicate(timeout=120)[0] for p in procs]
    assert procs[1].returncode == 9
    assert procs[0].returncode == 70, outs[0]
    assert "peer rank 1" in outs[0] and "should not get here" not in outs[0]


def _run_fault(env_extra, n=3, timeout=90):
    import time

    port = free_port()
    procs = []
    t0 = time.time()
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), MPIT_CPU_ONLY="1", PYTHONPATH=ROOT, **env_extra)
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "mp", "ps_fault.py")], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=timeout)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise AssertionError("a rank hung after a server fault")
    return [p.returncode for p in procs], outs, time.time() - t0


def test_server_fault_aborts_every_rank():
    """A failing server handler (injected HIP-style error in the update) ends the whole
    job: the failing rank exits 71 with the reason, every other rank exits 71 printing
    the same reason, nobody prints past the training loop."""
    rcs, outs, dt = _run_fault({"MPIT_PS_FAULT": "grad:3", "MPIT_PS_FAULT_RANK": "1"})
    assert all(rc == 71 for rc in rcs), (rcs, outs)
    assert "fatal: active-message handler" in outs[1] and "injected fault" in outs[1], outs[1]
    for r in (0, 2):
        assert "job aborted by rank 1 (code 71)" in outs[r] and "injected fault" in outs[r], outs[r]
    assert not any("should not get here" in o for o in outs)


def test_stuck_server_times_out():
    """A server that silently stops answering (drops pushes) trips the clients' PS wait
    deadline: the waiting rank raises with what is missing, the job ends non-zero."""
    rcs, outs, dt = _run_fault({"MPIT_PS_FAULT": "drop:4", "MPIT_PS_FAULT_RANK": "0", "MPIT_PS_TIMEOUT_S": "3"})
    assert all(rc != 0 for rc in rcs), (rcs, outs)
    assert any("MPIT_PS_TIMEOUT_S" in o for o in outs), outs
    assert not any("should not get here" in o for o in outs)
    assert dt < 60, dt


def _run_barrier_sleep(env_extra, n=2, timeout=90):
    port = free_port()
    procs = []
    for r in range(n):
        env = {k: v for k, v in os.environ.items() if k != "MPIT_WAIT_TIMEOUT_S"}
        env.update(RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), MPIT_CPU_ONLY="1", PYTHONPATH=ROOT, **env_extra)
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "mp", "barrier_sleep.py")], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = [p.communicate(timeout=timeout)[0] for p in procs]
    return [p.returncode for p in procs], outs


def test_long_barrier_has_no_default_deadline():
    """a rank legitimately waiting in Barrier longer than any deadline must
    not kill the job by default (MPI blocks without one); the deadline is opt-in."""
    rcs, outs = _run_barrier_sleep({"T_SLEEP": "4"})
    assert rcs == [0, 0], (rcs, outs)
    assert all("barrier passed" in o for o in outs), outs
    rcs, outs = _run_barrier_sleep({"T_SLEEP": "6", "MPIT_WAIT_TIMEOUT_S": "1"})
    assert rcs[0] != 0 and "MPIT_WAIT_TIMEOUT_S" in outs[0], (rcs, outs)


def test_preflight_names_the_broken_pair():
    """Verdict r03 #5: the pre-timing check pulls every shard once and names the (worker,
    server) pair whose pulled bits differ from the server's; a healthy job reports ok."""
    import re

    from mp_util import run_ranks

    out = run_ranks("preflight_check.py", 3, {"MPIT_CPU_ONLY": "1"}, timeout=240)
    rep = eval(re.search(r"PREFLIGHT (.*)", out).group(1))
    assert rep["ok"] and rep["mismatches"] == [] and rep["shards"] == 3 and rep["workers"] == 3, rep
    out = run_ranks("preflight_check.py", 3, {"MPIT_CPU_ONLY": "1", "MPIT_PS_FAULT": "badpull",
                                              "MPIT_PS_FAULT_RANK": "1", "MPIT_PS_FAULT_CLIENT": "2"}, timeout=240)
    rep = eval(re.search(r"PREFLIGHT (.*)", out).group(1))
    assert not rep["ok"] and rep["mismatches"] == [[2, 1]], rep

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

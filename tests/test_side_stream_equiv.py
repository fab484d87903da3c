"""Downpour training with the side-stream backward (ops/conv.py WgradStream) reaches the
same parameters, bit for bit, as the single-stream step (scripts/ws_equiv.py, run in two
child processes: the runtime is initialised once per process)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(flag):
    env = dict(os.environ, MPIT_WGRAD_STREAM=flag)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "ws_equiv.py")], env=env,
                         capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("side=")][-1]
    return line.split(" ", 1)


def test_side_stream_training_is_bitwise_identical():
    s0, r0 = _run("0")
    s1, r1 = _run("1")
    assert (s0, s1) == ("side=False", "side=True")
    assert r0 == r1

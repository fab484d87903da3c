"""The precast of the next step's weight casts (mpit_amd/train.py Trainer._precast_next: queued
when step() returns in Downpour su = 1) trains to the same parameters, bit for bit, as casting
at the start of each step (scripts/ws_equiv.py in two child processes, MPIT_PRECAST=0 / 1)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(flag):
    env = dict(os.environ, MPIT_PRECAST=flag)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "ws_equiv.py")], env=env,
                         capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("side=")][-1]
    return line.split(" ", 1)[1]


def test_precast_training_is_bitwise_identical():
    assert _run("0") == _run("1")


_INVALIDATE = """
import mpit_amd as mp
from mpit_amd.train import TrainConfig, Trainer
mp.Init()
tr = Trainer(TrainConfig(model="resnet18", batch=8, num_classes=10, lr=0.0))
tr.step()
states = [tr._precast_ok, tr._precast]
tr.invalidate_precast()
states += [tr._precast, tr.wcast.valid]
tr.step()  # casts anew at the forward, then precasts again
states.append(tr._precast)
print("STATES", states, flush=True)
tr.stop()
mp.Finalize()
"""


def test_precast_invalidated_when_weights_change():
    """After invalidate_precast() (what load_checkpoint / set_amp / verify_ps call when the
    weights are written between steps) the next step casts anew; step() precasts again."""
    out = subprocess.run([sys.executable, "-c", _INVALIDATE], env=dict(os.environ, PYTHONPATH=ROOT),
                         capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("STATES")][-1]
    assert line == "STATES [True, True, False, False, True]", line

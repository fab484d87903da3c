"""Stream hygiene of the trainer step: autograd must never find an
AccumulateGrad node made on another stream than the step's (a graph edge kept alive from
model build time), which would insert cross-stream waits and run the push hooks on the
default stream. The warning fires once per process, so the check runs in a fresh one."""
import json
import os
import subprocess
import sys

import pytest

from mp_util import ROOT


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["default", "bf16"])
def test_no_accumulate_grad_stream_mismatch(variant):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "benchmarks", "diag_accgrad.py"), variant],
                       capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    assert json.loads(line)["warnings_per_step"] == [0, 0, 0, 0], line

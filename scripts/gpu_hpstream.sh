#!/bin/bash
# High-priority critical-path stream (MPIT_HP_STREAM): trainer GPU tests, then bench A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/hp
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_side_stream_equiv.py tests/test_overlap.py tests/test_checkpoint.py tests/test_ps.py tests/test_wgrad_stream.py -m gpu -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1; rc=$?
tail -3 $D/pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do for h in 0 1; do
  MPIT_HP_STREAM=$h timeout -k 10 300 python -u bench.py > $D/b_${h}_$i.log 2>&1 || { tail -20 $D/b_${h}_$i.log; exit 1; }
  echo "hp=$h run=$i $(tail -1 $D/b_${h}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["secondary"]["bf16_autocast"]["value"])')"
done; done

#!/bin/bash
# MPIT_TN_OCC=1 (one backward-weight GEMM block per CU): wgrad numerics under the knob, then
# a same-box bench A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/tnocc
mkdir -p $D
MPIT_TN_OCC=1 timeout -k 10 300 python3 -u -m pytest tests/test_gemm.py tests/test_fp32_path.py -m gpu -q -x -k "tn or wgrad" --timeout 120 --timeout-method thread > $D/pytest.log 2>&1; rc=$?
tail -3 $D/pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do for o in 0 1; do
  MPIT_TN_OCC=$o timeout -k 10 300 python3 -u bench.py > $D/b_${o}_$i.log 2>&1 || { tail -20 $D/b_${o}_$i.log; exit 1; }
  echo "occ=$o run=$i $(tail -1 $D/b_${o}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["secondary"]["bf16_autocast"]["value"])')"
done; done

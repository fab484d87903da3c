#!/bin/bash
# A/B: fewer backward-weight splits (longer side-stream blocks, less partial traffic), MPIT_TN_SPLIT_DIV=1/2/4
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/splitmul
mkdir -p $D
MPIT_TN_SPLIT_DIV=4 timeout -k 10 300 python3 -u -m pytest tests/test_gemm.py -m gpu -q -x -k "tn" --timeout 120 --timeout-method thread > $D/pytest.log 2>&1; rc=$?
tail -2 $D/pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do for k in 1 2 4; do export MPIT_TN_SPLIT_DIV=$k;
  timeout -k 10 300 python3 -u bench.py > $D/b_${k}_$i.log 2>&1 || { tail -20 $D/b_${k}_$i.log; exit 1; }
  echo "div=$k run=$i $(tail -1 $D/b_${k}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["secondary"]["bf16_autocast"]["value"])')"
done; done

#!/bin/bash
# BN backward finalize folded into the backward-data GEMM: numerics tests, then a same-box
# bench A/B (MPIT_BN_FOLD=0 = separate finalize launch).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/bnfold
mkdir -p $D
timeout -k 10 600 python3 -u -m pytest tests/test_resnet_fused.py tests/test_bn_act.py tests/test_fp32_path.py tests/test_side_stream_equiv.py -m gpu -x -v --timeout 200 --timeout-method thread > $D/pytest.log 2>&1; rc=$?
grep -E "passed|failed|FAIL|Error" $D/pytest.log | tail -8; [ $rc -ne 0 ] && { tail -40 $D/pytest.log; exit $rc; }
for i in 1 2; do for f in 0 1; do
  MPIT_BN_FOLD=$f timeout -k 10 300 python3 -u bench.py > $D/b_${f}_$i.log 2>&1 || { tail -20 $D/b_${f}_$i.log; exit 1; }
  echo "fold=$f run=$i $(tail -1 $D/b_${f}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["secondary"]["bf16_autocast"]["value"], d["ps_check"]["ok"])')"
done; done

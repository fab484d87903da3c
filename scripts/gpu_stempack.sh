#!/bin/bash
# stem pack buffer reuse: tests, then same-box bench A/B (MPIT_STEM_PACK_REUSE)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/stempack
mkdir -p $D
timeout -k 10 400 python3 -u -m pytest tests/test_stem.py tests/test_resnet_fused.py tests/test_fp32_path.py -m gpu -q -x --timeout 250 --timeout-method thread > $D/pytest.log 2>&1; rc=$?
tail -2 $D/pytest.log; [ $rc -ne 0 ] && { tail -30 $D/pytest.log; exit $rc; }
for i in 1 2; do for r in 0 1; do
  MPIT_STEM_PACK_REUSE=$r timeout -k 10 300 python3 -u bench.py > $D/b_${r}_$i.log 2>&1 || { tail -20 $D/b_${r}_$i.log; exit 1; }
  echo "reuse=$r run=$i $(tail -1 $D/b_${r}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["secondary"]["bf16_autocast"]["value"], d["ps_check"]["ok"])')"
done; done

#!/bin/bash
# bn_tiles_finalize block width (MPIT_BN_FIN_LANES 4 vs 16): BN tests, then bench A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/finl
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_bn_act.py tests/test_resnet_fused.py tests/test_fp32_path.py -m gpu -q --timeout 200 --timeout-method thread > $D/pytest.log 2>&1; rc=$?
tail -2 $D/pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do for l in 16 4; do
  MPIT_BN_FIN_LANES=$l timeout -k 10 300 python -u bench.py > $D/b_${l}_$i.log 2>&1 || { tail -20 $D/b_${l}_$i.log; exit 1; }
  echo "lanes=$l run=$i $(tail -1 $D/b_${l}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["secondary"]["bf16_autocast"]["value"])')"
done; done

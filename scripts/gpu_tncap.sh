#!/bin/bash
# A/B: fp32 gemm_tn capped at 224 VGPRs (ab/_mpit_tncap.so, a few spills) so BN kernels
# (<= 64 VGPRs) can co-reside with two GEMM blocks per CU, vs the default build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/tncap
mkdir -p $D
MPIT_NATIVE_SO=ab/_mpit_tncap.so timeout -k 10 300 python3 -u -m pytest tests/test_gemm.py tests/test_fp32_path.py -m gpu -q -x -k "tn or wgrad" --timeout 120 --timeout-method thread > $D/pytest.log 2>&1; rc=$?
tail -2 $D/pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do for v in def cap; do
  if [ $v = cap ]; then export MPIT_NATIVE_SO=ab/_mpit_tncap.so; else unset MPIT_NATIVE_SO; fi
  timeout -k 10 300 python3 -u bench.py > $D/b_${v}_$i.log 2>&1 || { tail -20 $D/b_${v}_$i.log; exit 1; }
  echo "$v run=$i $(tail -1 $D/b_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["secondary"]["bf16_autocast"]["value"])')"
done; done

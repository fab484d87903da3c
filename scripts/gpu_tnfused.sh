#!/bin/bash
# In-kernel split reduction of gemm_tn: bitwise test vs split_reduce, wgrad probes, benches.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/tnfused
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gemm.py -m gpu -q -k "tn" --timeout 300 --timeout-method thread > $D/pytest.log 2>&1; rc=$?
tail -3 $D/pytest.log; [ $rc -ge 124 ] && exit $rc; [ $rc -ne 0 ] && exit $rc
P=benchmarks/gemm_probe.py
: > $D/sweep.jsonl
for f in 0 1; do for a in "--f32 wgrad 256 56 56 64 64 3 1" "--f32 wgrad 256 14 14 256 256 3 1" "--f32 tn 50176 512 2048" \
         "wgrad 256 56 56 64 64 3 1" "tn 802816 64 256"; do
  MPIT_TN_FUSED=$f timeout -k 10 60 python3 $P $a 20 | sed "s/^{/{\"fused\": $f, /" >> $D/sweep.jsonl || exit 1
done; done
cat $D/sweep.jsonl
for i in 1 2; do for f in 0 1; do
  MPIT_TN_FUSED=$f timeout -k 10 300 python -u bench.py > $D/b_${f}_$i.log 2>&1 || { tail -20 $D/b_${f}_$i.log; exit 1; }
  echo "fused=$f run=$i $(tail -1 $D/b_${f}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["secondary"]["bf16_autocast"]["value"])')"
done; done

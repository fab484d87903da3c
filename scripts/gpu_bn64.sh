#!/bin/bash
# fp32 gemm_nt 128x128 (2 blocks/CU) vs 128x64 (3 blocks/CU, MPIT_F32_BN64=1): probes + bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/bn64
mkdir -p $D
MPIT_F32_BN64=1 timeout -k 10 300 python -u -m pytest tests/test_fp32_path.py -m gpu -q --timeout 120 --timeout-method thread > $D/pytest.log 2>&1; rc=$?
tail -1 $D/pytest.log; [ $rc -ge 124 ] && exit $rc
P=benchmarks/gemm_probe.py
: > $D/sweep.jsonl
for v in 0 1; do
for a in "nt 802816 256 64" "nt 200704 512 128" "nt 50176 2048 512" "nt 50176 256 1024" \
         "conv 256 56 56 64 64 3 1" "conv 256 28 28 128 128 3 1" "conv 256 14 14 256 256 3 1" "dgrad 256 14 14 256 256 3 1"; do
  MPIT_F32_BN64=$v timeout -k 10 60 python3 $P --f32 $a 20 | sed "s/^{/{\"bn64\": $v, /" >> $D/sweep.jsonl || exit 1
done; done
cat $D/sweep.jsonl
: > $D/ab.txt
for i in 1 2; do for v in 0 1; do
  MPIT_F32_BN64=$v timeout -k 10 300 python -u bench.py --no-secondary > $D/b_${v}_$i.log 2>&1 || { tail -20 $D/b_${v}_$i.log; exit 1; }
  echo "bn64=$v run=$i $(tail -1 $D/b_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $D/ab.txt
done; done

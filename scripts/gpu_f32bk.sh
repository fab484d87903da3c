#!/bin/bash
# fp32 bf16x6 gemm_nt: 16-deep (default) vs 32-deep k-tiles (MPIT_F32_BK=32, 2 or 3 stages).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/f32bk
mkdir -p $D
MPIT_F32_BK=32 timeout -k 10 300 python -u -m pytest tests/test_fp32_path.py -m gpu -v --timeout 120 --timeout-method thread > $D/pytest_bk32.log 2>&1; rc=$?
grep -E "passed|failed" $D/pytest_bk32.log | tail -2; [ $rc -ge 124 ] && exit $rc
P=benchmarks/gemm_probe.py
: > $D/sweep.jsonl
for cfg in "16 0" "32 2" "32 3"; do set -- $cfg
for a in "nt 8192 8192 8192" "nt 200704 512 128" "nt 50176 2048 512" \
         "conv 256 56 56 64 64 3 1" "conv 256 28 28 128 128 3 1" "conv 256 14 14 256 256 3 1" "dgrad 256 14 14 256 256 3 1"; do
  if [ $2 = 0 ]; then MPIT_F32_BK=$1 timeout -k 10 60 python3 $P --f32 $a 20 | sed "s/^{/{\"bk\": $1, \"st\": $2, /" >> $D/sweep.jsonl || exit 1
  else MPIT_F32_BK=$1 MPIT_F32_STAGES=$2 timeout -k 10 60 python3 $P --f32 $a 20 | sed "s/^{/{\"bk\": $1, \"st\": $2, /" >> $D/sweep.jsonl || exit 1; fi
done; done
cat $D/sweep.jsonl
MPIT_F32_BK=32 timeout -k 10 300 python -u bench.py --no-secondary > $D/bench_bk32.log 2>&1 || { tail -30 $D/bench_bk32.log; exit 1; }
tail -1 $D/bench_bk32.log

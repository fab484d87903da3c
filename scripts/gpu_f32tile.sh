#!/bin/bash
# fp32 bf16x6 gemm_nt variants: accumulators (dual / single) x tile (128x128 / 256x128).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/f32tile
mkdir -p $D
MPIT_F32_ACC=single MPIT_F32_TILE=256x128 timeout -k 10 300 python -u -m pytest tests/test_fp32_path.py -m gpu -v --timeout 120 --timeout-method thread > $D/pytest.log 2>&1; rc=$?
grep -E "passed|failed" $D/pytest.log | tail -2; [ $rc -ge 124 ] && exit $rc
P=benchmarks/gemm_probe.py
: > $D/sweep.jsonl
for cfg in "dual 128" "single 128" "dual 256x128" "single 256x128"; do set -- $cfg
for a in "nt 8192 8192 8192" "nt 200704 512 128" "nt 50176 2048 512" \
         "conv 256 56 56 64 64 3 1" "conv 256 28 28 128 128 3 1" "conv 256 14 14 256 256 3 1" "dgrad 256 14 14 256 256 3 1"; do
  MPIT_F32_ACC=$1 MPIT_F32_TILE=$2 timeout -k 10 60 python3 $P --f32 $a 20 | sed "s/^{/{\"acc\": \"$1\", \"tile\": \"$2\", /" >> $D/sweep.jsonl || exit 1
done; done
cat $D/sweep.jsonl
for cfg in "single 128" "single 256x128"; do set -- $cfg
MPIT_F32_ACC=$1 MPIT_F32_TILE=$2 timeout -k 10 300 python -u bench.py --no-secondary > $D/bench_$1_$2.log 2>&1 || { tail -30 $D/bench_$1_$2.log; exit 1; }
echo "$cfg $(tail -1 $D/bench_$1_$2.log | cut -c1-200)"
done

#!/bin/bash
# bf16x6 fp32 GEMMs after a kernel change: numerics tests, shape sweep, fp32 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/${X3_TAG:-x3b}
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_fp32_path.py -m gpu -v --timeout 120 --timeout-method thread > $D/pytest.log 2>&1; rc=$?
grep -E "passed|failed" $D/pytest.log | tail -2; [ $rc -ge 124 ] && exit $rc
P=benchmarks/gemm_probe.py
: > $D/sweep.jsonl
for a in "nt 8192 8192 8192" "nt 200704 512 128" "nt 50176 2048 512" "tn 50176 512 2048" \
         "conv 256 56 56 64 64 3 1" "conv 256 28 28 128 128 3 1" "conv 256 14 14 256 256 3 1" "dgrad 256 14 14 256 256 3 1" \
         "wgrad 256 56 56 64 64 3 1" "wgrad 256 28 28 128 128 3 1" "wgrad 256 14 14 256 256 3 1"; do
  timeout -k 10 60 python3 $P --f32 $a 20 >> $D/sweep.jsonl || exit 1
done
cat $D/sweep.jsonl
timeout -k 10 300 python -u bench.py --no-secondary > $D/bench.log 2>&1 || { tail -30 $D/bench.log; exit 1; }
tail -1 $D/bench.log

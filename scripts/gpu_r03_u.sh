#!/bin/bash
# Round 3 (session 2): fp16x3 split products (FM 11) — fp32 numerics tier, then the bench
# A/B against the bf16x6 kernels (MPIT_F32_SPLIT=bf16x6), then the whole GPU tier.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03u
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fp32_path.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_fp32.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/pytest_fp32.log | tail -15; [ $rc -ne 0 ] && exit 1
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
echo "f16x3: $(tail -1 $O/bench.json | cut -c1-300)"
MPIT_F32_SPLIT=bf16x6 timeout -k 10 300 python -u bench.py --no-secondary > $O/bench_b6.json 2> $O/bench_b6.err || { tail -30 $O/bench_b6.err; exit 1; }
echo "bf16x6: $(tail -1 $O/bench_b6.json | cut -c1-300)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest_gpu.log | head; exit 1; }
echo ALL OK

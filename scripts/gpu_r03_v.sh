#!/bin/bash
# Round 3 (session 2): fp16x3 (FM 11) bench A/B against the bf16x6 kernels, the two plan tests,
# then the whole GPU tier.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03v
mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
echo "f16x3: $(tail -1 $O/bench.json | cut -c1-300)"
MPIT_F32_SPLIT=bf16x6 timeout -k 10 300 python -u bench.py --no-secondary > $O/bench_b6.json 2> $O/bench_b6.err || { tail -30 $O/bench_b6.err; exit 1; }
echo "bf16x6: $(tail -1 $O/bench_b6.json | cut -c1-300)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest_gpu.log | head; exit 1; }
echo ALL OK

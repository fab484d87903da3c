#!/bin/bash
# Full GPU test tier (what the driver runs at round end) + the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { grep -E "PASS|FAIL" gpurun_out/pytest_gpu.log | tail -5; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1 || { tail -30 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log

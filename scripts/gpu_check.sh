#!/bin/bash
# One GPU-box session: gpu tests, N=1 bench, steady-state kernel profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err || { tail -30 gpurun_out/bench_n1.err; exit 1; }
cat gpurun_out/bench_n1.json
if [ "${CONVB:-0}" = 1 ]; then
  timeout -k 10 400 python -u benchmarks/conv_vs_gemm.py 256 > gpurun_out/conv_bench.jsonl 2> gpurun_out/conv_bench.err || { tail -30 gpurun_out/conv_bench.err; exit 1; }
  tail -1 gpurun_out/conv_bench.jsonl
fi
if [ "${PROFILE:-1}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --gpus 1 --steps 6 --warmup 3 > gpurun_out/prof.log 2>&1 || { tail -30 gpurun_out/prof.log; exit 1; }
  echo prof done
fi

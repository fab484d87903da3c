#!/bin/bash
# conv kernels: numerics, per-shape timing vs MIOpen, end-to-end bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gemm.log 2>&1 || { tail -40 gpurun_out/pytest_gemm.log; exit 1; }
tail -3 gpurun_out/pytest_gemm.log
timeout -k 10 400 python -u benchmarks/conv_vs_gemm.py 256 > gpurun_out/conv_bench.jsonl 2> gpurun_out/conv_bench.err || { tail -30 gpurun_out/conv_bench.err; exit 1; }
tail -1 gpurun_out/conv_bench.jsonl
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err || { tail -30 gpurun_out/bench_n1.err; exit 1; }
cat gpurun_out/bench_n1.json

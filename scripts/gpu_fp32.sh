#!/bin/bash
# fp32 MFMA path: numerics tests, the bf16 regression tests on the shared kernels, then the
# fp32 ResNet-50 bench step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_fp32_path.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_fp32only.log 2>&1; grep -E "PASS|FAIL|Error|assert" gpurun_out/pytest_fp32only.log | tail -40; timeout -k 10 400 python -u -m pytest tests/test_gemm.py tests/test_bn_act.py tests/test_pool.py tests/test_stem.py tests/test_resnet_fused.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_fp32.log 2>&1 || { tail -60 gpurun_out/pytest_fp32.log; exit 1; }
tail -3 gpurun_out/pytest_fp32.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 10 --warmup 3 --no-amp > gpurun_out/bench_fp32.log 2>&1 || { tail -30 gpurun_out/bench_fp32.log; exit 1; }
tail -1 gpurun_out/bench_fp32.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/bench_bf16.log 2>&1 || { tail -30 gpurun_out/bench_bf16.log; exit 1; }
tail -1 gpurun_out/bench_bf16.log

#!/bin/bash
# Comparator runs: ResNet-50 step on stock PyTorch fp32 (MIOpen convs, --no-amp) and the
# current bf16 headline, same box, one after the other.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --gpus 1 --steps 10 --warmup 3 --no-amp > gpurun_out/base_fp32_miopen.log 2>&1 || { tail -30 gpurun_out/base_fp32_miopen.log; exit 1; }
tail -1 gpurun_out/base_fp32_miopen.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/base_bf16.log 2>&1 || { tail -30 gpurun_out/base_bf16.log; exit 1; }
tail -1 gpurun_out/base_bf16.log

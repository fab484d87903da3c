#!/bin/bash
# bf16x6 fp32 GEMMs: numerics tests, shape sweep (split vs native fp32 MFMA), fp32 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/x3
timeout -k 10 300 python -u -m pytest tests/test_fp32_path.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/x3/pytest.log 2>&1; grep -E "PASS|FAIL|Error|assert" gpurun_out/x3/pytest.log | tail -40
P=benchmarks/gemm_probe.py
: > gpurun_out/x3/sweep.jsonl
for mode in x3; do
for a in "nt 8192 8192 8192" "nt 802816 64 256" "nt 50176 2048 512" "tn 50176 512 2048" \
         "conv 256 56 56 64 64 3 1" "conv 256 14 14 256 256 3 1" "dgrad 256 14 14 256 256 3 1" \
         "wgrad 256 56 56 64 64 3 1" "wgrad 256 14 14 256 256 3 1"; do
  MPIT_F32_MFMA=$mode timeout -k 10 60 python3 $P --f32 $a 20 | sed "s/^{/{\"mode\": \"$mode\", /" >> gpurun_out/x3/sweep.jsonl || exit 1
done; done
cat gpurun_out/x3/sweep.jsonl
timeout -k 10 300 python -u bench.py --no-secondary > gpurun_out/x3/bench.log 2>&1 || { tail -30 gpurun_out/x3/bench.log; exit 1; }
tail -1 gpurun_out/x3/bench.log

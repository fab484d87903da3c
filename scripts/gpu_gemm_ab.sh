#!/bin/bash
# A/B of GEMM tile shapes (MPIT_GEMM_BM) on ResNet-50 conv shapes at batch 256, after a
# correctness pass of the GEMM / fused-block tests with the forced variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
MPIT_GEMM_BM=256 timeout -k 10 300 python -u -m pytest tests/test_gemm.py tests/test_resnet_fused.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_bm256.log 2>&1 || { tail -30 gpurun_out/pytest_bm256.log; exit 1; }
tail -1 gpurun_out/pytest_bm256.log
out=gpurun_out/gemm_ab.jsonl; : > $out
for bm in 128; do
  for shp in "conv 256 14 14 256 256 3 1" "conv 256 7 7 512 512 3 1" "conv 256 28 28 128 128 3 1" "nt 50176 1024 256" "nt 12544 2048 512" "nt 50176 256 1024" "nt 200704 128 512" "nt 200704 512 128" "nt 802816 256 64" "nt 802816 128 128"; do
    MPIT_GEMM_BM=$bm timeout -k 10 60 python3 benchmarks/gemm_probe.py $shp 50 | sed "s/^/{\"bm\": $bm, \"r\": /; s/$/}/" >> $out || exit 1
  done
done
cat $out

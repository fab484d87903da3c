#!/bin/bash
# gemm_nt block-tile A/B: the GEMM tests under each forced tile, then per-shape probes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/tile_ab.jsonl
: > $out
for t in 256 256x128; do
  MPIT_GEMM_TILE=$t timeout -k 10 300 python -u -m pytest tests/test_gemm.py tests/test_resnet_fused.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_tile_$t.log 2>&1 || { echo "tests FAILED under tile $t"; tail -30 gpurun_out/pytest_tile_$t.log; exit 1; }
  tail -1 gpurun_out/pytest_tile_$t.log
done
for t in 128 256x128 256; do
  for a in "conv 256 14 14 256 256 3 1" "conv 256 7 7 512 512 3 1" "conv 256 28 28 128 128 3 1" "conv 256 56 56 64 64 3 1" "nt 50176 256 2304" "nt 50176 256 1024" "nt 12544 512 2048" "nt 12544 2048 512" "nt 8192 8192 8192 20"; do
    r=$(MPIT_GEMM_TILE=$t timeout -k 10 60 python benchmarks/gemm_probe.py $a) || { echo "probe FAILED $t $a"; exit 1; }
    echo "{\"tile\": \"$t\", \"r\": $r}" | tee -a $out
  done
done

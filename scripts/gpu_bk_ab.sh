#!/bin/bash
# 128x128 gemm_nt staged 64 deep (2 slots) vs 32 deep: tests under BK64, probes, bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/bk_ab.jsonl
: > $out
MPIT_GEMM_BK64=1 timeout -k 10 300 python -u -m pytest tests/test_gemm.py tests/test_resnet_fused.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_bk64.log 2>&1 || { echo "tests FAILED under BK64"; tail -30 gpurun_out/pytest_bk64.log; exit 1; }
tail -1 gpurun_out/pytest_bk64.log
for b in 0 1; do
  for a in "conv 256 14 14 256 256 3 1" "conv 256 7 7 512 512 3 1" "conv 256 28 28 128 128 3 1" "conv 256 56 56 64 64 3 1" "nt 50176 256 2304" "nt 200704 128 512" "nt 12544 512 2048" "nt 12544 2048 512" "nt 8192 8192 8192 20"; do
    r=$(MPIT_GEMM_BK64=$b timeout -k 10 60 python benchmarks/gemm_probe.py $a) || { echo "probe FAILED $b $a"; exit 1; }
    echo "{\"bk64\": $b, \"r\": $r}" | tee -a $out
  done
done
for b in 0 1 0 1; do
  r=$(MPIT_GEMM_BK64=$b timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 2>/dev/null) || { echo "bench FAILED $b"; exit 1; }
  echo "{\"bk64\": $b, \"bench\": $r}" | tee -a $out
done

#!/bin/bash
# bf16 step kernel traces with the default 128-row tiles and with MPIT_GEMM_TILE=256
# (256x256 where N % 256 == 0, else 256x128 / 128-row), for a call-by-call comparison.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/t256
mkdir -p $D
for cfg in 128 256; do
  MPIT_GEMM_TILE=$cfg timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/t$cfg -o t -- python3 bench.py --steps 6 --warmup 3 --no-secondary --dtype bf16 > $D/run$cfg.log 2>&1 || { tail -20 $D/run$cfg.log; exit 1; }
  tail -1 $D/run$cfg.log | cut -c1-200
done

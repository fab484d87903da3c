#!/bin/bash
# End-to-end A/B of an environment switch on the N=1 bench: A B A B (same box).
# usage: bash scripts/gpu_bench_ab.sh "VAR=value"
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/bench_ab.txt; : > $out
for i in 1 2; do
  for v in "" "$1"; do
    r=$(env $v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 2>/dev/null | tail -1) || exit 1
    echo "[$v] $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $out
  done
done

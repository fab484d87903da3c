#!/bin/bash
# Per-call GEMM tables of the fp32 ResNet-50 step: default (side stream for the weight
# gradients) and everything on one stream (MPIT_WGRAD_STREAM=0: uncontended per-call times).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/gcalls
mkdir -p $D
for v in side one; do
  ws=1; [ $v = one ] && ws=0
  MPIT_WGRAD_STREAM=$ws MPIT_GEMM_LOG=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $D/t_$v -o t --output-format csv -- \
    python3 bench.py --steps 4 --warmup 2 --no-secondary > $D/log_$v.txt 2>&1 || { tail -20 $D/log_$v.txt; exit 1; }
  python3 scripts/gemm_calls.py $D/log_$v.txt $D/t_$v $D/calls_$v.md "fp32 ResNet-50 step GEMM calls ($v)" || exit 1
done

#!/bin/bash
# step-boundary host stall: Python threads present, GIL switch interval A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/gil
mkdir -p $D
for sw in 5000 100; do
  MPIT_THREAD_DUMP=1 MPIT_SWITCH_US=$sw MPIT_TRACE=1 timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --output-format csv -d $D/t$sw -o b -- python3 bench.py --dtype bf16 --steps 8 --warmup 3 --no-secondary > $D/t$sw.log 2>&1 || { tail -20 $D/t$sw.log; exit 1; }
  grep "mpit threads" $D/t$sw.log | head -1
  echo "== switch interval $sw us (bf16)"; python3 scripts/boundary_summary.py $D/t$sw || exit 1
done
find $D -name "*.csv" -size +30M -delete

#!/bin/bash
# step-boundary latency chain (roctx + kernel trace), fp32 and bf16
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/boundary
mkdir -p $D
for dt in fp32 bf16; do
  MPIT_TRACE=1 timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --output-format csv -d $D/$dt -o b -- python3 bench.py --dtype $dt --steps 8 --warmup 3 --no-secondary > $D/$dt.log 2>&1 || { tail -20 $D/$dt.log; exit 1; }
  echo "== $dt"; python3 scripts/boundary_summary.py $D/$dt || exit 1
done
find $D -name "*.csv" -size +30M -delete

#!/bin/bash
# Steady-state kernel tables of the fp32 and bf16 steps (current defaults).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/prof2
mkdir -p $D
for dt in fp32 bf16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/$dt -o t -- python3 bench.py --steps 6 --warmup 3 --no-secondary --dtype $dt > $D/$dt.log 2>&1 || { tail -20 $D/$dt.log; exit 1; }
  python3 scripts/prof_summary.py $D/$dt $D/${dt}_steady.md --top 30 > /dev/null || exit 1
  head -3 $D/${dt}_steady.md
done

#!/bin/bash
# roctx phase table of the bf16 step incl. the step-start ranges (hp_wait, push_arm, wcast)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/ranges
mkdir -p $D
MPIT_TRACE=1 timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --output-format csv -d $D/t -o b -- python3 bench.py --dtype bf16 --steps 8 --warmup 3 --no-secondary > $D/t.log 2>&1 || { tail -20 $D/t.log; exit 1; }
python3 scripts/phase_summary.py $D/t $D/phase.md --skip 3 || exit 1
python3 scripts/boundary_summary.py $D/t || exit 1
cat $D/phase.md | head -30
find $D -name "*.csv" -size +30M -delete

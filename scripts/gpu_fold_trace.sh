#!/bin/bash
# fp32 step kernel traces with the BN finalize fold on and off (same box)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/foldtr
mkdir -p $D
for f in 0 1; do
  MPIT_BN_FOLD=$f timeout -k 10 300 rocprofv3 --kernel-trace -d $D/t$f -o t --output-format csv -- \
    python3 bench.py --steps 6 --warmup 3 --no-secondary > $D/log$f.txt 2>&1 || { tail -20 $D/log$f.txt; exit 1; }
  python3 scripts/step_gaps.py $D/t$f 2
done

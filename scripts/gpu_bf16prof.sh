#!/bin/bash
# bf16-autocast step: steady-state kernel table (copy dispatches included).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/bf16p
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $D/t -o t -- python3 bench.py --steps 6 --warmup 3 --no-secondary --dtype bf16 > $D/run.log 2>&1 || { tail -20 $D/run.log; exit 1; }
tail -1 $D/run.log | cut -c1-300
python3 scripts/prof_summary.py $D/t $D/bf16_steady.md --top 40 > /dev/null || exit 1
ls $D/t
find $D/t -name "*.csv" -size +30M -delete

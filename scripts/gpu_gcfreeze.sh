#!/bin/bash
# A/B: gc.freeze() after warmup (MPIT_GC_FREEZE) — step-boundary chain and bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/gcf
mkdir -p $D
for g in 0 1; do
  MPIT_GC_FREEZE=$g MPIT_TRACE=1 timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --output-format csv -d $D/t$g -o b -- python3 bench.py --dtype bf16 --steps 8 --warmup 3 --no-secondary > $D/t$g.log 2>&1 || { tail -20 $D/t$g.log; exit 1; }
  echo "== gc_freeze=$g (bf16)"; python3 scripts/boundary_summary.py $D/t$g || exit 1
done
find $D -name "*.csv" -size +30M -delete
for i in 1 2; do for g in 0 1; do
  MPIT_GC_FREEZE=$g timeout -k 10 300 python3 -u bench.py > $D/b_${g}_$i.log 2>&1 || { tail -20 $D/b_${g}_$i.log; exit 1; }
  echo "freeze=$g run=$i $(tail -1 $D/b_${g}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["secondary"]["bf16_autocast"]["value"])')"
done; done

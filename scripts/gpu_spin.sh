#!/bin/bash
# step-start host stall: the worker's PS wait polls before sleeping (MPIT_WAIT_SPIN_US, default 200 ms) vs sleeping at once (0)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/spin
mkdir -p $D
echo "cpus: $(nproc) affinity: $(python3 -c 'import os; print(len(os.sched_getaffinity(0)))')"
for y in 0 200000; do
  MPIT_WAIT_SPIN_US=$y MPIT_TRACE=1 timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --output-format csv -d $D/t$y -o b -- python3 bench.py --dtype bf16 --steps 8 --warmup 3 --no-secondary > $D/t$y.log 2>&1 || { tail -20 $D/t$y.log; exit 1; }
  python3 scripts/phase_summary.py $D/t$y $D/phase$y.md --skip 3 || exit 1
  echo "== wait spin $y us"; grep -E "push_arm|ps_wait|wcast" $D/phase$y.md; python3 scripts/boundary_summary.py $D/t$y | tail -1
done
find $D -name "*.csv" -size +30M -delete
for i in 1 2; do for y in 0 200000; do
  MPIT_WAIT_SPIN_US=$y timeout -k 10 300 python3 -u bench.py > $D/b_${y}_$i.log 2>&1 || { tail -20 $D/b_${y}_$i.log; exit 1; }
  echo "spin=$y run=$i $(tail -1 $D/b_${y}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["secondary"]["bf16_autocast"]["value"])')"
done; done

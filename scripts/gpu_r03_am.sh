#!/bin/bash
# Round 3 (session 2): bf16 step host-side knobs A/B (standalone bench --dtype bf16): default vs no
# deferred PS wait vs round-2 progress idle loop (no futex park) vs no gc.freeze vs 40 steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03am
mkdir -p $O
one() {
  local V=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --dtype bf16 --no-secondary > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; return 1; }
  echo "$V: $(tail -1 $O/b.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
for rep in 1 2; do
  one default || exit 1
  one nodefer MPIT_DEFER_PS_WAIT=0 || exit 1
  one nopark MPIT_PROGRESS_PARK=0 || exit 1
  one nofreeze MPIT_GC_FREEZE=0 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace -d $O/prof -o t --output-format csv -- python3 bench.py --dtype bf16 --steps 6 --warmup 3 --no-secondary > $O/prof.log 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
python3 scripts/step_gaps.py $O/prof > $O/gaps.txt 2>&1 || true
tail -30 $O/gaps.txt
find $O/prof -name "*.csv" -size +40M -delete
echo ALL OK

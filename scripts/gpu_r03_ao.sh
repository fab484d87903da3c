#!/bin/bash
# Round 3 (session 2): PS client poll-before-sleep (MPIT_WAIT_SPIN_US) A/B on the round-3 engine,
# fp32 and bf16 standalone benches, interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03ao
mkdir -p $O
one() {
  local V=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-secondary $BARGS > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; return 1; }
  echo "$V $BARGS: $(tail -1 $O/b.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
for BARGS in "--dtype fp32" "--dtype bf16"; do
  for rep in 1 2 3; do
    one default || exit 1
    one spin200 MPIT_WAIT_SPIN_US=200 || exit 1
  done
done
echo ALL OK

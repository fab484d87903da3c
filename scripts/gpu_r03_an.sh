#!/bin/bash
# Round 3 (session 2): deferred PS wait A/B in the fp32 headline (interleaved, 3 rounds).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03an
mkdir -p $O
one() {
  local V=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-secondary > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; return 1; }
  echo "$V: $(tail -1 $O/b.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
for rep in 1 2 3; do
  one defer MPIT_DEFER_PS_WAIT=1 || exit 1
  one nodefer MPIT_DEFER_PS_WAIT=0 || exit 1
done
echo ALL OK

#!/bin/bash
# Round 3 (session 2): BN apply passes A/B in the fp32 bench: grid-stride cap (MPIT_BN_GRID 2048 / 4096
# (default) / 8192 / 16384) and a 2x-unrolled grid-stride loop (varso/bnunroll.so).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03aj
mkdir -p $O
: > $O/ab.txt
one() {  # name, env...
  local V=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-secondary > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; return 1; }
  echo "$V $(tail -1 $O/b.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $O/ab.txt
}
for rep in 1 2; do
  one base MPIT_BN_GRID=4096 || exit 1
  one g2048 MPIT_BN_GRID=2048 || exit 1
  one g8192 MPIT_BN_GRID=8192 || exit 1
  one g16384 MPIT_BN_GRID=16384 || exit 1
  one unroll2 MPIT_NATIVE_SO=varso/bnunroll.so || exit 1
done
echo ALL OK

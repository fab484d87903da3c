#!/bin/bash
# Round 3 (session 2): bf16 step standalone (bench --dtype bf16) vs as the fp32 job's secondary
# (same trainer after set_amp), interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03al
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --dtype bf16 --no-secondary > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  echo "standalone bf16: $(tail -1 $O/b.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  timeout -k 10 300 python -u bench.py > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  echo "fp32 + secondary: $(tail -1 $O/b.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["secondary"]["bf16_autocast"]["value"], d["secondary"]["bf16_autocast"]["ms_per_step"])')"
done
echo ALL OK

#!/bin/bash
# Round 3: GPU test tier on the fail-fast runtime, default bench line, AccumulateGrad
# stream diagnostic, and the K-shard emulation (bench.py --emulate-shards K).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20; tail -2 $O/pytest_gpu.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-300; echo "accgrad warnings: $(grep -c AccumulateGrad $O/bench.err)"
timeout -k 10 300 python -u benchmarks/diag_accgrad.py > $O/diag_accgrad.jsonl 2> $O/diag_accgrad.err || { tail -30 $O/diag_accgrad.err; exit 1; }
cat $O/diag_accgrad.jsonl
for k in 1 2 4 8; do
  timeout -k 10 240 python -u bench.py --no-secondary --steps 20 --warmup 5 --emulate-shards $k > $O/emu$k.json 2> $O/emu$k.err || { tail -30 $O/emu$k.err; exit 1; }
  echo "K=$k $(tail -1 $O/emu$k.json | cut -c1-200)"
done
echo ALL OK

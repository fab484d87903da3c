#!/bin/bash
# Round 3: pre-split weight planes (FM 4): fp32 numerics tier, per-shape timing vs the
# in-register split, and the default bench line on the new path.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03g
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fp32_path.py tests/test_resnet_fused.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_fp32.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/pytest_fp32.log | tail -12; [ $rc -ne 0 ] && exit 1
: > $O/probe.jsonl
for P in "nt 50176 1024 512" "nt 200704 512 128" "nt 802816 256 64" "conv 256 14 14 256 256 3 1" "conv 256 56 56 64 64 3 1" "conv 256 7 7 512 512 3 1" "dgrad 256 28 28 128 128 3 1"; do
  for B in "" "--bsplit"; do
    timeout -k 10 120 python3 benchmarks/gemm_probe.py --f32 $B $P 20 > $O/t.json || exit 1
    echo "{\"b\": \"$B\", \"r\": $(cat $O/t.json)}" >> $O/probe.jsonl
  done
done
cat $O/probe.jsonl
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
MPIT_F32_BSPLIT=0 timeout -k 10 300 python -u bench.py --no-secondary > $O/bench_regsplit.json 2> $O/bench_regsplit.err || { tail -30 $O/bench_regsplit.err; exit 1; }
echo "planes:   $(tail -1 $O/bench.json | cut -c1-200)"
echo "regsplit: $(tail -1 $O/bench_regsplit.json | cut -c1-200)"
echo ALL OK

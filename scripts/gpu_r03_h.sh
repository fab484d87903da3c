#!/bin/bash
# Round 3: pre-split planes on the 4x1 wave grid (FM 9) vs 2x2 (FM 4) vs in-register split
# (FM 3): fp32 numerics tier, per-shape timing, bench lines, and a per-stream kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fp32_path.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_fp32.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/pytest_fp32.log | tail -12; [ $rc -ne 0 ] && exit 1
: > $O/probe.jsonl
for P in "nt 50176 1024 512" "nt 200704 512 128" "nt 802816 256 64" "conv 256 14 14 256 256 3 1" "conv 256 7 7 512 512 3 1" "dgrad 256 28 28 128 128 3 1" "dgrad 256 14 14 256 256 3 1"; do
  for V in reg 2x2 4x1; do
    if [ $V = reg ]; then B=""; else B="--bsplit"; fi
    MPIT_F32_WAVES=$V timeout -k 10 120 python3 benchmarks/gemm_probe.py --f32 $B $P 20 > $O/t.json || exit 1
    echo "{\"v\": \"$V\", \"r\": $(cat $O/t.json)}" >> $O/probe.jsonl
  done
done
cat $O/probe.jsonl
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
MPIT_F32_WAVES=2x2 timeout -k 10 300 python -u bench.py --no-secondary > $O/bench_22.json 2> $O/bench_22.err || { tail -30 $O/bench_22.err; exit 1; }
echo "4x1: $(tail -1 $O/bench.json | cut -c1-220)"
echo "2x2: $(tail -1 $O/bench_22.json | cut -c1-220)"
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o t --output-format csv -- python3 bench.py --steps 6 --warmup 3 --no-secondary > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/stream_summary.py $O/prof $O/streams.md cast_batch_kernel 3 || exit 1
find $O/prof -name "*kernel_trace.csv" -size +40M -delete
echo ALL OK

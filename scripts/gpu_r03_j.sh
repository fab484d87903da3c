#!/bin/bash
# Round 3: split-once fp32 wgrad (gemm_tn_f32s_kernel) — bitwise vs the per-tile split,
# fp32 numerics tier, per-shape timing (MPIT_TN_F32S=0 vs 1), bench A/B, per-stream trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03j
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_fp32_path.py -m gpu -k "split_once or gemm_tn" -v --timeout 180 --timeout-method thread > $O/pytest_wg.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed|Error" $O/pytest_wg.log | tail -12; [ $rc -ne 0 ] && exit 1
: > $O/probe.jsonl
for P in "tn 200704 512 128" "tn 200704 128 512" "tn 50176 1024 256" "tn 50176 256 1024" "tn 12544 2048 512" "tn 12544 512 2048" "wgrad 256 28 28 128 128 3 1" "wgrad 256 14 14 256 256 3 1" "wgrad 256 7 7 512 512 3 1" "wgrad 256 56 56 128 128 3 2"; do
  for V in 0 1; do
    MPIT_TN_F32S=$V timeout -k 10 120 python3 benchmarks/gemm_probe.py --f32 $P 20 > $O/t.json || exit 1
    echo "{\"f32s\": $V, \"r\": $(cat $O/t.json)}" >> $O/probe.jsonl
  done
done
cat $O/probe.jsonl
timeout -k 10 300 python -u bench.py --no-secondary > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
MPIT_TN_F32S=0 timeout -k 10 300 python -u bench.py --no-secondary > $O/bench_old.json 2> $O/bench_old.err || { tail -30 $O/bench_old.err; exit 1; }
MPIT_F32_PLANES_N=64 timeout -k 10 300 python -u bench.py --no-secondary > $O/bench_p64.json 2> $O/bench_p64.err || { tail -30 $O/bench_p64.err; exit 1; }
echo "f32s: $(tail -1 $O/bench.json | cut -c1-200)"
echo "old : $(tail -1 $O/bench_old.json | cut -c1-200)"
echo "p64 : $(tail -1 $O/bench_p64.json | cut -c1-200)"
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o t --output-format csv -- python3 bench.py --steps 6 --warmup 3 --no-secondary > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/stream_summary.py $O/prof $O/streams.md cast_batch_kernel 3 || exit 1
find $O/prof -name "*kernel_trace.csv" -size +40M -delete
echo ALL OK

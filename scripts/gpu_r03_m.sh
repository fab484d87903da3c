#!/bin/bash
# Round 3: fp32 NT kernels with asm LDS DMA (stage kt+1 load overlaps stage kt MFMAs) and
# the split-once wgrad without scratch: numerics tier, per-shape timing, bench A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03m
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fp32_path.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_fp32.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/pytest_fp32.log | tail -12; [ $rc -ne 0 ] && { grep -E "^E " $O/pytest_fp32.log | head -20; exit 1; }
: > $O/probe.jsonl
for P in "nt 50176 1024 512" "nt 200704 512 128" "nt 802816 256 64" "conv 256 14 14 256 256 3 1" "conv 256 7 7 512 512 3 1" "conv 256 56 56 64 64 3 1" "dgrad 256 28 28 128 128 3 1"; do
  timeout -k 10 120 python3 benchmarks/gemm_probe.py --f32 --bsplit $P 20 > $O/t.json || exit 1
  echo "{\"v\": \"fm9\", \"r\": $(cat $O/t.json)}" >> $O/probe.jsonl
done
for P in "tn 200704 512 128" "tn 50176 1024 256" "tn 12544 512 2048" "wgrad 256 14 14 256 256 3 1" "wgrad 256 28 28 128 128 3 1"; do
  for V in 0 1; do
    MPIT_TN_F32S=$V timeout -k 10 120 python3 benchmarks/gemm_probe.py --f32 $P 20 > $O/t.json || exit 1
    echo "{\"f32s\": $V, \"r\": $(cat $O/t.json)}" >> $O/probe.jsonl
  done
done
cat $O/probe.jsonl
timeout -k 10 300 python -u bench.py --no-secondary > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
echo "dflt: $(tail -1 $O/bench.json | cut -c1-200)"
MPIT_TN_F32S=1 timeout -k 10 300 python -u bench.py --no-secondary > $O/bench_f32s.json 2> $O/bench_f32s.err || { tail -30 $O/bench_f32s.err; exit 1; }
echo "f32s: $(tail -1 $O/bench_f32s.json | cut -c1-200)"
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o t --output-format csv -- python3 bench.py --steps 6 --warmup 3 --no-secondary > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/stream_summary.py $O/prof $O/streams.md cast_batch_kernel 3 || exit 1
find $O/prof -name "*kernel_trace.csv" -size +40M -delete
echo ALL OK

#!/bin/bash
# Round 3 (session 2): final-tree evidence — smoke, bench (fp32 headline + bf16 secondary), fp32 and
# bf16 per-stream kernel tables, whole GPU tier.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03ak
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
echo "bench: $(tail -1 $O/bench.json | cut -c1-300)"
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o t --output-format csv -- python3 bench.py --steps 4 --warmup 3 --no-secondary > $O/prof.log 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
python3 scripts/stream_summary.py $O/prof $O/streams_fp32.md cast_batch_kernel 3 || exit 1
find $O/prof -name "*kernel_trace.csv" -size +40M -delete
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/profb -o t --output-format csv -- python3 bench.py --dtype bf16 --steps 4 --warmup 3 --no-secondary > $O/profb.log 2> $O/profb.err || { tail -20 $O/profb.err; exit 1; }
python3 scripts/stream_summary.py $O/profb $O/streams_bf16.md cast_batch_kernel 3 || exit 1
find $O/profb -name "*kernel_trace.csv" -size +40M -delete
grep -E "step wall" $O/streams_fp32.md $O/streams_bf16.md
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest_gpu.log | head; exit 1; }
echo ALL OK

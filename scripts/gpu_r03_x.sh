#!/bin/bash
# Round 3 (session 2): producer bounds by one atomic per block (zeroed by the finalize):
# bound tests, bench, per-stream table, whole GPU tier.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03x
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_f16x3.py tests/test_fp32_path.py -m gpu -q --timeout 200 --timeout-method thread > $O/pytest_f16.log 2>&1
rc=$?; tail -4 $O/pytest_f16.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest_f16.log | head; exit 1; }
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
echo "f16x3: $(tail -1 $O/bench.json | cut -c1-300)"
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o t --output-format csv -- python3 bench.py --steps 4 --warmup 3 --no-secondary > $O/prof.log 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
python3 scripts/stream_summary.py $O/prof $O/streams.md cast_batch_kernel 3 || exit 1
find $O/prof -name "*kernel_trace.csv" -size +40M -delete
head -34 $O/streams.md
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest_gpu.log | head; exit 1; }
echo ALL OK

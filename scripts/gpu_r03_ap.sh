#!/bin/bash
# Round 3 (session 2): the weight plan's fp16-plane bound computed natively (cast_amax_kernel, one
# memset + one launch before cast_batch) instead of torch _foreach_norm + stack + amax: numerics,
# step-boundary gaps, bench x3.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03ap
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_f16x3.py tests/test_fp32_path.py -m gpu -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest.log | head; exit 1; }
for rep in 1 2 3; do
  timeout -k 10 300 python -u bench.py > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  echo "bench: $(tail -1 $O/b.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["secondary"]["bf16_autocast"]["value"])')"
done
cp $O/b.json $O/bench_last.json
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o t --output-format csv -- python3 bench.py --steps 4 --warmup 3 --no-secondary > $O/prof.log 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
python3 scripts/step_gaps.py $O/prof 3 > $O/gaps.txt 2>&1 || true
python3 scripts/stream_summary.py $O/prof $O/streams_fp32.md cast_batch_kernel 3 || exit 1
grep -E "step wall" $O/gaps.txt $O/streams_fp32.md
find $O/prof -name "*kernel_trace.csv" -size +40M -delete
echo ALL OK

#!/bin/bash
# Round 3 (session 2): GPU tier on the restored tree, then per-call GEMM tables of the
# fp32 bench step with both streams (default) and with the weight gradients on the
# compute stream (MPIT_WGRAD_STREAM=0: per-call times without side-stream contention).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03t
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest_gpu.log | head; exit 1; }
for V in 2s 1s; do
  if [ $V = 1s ]; then W=0; else W=1; fi
  MPIT_WGRAD_STREAM=$W MPIT_GEMM_LOG=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_$V -o t --output-format csv -- python3 bench.py --steps 4 --warmup 3 --no-secondary > $O/prof_$V.log 2> $O/prof_$V.err || { tail -20 $O/prof_$V.err; exit 1; }
  python3 scripts/gemm_calls.py $O/prof_$V.err $O/prof_$V $O/gemm_calls_$V.md "fp32 ResNet-50 step GEMM calls ($V)" || exit 1
  python3 scripts/stream_summary.py $O/prof_$V $O/streams_$V.md cast_batch_kernel 3 || exit 1
  find $O/prof_$V -name "*kernel_trace.csv" -size +40M -delete
done
echo ALL OK

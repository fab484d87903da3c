#!/bin/bash
# Round 3 (session 2): fp16 plane diagnostic, then per-call GEMM tables and per-stream kernel
# time of the fp16x3 fp32 step (both streams / one stream).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03w
mkdir -p $O
timeout -k 10 120 python -u benchmarks/f16_plane_diag.py > $O/diag.txt 2>&1 || { tail -20 $O/diag.txt; exit 1; }
cat $O/diag.txt | grep -v amdgpu.ids
for V in 2s 1s; do
  if [ $V = 1s ]; then W=0; else W=1; fi
  MPIT_WGRAD_STREAM=$W MPIT_GEMM_LOG=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_$V -o t --output-format csv -- python3 bench.py --steps 4 --warmup 3 --no-secondary > $O/prof_$V.log 2> $O/prof_$V.err || { tail -20 $O/prof_$V.err; exit 1; }
  python3 scripts/gemm_calls.py $O/prof_$V.err $O/prof_$V $O/gemm_calls_$V.md "fp32 (fp16x3) ResNet-50 step GEMM calls ($V)" || exit 1
  python3 scripts/stream_summary.py $O/prof_$V $O/streams_$V.md cast_batch_kernel 3 || exit 1
  find $O/prof_$V -name "*kernel_trace.csv" -size +40M -delete
done
grep total $O/gemm_calls_1s.md
head -30 $O/streams_2s.md
echo ALL OK

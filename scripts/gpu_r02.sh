#!/bin/bash
# Round-2 validation: GPU test tier, smoke(), default bench line, fp32 step kernel table.
# Test failures do not stop the run; crashes / time limits (rc >= 124) do.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r02
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r02/pytest_gpu.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/r02/pytest_gpu.log | head -20; tail -2 gpurun_out/r02/pytest_gpu.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02/smoke.log 2>&1 || { tail -30 gpurun_out/r02/smoke.log; exit 1; }
tail -1 gpurun_out/r02/smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/r02/bench_default.log 2>&1 || { tail -30 gpurun_out/r02/bench_default.log; exit 1; }
tail -1 gpurun_out/r02/bench_default.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02/prof -o run -- python3 bench.py --gpus 1 --steps 6 --warmup 3 --no-secondary > gpurun_out/r02/prof.log 2>&1 || { tail -30 gpurun_out/r02/prof.log; exit 1; }
python3 scripts/prof_summary.py gpurun_out/r02/prof gpurun_out/r02/fp32_steady.md > /dev/null
find gpurun_out/r02/prof -name "*kernel_trace.csv" -size +20M -delete
echo prof done
: > gpurun_out/r02/ew.jsonl
for u in auto 1 2 4; do
  if [ $u = auto ]; then timeout -k 10 120 python3 benchmarks/ew_probe.py 25.6 3.2 0.8 >> gpurun_out/r02/ew.jsonl || exit 1
  else MPIT_EW_UNROLL=$u timeout -k 10 120 python3 benchmarks/ew_probe.py 25.6 3.2 0.8 >> gpurun_out/r02/ew.jsonl || exit 1; fi
done
cat gpurun_out/r02/ew.jsonl

#!/bin/bash
# Round-2 validation: GPU test tier, smoke(), default bench line, fp32 step kernel table.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r02
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02/pytest_gpu.log 2>&1 || { grep -E "PASS|FAIL" gpurun_out/r02/pytest_gpu.log | tail -5; tail -40 gpurun_out/r02/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r02/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02/smoke.log 2>&1 || { tail -30 gpurun_out/r02/smoke.log; exit 1; }
tail -1 gpurun_out/r02/smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/r02/bench_default.log 2>&1 || { tail -30 gpurun_out/r02/bench_default.log; exit 1; }
tail -1 gpurun_out/r02/bench_default.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02/prof -o run -- python3 bench.py --gpus 1 --steps 6 --warmup 3 --no-secondary > gpurun_out/r02/prof.log 2>&1 || { tail -30 gpurun_out/r02/prof.log; exit 1; }
python3 scripts/prof_summary.py gpurun_out/r02/prof gpurun_out/r02/fp32_steady.md > /dev/null
rm -rf gpurun_out/r02/prof/*/*kernel_trace.csv.bak
echo prof done

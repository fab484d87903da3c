#!/bin/bash
# Round-end rehearsal: GPU test tier, smoke(), default bench line, steady-state fp32 kernel table.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/final
D=gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { grep -E "PASS|FAIL" $D/pytest_gpu.log | tail -5; tail -40 $D/pytest_gpu.log; exit 1; }
tail -3 $D/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -30 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 300 python -u bench.py > $D/bench.log 2>&1 || { tail -30 $D/bench.log; exit 1; }
tail -1 $D/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o p --output-format csv -- python3 bench.py --steps 6 --warmup 3 --no-secondary > $D/prof.log 2>&1 || { tail -20 $D/prof.log; exit 1; }
python3 scripts/prof_summary.py $D/prof $D/kernels.md > $D/ps.log 2>&1 || { tail -5 $D/ps.log; exit 1; }
head -12 $D/kernels.md

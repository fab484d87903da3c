#!/bin/bash
# bf16 step: GPU idle gaps (kernel trace) and host-side Python profile (cProfile) of the step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/bf16gaps
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace -d $D/t -o t --output-format csv -- \
  python3 bench.py --dtype bf16 --steps 6 --warmup 3 --no-secondary > $D/trace.log 2>&1 || { tail -20 $D/trace.log; exit 1; }
tail -1 $D/trace.log
timeout -k 10 300 python3 -m cProfile -o $D/prof.out bench.py --dtype bf16 --steps 30 --warmup 5 --no-secondary > $D/cprof.log 2>&1 || { tail -20 $D/cprof.log; exit 1; }
tail -1 $D/cprof.log
python3 - <<'PY' > $D/cprof_top.txt
import pstats
p = pstats.Stats("gpurun_out/bf16gaps/prof.out")
p.sort_stats("tottime").print_stats(45)
PY
head -80 $D/cprof_top.txt

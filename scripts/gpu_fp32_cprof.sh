#!/bin/bash
# host-side Python profile of the fp32 bench step (cProfile)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/fp32cprof
mkdir -p $D
timeout -k 10 300 python3 -m cProfile -o $D/prof.out bench.py --steps 20 --warmup 5 --no-secondary > $D/cprof.log 2>&1 || { tail -20 $D/cprof.log; exit 1; }
tail -1 $D/cprof.log | cut -c1-200

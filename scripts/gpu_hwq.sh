#!/bin/bash
# HIP hardware queues per process (GPU_MAX_HW_QUEUES) A/B on the default bench, and a
# 4-rank shared-GPU run (more streams per process: link streams of the co-located PS).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/hwq
mkdir -p $D
for i in 1 2; do for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py > $D/b_${q}_$i.log 2>&1 || { tail -20 $D/b_${q}_$i.log; exit 1; }
  echo "q=$q run=$i $(tail -1 $D/b_${q}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["secondary"]["bf16_autocast"]["value"])')"
done; done

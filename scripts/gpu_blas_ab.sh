#!/bin/bash
# A/B of step-boundary host latency fixes: progress-thread timer slack (MPIT_TIMER_SLACK_NS=0
# restores the default 50 us) and the fc layer's library GEMMs on rocBLAS (MPIT_BLAS=rocblas)
# instead of hipBLASLt; then the bf16 GPU idle gaps of the best arm.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/blas
mkdir -p $D
arm() { case $1 in base) echo "MPIT_TIMER_SLACK_NS=0 MPIT_BLAS=lt";; slack) echo "MPIT_BLAS=lt";; roc) echo "MPIT_BLAS=rocblas";; esac; }
for i in 1 2; do for a in base slack roc; do
  env $(arm $a) timeout -k 10 300 python3 -u bench.py > $D/b_${a}_$i.log 2>&1 || { tail -20 $D/b_${a}_$i.log; exit 1; }
  echo "arm=$a run=$i $(tail -1 $D/b_${a}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["secondary"]["bf16_autocast"]["value"])')"
done; done
MPIT_BLAS=rocblas timeout -k 10 300 rocprofv3 --kernel-trace -d $D/t -o t --output-format csv -- \
  python3 bench.py --dtype bf16 --steps 6 --warmup 3 --no-secondary > $D/trace.log 2>&1 || { tail -20 $D/trace.log; exit 1; }
tail -1 $D/trace.log | cut -c1-200

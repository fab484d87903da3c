#!/bin/bash
# ShardPusher overlap equivalence diagnostics (3 ranks on the box's GPU).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/ovl
run() { timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=3 --master-addr=127.0.0.1 --master-port=$1 tests/mp/overlap_equiv.py; }
for i in 1 2 3; do
MPIT_WGRAD_STREAM=force T_STEPS=4 run 2961$i > gpurun_out/ovl/force_s4_$i.log 2>&1 || { tail -30 gpurun_out/ovl/force_s4_$i.log; exit 1; }
grep -E "DIFF|RESULT" gpurun_out/ovl/force_s4_$i.log
done

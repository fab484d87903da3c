#!/bin/bash
# Default bench line, then roctx phase breakdowns: 1 rank, and 2 ranks sharing the GPU
# (co-located PS: every step pushes a shard to the other rank's server).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/phase
mkdir -p $D
timeout -k 10 300 python -u bench.py > $D/bench.log 2>&1 || { tail -20 $D/bench.log; exit 1; }
tail -1 $D/bench.log
MPIT_TRACE=1 timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --output-format csv -d $D/n1 -o ph -- python3 bench.py --steps 6 --warmup 2 --no-secondary > $D/n1.log 2>&1 || { tail -20 $D/n1.log; exit 1; }
python3 scripts/phase_summary.py $D/n1 $D/phase_n1.md --skip 2 || exit 1
MPIT_TRACE=1 timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --output-format csv -d $D/n2 -o ph -- python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29731 bench.py --gpus 2 --steps 6 --warmup 2 --no-secondary --batch 128 > $D/n2.log 2>&1 || { tail -20 $D/n2.log; exit 1; }
python3 scripts/phase_summary.py $D/n2 $D/phase_n2_shared.md --skip 2 || exit 1
find $D -name "*.csv" -size +30M -delete

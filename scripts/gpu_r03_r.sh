#!/bin/bash
# Round 3: VGG-16 bf16 operator table, then the FM 9 wave-cycle breakdown (scripts/gpu_r03_q.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03r
mkdir -p $O
timeout -k 10 300 python3 -u benchmarks/op_profile.py --model vgg16 --batch 64 --optimizer eamsgd --su 2 --dtype bf16 > $O/vgg_ops.txt 2> $O/vgg_ops.err || { tail -20 $O/vgg_ops.err; exit 1; }
head -60 $O/vgg_ops.txt
bash scripts/gpu_r03_q.sh || exit 1

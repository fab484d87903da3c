#!/bin/bash
# Rehearsal of the multi-rank paths on one GPU (ranks share the card) and the other
# BASELINE.json configs at N=1. Every step has its own time limit; stop at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/cfg_r03ae
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/cfg_r03ae/$name.json" 2> "gpurun_out/cfg_r03ae/$name.err" || { echo "FAILED $name rc=$?"; tail -25 "gpurun_out/cfg_r03ae/$name.err"; exit 1; }
  tail -1 "gpurun_out/cfg_r03ae/$name.json"
}
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --master-port 29533"
run n8_downpour 400 $TR --nproc-per-node 8 bench.py --gpus 8 --batch 32 --steps 4 --warmup 2
run n4_downpour 300 $TR --nproc-per-node 4 bench.py --gpus 4 --batch 64 --steps 5 --warmup 2
run n3_dedicated 300 $TR --nproc-per-node 3 bench.py --gpus 3 --batch 64 --steps 5 --warmup 2 --topology dedicated --servers 1
run n2_eamsgd 300 $TR --nproc-per-node 2 bench.py --gpus 2 --batch 64 --steps 5 --warmup 2 --optimizer eamsgd --su 2 --wire bf16
run n2_allreduce_bf16wire 300 $TR --nproc-per-node 2 bench.py --gpus 2 --batch 64 --steps 5 --warmup 2 --optimizer allreduce --wire bf16
run n1_allreduce 300 python -u bench.py --optimizer allreduce --steps 10 --warmup 3
run n1_alexnet_ssp 300 python -u bench.py --model alexnet --batch 256 --staleness 2 --steps 10 --warmup 3
run n1_vgg16_easgd_bf16 300 python -u bench.py --model vgg16 --batch 64 --optimizer eamsgd --su 2 --steps 10 --warmup 3 --dtype bf16
run n1_vgg16_easgd_fp32 300 python -u bench.py --model vgg16 --batch 64 --optimizer eamsgd --su 2 --steps 10 --warmup 3
echo ALL OK

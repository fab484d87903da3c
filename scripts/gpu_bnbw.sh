#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/bnbw
timeout -k 10 180 python3 benchmarks/bn_bw_probe.py > gpurun_out/bnbw/probe.jsonl 2>&1 || { tail -20 gpurun_out/bnbw/probe.jsonl; exit 1; }
cat gpurun_out/bnbw/probe.jsonl

#!/bin/bash
# A/B of GEMM ring depths (MPIT_GEMM_STAGES) on ResNet-50 conv shapes at batch 256.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/gemm_ab.jsonl; : > $out
for st in 2; do
  for shp in "conv 256 14 14 256 256 3 1" "conv 256 7 7 512 512 3 1" "conv 256 28 28 128 128 3 1" "nt 50176 1024 256" "nt 12544 2048 512" "nt 50176 256 1024" "nt 200704 128 512" "nt 200704 512 128" "nt 802816 256 64" "nt 802816 128 128"; do
    MPIT_GEMM_STAGES=$st timeout -k 10 60 python3 benchmarks/gemm_probe.py $shp 50 | sed "s/^/{\"stages\": $st, \"r\": /; s/$/}/" >> $out || exit 1
  done
done
cat $out

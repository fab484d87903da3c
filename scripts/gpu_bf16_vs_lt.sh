#!/bin/bash
# bf16 GEMMs on the ResNet-50 shapes: hipBLASLt (torch.matmul) vs ours (gemm_nt / implicit-GEMM conv)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/bf16lt
mkdir -p $D
SH="4096 4096 4096 8192 8192 8192 802816 64 256 802816 256 64 50176 2048 512 200704 512 128 802816 64 576 50176 256 2304 12544 512 4608"
timeout -k 10 120 python3 benchmarks/mm_probe.py $SH > $D/hipblaslt_bf16.jsonl 2>&1 || { tail -5 $D/hipblaslt_bf16.jsonl; exit 1; }
: > $D/ours_bf16.jsonl
for a in "nt 4096 4096 4096" "nt 8192 8192 8192" "nt 802816 64 256" "nt 802816 256 64" "nt 50176 2048 512" \
         "nt 200704 512 128" "conv 256 56 56 64 64 3 1" "conv 256 14 14 256 256 3 1" "conv 256 7 7 512 512 3 1"; do
  timeout -k 10 60 python3 benchmarks/gemm_probe.py $a 20 >> $D/ours_bf16.jsonl || exit 1
done
cat $D/hipblaslt_bf16.jsonl $D/ours_bf16.jsonl

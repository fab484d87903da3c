#!/bin/bash
# (1) fp32 library reference: hipBLASLt fp32 (torch.matmul) vs our bf16x6 gemm_nt on the
#     ResNet-50 GEMM shapes (convs as their implicit-GEMM M x N x K);
# (2) stock PyTorch-ROCm ResNet-50 (MIOpen + SGD foreach), fp32 and bf16 autocast;
# (3) same-box A/B of the CU-reserved side stream (MPIT_SIDE_CU_RESERVE=0/16/32).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/stock
mkdir -p $D
if [ "$1" != "--skip-gemm" ]; then
SH="4096 4096 4096 8192 8192 8192 802816 64 256 802816 256 64 50176 2048 512 200704 512 128 802816 64 576 50176 256 2304 12544 512 4608"
timeout -k 10 120 python3 benchmarks/mm_probe.py --f32 $SH > $D/hipblaslt_f32.jsonl 2>&1 || { tail -5 $D/hipblaslt_f32.jsonl; exit 1; }
: > $D/ours_f32.jsonl
for a in "nt 4096 4096 4096" "nt 8192 8192 8192" "nt 802816 64 256" "nt 802816 256 64" "nt 50176 2048 512" \
         "nt 200704 512 128" "conv 256 56 56 64 64 3 1" "conv 256 14 14 256 256 3 1" "conv 256 7 7 512 512 3 1"; do
  timeout -k 10 60 python3 benchmarks/gemm_probe.py --f32 $a 20 >> $D/ours_f32.jsonl || exit 1
done
cat $D/hipblaslt_f32.jsonl $D/ours_f32.jsonl
fi
for dt in fp32 bf16; do
  timeout -k 10 400 python3 -u benchmarks/torch_stock_resnet50.py --dtype $dt > $D/stock_$dt.log 2>&1 || { tail -5 $D/stock_$dt.log; exit 1; }
  tail -1 $D/stock_$dt.log
done
for i in 1 2; do for r in 0 32; do
  MPIT_SIDE_CU_RESERVE=$r timeout -k 10 300 python3 -u bench.py > $D/b_${r}_$i.log 2>&1 || { tail -20 $D/b_${r}_$i.log; exit 1; }
  echo "reserve=$r run=$i $(tail -1 $D/b_${r}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["secondary"]["bf16_autocast"]["value"])')"
done; done
bash scripts/gpu_gemm_calls.sh

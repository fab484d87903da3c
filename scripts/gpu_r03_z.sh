#!/bin/bash
# Round 3 (session 2): fp32 GEMMs against hipBLASLt fp32 (torch.matmul) per ResNet-50 shape,
# bf16x6 (FM 9, weight planes) vs fp16x3 (FM 11); then the whole GPU tier.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03z
mkdir -p $O
SH="4096 4096 4096 8192 8192 8192 802816 64 256 802816 256 64 50176 2048 512 200704 512 128 802816 64 576 50176 256 2304 12544 512 4608"
timeout -k 10 120 python3 benchmarks/mm_probe.py --f32 $SH > $O/hipblaslt_f32.jsonl 2>&1 || { tail -5 $O/hipblaslt_f32.jsonl; exit 1; }
: > $O/ours.jsonl
for a in "nt 4096 4096 4096" "nt 8192 8192 8192" "nt 802816 64 256" "nt 802816 256 64" "nt 50176 2048 512" \
         "nt 200704 512 128" "conv 256 56 56 64 64 3 1" "conv 256 14 14 256 256 3 1" "conv 256 7 7 512 512 3 1" \
         "dgrad 256 14 14 256 256 3 1" "wgrad 256 14 14 256 256 3 1" "tn 50176 1024 256"; do
  for V in --bsplit --f16x3; do
    timeout -k 10 60 python3 benchmarks/gemm_probe.py --f32 $V $a 20 > $O/t.json 2> $O/t.err || { tail -5 $O/t.err; exit 1; }
    echo "{\"v\": \"$V\", \"r\": $(cat $O/t.json)}" >> $O/ours.jsonl
  done
done
cat $O/hipblaslt_f32.jsonl | grep -v amdgpu; cat $O/ours.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest_gpu.log | head; exit 1; }
echo ALL OK

#!/bin/bash
# fp32 MFMA GEMM / conv shape sweep (+ one PMC pass on the layer-3 3x3 forward)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/f32g
P=benchmarks/gemm_probe.py
: > gpurun_out/f32g/sweep.jsonl
for a in "nt 4096 4096 4096" "nt 8192 8192 8192" "nt 802816 64 256" "nt 802816 256 64" "nt 50176 2048 512" \
         "tn 802816 64 256" "tn 50176 512 2048" "tn 4096 4096 4096" \
         "conv 256 56 56 64 64 3 1" "conv 256 14 14 256 256 3 1" "conv 256 7 7 512 512 3 1" "conv 256 56 56 128 128 3 2" \
         "dgrad 256 56 56 64 64 3 1" "dgrad 256 14 14 256 256 3 1" \
         "wgrad 256 56 56 64 64 3 1" "wgrad 256 14 14 256 256 3 1" "wgrad 256 7 7 512 512 3 1"; do
  timeout -k 10 60 python3 $P --f32 $a 20 >> gpurun_out/f32g/sweep.jsonl || exit 1
done
cat gpurun_out/f32g/sweep.jsonl
Q="python3 $P --f32 conv 256 14 14 256 256 3 1 10"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --kernel-trace -d gpurun_out/f32g/p1 -o p1 --output-format csv -- $Q > gpurun_out/f32g/p1.log 2>&1 || { tail -5 gpurun_out/f32g/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum --kernel-trace -d gpurun_out/f32g/p2 -o p2 --output-format csv -- $Q > gpurun_out/f32g/p2.log 2>&1 || { tail -5 gpurun_out/f32g/p2.log; exit 1; }
echo pmc done

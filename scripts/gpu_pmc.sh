#!/bin/bash
# Counter passes over one compute-bound conv shape (layer3 3x3 of ResNet-50 at batch 256).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
P="python3 benchmarks/gemm_probe.py conv 256 14 14 256 256 3 1 20"
timeout -k 10 120 python3 benchmarks/gemm_probe.py conv 256 14 14 256 256 3 1 50 > gpurun_out/pmc/time.json || exit 1
cat gpurun_out/pmc/time.json
timeout -k 10 60 rocprofv3 -L > gpurun_out/pmc/avail.txt 2>&1 || echo "list failed"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU --kernel-trace -d gpurun_out/pmc/p1 -o p1 --output-format csv -- $P > gpurun_out/pmc/p1.log 2>&1 || { tail -5 gpurun_out/pmc/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum --kernel-trace -d gpurun_out/pmc/p2 -o p2 --output-format csv -- $P > gpurun_out/pmc/p2.log 2>&1 || { tail -5 gpurun_out/pmc/p2.log; exit 1; }
echo pmc done

#!/bin/bash
# Counter passes over the fp32 (bf16x6) GEMMs: a 3x3 conv forward, its wgrad, a 1x1 GEMM.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcf
i=0
for P in "conv 256 28 28 128 128 3 1" "wgrad 256 28 28 128 128 3 1" "nt 200704 512 128"; do
  i=$((i+1))
  timeout -k 10 120 python3 benchmarks/gemm_probe.py --f32 $P 20 > gpurun_out/pmcf/time$i.json || exit 1
  cat gpurun_out/pmcf/time$i.json
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU --kernel-trace -d gpurun_out/pmcf/a$i -o a --output-format csv -- python3 benchmarks/gemm_probe.py --f32 $P 5 > gpurun_out/pmcf/a$i.log 2>&1 || { tail -5 gpurun_out/pmcf/a$i.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmcf/b$i -o b --output-format csv -- python3 benchmarks/gemm_probe.py --f32 $P 5 > gpurun_out/pmcf/b$i.log 2>&1 || { tail -5 gpurun_out/pmcf/b$i.log; exit 1; }
done
echo pmc done

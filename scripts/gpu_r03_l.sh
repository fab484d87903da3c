#!/bin/bash
# Round 3: split-once wgrad with a 2-step prefetch — timing vs gemm_tn_kernel, and one PMC
# pass per arm on one shape (wave-cycle breakdown, LDS bank conflicts, MFMA busy).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03l
mkdir -p $O
: > $O/probe.jsonl
for P in "tn 200704 512 128" "tn 50176 1024 256" "tn 12544 512 2048" "wgrad 256 14 14 256 256 3 1"; do
  for V in 0 1; do
    MPIT_TN_F32S=$V timeout -k 10 120 python3 benchmarks/gemm_probe.py --f32 $P 20 > $O/t.json || exit 1
    echo "{\"f32s\": $V, \"r\": $(cat $O/t.json)}" >> $O/probe.jsonl
  done
done
cat $O/probe.jsonl
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_LDS"
for V in 0 1; do
  MPIT_TN_F32S=$V timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --stats -d $O/pmc$V -o p --output-format csv -- python3 benchmarks/gemm_probe.py --f32 tn 200704 512 128 5 > $O/pmc$V.log 2>&1 || { tail -20 $O/pmc$V.log; exit 1; }
done
bash scripts/gpu_r03_k.sh || exit 1

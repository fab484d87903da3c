#!/bin/bash
# A/B: weight-gradient GEMMs start before (default) or after (MPIT_WGRAD_AFTER=1) the input-
# gradient GEMM of the same convolution; then one PMC pass over the fp32 step (MFMA busy per kernel).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/wafter
mkdir -p $D
for i in 1 2; do for a in 0 1; do
  MPIT_WGRAD_AFTER=$a timeout -k 10 300 python3 -u bench.py > $D/b_${a}_$i.log 2>&1 || { tail -20 $D/b_${a}_$i.log; exit 1; }
  echo "after=$a run=$i $(tail -1 $D/b_${a}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["secondary"]["bf16_autocast"]["value"])')"
done; done
mkdir -p gpurun_out/pmc_f32
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES \
  -d gpurun_out/pmc_f32 -o pmc --output-format csv -- python3 bench.py --steps 3 --warmup 2 --no-secondary > gpurun_out/pmc_f32/bench.log 2>&1 || { tail -5 gpurun_out/pmc_f32/bench.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmc_f32/pmc_counter_collection.csv > gpurun_out/pmc_f32/mfma_util.md || exit 1
head -30 gpurun_out/pmc_f32/mfma_util.md

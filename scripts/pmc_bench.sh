#!/usr/bin/env bash
# One rocprofv3 --pmc pass over a short ResNet-50 bench, then a per-kernel MFMA table.
# Run on the GPU box:  gpurun --timeout 300 -- 'bash scripts/pmc_bench.sh'
# (counters only, no trace domains; one pass fits the SQ/GRBM counter limits)
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES \
  -d "$OUT" -o pmc --output-format csv -- python3 "$ROOT/bench.py" --steps 3 --warmup 2 > "$OUT/bench.log" 2>&1
python3 "$ROOT/scripts/pmc_summary.py" "$OUT/pmc_counter_collection.csv" > "$OUT/mfma_util.md"

#!/bin/bash
# bf16 step on the final tree: steady-state kernel table and one PMC MFMA pass
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/bf16final
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o p --output-format csv -- python3 bench.py --dtype bf16 --steps 6 --warmup 3 --no-secondary > $D/prof.log 2>&1 || { tail -20 $D/prof.log; exit 1; }
python3 scripts/prof_summary.py $D/prof $D/kernels.md > $D/ps.log 2>&1 || { tail -5 $D/ps.log; exit 1; }
python3 scripts/step_gaps.py $D/prof 2
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES -d $D/pmc -o pmc --output-format csv -- python3 bench.py --dtype bf16 --steps 3 --warmup 2 --no-secondary > $D/pmc.log 2>&1 || { tail -5 $D/pmc.log; exit 1; }
python3 scripts/pmc_summary.py $D/pmc/pmc_counter_collection.csv > $D/mfma_util.md || exit 1
head -14 $D/mfma_util.md
find $D -name "*.csv" -size +30M -delete

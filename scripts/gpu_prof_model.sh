#!/bin/bash
# Steady-state kernel profile of one bench configuration: bash scripts/gpu_prof_model.sh <name> <bench args...>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
name=$1; shift
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$name -o run -- python3 bench.py "$@" > gpurun_out/prof_$name.log 2>&1 || { tail -30 gpurun_out/prof_$name.log; exit 1; }
tail -1 gpurun_out/prof_$name.log

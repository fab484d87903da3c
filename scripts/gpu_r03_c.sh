#!/bin/bash
# Round 3: new GPU tests (clamp_scan kernel, BiCNN parity rule), per-process AccumulateGrad
# stream diagnostic.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels.py tests/test_apps.py -m gpu -k "clamp_scan or parity" -v --timeout 120 --timeout-method thread > $O/pytest_new.log 2>&1
rc=$?; tail -3 $O/pytest_new.log; [ $rc -ne 0 ] && { grep -E "^E " $O/pytest_new.log | head; exit 1; }
timeout -k 10 900 python -u benchmarks/diag_accgrad.py > $O/diag_accgrad.jsonl 2> $O/diag_accgrad.err || { tail -30 $O/diag_accgrad.err; exit 1; }
cat $O/diag_accgrad.jsonl
echo ALL OK

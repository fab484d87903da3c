#!/bin/bash
# fp32 training parity vs fp64 (mpit kernels and stock PyTorch): benchmark + GPU test
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/parity
mkdir -p $D
timeout -k 10 300 python3 -u -m pytest tests/test_fp32_path.py -m gpu -v -x -k "tracks_fp64" --timeout 250 --timeout-method thread > $D/pytest.log 2>&1; rc=$?
grep -E "passed|failed|PASS|FAIL" $D/pytest.log | tail -3; [ $rc -ne 0 ] && { tail -30 $D/pytest.log; exit $rc; }
timeout -k 10 500 python3 -u benchmarks/loss_parity.py --batch 16 --size 96 --steps 10 --out $D/parity.json > $D/parity.log 2>&1 || { tail -20 $D/parity.log; exit 1; }
python3 -c "import json; d=json.load(open('$D/parity.json')); print(d['step0_grad_rel_err'], d['step0_grad_worst_tensor_rel_err'], d['max_rel_loss_dev'])"

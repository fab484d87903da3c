#!/bin/bash
# fp32 gemm_nt change check: numerics, probes, bench x2 (TAG names the output dir).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=gpurun_out/${TAG:-f32check}
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_fp32_path.py -m gpu -q --timeout 120 --timeout-method thread > $D/pytest.log 2>&1; rc=$?
tail -1 $D/pytest.log; [ $rc -ge 124 ] && exit $rc
P=benchmarks/gemm_probe.py
: > $D/sweep.jsonl
for a in "nt 8192 8192 8192" "nt 802816 256 64" "nt 200704 512 128" "nt 50176 2048 512" \
         "conv 256 56 56 64 64 3 1" "conv 256 28 28 128 128 3 1" "conv 256 14 14 256 256 3 1" "dgrad 256 14 14 256 256 3 1"; do
  timeout -k 10 60 python3 $P --f32 $a 20 >> $D/sweep.jsonl || exit 1
done
cat $D/sweep.jsonl
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-secondary > $D/b_$i.log 2>&1 || { tail -20 $D/b_$i.log; exit 1; }
  tail -1 $D/b_$i.log | cut -c1-160
done

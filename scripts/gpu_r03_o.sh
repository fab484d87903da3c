#!/bin/bash
# Round 3: multi-segment apply tests + bandwidth; FM 10 (one accumulator + fragment
# prefetch) vs FM 9: fp32 numerics vs fp64, per-shape timing, bench A/B; split-once wgrad.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03o
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels.py tests/test_ps.py -m gpu -k "multi or batched" -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -12; [ $rc -ne 0 ] && { grep -E "^E " $O/pytest.log | head -20; exit 1; }
MPIT_F32_NT=acc1 timeout -k 10 500 python -u -m pytest tests/test_fp32_path.py -m gpu -k "vs_fp64 or within_2x or tracks_fp64" -v --timeout 300 --timeout-method thread > $O/pytest_acc1.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/pytest_acc1.log | tail -12; [ $rc -ne 0 ] && { grep -E "^E " $O/pytest_acc1.log | head -20; }
timeout -k 10 300 python3 -u benchmarks/ew_probe.py 25.6 3.2 0.8 > $O/ew.jsonl 2> $O/ew.err || { tail -20 $O/ew.err; exit 1; }
cat $O/ew.jsonl
: > $O/probe.jsonl
for P in "nt 50176 1024 512" "nt 200704 512 128" "conv 256 14 14 256 256 3 1" "conv 256 7 7 512 512 3 1" "dgrad 256 28 28 128 128 3 1"; do
  for V in fm9 acc1; do
    MPIT_F32_NT=$V timeout -k 10 120 python3 benchmarks/gemm_probe.py --f32 --bsplit $P 20 > $O/t.json || exit 1
    echo "{\"v\": \"$V\", \"r\": $(cat $O/t.json)}" >> $O/probe.jsonl
  done
done
for P in "tn 200704 512 128" "tn 50176 1024 256" "tn 12544 512 2048"; do
  for V in 0 1; do
    MPIT_TN_F32S=$V timeout -k 10 120 python3 benchmarks/gemm_probe.py --f32 $P 20 > $O/t.json || exit 1
    echo "{\"f32s\": $V, \"r\": $(cat $O/t.json)}" >> $O/probe.jsonl
  done
done
cat $O/probe.jsonl
timeout -k 10 300 python -u bench.py --no-secondary > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
echo "fm9 : $(tail -1 $O/bench.json | cut -c1-200)"
MPIT_F32_NT=acc1 timeout -k 10 300 python -u bench.py --no-secondary > $O/bench_acc1.json 2> $O/bench_acc1.err || { tail -30 $O/bench_acc1.err; exit 1; }
echo "acc1: $(tail -1 $O/bench_acc1.json | cut -c1-200)"
echo ALL OK

#!/bin/bash
# Round 3: multi-segment server apply (kernel test, batched server bitwise test, bandwidth of
# 8 x 3.2 M pieces one launch vs 8), split-once wgrad with the conflict-free image swizzle.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03n
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels.py tests/test_ps.py -m gpu -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -12; [ $rc -ne 0 ] && { grep -E "^E " $O/pytest.log | head -20; exit 1; }
timeout -k 10 300 python3 -u benchmarks/ew_probe.py 25.6 3.2 0.8 > $O/ew.jsonl 2> $O/ew.err || { tail -20 $O/ew.err; exit 1; }
cat $O/ew.jsonl
: > $O/probe.jsonl
for P in "tn 200704 512 128" "tn 50176 1024 256" "tn 12544 512 2048" "wgrad 256 14 14 256 256 3 1"; do
  for V in 0 1; do
    MPIT_TN_F32S=$V timeout -k 10 120 python3 benchmarks/gemm_probe.py --f32 $P 20 > $O/t.json || exit 1
    echo "{\"f32s\": $V, \"r\": $(cat $O/t.json)}" >> $O/probe.jsonl
  done
done
cat $O/probe.jsonl
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_LDS"
MPIT_TN_F32S=1 timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --stats -d $O/pmc1 -o p --output-format csv -- python3 benchmarks/gemm_probe.py --f32 tn 200704 512 128 5 > $O/pmc1.log 2>&1 || { tail -20 $O/pmc1.log; exit 1; }
echo ALL OK

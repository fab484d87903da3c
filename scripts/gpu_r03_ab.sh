#!/bin/bash
# Round 3 (session 2): split-once fp16x3 wgrad (MPIT_TN_F32S=1: each operand element scaled and
# split once into fp16 planes in LDS) vs the per-fragment split (default): bitwise-free numerics
# check, probes, same-box bench A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03ab
mkdir -p $O
MPIT_TN_F32S=1 timeout -k 10 300 python -u -m pytest tests/test_f16x3.py tests/test_fp32_path.py -m gpu -q --timeout 200 --timeout-method thread -k "tn or bottleneck or resnet50 or fp64" > $O/pytest_f32s.log 2>&1
rc=$?; tail -2 $O/pytest_f32s.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest_f32s.log | head; exit 1; }
: > $O/probe.jsonl
for a in "tn 50176 1024 256" "tn 200704 512 128" "tn 802816 256 64" "wgrad 256 14 14 256 256 3 1" "wgrad 256 28 28 128 128 3 1" "tn 12544 2048 512"; do
  for V in 0 1; do
    MPIT_TN_F32S=$V timeout -k 10 60 python3 benchmarks/gemm_probe.py --f32 --f16x3 $a 30 > $O/t.json 2> $O/t.err || { tail -5 $O/t.err; exit 1; }
    echo "{\"f32s\": $V, \"r\": $(cat $O/t.json)}" >> $O/probe.jsonl
  done
done
cat $O/probe.jsonl
b() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-secondary > $O/b_$n.json 2> $O/b_$n.err || { tail -20 $O/b_$n.err; return 1; }
  echo "$n: $(tail -1 $O/b_$n.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
b base MPIT_X=0 || exit 1
b f32s MPIT_TN_F32S=1 || exit 1
b base2 MPIT_X=0 || exit 1
b f32s2 MPIT_TN_F32S=1 || exit 1
echo ALL OK

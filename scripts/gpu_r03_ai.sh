#!/bin/bash
# Round 3 (session 2): fp16x3 NT kernel A/B on one box: 2-deep ring (2 blocks/CU, base) vs 3-deep
# (MPIT_F16X3_STAGES=3, 1 block/CU) vs s_setprio(1) around the MFMA burst (varso/prio.so) vs 128x64
# tiles (MPIT_F32_BN64=1).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03ai
mkdir -p $O
: > $O/ab.jsonl
run() {  # name, env..., then shapes from the list
  local V=$1; shift
  for a in "nt 4096 4096 4096" "nt 50176 2048 512" "nt 200704 512 128" "conv 256 14 14 256 256 3 1" "conv 256 7 7 512 512 3 1" \
           "conv 256 56 56 64 64 3 1" "dgrad 256 14 14 256 256 3 1"; do
    env "$@" timeout -k 10 60 python3 benchmarks/gemm_probe.py --f32 --f16x3 $a 20 > $O/t.json 2> $O/t.err || { tail -5 $O/t.err; return 1; }
    echo "{\"v\": \"$V\", \"a\": \"$a\", \"r\": $(cat $O/t.json)}" >> $O/ab.jsonl
  done
}
for rep in 1 2; do
  run base MPIT_NATIVE_SO=varso/base.so || exit 1
  run st3 MPIT_NATIVE_SO=varso/base.so MPIT_F16X3_STAGES=3 || exit 1
  run prio MPIT_NATIVE_SO=varso/prio.so || exit 1
  run bn64 MPIT_NATIVE_SO=varso/base.so MPIT_F32_BN64=1 || exit 1
done
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r03ai/ab.jsonl")]
t = collections.defaultdict(list)
for r in rows: t[(r["a"], r["v"])].append(r["r"]["tflops"])
vs = list(dict.fromkeys(r["v"] for r in rows))
print("shape | " + " | ".join(vs))
for a in dict.fromkeys(r["a"] for r in rows):
    print(a, "|", " | ".join(f"{max(t[(a, v)]):.1f}" for v in vs))
PY
timeout -k 10 500 python -u -m pytest tests/test_overlap.py -m gpu -q --timeout 450 --timeout-method thread > $O/overlap.log 2>&1
rc=$?; tail -2 $O/overlap.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|DIFF" $O/overlap.log | head; exit 1; }
echo ALL OK

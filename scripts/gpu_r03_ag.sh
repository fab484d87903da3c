#!/bin/bash
# Round 3 (session 2): scalar f32 split (v_fma_mix, no v_pk_*_f32; gemm.hip built with
# -fno-slp-vectorize): numerics, per-shape fp16x3 GEMM TF (vs gemm_fp32_vs_hipblaslt_r03.md), bench x2.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03ag
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_f16x3.py tests/test_fp32_path.py -m gpu -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest.log | head; exit 1; }
: > $O/ours.jsonl
for a in "nt 4096 4096 4096" "nt 802816 64 256" "nt 802816 256 64" "nt 50176 2048 512" \
         "nt 200704 512 128" "conv 256 56 56 64 64 3 1" "conv 256 14 14 256 256 3 1" "conv 256 7 7 512 512 3 1" \
         "dgrad 256 14 14 256 256 3 1" "wgrad 256 14 14 256 256 3 1" "tn 50176 1024 256"; do
  timeout -k 10 60 python3 benchmarks/gemm_probe.py --f32 --f16x3 $a 20 > $O/t.json 2> $O/t.err || { tail -5 $O/t.err; exit 1; }
  echo "{\"a\": \"$a\", \"r\": $(cat $O/t.json)}" >> $O/ours.jsonl
done
cat $O/ours.jsonl
for i in 1 2; do
  timeout -k 10 300 python -u bench.py > $O/bench_$i.json 2> $O/bench_$i.err || { tail -30 $O/bench_$i.err; exit 1; }
  echo "bench $i: $(tail -1 $O/bench_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["secondary"]["bf16_autocast"]["value"])')"
done
echo ALL OK

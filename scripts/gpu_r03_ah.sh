#!/bin/bash
# Round 3 (session 2): fp32 split A/B on one box — HEAD split (v_pk f32) vs scalar split (v_fma_mix),
# each with and without -fno-slp-vectorize on gemm.hip (variant modules under varso/, MPIT_NATIVE_SO).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03ah
mkdir -p $O
: > $O/ab.jsonl
for rep in 1 2; do
for V in base scal_noslp base_noslp scal_slp; do
  for a in "nt 4096 4096 4096" "nt 50176 2048 512" "conv 256 14 14 256 256 3 1" "conv 256 56 56 64 64 3 1" \
           "dgrad 256 14 14 256 256 3 1" "wgrad 256 14 14 256 256 3 1" "tn 50176 1024 256"; do
    MPIT_NATIVE_SO=varso/$V.so timeout -k 10 60 python3 benchmarks/gemm_probe.py --f32 --f16x3 $a 20 > $O/t.json 2> $O/t.err || { tail -5 $O/t.err; exit 1; }
    echo "{\"v\": \"$V\", \"rep\": $rep, \"a\": \"$a\", \"r\": $(cat $O/t.json)}" >> $O/ab.jsonl
  done
done
done
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r03ah/ab.jsonl")]
t = collections.defaultdict(list)
for r in rows: t[(r["a"], r["v"])].append(r["r"]["tflops"])
vs = ["base", "scal_noslp", "base_noslp", "scal_slp"]
print("shape | " + " | ".join(vs))
for a in dict.fromkeys(r["a"] for r in rows):
    print(a, "|", " | ".join(f"{max(t[(a, v)]):.1f}" for v in vs))
PY
for V in base scal_noslp; do
  MPIT_NATIVE_SO=varso/$V.so timeout -k 10 300 python -u bench.py --no-secondary > $O/bench_$V.json 2> $O/bench_$V.err || { tail -30 $O/bench_$V.err; exit 1; }
  echo "bench $V: $(tail -1 $O/bench_$V.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
echo ALL OK

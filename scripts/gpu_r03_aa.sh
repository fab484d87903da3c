#!/bin/bash
# Round 3 (session 2): prefetch-all k-tiles for short-K GEMMs (MPIT_GEMM_PREFETCH_ALL) and the
# in-kernel wgrad split reduction (MPIT_TN_FUSED) on the fp16x3 kernels: numerics, same-box
# bench A/B, short-K probes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03aa
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_f16x3.py tests/test_fp32_path.py tests/test_resnet_fused.py -m gpu -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest.log | head; exit 1; }
b() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-secondary > $O/b_$n.json 2> $O/b_$n.err || { tail -20 $O/b_$n.err; return 1; }
  echo "$n: $(tail -1 $O/b_$n.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
b base MPIT_X=0 || exit 1
b nopall MPIT_GEMM_PREFETCH_ALL=0 || exit 1
b tnfused MPIT_TN_FUSED=1 || exit 1
b base2 MPIT_X=0 || exit 1
b nopall2 MPIT_GEMM_PREFETCH_ALL=0 || exit 1
b tnfused2 MPIT_TN_FUSED=1 || exit 1
: > $O/probe.jsonl
for a in "nt 802816 256 64" "nt 200704 512 128" "nt 802816 256 128" "nt 802816 64 64"; do
  for V in pall nopall bn64; do
    E="MPIT_X=0"; [ $V = nopall ] && E="MPIT_GEMM_PREFETCH_ALL=0"; [ $V = bn64 ] && E="MPIT_F32_BN64=1"
    env $E timeout -k 10 60 python3 benchmarks/gemm_probe.py --f32 --f16x3 $a 50 > $O/t.json 2> $O/t.err || { tail -5 $O/t.err; exit 1; }
    echo "{\"v\": \"$V\", \"r\": $(cat $O/t.json)}" >> $O/probe.jsonl
  done
done
cat $O/probe.jsonl
echo ALL OK

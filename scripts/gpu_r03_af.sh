#!/bin/bash
# Round 3 (session 2): stem input bound cached on the (unchanged) batch; numerics + bench x2;
# fp32 GEMM accuracy per ResNet-50 shape (torch fp32 / bf16x6 / fp16x3 vs fp64) and the
# ResNet-50 training parity through the weight plan, fp16x3 and bf16x6.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03af
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_f16x3.py tests/test_fp32_path.py -m gpu -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest.log | head; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py > $O/bench_$i.json 2> $O/bench_$i.err || { tail -30 $O/bench_$i.err; exit 1; }
  echo "bench $i: $(tail -1 $O/bench_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["secondary"]["bf16_autocast"]["value"])')"
done
timeout -k 10 300 python -u benchmarks/split_accuracy.py > $O/split_accuracy.jsonl 2> $O/split_accuracy.err || { tail -20 $O/split_accuracy.err; exit 1; }
cat $O/split_accuracy.jsonl
timeout -k 10 600 python -u benchmarks/loss_parity.py --batch 16 --size 96 --steps 2 --out $O/parity_f16x3.json > $O/parity_f16x3.log 2>&1 || { tail -20 $O/parity_f16x3.log; exit 1; }
MPIT_F32_SPLIT=bf16x6 timeout -k 10 600 python -u benchmarks/loss_parity.py --batch 16 --size 96 --steps 2 --out $O/parity_bf16x6.json > $O/parity_bf16x6.log 2>&1 || { tail -20 $O/parity_bf16x6.log; exit 1; }
python3 -c "
import json
for m in ('f16x3', 'bf16x6'):
    d = json.load(open('$O/parity_' + m + '.json'))
    print(m, d['split'], 'grad0', d['step0_grad_rel_err'], 'worst', d['step0_grad_worst_tensor_rel_err'], 'loss0', d['loss_fp64_cpu'][0], d['loss_mpit_fp32'][0], d['loss_stock_fp32'][0])
"
echo ALL OK

#!/bin/bash
# Round 3 (session 2): the stem on fp16x3 (row-tap GEMM on 32-deep tiles with fp16 weight planes,
# fp16x3 wgrad) — numerics, bench, stream table; MFMA utilisation PMC pass of the fp16x3 step;
# a 2-rank bench on the one GPU (the N > 1 path); whole GPU tier.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03ac
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_f16x3.py tests/test_fp32_path.py -m gpu -q --timeout 200 --timeout-method thread > $O/pytest_f16.log 2>&1
rc=$?; tail -2 $O/pytest_f16.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest_f16.log | head; exit 1; }
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
echo "bench: $(tail -1 $O/bench.json | cut -c1-230)"
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o t --output-format csv -- python3 bench.py --steps 4 --warmup 3 --no-secondary > $O/prof.log 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
python3 scripts/stream_summary.py $O/prof $O/streams.md cast_batch_kernel 3 || exit 1
find $O/prof -name "*kernel_trace.csv" -size +40M -delete
grep -E "step wall|stem|gemm_nt_kernel<float, 128, 64, 2, 1, true|gemm_tn_kernel<float, 64, 64" $O/streams.md | head
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES -d $O/pmc -o pmc --output-format csv -- python3 bench.py --steps 3 --warmup 2 --no-secondary > $O/pmc.log 2>&1 || { tail -10 $O/pmc.log; exit 1; }
python3 scripts/pmc_summary.py $(find $O/pmc -name "pmc_counter_collection.csv" | head -1) > $O/mfma_util.md || exit 1
head -16 $O/mfma_util.md
find $O/pmc -name "*.csv" -size +20M -delete
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 6 --warmup 3 > $O/bench_n2.json 2> $O/bench_n2.err || { tail -30 $O/bench_n2.err; exit 1; }
echo "n2: $(tail -1 $O/bench_n2.json | cut -c1-400)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest_gpu.log | head; exit 1; }
echo ALL OK

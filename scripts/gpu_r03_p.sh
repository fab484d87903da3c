#!/bin/bash
# Round 3: 3-rank one-GPU API suite (HBM ring all-reduce), fp32 step MFMA utilisation per
# kernel (PMC), bf16 ResNet-50 per-stream trace, VGG-16 bf16 operator table.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03p
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_api.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_api.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/pytest_api.log | tail -6; [ $rc -ne 0 ] && { grep -E "^E " $O/pytest_api.log | head -20; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES -d $O/pmc -o pmc --output-format csv -- python3 bench.py --steps 3 --warmup 2 --no-secondary > $O/pmc_bench.log 2>&1 || { tail -20 $O/pmc_bench.log; exit 1; }
python3 scripts/pmc_summary.py $(find $O/pmc -name "pmc_counter_collection.csv" | head -1) > $O/mfma_util.md || exit 1
head -20 $O/mfma_util.md
find $O/pmc -name "*.csv" -size +40M -delete
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/profb -o t --output-format csv -- python3 bench.py --steps 6 --warmup 3 --no-secondary --dtype bf16 > $O/profb.log 2>&1 || { tail -20 $O/profb.log; exit 1; }
python3 scripts/stream_summary.py $O/profb $O/streams_bf16.md cast_batch_kernel 3 || exit 1
head -40 $O/streams_bf16.md
find $O/profb -name "*kernel_trace.csv" -size +40M -delete
timeout -k 10 300 python3 -u benchmarks/op_profile.py --model vgg16 --batch 64 --optimizer eamsgd --su 2 --dtype bf16 > $O/vgg_ops.txt 2> $O/vgg_ops.err || { tail -20 $O/vgg_ops.err; exit 1; }
head -60 $O/vgg_ops.txt
echo ALL OK

#!/bin/bash
# Round 3: VGG-16 bf16 — per-layer kernels vs MIOpen, and a per-stream trace of the EASGD step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03k
mkdir -p $O
timeout -k 10 300 python3 -u benchmarks/vgg_layers.py 64 bf16 > $O/vgg_layers_bf16.jsonl 2> $O/vgg_layers.err || { tail -20 $O/vgg_layers.err; exit 1; }
cat $O/vgg_layers_bf16.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o t --output-format csv -- python3 bench.py --no-secondary --model vgg16 --batch 64 --optimizer eamsgd --su 2 --steps 6 --warmup 3 --dtype bf16 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 scripts/stream_summary.py $O/prof $O/streams.md cast_batch_kernel 4 || exit 1
find $O/prof -name "*kernel_trace.csv" -size +40M -delete
echo ALL OK

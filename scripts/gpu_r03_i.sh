#!/bin/bash
# Round 3: VGG / AlexNet conv layers on the weight plan — bitwise test, then the BASELINE
# config lines at N=1 (VGG-16 EASGD bf16 / fp32, AlexNet Downpour + SSP).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03i
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_fp32_path.py -m gpu -k "convact or presplit" -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -6; [ $rc -ne 0 ] && { grep -E "^E " $O/pytest.log | head; exit 1; }
run() {  # name args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py --no-secondary "$@" > $O/$name.json 2> $O/$name.err || { tail -20 $O/$name.err; exit 1; }
  echo "$name: $(tail -1 $O/$name.json | cut -c1-230)"
}
run vgg16_easgd_bf16 --model vgg16 --batch 64 --optimizer eamsgd --su 2 --steps 10 --warmup 3 --dtype bf16
run vgg16_easgd_fp32 --model vgg16 --batch 64 --optimizer eamsgd --su 2 --steps 10 --warmup 3
run alexnet_ssp --model alexnet --batch 256 --staleness 2 --steps 10 --warmup 3
run resnet50_bf16 --dtype bf16 --steps 20 --warmup 5
run resnet50_allreduce --optimizer allreduce --steps 10 --warmup 3
echo ALL OK

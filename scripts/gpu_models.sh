set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u -m pytest tests/test_gemm.py tests/test_pool.py tests/test_resnet_fused.py -m gpu -x -q --timeout 60 --timeout-method thread > gpurun_out/tg.log 2>&1 || { tail -30 gpurun_out/tg.log; exit 1; }
tail -2 gpurun_out/tg.log
timeout -k 10 200 python -u bench.py --model vgg16 --batch 64 --optimizer eamsgd --su 2 --steps 10 --warmup 3 > gpurun_out/vgg.json 2>gpurun_out/vgg.err || { tail -20 gpurun_out/vgg.err; exit 1; }
cat gpurun_out/vgg.json
timeout -k 10 200 python -u bench.py --model alexnet --batch 256 --staleness 2 --steps 10 --warmup 3 > gpurun_out/alex.json 2>gpurun_out/alex.err || { tail -20 gpurun_out/alex.err; exit 1; }
cat gpurun_out/alex.json

#!/bin/bash
# split-group split-K reduce: gemm / conv / stem tests, then ResNet-50 and GoogLeNet A/B (DLA_SPLITK_SG)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_conv3x3.py tests/test_gpu_stem.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3n_tests.log 2>&1 || { grep -E "Error|assert|FAIL" gpurun_out/r3n_tests.log | head; tail -20 gpurun_out/r3n_tests.log; exit 1; }
tail -1 gpurun_out/r3n_tests.log
for sg in 1 0 1 0; do
  DLA_SPLITK_SG=$sg timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/r3n_b.log 2>&1 && echo "resnet sg=$sg $(grep -o '"value": [0-9.]*' gpurun_out/r3n_b.log | head -1)"
  DLA_SPLITK_SG=$sg timeout -k 10 300 python bench.py --model googlenet --batch 128 --graph on --steps 30 --warmup 10 > gpurun_out/r3n_g.log 2>&1 && echo "gnet sg=$sg $(grep -o '"value": [0-9.]*' gpurun_out/r3n_g.log | head -1)"
done

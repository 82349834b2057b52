#!/bin/bash
# split-K gemm_nt for the fully connected heads: tests, then GoogLeNet / ResNet-50 A/B (DLA_GEMM_SPLITK)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_linear.py tests/test_gpu_inception.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3p_tests.log 2>&1 || { grep -E "Error|assert|FAIL" gpurun_out/r3p_tests.log | head; tail -20 gpurun_out/r3p_tests.log; exit 1; }
tail -1 gpurun_out/r3p_tests.log
for v in 1 0 1 0; do
  DLA_GEMM_SPLITK=$v timeout -k 10 300 python bench.py --model googlenet --batch 128 --graph on --steps 30 --warmup 10 > gpurun_out/r3p_g.log 2>&1 && echo "gnet splitk=$v $(grep -o '"value": [0-9.]*' gpurun_out/r3p_g.log | head -1)"
done
for v in 1 0; do
  DLA_GEMM_SPLITK=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/r3p_b.log 2>&1 && echo "resnet splitk=$v $(grep -o '"value": [0-9.]*' gpurun_out/r3p_b.log | head -1)"
done

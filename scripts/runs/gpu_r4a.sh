#!/bin/bash
# dgrad BN epilogue reading a strided BN input (reduction-branch links restored in the fused fan-in)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_inception.py tests/test_gpu_conv3x3.py tests/test_gpu_bn_epilogue.py tests/test_gpu_gemm.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4a_tests.log 2>&1 || { grep -E "Error|assert|FAIL" gpurun_out/r4a_tests.log | head -20; tail -20 gpurun_out/r4a_tests.log; exit 1; }
tail -1 gpurun_out/r4a_tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --model googlenet --batch 128 --graph on --steps 30 --warmup 10 > gpurun_out/r4a_g.log 2>&1 && echo "gnet $(grep -o '"value": [0-9.]*' gpurun_out/r4a_g.log | head -1)"
done

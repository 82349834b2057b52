#!/bin/bash
# grouped BN for the two reduction branches too (separate outputs, dgrad-epilogue partials): tests, GoogLeNet A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_inception.py tests/test_gpu_bn_act.py tests/test_gpu_model_parity.py tests/test_gpu_graph.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3s_tests.log 2>&1 || { grep -E "Error|assert|FAIL" gpurun_out/r3s_tests.log | head; tail -20 gpurun_out/r3s_tests.log; exit 1; }
tail -1 gpurun_out/r3s_tests.log
for v in 1 0 1 0; do
  DLA_BN_GROUPED=$v timeout -k 10 300 python bench.py --model googlenet --batch 128 --graph on --steps 30 --warmup 10 > gpurun_out/r3s_g.log 2>&1 && echo "gnet grouped=$v $(grep -o '"value": [0-9.]*' gpurun_out/r3s_g.log | head -1)"
done
DLA_BN_GROUPED=1 timeout -k 10 300 python bench.py --model googlenet --batch 512 --steps 20 --warmup 5 > gpurun_out/r3s_g512.log 2>&1 && echo "gnet512 grouped $(grep -o '"value": [0-9.]*' gpurun_out/r3s_g512.log | head -1)"

#!/bin/bash
# fused Inception fan-in (one GEMM for the three 1x1 convs, strided grouped BN, shared dY buffer): tests + A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_inception.py tests/test_gpu_model_parity.py tests/test_gpu_graph.py tests/test_gpu_bn_act.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3y_tests.log 2>&1 || { grep -E "Error|assert|FAIL" gpurun_out/r3y_tests.log | head -20; tail -30 gpurun_out/r3y_tests.log; exit 1; }
tail -1 gpurun_out/r3y_tests.log
for v in 1 0 1 0; do
  DLA_FANIN_CAT=$v timeout -k 10 300 python bench.py --model googlenet --batch 128 --graph on --steps 30 --warmup 10 > gpurun_out/r3y_g.log 2>&1 && echo "gnet cat=$v $(grep -o '"value": [0-9.]*' gpurun_out/r3y_g.log | head -1)"
done
for v in 1 0; do
  DLA_FANIN_CAT=$v timeout -k 10 300 python bench.py --model googlenet --batch 512 --steps 20 --warmup 5 > gpurun_out/r3y_g512.log 2>&1 && echo "gnet512 cat=$v $(grep -o '"value": [0-9.]*' gpurun_out/r3y_g512.log | head -1)"
done

#!/bin/bash
# persistent short-K gemm_nt: tests + per-layer fwd/dgrad A/B + whole step A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_conv.py tests/test_gpu_bn_epilogue.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2s_tests.log 2>&1 || { echo "tests failed"; grep -E "Error|assert|FAIL" gpurun_out/r2s_tests.log | head; tail -20 gpurun_out/r2s_tests.log; exit 1; }
tail -1 gpurun_out/r2s_tests.log
for x in 0 1 0 1; do
  DLA_GEMM_PERSIST=$x timeout -k 10 300 python scripts/bench_layers.py --only fwd,dgrad --out gpurun_out/r2s_layers_p$x.jsonl > gpurun_out/r2s_layers_p$x.log 2>&1 || { tail -20 gpurun_out/r2s_layers_p$x.log; exit 1; }
  echo "persist=$x"; grep -A8 "conv time" gpurun_out/r2s_layers_p$x.log | grep 1x1
done
for x in 0 1 0 1; do
  DLA_GEMM_PERSIST=$x timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2s_bench_p$x.log 2>&1 && echo "persist=$x $(grep -o '"value": [0-9.]*' gpurun_out/r2s_bench_p$x.log | head -1)"
done

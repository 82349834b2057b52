#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2u_tests.log 2>&1 || { tail -20 gpurun_out/r2u_tests.log; exit 1; }
tail -1 gpurun_out/r2u_tests.log
timeout -k 10 300 python scripts/bench_layers.py --only fwd,dgrad --out gpurun_out/r2u_layers.jsonl > gpurun_out/r2u_layers.log 2>&1 && grep -A8 "conv time" gpurun_out/r2u_layers.log | grep 1x1
for i in 1 2 3; do timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2u_bench$i.log 2>&1 && grep -o '"value": [0-9.]*' gpurun_out/r2u_bench$i.log | head -1; done

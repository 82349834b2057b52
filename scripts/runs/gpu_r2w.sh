#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv3x3.py tests/test_gpu_conv3x3_autograd.py tests/test_gpu_race.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2w_tests.log 2>&1 || { grep -E "Error|assert|FAIL" gpurun_out/r2w_tests.log | head; tail -20 gpurun_out/r2w_tests.log; exit 1; }
tail -1 gpurun_out/r2w_tests.log
timeout -k 10 300 python scripts/bench_layers.py --out gpurun_out/r2w_layers.jsonl > gpurun_out/r2w_layers.log 2>&1 && grep -A8 "conv time" gpurun_out/r2w_layers.log
for i in 1 2 3; do timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2w_bench$i.log 2>&1 && grep -o '"value": [0-9.]*' gpurun_out/r2w_bench$i.log | head -1; done

#!/bin/bash
# split-K wgrad grids: XCD-aware tile order A/B (per-layer wgrad + whole step)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv3x3.py tests/test_gpu_gemm.py tests/test_gpu_stem.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2r_tests.log 2>&1 || { echo "tests failed"; grep -E "Error|assert|FAIL" gpurun_out/r2r_tests.log | head; tail -20 gpurun_out/r2r_tests.log; exit 1; }
tail -1 gpurun_out/r2r_tests.log
for x in 0 1 0 1; do
  DLA_SPLITK_XCD=$x timeout -k 10 300 python scripts/bench_layers.py --only wgrad --out gpurun_out/r2r_wgrad_x$x.jsonl > gpurun_out/r2r_wgrad_x$x.log 2>&1 || { tail -20 gpurun_out/r2r_wgrad_x$x.log; exit 1; }
  echo "xcd=$x"; grep -A8 "conv time" gpurun_out/r2r_wgrad_x$x.log
done
for x in 0 1; do
  DLA_SPLITK_XCD=$x timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2r_bench_x$x.log 2>&1 && echo "xcd=$x $(grep -o '"value": [0-9.]*' gpurun_out/r2r_bench_x$x.log | head -1)"
done

#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pool.py tests/test_gpu_stem.py tests/test_gpu_model_parity.py tests/test_gpu_inception.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3h_tests.log 2>&1 || { grep -E "Error|assert|FAIL" gpurun_out/r3h_tests.log | head; tail -20 gpurun_out/r3h_tests.log; exit 1; }
tail -1 gpurun_out/r3h_tests.log
bash scripts/gpu_bench_prof.sh r3h_gnet --model googlenet --batch 128 --graph on || exit 1
grep -E "GPU wall|quad|PoolDy" gpurun_out/ksum_r3h_gnet.md | head
grep metric gpurun_out/bench_r3h_gnet.log | grep -o '"value": [0-9.]*' | head -1

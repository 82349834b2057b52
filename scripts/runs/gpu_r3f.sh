#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pool.py tests/test_gpu_stem.py tests/test_gpu_bn_act.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3f_tests.log 2>&1 || { grep -E "Error|assert|FAIL" gpurun_out/r3f_tests.log | head; tail -20 gpurun_out/r3f_tests.log; exit 1; }
tail -1 gpurun_out/r3f_tests.log
bash scripts/gpu_bench_prof.sh r3f || exit 1
grep -E "GPU wall|PoolDy|maxpool" gpurun_out/ksum_r3f.md | head
grep metric gpurun_out/bench_r3f.log | grep -o '"value": [0-9.]*'

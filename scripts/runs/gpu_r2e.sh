#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_conv3x3.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2e_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r2e_tests.log; exit 1; }
tail -2 gpurun_out/r2e_tests.log
timeout -k 10 300 python -u scripts/bench_tiles_r2.py > gpurun_out/r2e_tiles.log 2>&1; echo "tiles rc=$?"; tail -9 gpurun_out/r2e_tiles.log
timeout -k 10 300 python -u scripts/bench_layers.py --pipe 4 --out gpurun_out/layers_r2e_p4.jsonl > gpurun_out/layers_r2e_p4.log 2>&1; echo "layers rc=$?"; tail -8 gpurun_out/layers_r2e_p4.log

#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_engine_vranks.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2j_dp.log 2>&1 || { echo "dp tests failed"; tail -40 gpurun_out/r2j_dp.log; exit 1; }
tail -1 gpurun_out/r2j_dp.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --force_comm 1 > gpurun_out/r2j_force.log 2>&1 && grep -o '"value": [0-9.]*\|"allreduce_ms_per_step": [0-9.]*' gpurun_out/r2j_force.log

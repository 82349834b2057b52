#!/bin/bash
# halo dgrad default (DLA_HALO=1), forward opt-in: conv tests, then the full GPU suite + smoke + bench
set -o pipefail
mkdir -p gpurun_out/r5i
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv3x3.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5i/conv_tests.log 2>&1 || { tail -40 gpurun_out/r5i/conv_tests.log; exit 1; }
tail -1 gpurun_out/r5i/conv_tests.log
bash scripts/gpu_full.sh

#!/bin/bash
# Round 4, call g14: the new hand-off / graph tests, then per-kernel HBM bytes of the final bs1280 step
# (two single-counter rocprofv3 --pmc passes, scripts/gpu_pmc_bench.sh) for the r3 g42 comparison
set -o pipefail
O=gpurun_out/g14
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_gemm_dual.py tests/test_gpu_graph.py \
  > $O/pytest.log 2>&1 || exit 1
timeout -k 10 700 bash scripts/gpu_pmc_bench.sh > $O/pmc.log 2>&1 || exit 1

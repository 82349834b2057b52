#!/bin/bash
# full GPU suite + smoke + default bench (what the driver runs at round end)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full_gpu.log 2>&1 || { echo "GPU suite failed"; grep -E "Error|assert|FAIL|failed" gpurun_out/full_gpu.log | head -20; tail -30 gpurun_out/full_gpu.log; exit 1; }
tail -2 gpurun_out/full_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/full_smoke.log; exit 1; }
tail -3 gpurun_out/full_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/full_bench.log 2>&1 && grep metric gpurun_out/full_bench.log | cut -c1-300
